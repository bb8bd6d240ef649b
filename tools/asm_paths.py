#!/usr/bin/env python3
"""Which pass-4 path the config-5 batch's coordinates take (covt_assemble.hip): a column whose rings get
no closing vertex copies (or, ICE, gathers) source vertex v into coordinate v; the others expand ring
offsets per coordinate.  Decodes and assembles the batch once, then splits the coordinates by path and by
ICE / plain vertex buffers.  usage: asm_paths.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    import torch

    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    b = covt.DeviceBatch(plan, "cuda")
    b.decode()
    b.assemble()
    torch.cuda.synchronize()
    _, g = b.assembly_results()
    gi = plan.geom
    st = plan.streams
    ok = g["status"] == 0
    coords = g["num_coords"].astype(np.int64)
    ice = gi["stream"][:, 4] >= 0
    vb = gi["stream"][:, 5]
    # source vertices: ICE -> vertexOffsets entries, else vertexBuffer values / 2 (x, y)
    src = np.where(ice, st["num_values"][np.maximum(gi["stream"][:, 4], 0)],
                   st["num_values"][np.maximum(vb, 0)] // 2).astype(np.int64)
    src = np.where(vb >= 0, src, 0)
    copy = ok & (coords == src)
    expand = ok & (coords != src)
    tot = coords[ok].sum()
    print("columns %d (ok %d), coordinates %d" % (len(g), int(ok.sum()), int(tot)))
    for name, m in (("copy / gather (no closing vertex)", copy), ("ring expansion (closing vertices)", expand)):
        for kind, k in (("plain", ~ice), ("ICE", ice)):
            mm = m & k
            print("  %-36s %-5s columns %6d  coordinates %11d  (%.1f %%)" % (name, kind, int(mm.sum()),
                                                                          int(coords[mm].sum()),
                                                                          100.0 * coords[mm].sum() / max(tot, 1)))


if __name__ == "__main__":
    main()
