#!/usr/bin/env python3
"""Is batch assembly bound by its longest column?  Times the batch assembly kernel (one wave per column) on
(a) the tile holding the bench batch's largest geometry column plus enough small tiles to take the batch path
(> 4096 columns), (b) the small tiles alone, (c) the config-5 batch.  usage: asm_longpole.py [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def timed(covt, tiles, reps):
    import torch

    plan = covt.Plan.from_tiles(tiles)
    b = covt.DeviceBatch(plan, "cuda")
    s = torch.cuda.current_stream()
    b.decode(s)
    b.assemble(s)
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        b.assemble(s)
        e1.record(s)
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1))
    return float(np.median(t)), plan.num_geometry_columns


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    covt = bench.load_covt()
    lib = bench.tile_library()
    tiles = [t for z in lib.values() for _, t in z]
    coords = []
    for t in tiles:
        p = covt.Plan.from_tiles([t])
        n = p.num_geometry_columns
        rec = np.frombuffer(p.gdescs, dtype=np.uint8).reshape(n, -1) if n else np.zeros((0, 160), np.uint8)
        caps = rec[:, 144:156].copy().view(np.int32).reshape(n, 3)
        coords.append(int(caps[:, 2].max()) if n else 0)
    big = tiles[int(np.argmax(coords))]
    small = [t for t, c in sorted(zip(tiles, coords), key=lambda x: x[1])[:40]]
    filler = (small * 200)[:1200]
    ms_big, nb = timed(covt, [big] + filler, reps)
    ms_small, ns = timed(covt, filler, reps)
    print("largest column's tile (%d coords) + %d small tiles: %d columns, assembly %.3f ms" % (max(coords), len(filler), nb, ms_big))
    print("the small tiles alone: %d columns, assembly %.3f ms" % (ns, ms_small))
    picks = bench.sample_batch(lib, 10000, bench.SEED)
    ms_all, na = timed(covt, [t for _, t in picks], reps)
    print("config-5 batch: %d columns, assembly %.3f ms" % (na, ms_all))


if __name__ == "__main__":
    main()
