#!/usr/bin/env python3
"""Debug aid: the synthetic assembly columns of tests/test_gpu_assembly.py (seed 1), first mismatch per column
against the oracle, printed with the column's shape.  usage: asm_debug.py [seed]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import covt_asm as A  # noqa: E402


def main():
    import torch
    import oracle as O

    covt = bench.load_covt()
    O.build()
    orc = O
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    rng = np.random.default_rng(seed)
    cols = []
    for i in range(48):
        big = i % 8 == 7
        n = int(rng.choice([1, 2, 5, 8])) if big else int(rng.choice([0, 1, 5, 63, 64, 65, 200, 1000, 5000]))
        cols.append(A.synth_column(rng, n, ice=bool(i & 1), closed=bool(i & 2), big=big))
    dec, desc, asm_bytes, lay = A.pack_columns(covt, cols)
    dev = torch.device("cuda:0")
    d_dec = torch.from_numpy(dec).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    d_asm = torch.full((asm_bytes,), 0x5A, dtype=torch.uint8, device=dev)
    d_gres = torch.zeros(4 * len(cols), dtype=torch.int32, device=dev)
    d_res = torch.zeros(2, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    st = covt.lib().covt_assemble_geometry_device(d_dec.data_ptr(), d_res.data_ptr(), d_desc.data_ptr(), len(cols),
                                                  d_asm.data_ptr(), d_gres.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    asm, gres = d_asm.cpu().numpy(), d_gres.cpu().numpy().view(covt.GEOM_RESULT_DTYPE)
    for ci, col in enumerate(cols):
        o = orc.assemble_geometry(col["types"], col["go"], col["po"], col["ro"], col["vo"], col["vb"], col["closed"],
                                  A.caps(col))
        g = A.unpack_column(asm, lay[ci], col["types"].size, gres[ci])
        if g[0] != o[0]:
            print(ci, "status", g[0], o[0])
            continue
        if o[0]:
            continue
        for k, name in ((1, "geo"), (2, "part"), (3, "ring"), (4, "coords")):
            a, b = np.asarray(g[k]), np.asarray(o[k])
            if a.shape != b.shape or not np.array_equal(a, b):
                bad = np.nonzero(a.ravel()[:b.size] != b.ravel()[:a.size])[0] if a.size and b.size else []
                print("col %d n=%d %s: sizes %d/%d, %d bad, first %s; got %s want %s" % (
                    ci, col["types"].size, name, a.size, b.size, len(bad), bad[:8].tolist(),
                    a.ravel()[bad[:4]].tolist() if len(bad) else None, b.ravel()[bad[:4]].tolist() if len(bad) else None))
                break


if __name__ == "__main__":
    main()
