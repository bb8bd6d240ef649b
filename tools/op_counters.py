#!/usr/bin/env python3
"""Launches the config-5 batch once per (op, kernel family) subset -- a rocprofv3 --pmc target that
gives instruction counts per op.  Dispatch k of the printed order is the k-th decode kernel after the
warmup launch.  usage: op_counters.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

OPS = {1: "BYTE_RLE", 2: "RLE_U64", 3: "RLE_I32", 4: "RLE_S64", 7: "VAR_ZZD", 8: "VAR_XY", 9: "VAR_MORTON",
       10: "FPF_ZZD", 11: "FPF_XY", 12: "FPF_MORTON", 13: "VAR_U64", 14: "VAR_I32_AS_I64", 15: "VAR_ZZD_I64"}


def main():
    import torch

    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    batch = covt.DeviceBatch(plan, "cuda")
    L = covt.lib()
    s = torch.cuda.current_stream()
    D = plan.descs.reshape(-1, 32)
    op = D[:, 24]
    flags = D[:, 26].astype(np.int32) | (D[:, 27].astype(np.int32) << 8)
    nv = D[:, 20:24].copy().view(np.int32).ravel()
    bl = D[:, 28:32].copy().view(np.int32).ravel()
    fam_of = np.zeros(len(D), np.int64)
    off = 0
    for f in range(covt.NUM_FAMILIES):
        n = int(plan.family_counts[f])
        fam_of[off:off + n] = f
        off += n
    jobs = []
    for f in range(covt.NUM_FAMILIES):
        for o in sorted(OPS):
            sel = (fam_of == f) & (op == o)
            if sel.sum() == 0:
                continue
            sub = D[sel]
            counts = np.zeros(covt.NUM_FAMILIES, np.int64)
            counts[f] = len(sub)
            full = np.zeros((int(counts.sum()), 32), np.uint8)
            full[:len(sub)] = sub
            jobs.append((f, o, int(sel.sum()), int(nv[sel].sum()), int(bl[sel].sum()),
                         torch.from_numpy(full.reshape(-1)).cuda(), counts))
    del flags

    def run(d, counts):
        L.covt_decode_streams_device_grouped(batch.d_in.data_ptr(), d.data_ptr(),
                                             counts.ctypes.data_as(C.POINTER(C.c_int64)), batch.d_out.data_ptr(),
                                             batch.d_res.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()

    run(batch.d_desc, plan.family_counts.copy())  # warmup (all families)
    for k, (f, o, ns, v, b, d, counts) in enumerate(jobs):
        run(d, counts)
        print("dispatch %d fam %d op %-14s streams %7d values %10d bytes %10d" % (k, f, OPS[o], ns, v, b), flush=True)


if __name__ == "__main__":
    main()
