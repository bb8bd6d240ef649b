#!/usr/bin/env python3
"""Runs one codec family (or all) of the config-5 batch N times -- a profiling target for rocprofv3.
usage: family_run.py {rle,varint,fastpfor,all} [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import ctypes as C

    import torch

    fam = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    # OPB_PROPS=1: the plan also decodes every property column's streams (COVT_PLAN_PROPERTIES)
    plan = covt.Plan.from_tiles([t for _, t in picks], flags=covt.PLAN_PROPERTIES if os.environ.get("OPB_PROPS") else 0)
    batch = covt.DeviceBatch(plan, "cuda")
    counts = plan.family_counts.copy()
    if fam != "all":
        keep = {"rle": 0, "varint": 1, "fastpfor": 2, "lane": 3}[fam]
        for f in range(covt.NUM_FAMILIES):
            if f != keep:
                counts[f] = 0
        # move the kept family's descriptors to the front ranges the grouped launch expects
        off = int(plan.family_counts[:keep].sum())
        n = int(plan.family_counts[keep])
        sub = np.zeros_like(plan.descs.reshape(-1, 32))
        lo = int(counts[:keep].sum())
        sub[lo:lo + n] = plan.descs.reshape(-1, 32)[off:off + n]
        batch.d_desc = torch.from_numpy(sub.reshape(-1)).cuda()
    L = covt.lib()
    s = torch.cuda.current_stream()
    for _ in range(reps):
        L.covt_decode_streams_device_grouped(batch.d_in.data_ptr(), batch.d_desc.data_ptr(),
                                             counts.ctypes.data_as(C.POINTER(C.c_int64)), batch.d_out.data_ptr(),
                                             batch.d_res.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    print("ok", fam, counts)


if __name__ == "__main__":
    main()
