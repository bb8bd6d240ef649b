#!/usr/bin/env python3
"""Per family: the streams' byteLength total against the bytes their decode consumed (the results'
consumed field) on the bench batch with property columns -- what a read-traffic ratio should be
measured against.  usage: consumed_check.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    for flags in (0, covt.PLAN_PROPERTIES):
        plan = covt.Plan.from_tiles([t for _, t in picks], flags=flags)
        batch = covt.DeviceBatch(plan, "cuda")
        batch.decode()
        torch.cuda.synchronize()
        res = batch.d_res.cpu().numpy().reshape(-1, 2)[:plan.num_descs]
        d = plan.descs.reshape(-1, 32)
        bl = d[:, 28:32].copy().view(np.int32).ravel().astype(np.int64)
        ops = d[:, 24]
        off = np.concatenate([[0], np.cumsum(plan.family_counts)])
        for f in range(covt.NUM_FAMILIES):
            sl = slice(off[f], off[f + 1])
            if off[f + 1] == off[f]:
                continue
            print("flags=%d family %d: %7d descs  byteLength %8.1f MB  consumed %8.1f MB  errors %d" % (
                flags, f, off[f + 1] - off[f], bl[sl].sum() / 1e6, res[sl, 1].astype(np.int64).sum() / 1e6,
                int((res[sl, 0] != 0).sum())))
        for op in np.unique(ops):
            m = ops == op
            print("   op %2d: %7d  byteLength %8.1f MB consumed %8.1f MB" % (op, m.sum(), bl[m].sum() / 1e6,
                                                                          res[m, 1].astype(np.int64).sum() / 1e6))


if __name__ == "__main__":
    main()
