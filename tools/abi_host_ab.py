#!/usr/bin/env python3
"""C-ABI host entry (covt_plan_decode_host, pageable in/out) on the config-5 batch: fresh output buffers
per call vs caller buffers reused, for prefault settings given as KNOB=VALUE[,KNOB=VALUE] arguments
(e.g. COVT_HOST_PREFAULT=0  COVT_HOST_PREFAULT_THREADS=8); variants interleaved, median of 3 each."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    plan.decode_host()  # device buffers cached on the plan, HIP warm
    variants = sys.argv[1:] or ["COVT_HOST_PREFAULT_THREADS=16"]
    res = {v: ([], []) for v in variants}
    out = np.zeros(max(plan.output_bytes, 1), dtype=np.uint8)
    rs = np.zeros((max(plan.num_streams, 1), 2), dtype=np.int32)
    for _ in range(3):
        for v in variants:
            for kv in v.split(","):
                k, val = kv.split("=", 1)
                os.environ[k] = val
            t = time.perf_counter()
            o, r = plan.decode_host()
            res[v][0].append((time.perf_counter() - t) * 1e3)
            del o, r
            t = time.perf_counter()
            plan.decode_host(out=out, res=rs)
            res[v][1].append((time.perf_counter() - t) * 1e3)
            for kv in v.split(","):
                os.environ.pop(kv.split("=", 1)[0], None)
    for v in variants:
        print("%-48s fresh %8.1f ms   reused %8.1f ms" % (v, np.median(res[v][0]), np.median(res[v][1])))


if __name__ == "__main__":
    main()
