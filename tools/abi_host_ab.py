#!/usr/bin/env python3
"""C-ABI host entry (covt_plan_decode_host, pageable in/out) on the config-5 batch: fresh output buffers
per call vs caller buffers reused, for prefault settings given as covt_plan_options FIELD=VALUE[,...]
arguments (e.g. host_prefault=0  prefault_threads=8); variants interleaved, median of 3 each."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    variants = sys.argv[1:] or ["prefault_threads=16"]
    blob, offs, sizes = covt.pack_tiles([t for _, t in picks])
    plans = {v: covt.Plan(blob, offs, sizes, options=covt.PlanOptions(
        **{kv.split("=")[0]: int(kv.split("=")[1]) for kv in v.split(",")})) for v in variants}
    for p in plans.values():
        p.decode_host()  # device buffers cached on the plan, HIP warm
    plan = plans[variants[0]]
    res = {v: ([], []) for v in variants}
    out = np.zeros(max(plan.output_bytes, 1), dtype=np.uint8)
    rs = np.zeros((max(plan.num_streams, 1), 2), dtype=np.int32)
    for _ in range(3):
        for v in variants:
            plan = plans[v]
            t = time.perf_counter()
            o, r = plan.decode_host()
            res[v][0].append((time.perf_counter() - t) * 1e3)
            del o, r
            t = time.perf_counter()
            plan.decode_host(out=out, res=rs)
            res[v][1].append((time.perf_counter() - t) * 1e3)
    for v in variants:
        print("%-48s fresh %8.1f ms   reused %8.1f ms" % (v, np.median(res[v][0]), np.median(res[v][1])))


if __name__ == "__main__":
    main()
