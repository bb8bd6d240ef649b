#!/usr/bin/env python3
"""Profiling target: covt_device_plan_create on the bench batch (BASELINE config 5) N times, wall-clock per
creation printed (run under rocprofv3 --kernel-trace --stats [--hip-trace] for the per-kernel / per-call
breakdown).  usage: device_plan_prof.py [reps] [--sweep | --small | --n256] [--nosplit] [--sorted] [--geometry] [--drop=K,...]
--sweep: also batches of 1 tile (the library's largest), 256, 2048 and 4096 tiles (latency vs. occupancy).
--geometry: also time covt_device_plan_geometry (the geometry-column planning) after each creation.
--props: plans with COVT_PLAN_PROPERTIES (property columns planned on the device too).
--drop=K,...: also the batch without its K largest tiles (is the walk bound by its longest tiles?)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = int(args[0]) if args else 10
    covt = bench.load_covt()
    lib = bench.tile_library()
    if "--sweep" in sys.argv:
        big = max((t for z in lib.values() for _, t in z), key=len)
        for n in (1, 256, 2048, 4096):
            tiles = [big] if n == 1 else [t for _, t in bench.sample_batch(lib, n, bench.SEED)]
            run(covt, tiles, reps, "%5d tiles" % n)
    if "--small" in sys.argv:  # the single largest tile only (a split plan)
        run(covt, [max((t for z in lib.values() for _, t in z), key=len)], reps, "    1 tiles")
        return
    if "--n256" in sys.argv:  # 256 sampled tiles (a split plan)
        run(covt, [t for _, t in bench.sample_batch(lib, 256, bench.SEED)], reps, "  256 tiles")
        return
    picks = bench.sample_batch(lib, 10000, bench.SEED)
    run(covt, [t for _, t in picks], reps, "10000 tiles")
    for a in sys.argv[1:]:
        if a.startswith("--drop="):
            tl = [t for _, t in picks]
            by = np.argsort([-len(t) for t in tl], kind="stable")
            for k in (int(x) for x in a[7:].split(",")):
                keep = sorted(by[k:])
                sub = [tl[i] for i in keep]
                run(covt, sub, reps, "%5d tiles (%d largest dropped, %.1f %% of the bytes)"
                    % (len(sub), k, 100.0 * sum(len(t) for t in sub) / sum(len(t) for t in tl)))
    if "--sorted" in sys.argv:  # the same batch, largest tiles first (walk launch order experiment)
        run(covt, sorted((t for _, t in picks), key=len, reverse=True), reps, "10000 tiles, largest first")


def run(covt, tiles, reps, label):
    import torch

    blob, offs, sizes = covt.pack_tiles(tiles)
    d_blob = torch.from_numpy(blob).cuda()
    d_off = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_size = torch.from_numpy(sizes.astype(np.int64)).cuda()
    ts, tg = [], []
    for _ in range(reps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kw = {}
        if "--nosplit" in sys.argv:
            kw["split_min"] = -1
        if "--props" in sys.argv:
            kw["flags"] = covt.PLAN_PROPERTIES
        dp = covt.DevicePlan(d_blob, d_off, d_size, options=covt.PlanOptions(**kw) if kw else None)
        ts.append(time.perf_counter() - t0)
        if "--geometry" in sys.argv:
            t0 = time.perf_counter()
            dp.geometry()
            tg.append(time.perf_counter() - t0)
        dp.close()
    print("%s %s device plan: median %.3f ms, min %.3f ms over %d" % (os.environ.get("COVT_LIB_VARIANT", "libcovt.so"), label,
                                                                   np.median(ts[2:]) * 1e3, min(ts[2:]) * 1e3, reps))
    if tg:
        print("%s %s geometry planning: median %.3f ms, min %.3f ms (%d columns)"
              % (os.environ.get("COVT_LIB_VARIANT", "libcovt.so"), label, np.median(tg[2:]) * 1e3, min(tg[2:]) * 1e3,
                 dp.num_geometry_columns))


if __name__ == "__main__":
    main()
