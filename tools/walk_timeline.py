#!/usr/bin/env python3
"""Per-tile timeline of the device plan's Id / Geometry walk (walk_count) over the bench batch.

Loads libcovt_plan_timing.so (make -C cov-tiles_amd plan_var PV=timing PFLAGS=-DCOVT_PLAN_TIMING), whose
walk writes each tile's (start, end) s_memrealtime ticks (100 MHz) into a buffer registered with
covt_debug_walk_clock, creates the plan a few times and prints the walk's span, the tiles in flight over
it, the duration distribution and the tiles that end last.  usage: walk_timeline.py [reps]"""
import ctypes
import os
import sys

os.environ["COVT_LIB_VARIANT"] = "libcovt_plan_timing.so"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402

TICK_US = 0.01


def main():
    import torch

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    tiles = [t for _, t in picks]
    blob, offs, sizes = covt.pack_tiles(tiles)
    d_blob = torch.from_numpy(blob).cuda()
    d_off = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_size = torch.from_numpy(sizes.astype(np.int64)).cuda()
    clock = torch.zeros(2 * len(tiles), dtype=torch.int64, device="cuda")
    L = covt.lib()
    L.covt_debug_walk_clock.argtypes = [ctypes.c_void_p]
    assert L.covt_debug_walk_clock(clock.data_ptr()) == 0
    spans = []
    for r in range(reps):
        clock.zero_()
        dp = covt.DevicePlan(d_blob, d_off, d_size)
        torch.cuda.synchronize()
        dp.close()
        c = clock.cpu().numpy().reshape(-1, 2).astype(np.int64)
        t0 = c[:, 0].min()
        st, en = (c[:, 0] - t0) * TICK_US, (c[:, 1] - t0) * TICK_US
        spans.append(en.max())
    L.covt_debug_walk_clock(None)
    dur = en - st
    nb = np.array([len(t) for t in tiles])
    print("walk span (first start -> last end) over %d plans: %s us" % (reps, " ".join("%.1f" % x for x in spans)))
    print("last plan: tile walk durations p50 %.1f  p90 %.1f  p99 %.1f  max %.1f us; mean %.1f us; sum %.0f us"
          % (np.percentile(dur, 50), np.percentile(dur, 90), np.percentile(dur, 99), dur.max(), dur.mean(), dur.sum()))
    span = en.max()
    print("tiles in flight per 5 %% of the span (starts / running at the slice's midpoint):")
    cuts = np.linspace(0, span, 21)
    print("  starts ", " ".join("%5d" % ((st >= a) & (st < b)).sum() for a, b in zip(cuts[:-1], cuts[1:])))
    mids = (cuts[:-1] + cuts[1:]) / 2
    print("  running", " ".join("%5d" % ((st <= m) & (en > m)).sum() for m in mids))
    print("last 10 tiles to finish (bytes, start us, duration us):")
    for i in np.argsort(-en)[:10]:
        print("  %8d  start %7.1f  dur %7.1f" % (nb[i], st[i], dur[i]))
    print("longest 10 walks (bytes, start us, duration us):")
    for i in np.argsort(-dur)[:10]:
        print("  %8d  start %7.1f  dur %7.1f" % (nb[i], st[i], dur[i]))
    cc = np.corrcoef(nb, dur)[0, 1]
    print("duration vs tile bytes: corr %.2f; by size class (bytes: n, mean us):" % cc)
    for lo, hi in ((0, 4096), (4096, 16384), (16384, 65536), (65536, 262144), (262144, 1 << 30)):
        m = (nb >= lo) & (nb < hi)
        if m.any():
            print("  [%7d, %9d): %5d  %.1f" % (lo, hi, m.sum(), dur[m].mean()))


if __name__ == "__main__":
    main()
