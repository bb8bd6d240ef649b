#!/usr/bin/env python3
"""Profiling target: BASELINE config 1 (omt/5_16_20 decoded whole: decode launch + geometry assembly +
property materialization on one stream) N times; run under rocprofv3 --kernel-trace --stats for the
per-kernel split of bench.py's configs.config1.gpu_full_ms.  usage: config1_prof.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    covt = bench.load_covt()
    tile = bench.config1_tile(bench.tile_library())
    plan = covt.Plan.from_tiles([tile], covt.FORMAT_GENC, 0, covt.PLAN_PROPERTIES)
    batch = covt.DeviceBatch(plan, "cuda")
    s = torch.cuda.current_stream()
    for _ in range(reps):
        batch.decode(s)
        batch.assemble(s)
        batch.materialize_properties(s)
    torch.cuda.synchronize()
    print("config1: %d streams, %d property columns" % (plan.num_streams, plan.num_property_columns))


if __name__ == "__main__":
    main()
