#!/usr/bin/env python3
"""Times the property materialization kernel alone on the bench batch (A/B of library variants via
COVT_LIB_VARIANT): one decode launch over all streams with COVT_PLAN_PROPERTIES, then 5 trials of 10
materializations, median printed.  usage: props_run.py [tiles]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    covt = bench.load_covt()
    tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    picks = bench.sample_batch(bench.tile_library(), tiles, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks], flags=covt.PLAN_PROPERTIES)
    batch = covt.DeviceBatch(plan, "cuda")
    stream = torch.cuda.current_stream()
    batch.decode(stream)
    for _ in range(2):
        batch.materialize_properties(stream)
    torch.cuda.synchronize()
    trials = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            batch.materialize_properties(stream)
        e1.record(stream)
        torch.cuda.synchronize()
        trials.append(e0.elapsed_time(e1) / 10)
    trials.sort()
    _, pres = batch.property_results()
    print("%s: materialize %.3f ms (min %.3f) over %d columns, %d not OK"
          % (os.environ.get("COVT_LIB_VARIANT", "libcovt.so"), trials[2], trials[0], plan.num_property_columns,
             int((pres["status"] != 0).sum())))


if __name__ == "__main__":
    main()
