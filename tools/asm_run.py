#!/usr/bin/env python3
"""Geometry assembly over the config-5 batch: decode once, then time `reps` assembly launches with HIP
events (a profiling / A-B target).  usage: asm_run.py [reps]   (COVT_LIB_VARIANT picks the library)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    b = covt.DeviceBatch(plan, "cuda")
    s = torch.cuda.current_stream()
    b.decode(s)
    b.assemble(s)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(s)
        b.assemble(s)
        e1.record(s)
    torch.cuda.synchronize()
    t = [a.elapsed_time(c) for a, c in ev]
    print("%s assembly ms: median %.4f min %.4f" % (os.environ.get("COVT_LIB_VARIANT", "libcovt.so"),
                                                    float(np.median(t)), min(t)))


if __name__ == "__main__":
    main()
