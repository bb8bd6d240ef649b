#!/usr/bin/env python3
"""BASELINE configs 2-4 under plan-time knobs (KNOB=VALUE[,KNOB=VALUE] per variant; the first argument
'-' is the default plan): every variant's plan and launch built in this process, launches timed
interleaved (4 rounds x 200 launches, HIP events on the launch stream), mean per variant."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    covt = bench.load_covt()
    lib = bench.tile_library()
    s = torch.cuda.current_stream()
    variants = sys.argv[1:] or ["-"]
    for name in bench.CONFIG_LEGS:
        picks = bench.config_tiles(lib, name)
        subs = []
        for v in variants:
            kv = [] if v == "-" else [x.split("=", 1) for x in v.split(",")]
            for k, val in kv:
                os.environ[k] = val
            plan = covt.Plan.from_tiles([t for _, t in picks])
            for k, _ in kv:
                del os.environ[k]
            batch = covt.DeviceBatch(plan, "cuda")
            subs.append((batch, batch.subset(bench.config_mask(plan, name))))
        times = [[] for _ in variants]
        for _ in range(4):
            for i, (_, sub) in enumerate(subs):
                for _ in range(20):
                    sub.decode(s)
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
                for a, b in ev:
                    a.record(s)
                    sub.decode(s)
                    b.record(s)
                torch.cuda.synchronize()
                times[i] += [a.elapsed_time(b) for a, b in ev]
        for i, v in enumerate(variants):
            _, r, _ = subs[i][1].results()
            print("%s %-44s mean %.4f ms  median %.4f ms  statuses ok %s" % (
                name, v, np.mean(times[i]), np.median(times[i]), bool((r[:, 0] == 0).all())), flush=True)


if __name__ == "__main__":
    main()
