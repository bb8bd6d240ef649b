#!/usr/bin/env python3
"""The config-5 decode launch in its three shapes (covt_decode_streams_device_grouped_mode): auto (the four
family kernels on forked queues for this batch), fused (every family in one kernel) and forked; paired rounds
in one process.  --shard=N/k: shard k of the N-way LPT split of the batch (bench.py's strong scaling) instead.
usage: python tools/launch_mode_ab.py [rounds] [launches] [--shard=N/k]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds = int(args[0]) if len(args) > 0 else 5
    per = int(args[1]) if len(args) > 1 else 10
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    for a in sys.argv[1:]:
        if a.startswith("--shard="):
            n, k = (int(x) for x in a[8:].split("/"))
            picks = [picks[i] for i in bench.lpt_shards([len(t) for _, t in picks], n)[k]]
            print("shard %d/%d: %d tiles" % (k, n, len(picks)))
    plan = covt.Plan.from_tiles([t for _, t in picks])
    batch = covt.DeviceBatch(plan, "cuda")

    def run(mode):
        for _ in range(2):
            batch.decode(launch=mode)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(per):
            batch.decode(launch=mode)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / per

    names = {covt.LAUNCH_AUTO: "auto", covt.LAUNCH_FUSED: "fused", covt.LAUNCH_FORKED: "forked"}
    ts = {m: [] for m in names}
    for _ in range(rounds):
        for m in names:
            ts[m].append(run(m))
    for m, v in ts.items():
        print("%-6s median %.4f ms (%s)" % (names[m], float(np.median(v)), " ".join("%.4f" % x for x in v)))


if __name__ == "__main__":
    main()
