#!/usr/bin/env python3
"""Long poles of a strong-scaling shard: how long the shard's K longest streams take
decoded alone (one launch over just them: each gets a wave to itself), how long the other streams take
alone, and the whole shard -- per K.  If the longest streams alone finish well before the whole shard,
the shard's time is set by where those streams run (sharing SIMDs with the crowd), not by their length.
usage: long_poles.py [steps] [--shard=N/k] [--opts=k=v,...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    import torch

    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[0]) if args else 20
    n, k = 4, 0
    opts = {}
    for a in sys.argv[1:]:
        if a.startswith("--shard="):
            n, k = (int(x) for x in a[8:].split("/"))
        if a.startswith("--opts="):
            opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a[7:].split(",") if kv}
    covt = bench.load_covt()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    allp = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    sh = bench.lpt_shards([len(t) for _, t in allp], n)[k]
    blob, offs, sizes = covt.pack_tiles([allp[i][1] for i in sh])
    plan = covt.Plan(blob, offs, sizes, covt.FORMAT_GENC, 0, options=covt.PlanOptions(**opts))
    batch = covt.DeviceBatch(plan, dev)
    st = plan.streams
    cost = st["byte_length"].astype(np.int64) + st["out_elems"].astype(np.int64) * st["elem_bytes"] // 4
    order = np.argsort(-cost, kind="stable")

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for s, e in ev:
            s.record(stream)
            fn()
            e.record(stream)
        torch.cuda.synchronize(dev)
        return float(np.mean([s.elapsed_time(e) for s, e in ev]))

    full = timed(lambda: batch.decode(stream))
    print("shard %d/%d: %d tiles, %d streams, whole shard %.4f ms" % (k, n, len(sh), plan.num_streams, full),
          flush=True)
    print("%6s %12s %12s %12s %10s" % ("K", "min bytes", "top K ms", "rest ms", "max(2)"), flush=True)
    for kk in (1, 16, 64, 256, 512, 1024, 2048):
        top = np.zeros(plan.num_streams, dtype=bool)
        top[order[:kk]] = True
        a = batch.subset(top)
        b = batch.subset(~top)
        ta = timed(lambda: a.decode(stream))
        tb = timed(lambda: b.decode(stream))
        print("%6d %12d %12.4f %12.4f %10.4f" % (kk, int(st["byte_length"][order[kk - 1]]), ta, tb, max(ta, tb)),
              flush=True)
        del a, b


if __name__ == "__main__":
    main()
