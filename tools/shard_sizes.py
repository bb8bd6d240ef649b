#!/usr/bin/env python3
"""Strong-scaling shard sizes of BASELINE config 5 timed on ONE GPU.

The 10k-tile bench batch is split over N = 1, 2, 4, 8 ranks exactly as `bench.py --gpus N` (default strong
scaling) splits it (LPT byte balance, bench.lpt_shards); every shard of each split is planned and its
decode launch timed alone on this GPU (HIP events, mean of --steps after --warmup).  An N-GPU run takes as
long as its slowest shard, so `projected_gbps` = the whole batch's stream bytes / the slowest shard's
launch: what the strong-scaling line would report with no host-side effects.  `frac` is each shard's own
algorithmic bytes over its launch time against the 8 TB/s peak; `vs_full` its GB/s against the full batch's.
usage: shard_sizes.py [steps] [--ns=1,2,4,8] [--configs] [--opts=split_ratio=12000,split_min=4096 ...] (several --opts: each a
variant, the slowest shard per N of each printed at the end)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    import torch

    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[0]) if args else 30
    ns = [1, 2, 4, 8]
    variants = []
    for a in sys.argv[1:]:
        if a.startswith("--ns="):
            ns = [int(x) for x in a[5:].split(",")]
        if a.startswith("--opts="):
            variants.append({kv.split("=")[0]: int(kv.split("=")[1]) for kv in a[7:].split(",") if kv})
    if not variants:
        variants = [{}]
    summary = []
    for opts in variants:
        summary.append((opts, run(ns, steps, opts)))
    if len(variants) > 1:
        print("slowest shard ms per N:", flush=True)
        for opts, worst in summary:
            print("  %-40s %s" % (opts or "defaults", "  ".join(w for _, w in worst)), flush=True)


def run(ns, steps, opts):
    import torch

    print("== plan options:", opts or "defaults", flush=True)
    covt = bench.load_covt()
    opts = dict(opts)
    launch = opts.pop("launch", 0)  # covt_decode_streams_device_grouped_mode: 0 auto, 1 fused, 2 forked
    popts = covt.PlanOptions(**opts)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    allp = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    full_bytes = None
    full_gbps = None
    worsts = []
    print("%3s %5s %6s %10s %10s %9s %8s %8s %7s" % ("N", "shard", "tiles", "in MB", "out MB", "ms", "GB/s",
                                                    "frac", "vs_full"))
    for n in ns:
        shards = bench.lpt_shards([len(t) for _, t in allp], n)
        worst = 0.0
        for k, sh in enumerate(shards):
            blob, offs, sizes = covt.pack_tiles([allp[i][1] for i in sh])
            plan = covt.Plan(blob, offs, sizes, covt.FORMAT_GENC, 0, options=popts)
            batch = covt.DeviceBatch(plan, dev)
            for _ in range(5):
                batch.decode(stream, launch=launch)
            torch.cuda.synchronize(dev)
            _, res = batch.results()
            assert (res[:, 0] == 0).all()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
            for s, e in ev:
                s.record(stream)
                batch.decode(stream, launch=launch)
                e.record(stream)
            torch.cuda.synchronize(dev)
            ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
            gbps = plan.in_bytes / (ms * 1e-3) / 1e9
            frac = (plan.in_bytes + plan.out_bytes) / (ms * 1e-3) / 8e12
            if n == 1:
                full_bytes, full_gbps = plan.in_bytes, gbps
            worst = max(worst, ms)
            print("%3d %5d %6d %10.1f %10.1f %9.4f %8.1f %8.4f %7.3f" % (
                n, k, len(sh), plan.in_bytes / 1e6, plan.out_bytes / 1e6, ms, gbps, frac,
                gbps / full_gbps if full_gbps else float("nan")), flush=True)
            del batch, plan
        worsts.append((n, "N=%d %.4f" % (n, worst)))
        if full_bytes:
            print("    N=%d: slowest shard %.4f ms -> projected strong-scaling value %.1f GB/s (%.2fx of N=1, "
                  "efficiency %.3f)" % (n, worst, full_bytes / (worst * 1e-3) / 1e9,
                                         full_bytes / (worst * 1e-3) / 1e9 / full_gbps,
                                         full_bytes / (worst * 1e-3) / 1e9 / full_gbps / n), flush=True)


    if "--configs" in sys.argv:  # BASELINE configs 2-4: the config leg's subset launch under these options
        lib = bench.tile_library()
        for name in ("config2", "config3", "config4"):
            picks = bench.config_tiles(lib, name)
            plan = covt.Plan.from_tiles([t for _, t in picks], covt.FORMAT_GENC, 0, options=popts)
            batch = covt.DeviceBatch(plan, dev)
            sub = batch.subset(bench.config_mask(plan, name))
            for _ in range(5):
                sub.decode(stream)
            torch.cuda.synchronize(dev)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
            for s_, e_ in ev:
                s_.record(stream)
                sub.decode(stream)
                e_.record(stream)
            torch.cuda.synchronize(dev)
            ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
            print("%s: %.4f ms" % (name, ms), flush=True)
            worsts.append((name, "%s %.4f" % (name, ms)))
            del sub, batch, plan
    return worsts


if __name__ == "__main__":
    main()
