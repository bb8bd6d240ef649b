#!/usr/bin/env python3
"""Paired A/B of libcovt builds on one GPU (each variant in its own process, variants interleaved
twice to average out drift): config-5 grouped launch, each family alone, BASELINE configs 2-4.

  python tools/ab.py libcovt_base.so libcovt.so [...]      (files in cov-tiles_amd/)
  python tools/ab.py libcovt.so libcovt.so:split_min=0       (same build, plan options per variant)
  python tools/ab.py --one libcovt.so                        (one measurement, internal)
  AB_PROPS=1 python tools/ab.py ...                          (the property plan: every column's streams)
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def measure():
    import ctypes as C

    import torch

    sys.path.insert(0, ROOT)
    import bench

    covt = bench.load_covt()
    lib = bench.tile_library()
    picks = bench.sample_batch(lib, 10000, bench.SEED)
    opts = covt.PlanOptions(**json.loads(os.environ.get("AB_PLAN_OPTIONS", "{}")))
    # AB_PROPS=1: the plan also decodes every property column's streams (COVT_PLAN_PROPERTIES)
    flags = covt.PLAN_PROPERTIES if os.environ.get("AB_PROPS") else 0
    plan = covt.Plan.from_tiles([t for _, t in picks], options=opts, flags=flags)
    batch = covt.DeviceBatch(plan, "cuda")
    s = torch.cuda.current_stream()
    L = covt.lib()

    def timed(fn, reps=20, warm=5):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(s)
            fn()
            b.record(s)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    out = {"all": timed(lambda: batch.decode(s))}
    fams = {"rle": covt.FAMILY_RLE, "varint": covt.FAMILY_VARINT, "fastpfor": covt.FAMILY_FASTPFOR,
            "lane": covt.FAMILY_LANE}
    for name, f in fams.items():
        sub = batch.subset(np.isin(np.arange(plan.num_streams), np.nonzero(
            np.repeat(np.arange(covt.NUM_FAMILIES), plan.family_counts)[plan.streams["desc_index"]] == f)[0]))
        out[name] = timed(lambda: sub.decode(s))
        del sub
    for name in ([] if flags else bench.CONFIG_LEGS):
        cp = bench.config_tiles(lib, name)
        cplan = covt.Plan.from_tiles([t for _, t in cp], options=opts)
        cb = covt.DeviceBatch(cplan, "cuda")
        sub = cb.subset(bench.config_mask(cplan, name))
        out[name] = timed(lambda: sub.decode(s), reps=50)
        del sub, cb, cplan
    _ = L, C
    return out


def main():
    if sys.argv[1] == "--one":
        os.environ["COVT_LIB_VARIANT"] = sys.argv[2]
        print(json.dumps(measure()), flush=True)
        return
    variants = sys.argv[1:]
    res = {v: [] for v in variants}
    for _ in range(2):
        for v in variants:
            lib, *kv = v.split(":")  # "libcovt.so:split_min=0:split_chunk=1024" -> plan options of that variant
            env = dict(os.environ, COVT_LIB_VARIANT=lib,
                       AB_PLAN_OPTIONS=json.dumps({k: int(x) for k, x in (y.split("=", 1) for y in kv)}))
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", lib], capture_output=True,
                               text=True, timeout=600, env=env)
            if p.returncode != 0:
                print(p.stderr[-3000:])
                sys.exit(p.returncode)
            res[v].append(json.loads(p.stdout.strip().splitlines()[-1]))
    keys = list(res[variants[0]][0].keys())
    print("%-28s" % "ms (median of 20, 2 runs)" + "".join("%14s" % k for k in keys))
    for v in variants:
        print("%-28s" % v + "".join("%14s" % ("%.4f/%.4f" % (r0[k], r1[k])) for k, r0, r1 in
                                      [(k, res[v][0], res[v][1]) for k in keys]))


if __name__ == "__main__":
    main()
