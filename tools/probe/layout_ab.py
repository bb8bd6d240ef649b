#!/usr/bin/env python3
"""Paired A/B of the real decode launch with two output layouts of the same plan (round 4):
tile order (the plan's layout) against launch order (every descriptor's output slice re-assigned in
descriptor order, i.e. in the order the waves run).  Same kernels, same inputs; only out_off moves.
Checks that every stream's bytes are identical in both layouts, then alternates the two in rounds.
usage: python tools/probe/layout_ab.py [rounds] [launches_per_round]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import bench  # noqa: E402


def launch_order_descs(plan, nbytes):
    d = plan.descs.reshape(-1, 32).copy()
    flags = d[:, 26:28].copy().view(np.uint16).ravel()
    assert plan.num_descs == plan.num_streams, "plan has split chunks"
    sz = (nbytes + 15) // 16 * 16
    oo = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
    d[:, 8:16] = oo.view(np.uint8).reshape(-1, 8)
    return d.ravel().copy(), oo, flags


def main():
    import torch

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    batch = covt.DeviceBatch(plan, "cuda")
    s = plan.streams
    nbytes = np.zeros(plan.num_streams, dtype=np.int64)
    nbytes[s["desc_index"]] = (s["out_elems"] * s["elem_bytes"]).astype(np.int64)
    ld, new_off, _ = launch_order_descs(plan, nbytes)
    tile_desc = batch.d_desc
    launch_desc = torch.from_numpy(ld).cuda()
    old_off = plan.descs.reshape(-1, 32)[:, 8:16].copy().view(np.uint64).ravel()

    # parity: the same bytes per stream in both layouts
    batch.d_desc = tile_desc
    batch.decode()
    torch.cuda.synchronize()
    a = batch.d_out.cpu().numpy()
    ra = batch.d_res.cpu().numpy().copy()
    batch.d_out.zero_()
    batch.d_desc = launch_desc
    batch.decode()
    torch.cuda.synchronize()
    b = batch.d_out.cpu().numpy()
    rb = batch.d_res.cpu().numpy().copy()
    bad = 0
    for i in range(plan.num_streams):
        n = int(nbytes[i])
        if not np.array_equal(a[int(old_off[i]):int(old_off[i]) + n], b[int(new_off[i]):int(new_off[i]) + n]):
            bad += 1
    print("parity: %d of %d streams differ; results equal: %s" % (bad, plan.num_streams, np.array_equal(ra, rb)))
    del a, b

    def run(desc):
        batch.d_desc = desc
        for _ in range(3):
            batch.decode()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(per):
            batch.decode()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / per

    ts = {"tile": [], "launch": []}
    for r in range(rounds):
        ts["tile"].append(run(tile_desc))
        ts["launch"].append(run(launch_desc))
    alg = int(nbytes.sum()) + int(plan.descs.reshape(-1, 32)[:, 28:32].copy().view(np.int32).astype(np.int64).sum())
    for k, v in ts.items():
        m = float(np.median(v))
        print("%-7s layout: median %.4f ms  (%s)  %.0f GB/s algorithmic, frac %.3f" % (
            k, m, " ".join("%.4f" % x for x in v), alg / m / 1e6, alg / m / 1e6 / 8000))


if __name__ == "__main__":
    main()
