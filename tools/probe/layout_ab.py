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


def layout_descs(plan, nbytes, order, align):
    """descriptors with every output slice re-assigned: slices in `order` (descriptor indices), each
    starting on an `align`-byte boundary -> (descriptor bytes, new out_off per descriptor, buffer bytes)"""
    d = plan.descs.reshape(-1, 32).copy()
    assert plan.num_descs == plan.num_streams, "plan has split chunks"
    sz = (nbytes[order] + align - 1) // align * align
    oo = np.zeros(plan.num_streams, dtype=np.uint64)
    oo[order] = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
    d[:, 8:16] = oo.view(np.uint8).reshape(-1, 8)
    return d.ravel().copy(), oo, int(sz.sum())


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
    tile_order = s["desc_index"].astype(np.int64)  # descriptor index of each stream, in tile order
    launch_order = np.arange(plan.num_streams)
    layouts = {}
    for name, order, align in (("tile16", tile_order, 16), ("launch16", launch_order, 16),
                               ("tile128", tile_order, 128), ("launch128", launch_order, 128),
                               ("launch256", launch_order, 256)):
        ld, off, total = layout_descs(plan, nbytes, order, align)
        layouts[name] = (torch.from_numpy(ld).cuda(), off, total)
    need = max(v[2] for v in layouts.values())
    if need > batch.d_out.numel():
        batch.d_out = torch.zeros(need + 16, dtype=torch.uint8, device="cuda")
    tile_desc = layouts["tile16"][0]
    launch_desc = layouts["launch16"][0]
    new_off = layouts["launch16"][1]
    old_off = layouts["tile16"][1]
    assert np.array_equal(old_off, plan.descs.reshape(-1, 32)[:, 8:16].copy().view(np.uint64).ravel())
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

    ts = {k: [] for k in layouts}
    for r in range(rounds):
        for k, v in layouts.items():
            ts[k].append(run(v[0]))
    alg = int(nbytes.sum()) + int(plan.descs.reshape(-1, 32)[:, 28:32].copy().view(np.int32).astype(np.int64).sum())
    for k, v in ts.items():
        m = float(np.median(v))
        print("%-9s layout: median %.4f ms  (%s)  %.0f GB/s algorithmic, frac %.3f" % (
            k, m, " ".join("%.4f" % x for x in v), alg / m / 1e6, alg / m / 1e6 / 8000))


if __name__ == "__main__":
    main()
