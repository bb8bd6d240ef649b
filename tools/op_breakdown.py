#!/usr/bin/env python3
"""Times the decode kernel on the config-5 batch restricted to one op class at a time (GPU).
Prints per-op stream bytes, output bytes, kernel time and achieved GB/s (algorithmic bytes)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

NAMES = {1: "BYTE_RLE", 2: "RLE_U64", 3: "RLE_I32", 7: "VAR_ZZD", 8: "VAR_XY", 9: "VAR_MORTON", 10: "FPF_ZZD",
         11: "FPF_XY", 12: "FPF_MORTON", 13: "VAR_U64", 14: "VAR_I32_I64", 15: "VAR_ZZD_I64"}


def main():
    import torch

    covt = bench.load_covt()
    tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    picks = bench.sample_batch(bench.tile_library(), tiles, bench.SEED)
    # OPB_PROPS=1: the plan also decodes every property column's streams (COVT_PLAN_PROPERTIES)
    flags = covt.PLAN_PROPERTIES if os.environ.get("OPB_PROPS") else 0
    plan = covt.Plan.from_tiles([t for _, t in picks], flags=flags)
    batch = covt.DeviceBatch(plan, "cuda")
    descs = plan.descs.reshape(-1, 32)
    ops = descs[:, 24]
    s = plan.streams
    order = np.argsort(s["desc_index"])
    s_launch = s[order]
    res = torch.zeros(2 * plan.num_streams, dtype=torch.int32, device="cuda")
    L = covt.lib()
    stream = torch.cuda.current_stream()

    def run(d_desc, n, reps=5):
        for _ in range(2):
            L.covt_decode_streams_device(batch.d_in.data_ptr(), d_desc.data_ptr(), n, batch.d_out.data_ptr(),
                                         res.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            L.covt_decode_streams_device(batch.d_in.data_ptr(), d_desc.data_ptr(), n, batch.d_out.data_ptr(),
                                         res.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    t_all = run(batch.d_desc, plan.num_streams)
    print("all ops, families back to back: %.3f ms  (%d streams)" % (t_all, plan.num_streams))
    for _ in range(2):
        batch.decode()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    trials = []
    for _ in range(5):
        e0.record(stream)
        for _ in range(10):
            batch.decode(stream)
        e1.record(stream)
        torch.cuda.synchronize()
        trials.append(e0.elapsed_time(e1) / 10)
    trials.sort()
    print("all ops, families concurrent (grouped launch): %.3f ms  (min %.3f, 5 trials of 10)" % (trials[2], trials[0]))
    import ctypes as C
    quick = os.environ.get("OPB_QUICK")
    for fam, name in enumerate(("RLE", "VARINT", "FASTPFOR", "LANE")):
        cnt = np.zeros(covt.NUM_FAMILIES, dtype=np.int64)
        off = int(plan.family_counts[:fam].sum())
        n = int(plan.family_counts[fam])
        sub = torch.from_numpy(np.ascontiguousarray(descs[off:off + n]).reshape(-1)).cuda()
        cnt[fam] = n
        sub_full = torch.zeros(plan.num_streams * 32, dtype=torch.uint8, device="cuda")
        lo = int(cnt[:fam].sum())
        sub_full[lo * 32:(lo + n) * 32] = sub
        def go():
            L.covt_decode_streams_device_grouped(batch.d_in.data_ptr(), sub_full.data_ptr(),
                                                 cnt.ctypes.data_as(C.POINTER(C.c_int64)), batch.d_out.data_ptr(),
                                                 res.data_ptr(), stream.cuda_stream)
        go(); go()
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(5):
            go()
        e1.record(stream)
        torch.cuda.synchronize()
        print("family %-8s alone: %.3f ms (%d streams)" % (name, e0.elapsed_time(e1) / 5, n))
    if quick:
        return
    # each descriptor's family (launch order groups the plan's descriptors by family, so an op's subset is
    # contiguous per family too)
    fl = descs[:, 26:28].copy().view(np.uint16).ravel()
    fam_of = np.zeros(len(descs), dtype=np.int64)
    for f in range(covt.NUM_FAMILIES):
        n = int(plan.family_counts[f])
        lo = int(plan.family_counts[:f].sum())
        fam_of[lo:lo + n] = f
    res_g = torch.zeros(2 * plan.num_streams, dtype=torch.int32, device="cuda")

    def run_grouped(sub, cnt, reps=5):
        def go():
            L.covt_decode_streams_device_grouped(batch.d_in.data_ptr(), sub.data_ptr(),
                                                 cnt.ctypes.data_as(C.POINTER(C.c_int64)), batch.d_out.data_ptr(),
                                                 res_g.data_ptr(), stream.cuda_stream)
        go(); go()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            go()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    print("per op: t = every family kernel over the op's descriptors back to back (covt_decode_streams_device: "
          "each kernel skips the other families' descriptors, so empty waves are dispatched); tg = the grouped "
          "launch the decode uses (covt_decode_streams_device_grouped: the op's own families, concurrent)")
    for op in sorted(set(ops.tolist())):
        m = ops == op
        sub = torch.from_numpy(np.ascontiguousarray(descs[m]).reshape(-1)).cuda()
        t = run(sub, int(m.sum()))
        cnt_op = np.bincount(fam_of[m], minlength=covt.NUM_FAMILIES).astype(np.int64)
        if (fl[m] & 0x1e).any():  # split chunks: their pads are descriptors of other ops
            tg = float("nan")
        else:
            tg = run_grouped(sub, cnt_op)
        ib = int(s_launch["byte_length"][m].sum())
        ob = int((s_launch["out_elems"][m] * s_launch["elem_bytes"][m]).sum())
        nv = int(s_launch["num_values"][m].sum())
        idx = np.nonzero(m)[0]  # launch order is largest first
        top = torch.from_numpy(np.ascontiguousarray(descs[idx[:1]]).reshape(-1)).cuda()
        t1 = run(top, 1)
        rest = torch.from_numpy(np.ascontiguousarray(descs[idx[64:]]).reshape(-1)).cuda()
        tr = run(rest, max(len(idx) - 64, 0)) if len(idx) > 64 else 0.0
        print("%-12s streams=%7d values=%11d in=%6.1fMB out=%7.1fMB  t=%7.3f ms  alg=%7.1f GB/s  %.2f Gval/s"
              "  | largest stream (%d B, %d vals) %.3f ms | all but top-64 %.3f ms | tg=%7.3f ms  alg=%7.1f GB/s"
              % (NAMES.get(op, op), int(m.sum()), nv, ib / 1e6, ob / 1e6, t, (ib + ob) / t / 1e6, nv / t / 1e6,
                 int(s_launch["byte_length"][idx[0]]), int(s_launch["num_values"][idx[0]]), t1, tr, tg,
                 (ib + ob) / tg / 1e6))


if __name__ == "__main__":
    main()


def fpf_scaling():
    """FastPFOR throughput by stream size class: large streams (steady-state block loop) vs small ones
    (per-stream and per-page overhead, VariableByte tail)."""
    import torch

    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    batch = covt.DeviceBatch(plan, "cuda")
    descs = plan.descs.reshape(-1, 32)
    ops = descs[:, 24]
    nv = descs[:, 20:24].copy().view(np.int32).ravel()
    res = torch.zeros(2 * plan.num_streams, dtype=torch.int32, device="cuda")
    L = covt.lib()
    import ctypes as C
    L.covt_launch_family.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
    stream = torch.cuda.current_stream()
    for lo, hi in ((0, 256), (256, 1024), (1024, 4096), (4096, 16384), (16384, 1 << 30)):
        m = (ops >= 10) & (ops <= 12) & (nv >= lo) & (nv < hi)
        if not m.any():
            continue
        sub = torch.from_numpy(np.ascontiguousarray(descs[m]).reshape(-1)).cuda()
        n = int(m.sum())
        for _ in range(2):
            L.covt_launch_family(2, batch.d_in.data_ptr(), sub.data_ptr(), n, batch.d_out.data_ptr(), res.data_ptr(),
                                 stream.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(5):
            L.covt_launch_family(2, batch.d_in.data_ptr(), sub.data_ptr(), n, batch.d_out.data_ptr(), res.data_ptr(),
                                 stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 5
        vals = int(nv[m].sum())
        print("FPF streams with %6d <= values < %9d: n=%6d values=%10d  t=%.3f ms  %.1f Gval/s  %.2f us/stream-slot"
              % (lo, hi, n, vals, t, vals / t / 1e6, t * 1e3 * 1024 * 7 / max(n, 1)))

