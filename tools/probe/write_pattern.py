#!/usr/bin/env python3
"""Times the decode batch's output write pattern alone (tools/probe/write_pattern.hip): per family,
each wave writes its stream's region in 1 KiB steps, cached or nontemporal; plus a linear fill."""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import bench  # noqa: E402


def main():
    import torch

    covt = bench.load_covt()
    lib = C.CDLL(os.path.join(HERE, "libwrite_pattern.so"))
    lib.probe_write_regions.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    batch = covt.DeviceBatch(plan, "cuda")
    s = plan.streams
    nbytes_tile = (s["out_elems"] * s["elem_bytes"]).astype(np.int64)
    nbytes = np.zeros(plan.num_streams, dtype=np.int64)
    nbytes[s["desc_index"]] = nbytes_tile
    d_nb = torch.from_numpy(nbytes).cuda()
    stream = torch.cuda.current_stream()
    fc = plan.family_counts
    offs = np.concatenate([[0], np.cumsum(fc)])

    def run(lo, hi, nt, reps=5):
        n = hi - lo
        args = (batch.d_desc.data_ptr() + 32 * lo, d_nb.data_ptr() + 8 * lo, n, batch.d_out.data_ptr(), nt,
                stream.cuda_stream)
        for _ in range(2):
            lib.probe_write_regions(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            lib.probe_write_regions(*args)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    for nt in (0, 1):
        t = run(0, plan.num_streams, nt)
        tot = int(nbytes.sum())
        print("all streams  nt=%d: %.3f ms  %.0f GB/s (%d MB)" % (nt, t, tot / t / 1e6, tot // 1000000))
        for f, name in enumerate(("RLE", "VARINT", "FASTPFOR", "LANE")):
            b = int(nbytes[offs[f]:offs[f + 1]].sum())
            t = run(int(offs[f]), int(offs[f + 1]), nt)
            print("  %-8s nt=%d: %.3f ms  %.0f GB/s (%d MB)" % (name, nt, t, b / t / 1e6, b // 1000000))
    lib.probe_copy_regions.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p,
                                       C.c_void_p]
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")

    def runc(lo, hi, reps=5):
        args = (batch.d_in.data_ptr(), batch.d_desc.data_ptr() + 32 * lo, d_nb.data_ptr() + 8 * lo, hi - lo,
                batch.d_out.data_ptr(), 1, sink.data_ptr(), stream.cuda_stream)
        for _ in range(2):
            lib.probe_copy_regions(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            lib.probe_copy_regions(*args)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    ib = plan.descs.reshape(-1, 32)[:, 28:32].copy().view(np.int32).ravel().astype(np.int64)
    t = runc(0, plan.num_streams)
    print("read+write pattern, all streams (nt): %.3f ms  %.0f GB/s (r %d MB + w %d MB)" % (
        t, (ib.sum() + nbytes.sum()) / t / 1e6, ib.sum() // 1000000, nbytes.sum() // 1000000))
    for f, name in enumerate(("RLE", "VARINT", "FASTPFOR", "LANE")):
        lo, hi = int(offs[f]), int(offs[f + 1])
        t = runc(lo, hi)
        tb = int(ib[lo:hi].sum() + nbytes[lo:hi].sum())
        print("  %-8s read+write: %.3f ms  %.0f GB/s" % (name, t, tb / t / 1e6))
    x = torch.empty(int(nbytes.sum()) // 4, dtype=torch.int32, device="cuda")
    t = bench_fill(x)
    print("linear fill of the same bytes: %.3f ms  %.0f GB/s" % (t, 4 * x.numel() / t / 1e6))


def bench_fill(x, reps=5):
    import torch

    for _ in range(2):
        x.fill_(3)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        x.fill_(3)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


if __name__ == "__main__":
    main()
