#!/usr/bin/env python3
"""HBM ceiling for the decode launch's traffic (round 4).

Measured in one process, one box:
  * hand-written grid-stride streaming stores over the batch's 4.5 GB of output (tools/probe/hbm_ceiling.hip),
    nontemporal and cached, over a sweep of grid sizes; the same for the 0.9 GB of input (reads);
  * a proportional copy (each wave step: 1 KiB in, R KiB out, R = output / input of the batch);
  * the batch's own regions (tools/probe/write_pattern.hip: one wave per stream, its output slice front to back,
    input streamed in proportion) with the output slices laid out three ways: tile order (the plan's layout
    today), launch order (slices assigned in descriptor order, i.e. the order the waves run) and random order;
  * torch's fill_ for comparison.
Prints one line per measurement; `python tools/probe/hbm_ceiling.py > profiles/r04/practical_ceiling.txt`.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import bench  # noqa: E402


def timed(fn, reps=5, warm=2):
    import torch

    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    import torch

    covt = bench.load_covt()
    hc = C.CDLL(os.path.join(HERE, "libhbm_ceiling.so"))
    wp = C.CDLL(os.path.join(HERE, "libwrite_pattern.so"))
    hc.probe_store.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_void_p]
    hc.probe_read.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]
    hc.probe_copy.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    wp.probe_write_regions.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]
    wp.probe_copy_regions.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p,
                                      C.c_void_p]

    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    batch = covt.DeviceBatch(plan, "cuda")
    s = plan.streams
    nbytes = np.zeros(plan.num_streams, dtype=np.int64)
    nbytes[s["desc_index"]] = (s["out_elems"] * s["elem_bytes"]).astype(np.int64)
    descs = plan.descs.reshape(-1, 32).copy()
    ib = descs[:, 28:32].copy().view(np.int32).ravel().astype(np.int64)
    w_total, r_total = int(nbytes.sum()), int(ib.sum())
    stream = torch.cuda.current_stream().cuda_stream
    out = batch.d_out
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    print("# bench batch: %d streams, input %d B, output %d B, out buffer %d B" % (
        plan.num_streams, r_total, w_total, out.numel()))

    # 1. linear streaming stores / reads / copy, grid sweep
    n16 = w_total // 16
    for nt in (1, 0):
        for blocks in (1024, 2048, 4096, 8192, 16384, 65536):
            t = timed(lambda: hc.probe_store(out.data_ptr(), n16, nt, blocks, stream))
            print("store   nt=%d blocks=%6d: %.3f ms  %5.0f GB/s" % (nt, blocks, t, 16 * n16 / t / 1e6))
    inb = batch.d_in
    r16 = r_total // 16
    for blocks in (1024, 2048, 4096, 8192, 16384):
        t = timed(lambda: hc.probe_read(inb.data_ptr(), r16, sink.data_ptr(), blocks, stream))
        print("read         blocks=%6d: %.3f ms  %5.0f GB/s" % (blocks, t, 16 * r16 / t / 1e6))
    R = max(1, int(round(w_total / r_total)))
    units = min(r16 // 64, n16 // (64 * R))
    for nt in (1, 0):
        for blocks in (1024, 2048, 4096, 8192, 16384):
            t = timed(lambda: hc.probe_copy(inb.data_ptr(), units, R, out.data_ptr(), nt, blocks, stream))
            tb = units * 1024 * (1 + R)
            print("copy1:%d nt=%d blocks=%6d: %.3f ms  %5.0f GB/s (r %d MB + w %d MB)" % (
                R, nt, blocks, t, tb / t / 1e6, units * 1024 // 1000000, units * 1024 * R // 1000000))
    hc.probe_copy_depth.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    for depth in (2, 4):  # D loads in flight per lane (k_copy_d)
        for blocks in (1024, 2048, 4096, 8192, 16384):
            t = timed(lambda: hc.probe_copy_depth(inb.data_ptr(), units, R, out.data_ptr(), depth, blocks, stream))
            tb = units * 1024 * (1 + R)
            print("copy1:%d depth=%d blocks=%6d: %.3f ms  %5.0f GB/s" % (R, depth, blocks, t, tb / t / 1e6))
    # copy 1:1 (the guide's float4 copy shape)
    half = min(r16, n16 // 2) // 64
    for blocks in (4096, 8192, 16384):
        t = timed(lambda: hc.probe_copy(out.data_ptr(), half, 1, out.data_ptr() + half * 1024, 1, blocks, stream))
        print("copy1:1 nt=1 blocks=%6d: %.3f ms  %5.0f GB/s (r+w %d MB)" % (blocks, t, 2 * half * 1024 / t / 1e6,
                                                                           2 * half * 1024 // 1000000))
    for depth in (2, 4):
        for blocks in (2048, 4096, 8192, 16384):
            t = timed(lambda: hc.probe_copy_depth(out.data_ptr(), half, 1, out.data_ptr() + half * 1024, depth, blocks,
                                                  stream))
            print("copy1:1 depth=%d blocks=%6d: %.3f ms  %5.0f GB/s" % (depth, blocks, t, 2 * half * 1024 / t / 1e6))
    x = out[: 4 * (w_total // 4)].view(torch.int32)
    t = timed(lambda: x.fill_(3))
    print("torch fill_ of the output bytes: %.3f ms  %5.0f GB/s" % (t, w_total / t / 1e6))

    # 2. the batch's own regions in three output layouts
    def layout(order, align=16):
        d = descs.copy()
        oo = np.zeros(plan.num_streams, dtype=np.uint64)
        sz = (nbytes[order] + align - 1) // align * align
        oo[order] = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint64)
        d[:, 8:16] = oo.view(np.uint8).reshape(-1, 8)
        return torch.from_numpy(d.ravel().copy()).cuda()

    tile_d = torch.from_numpy(descs.ravel().copy()).cuda()
    launch_d = layout(np.arange(plan.num_streams))
    rand_d = layout(np.random.default_rng(1).permutation(plan.num_streams))
    d_nb = torch.from_numpy(nbytes).cuda()
    fc = plan.family_counts
    offs = np.concatenate([[0], np.cumsum(fc)])
    for name, dd in (("tile order", tile_d), ("launch order", launch_d), ("random order", rand_d)):
        t = timed(lambda: wp.probe_write_regions(dd.data_ptr(), d_nb.data_ptr(), plan.num_streams, out.data_ptr(), 1,
                                                 stream))
        print("regions write-only %-12s: %.3f ms  %5.0f GB/s" % (name, t, w_total / t / 1e6))
        t = timed(lambda: wp.probe_copy_regions(inb.data_ptr(), dd.data_ptr(), d_nb.data_ptr(), plan.num_streams,
                                                out.data_ptr(), 1, sink.data_ptr(), stream))
        print("regions read+write %-12s: %.3f ms  %5.0f GB/s" % (name, t, (w_total + r_total) / t / 1e6))
        for f, fname in enumerate(("RLE", "VARINT", "FASTPFOR", "LANE")):
            lo, hi = int(offs[f]), int(offs[f + 1])
            if hi <= lo:
                continue
            t = timed(lambda: wp.probe_copy_regions(inb.data_ptr(), dd.data_ptr() + 32 * lo, d_nb.data_ptr() + 8 * lo,
                                                    hi - lo, out.data_ptr(), 1, sink.data_ptr(), stream))
            tb = int(ib[lo:hi].sum() + nbytes[lo:hi].sum())
            print("   %-8s read+write %-12s: %.3f ms  %5.0f GB/s" % (fname, name, t, tb / t / 1e6))
    # 2b. several consecutive descriptors per wave (a longer contiguous write run in launch order)
    wp.probe_copy_regions_multi.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int,
                                            C.c_void_p, C.c_void_p]
    for name, dd in (("tile order", tile_d), ("launch order", launch_d)):
        for K in (1, 2, 4, 8, 16):
            t = timed(lambda: wp.probe_copy_regions_multi(inb.data_ptr(), dd.data_ptr(), d_nb.data_ptr(),
                                                          plan.num_streams, out.data_ptr(), K, sink.data_ptr(), stream))
            print("regions read+write %-12s %2d descriptors per wave: %.3f ms  %5.0f GB/s" % (
                name, K, t, (w_total + r_total) / t / 1e6))
    # 3. the real decode launch for reference, same process
    t = timed(lambda: batch.decode(), reps=10)
    print("decode launch (tile-order layout): %.3f ms  %5.0f GB/s algorithmic" % (t, (w_total + r_total) / t / 1e6))


if __name__ == "__main__":
    main()
