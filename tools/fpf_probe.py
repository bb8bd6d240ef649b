#!/usr/bin/env python3
"""FastPFOR family of the config-5 batch, split into its long poles and the rest (one GPU): the family
alone, its largest stream alone, its 64 largest alone, and all but those 64 -- so a change can be read as
throughput (the crowd) or latency (single long waves).  COVT_LIB_VARIANT picks the library.
usage: fpf_probe.py [reps]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    batch = covt.DeviceBatch(plan, "cuda")
    descs = plan.descs.reshape(-1, 32)
    fam = covt.FAMILY_FASTPFOR
    off = int(plan.family_counts[:fam].sum())
    n = int(plan.family_counts[fam])
    fd = descs[off:off + n]  # largest first (launch order)
    L = covt.lib()
    s = torch.cuda.current_stream()
    res = torch.zeros(2 * plan.num_descs, dtype=torch.int32, device="cuda")

    def timed(rows):
        cnt = np.zeros(covt.NUM_FAMILIES, dtype=np.int64)
        cnt[fam] = len(rows)
        full = np.zeros((int(cnt[:fam].sum()) + len(rows), 32), dtype=np.uint8)
        full[int(cnt[:fam].sum()):] = rows
        d = torch.from_numpy(full.reshape(-1)).cuda()

        def go():
            L.covt_decode_streams_device_grouped(batch.d_in.data_ptr(), d.data_ptr(),
                                                 cnt.ctypes.data_as(C.POINTER(C.c_int64)), batch.d_out.data_ptr(),
                                                 res.data_ptr(), s.cuda_stream)
        for _ in range(3):
            go()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(s)
            go()
            b.record(s)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    bl = fd.view(np.int32)[:, 7]
    print("variant %s: %d FastPFOR streams, largest %d B" % (os.environ.get("COVT_LIB_VARIANT", "libcovt.so"), n, bl[0]))
    print("  family alone      %.4f ms" % timed(fd))
    print("  largest alone     %.4f ms" % timed(fd[:1]))
    print("  top 64 alone      %.4f ms" % timed(fd[:64]))
    print("  all but top 64    %.4f ms" % timed(fd[64:]))
    print("  all but top 1024  %.4f ms" % timed(fd[1024:]))


if __name__ == "__main__":
    main()
