#!/usr/bin/env python3
"""Per-stream timeline of the BASELINE config 2-4 launches (GPU, profiling build libcovt_timing.so).

For each config: HIP-event time of the launch, the in-kernel span (first stream start -> last stream
end, s_memrealtime at 100 MHz), and the slowest streams -- to tell launch overhead from long poles.
Split streams (their chunks run in the split kernels, which keep real results) are listed apart:
only the whole-stream kernels write timestamps.  Phase clocks (thousands of shader clocks) per stream:
RLE 0 window 1 next[] 2 walk 3 runs 4 literals 5 long literal 7 loop; FastPFOR as stream_timeline.py."""
import ctypes
import os
import sys

os.environ["COVT_LIB_VARIANT"] = "libcovt_timing.so"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from stream_timeline import NAMES, TICK_US  # noqa: E402


def main():
    import torch

    covt = bench.load_covt()
    lib = bench.tile_library()
    for name in bench.CONFIG_LEGS:
        picks = bench.config_tiles(lib, name)
        plan = covt.Plan.from_tiles([t for _, t in picks])
        mask = bench.config_mask(plan, name)
        batch = covt.DeviceBatch(plan, "cuda")
        sub = batch.subset(mask)
        sub_descs = plan.subset_descs(mask)[0].view(np.uint8)
        s = torch.cuda.current_stream()
        phase = torch.zeros(max(sub.num_descs, 1) * 8, dtype=torch.int32, device="cuda")
        covt.lib().covt_debug_set_phase_buffer(ctypes.c_void_p(phase.data_ptr()), ctypes.c_void_p(sub.d_desc.data_ptr()))
        for _ in range(3):
            sub.decode(s)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(s)
        sub.decode(s)
        ev[1].record(s)
        torch.cuda.synchronize()
        _, res, idx = sub.results()
        ph = phase.cpu().numpy().view(np.uint32).reshape(-1, 8)[:sub.num_descs][sub.stream_index >= 0]
        st = plan.streams
        fam0 = int(plan.family_counts[:covt.FAMILY_SPLIT].sum())
        split = st["desc_index"][idx] >= fam0
        print("%s: %d split streams (%s)" % (name, int(split.sum()), ", ".join(
            "%s %d B" % (NAMES.get(int(st["op"][j]), st["op"][j]), st["byte_length"][j]) for j in idx[split][:8])))
        res, idx, ph = res[~split], idx[~split], ph[~split]
        # split chunks: (duration, start) in their chunk descriptor's phase row
        sd = sub_descs.reshape(-1, 32)
        flags = sd[:, 26].astype(np.int64) | (sd[:, 27].astype(np.int64) << 8)
        allph = phase.cpu().numpy().view(np.uint32).reshape(-1, 8)[:sub.num_descs]
        chunk_rows = np.nonzero((flags & covt.DESC_SPLIT) != 0)[0]
        dur = res[:, 0].astype(np.int64)
        start = res[:, 1].astype(np.int64) & 0xffffffff
        end = start + dur
        t0 = start.min()
        st = plan.streams
        ops = st["op"][idx]
        print("%s: %d streams, event %.1f us, in-kernel span %.1f us, last start %.1f us" % (
            name, len(idx), ev[0].elapsed_time(ev[1]) * 1e3, (end.max() - t0) * TICK_US, (start.max() - t0) * TICK_US))
        if chunk_rows.size:
            cdur = allph[chunk_rows, 0].astype(np.int64)
            cst = allph[chunk_rows, 1].astype(np.int64)
            kind = np.where((flags[chunk_rows] & covt.DESC_SPLIT_FPF) != 0, 1,
                            np.where((flags[chunk_rows] & covt.DESC_SPLIT_RLE) != 0, 2, 0))
            for f, fname in ((0, "SPLIT"), (1, "SPLIT_FPF"), (2, "SPLIT_RLE")):
                m = kind == f
                if not m.any():
                    continue
                k = np.nonzero(m)[0][np.argmax(cdur[m])]
                row = sd[chunk_rows[k]]
                op, nv, bl = int(row[24]), int(row[20:24].view(np.int32)[0]), int(row[28:32].view(np.int32)[0])
                if not cst[m].any():  # the fused kernel (small launches) records no chunk (duration, start)
                    print("   family %-9s chunks=%4d (in the fused kernel: chunk start / duration not recorded) of %s %d B "
                          "%d vals, phase kclk %s" % (fname, int(m.sum()), NAMES.get(op, op), bl, nv,
                                                      " ".join("%d" % (x // 1000) for x in allph[chunk_rows[k], 2:])))
                    continue
                print("   family %-9s chunks=%4d first start %6.1f last start %6.1f last end %6.1f us; longest chunk "
                      "%.1f us (start %.1f) of %s %d B %d vals, phase kclk %s" % (
                          fname, int(m.sum()), (cst[m].min() - t0) * TICK_US, (cst[m].max() - t0) * TICK_US,
                          (cst[m] + cdur[m] - t0).max() * TICK_US, cdur[k] * TICK_US, (cst[k] - t0) * TICK_US,
                          NAMES.get(op, op), bl, nv, " ".join("%d" % (x // 1000) for x in allph[chunk_rows[k], 2:])))
        for i in np.argsort(-end)[:6]:
            j = idx[i]
            print("   %-12s bytes %7d values %7d  start %7.1f us  dur %7.1f us" % (
                NAMES.get(int(ops[i]), ops[i]), st["byte_length"][j], st["num_values"][j], (start[i] - t0) * TICK_US,
                dur[i] * TICK_US) + "  phase kclk " + " ".join("%d" % (x // 1000) for x in ph[i]))
        fl = plan.descs.reshape(-1, 32)[st["desc_index"][idx], 26]
        fam = np.where(fl & 1, 3, np.where(np.isin(ops, (10, 11, 12)), 2,
                                           np.where(np.isin(ops, (1, 2, 3, 4, 16)), 0, 1)))
        for f, fname in enumerate(("RLE", "VARINT", "FASTPFOR", "LANE")):
            m = fam == f
            if not m.any():
                continue
            k = np.nonzero(m)[0][np.argmax(dur[m])]
            print("   family %-8s n=%4d first start %6.1f last start %6.1f last end %6.1f us; longest %s %d B %d vals "
                  "%.1f us (start %.1f)" % (fname, int(m.sum()), (start[m].min() - t0) * TICK_US,
                                            (start[m].max() - t0) * TICK_US, (end[m].max() - t0) * TICK_US,
                                            NAMES.get(int(ops[k]), ops[k]), st["byte_length"][idx[k]],
                                            st["num_values"][idx[k]], dur[k] * TICK_US, (start[k] - t0) * TICK_US))
        del sub, batch, plan


if __name__ == "__main__":
    main()
