#!/usr/bin/env python3
"""Per-stream timeline of one grouped decode launch over the bench batch (GPU, profiling build).

Loads libcovt_timing.so (make -C cov-tiles_amd timing), whose kernels write (duration, start) in
100 MHz s_memrealtime ticks in place of each stream's result, and prints per op: total wave time,
duration percentiles, the slowest streams and the launch's critical path.  The results are not
decode results, so this never runs in the product path."""
import ctypes
import os
import sys

os.environ["COVT_LIB_VARIANT"] = os.environ.get("TIMING_LIB", "libcovt_timing.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402

NAMES = {101: "L_BYTE_RLE", 102: "L_RLE_U64", 103: "L_RLE_I32", 104: "L_RLE_S64",
         1: "BYTE_RLE", 2: "RLE_U64", 3: "RLE_I32", 4: "RLE_S64", 7: "VAR_ZZD", 8: "VAR_XY", 9: "VAR_MORTON",
         10: "FPF_ZZD", 11: "FPF_XY", 12: "FPF_MORTON", 13: "VAR_U64", 14: "VAR_I32_I64", 15: "VAR_ZZD_I64",
         16: "BYTE_RLE_RAW", 116: "L_BYTE_RAW", 17: "VAR_ZZ_I64J", 18: "VAR_ZZ_S64", 19: "VAR_ZZD_S64"}
TICK_US = 0.01  # 100 MHz


def main():
    import torch

    covt = bench.load_covt()
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    tiles = int(args[0]) if args else 10000
    if "--omt" in sys.argv:  # the MVT-vs-COVT GPU set: decodable OMT fixtures replicated to `tiles`
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import mvt_vs_covt

        lib = [open(os.path.join(mvt_vs_covt.COVT_DIR, n + ".covt"), "rb").read() for n in mvt_vs_covt._decodable()]
        tile_bytes = [lib[i % len(lib)] for i in range(tiles)]
    else:
        tile_bytes = [t for _, t in bench.sample_batch(bench.tile_library(), tiles, bench.SEED)]
    for a in sys.argv[1:]:  # --shard=N/k: shard k of the N-way LPT split (bench.py's strong scaling)
        if a.startswith("--shard="):
            n, k = (int(x) for x in a[8:].split("/"))
            sh = bench.lpt_shards([len(t) for t in tile_bytes], n)[k]
            tile_bytes = [tile_bytes[i] for i in sh]
            print("shard %d of %d: %d tiles" % (k, n, len(tile_bytes)))
    # --props: the plan also decodes every property column's streams (COVT_PLAN_PROPERTIES)
    opts = {}
    for a in sys.argv[1:]:  # --opts=k=v,k=v: plan options (covt.PlanOptions)
        if a.startswith("--opts="):
            opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a[7:].split(",") if kv}
    plan = covt.Plan.from_tiles(tile_bytes, flags=covt.PLAN_PROPERTIES if "--props" in sys.argv else 0,
                                options=covt.PlanOptions(**opts))
    batch = covt.DeviceBatch(plan, "cuda")
    L = covt.lib()
    phase = torch.zeros(max(plan.num_streams, plan.descs.size // 32) * 8, dtype=torch.int32, device="cuda")  # (a row per descriptor)
    L.covt_debug_set_phase_buffer(ctypes.c_void_p(phase.data_ptr()), ctypes.c_void_p(batch.d_desc.data_ptr()))
    for _ in range(3):
        batch.decode()
    torch.cuda.synchronize()
    ph_launch = phase.cpu().numpy().view(np.uint32).reshape(-1, 8).astype(np.int64)
    _, res = batch.results()
    dur = res[:, 0].astype(np.int64)
    start = res[:, 1].astype(np.int64) & 0xffffffff
    if (dur < 0).any():
        print("streams with errors:", int((dur < 0).sum()))
    s = plan.streams
    di = s["desc_index"]
    ops = plan.descs.reshape(-1, 32)[:, 24]
    lane = (plan.descs.reshape(-1, 32)[:, 26] & 1).astype(bool)
    op_t = np.empty(len(s), dtype=np.int64)
    op_t[:] = ops[di] + 100 * lane[di]  # lane-kernel streams: op + 100
    d_t = dur  # results are in tile order
    st_t = start
    fl = plan.descs.reshape(-1, 32)[:, 26]
    heads = np.nonzero(((fl & covt.DESC_SPLIT) != 0) & ((fl & covt.DESC_SPLIT_PAD) == 0))[0]
    if heads.size:  # split streams: (duration, start) of each chunk in its head descriptor's phase row
        hs = plan.desc_streams[heads]
        c_st = ph_launch[heads, 1]
        c_en = c_st + ph_launch[heads, 0]
        sst = np.full(len(s), np.iinfo(np.int64).max)
        sen = np.zeros(len(s), dtype=np.int64)
        np.minimum.at(sst, hs, c_st)
        np.maximum.at(sen, hs, c_en)
        sp = np.unique(hs)
        st_t = st_t.copy()
        d_t = d_t.copy()
        st_t[sp] = sst[sp]
        d_t[sp] = sen[sp] - sst[sp]
        op_t[sp] += 200  # split streams: op + 200 (first chunk start -> last chunk end)
        print("split: %d streams in %d chunks, chunk wave-time %.1f us, p50 chunk %.1f us, max chunk %.1f us" % (
            sp.size, heads.size, ph_launch[heads, 0].sum() * TICK_US, np.percentile(ph_launch[heads, 0], 50) * TICK_US,
            ph_launch[heads, 0].max() * TICK_US))
    t0 = st_t.min()
    end_t = st_t - t0 + d_t
    print("launch span %.1f us (first start -> last end); %d streams" % (end_t.max() * TICK_US, len(s)))
    # concurrency profile: streams in flight per 5% of the span, and the output bytes finished per slice
    span = end_t.max()
    nb = 20
    ob = (s["out_elems"] * s["elem_bytes"]).astype(np.float64)
    line_w, line_b = [], []
    for q in range(nb):
        t0q, t1q = span * q / nb, span * (q + 1) / nb
        st_rel = st_t - t0
        live = ((st_rel < t1q) & (end_t > t0q)).sum()
        fin = ob[(end_t > t0q) & (end_t <= t1q)].sum()
        line_w.append("%5d" % live)
        line_b.append("%5.0f" % (fin / 1e6))
    print("streams in flight per 5%% of the launch: " + " ".join(line_w))
    print("output MB finished per 5%% slice:        " + " ".join(line_b))
    print("last 8 streams to finish (op, bytes, values, start us, duration us):")
    for i in np.argsort(-end_t)[:8]:
        print("   %-12s %8d %8d  start %7.1f  dur %7.1f" % (NAMES.get(int(op_t[i]), op_t[i]), s["byte_length"][i],
                                                          s["num_values"][i], (st_t[i] - t0) * TICK_US,
                                                          d_t[i] * TICK_US))
    for o, n in list(NAMES.items()):
        if o < 100:
            NAMES[o + 200] = "S_" + n
    fam_of = {1: 0, 2: 0, 3: 0, 4: 0, 16: 0}
    for fam, name in enumerate(("RLE", "VARINT", "FASTPFOR", "LANE")):
        m = np.array([(3 if 100 <= o < 200 else fam_of.get(int(o) % 200, 2 if o % 200 in (10, 11, 12) else 1)) == fam
                      for o in op_t])
        if m.any():
            print("  family %-8s first start %7.1f us  last start %7.1f us  last end %7.1f us  wave-time %9.1f us"
                  % (name, (st_t[m].min() - t0) * TICK_US, (st_t[m].max() - t0) * TICK_US, end_t[m].max() * TICK_US,
                     d_t[m].sum() * TICK_US))
    print("%-12s %7s %9s %9s %8s %8s %8s %8s  %s" % ("op", "streams", "MB", "wave-ms", "p50 us", "p99 us", "max us",
                                                    "ns/B", "slowest (bytes, values, us)"))
    for op in sorted(set(op_t.tolist())):
        m = op_t == op
        d = d_t[m] * TICK_US
        b = s["byte_length"][m]
        nv = s["num_values"][m]
        top = np.argsort(-d)[:3]
        print("%-12s %7d %9.1f %9.2f %8.2f %8.2f %8.1f %8.2f  %s" % (
            NAMES.get(op, op), int(m.sum()), b.sum() / 1e6, d.sum() / 1e3, np.percentile(d, 50),
            np.percentile(d, 99), d.max(), d.sum() * 1e3 / max(b.sum(), 1),
            " ".join("(%d,%d,%.1f)" % (b[i], nv[i], d[i]) for i in top)))
    print("wave time (ms) by op and stream size:")
    edges = (0, 64, 256, 1024, 4096, 16384, 65536, 1 << 30)
    print("%-12s" % "op" + "".join("%16s" % ("<%d" % e) for e in edges[1:]))
    for op in sorted(set(op_t.tolist())):
        m = op_t == op
        b = s["byte_length"]
        cells = []
        for lo, hi in zip(edges[:-1], edges[1:]):
            mm = m & (b >= lo) & (b < hi)
            cells.append("%7.1f/%-8d" % (d_t[mm].sum() * TICK_US / 1e3, int(mm.sum())))
        print("%-12s" % NAMES.get(op, op) + "".join("%16s" % c for c in cells))
    if len(ph_launch) < int(di.max()) + 1:  # (a split plan's descriptors outnumber its streams)
        return
    ph = ph_launch[di]  # tile order
    print("shader clocks by phase (G = 1e9 clocks; RLE: 0 window 1 next[] 2 walk 3 small-groups 4 big-groups "
          "5 long-literal 7 loop; FPF: 0 page-dir 1 stage 2 walk+prefetch 3 unpack 4 exceptions 5 sink 6 tail)")
    for op in sorted(set(op_t.tolist())):
        m = op_t == op
        tot = ph[m].sum(axis=0)
        if tot.sum() == 0:
            continue
        print("%-12s total %7.3f G  " % (NAMES.get(op, op), tot.sum() / 1e9) +
              " ".join("%d:%4.1f%%" % (k, 100.0 * tot[k] / tot.sum()) for k in range(8) if tot[k]))
    if heads.size:
        # split chunks: phase clocks of run_fastpfor / the varint decode in slots 2..7 of each chunk's row (phases
        # 0..5, s_memtime clocks), (duration, start) in slots 0, 1 (100 MHz ticks).  The clock rate is calibrated
        # on the whole streams (their phases cover their whole decode); a chunk's time outside its phases is its
        # setup, look-back and carry.
        whole = np.ones(len(s), dtype=bool)
        whole[np.unique(plan.desc_streams[heads])] = False
        clk = ph[whole].sum(axis=1)
        ok = (d_t[whole] > 0) & (clk > 0)
        ghz = (clk[ok].sum() / (d_t[whole][ok].sum() * TICK_US * 1e3)) if ok.any() else 0.0
        print("split chunks by phase (shader clock %.2f GHz from the whole streams; 'rest' = wall time outside the phases: "
              "setup, look-back, carry)" % ghz)
        hop = ops[heads]
        for op in sorted(set(hop.tolist())):
            m = hop == op
            tot = ph_launch[heads][m, 2:8].sum(axis=0)
            wall = ph_launch[heads][m, 0].sum() * TICK_US
            inph = tot.sum() / (ghz * 1e3) if ghz else 0.0
            print("  %-12s chunks %5d  wall %9.1f us  p50 %6.1f us  " % (
                NAMES.get(int(op), op), int(m.sum()), wall, np.percentile(ph_launch[heads][m, 0], 50) * TICK_US) +
                " ".join("%d:%4.1f%%" % (k, 100.0 * tot[k] * 1e-3 / ghz / wall) for k in range(6) if tot[k] and ghz) +
                "  rest:%4.1f%%" % (100.0 * max(wall - inph, 0.0) / wall if wall else 0.0))
    # duration vs size buckets
    print("duration by stream size (all ops):")
    b = s["byte_length"]
    for lo, hi in ((0, 64), (64, 256), (256, 1024), (1024, 4096), (4096, 16384), (16384, 65536), (65536, 1 << 30)):
        m = (b >= lo) & (b < hi)
        if m.any():
            d = d_t[m] * TICK_US
            print("  [%6d,%9d) n=%7d  mean %7.2f us  p99 %7.2f us  ns/B %7.2f" % (
                lo, hi, int(m.sum()), d.mean(), np.percentile(d, 99), d.sum() * 1e3 / b[m].sum()))


if __name__ == "__main__":
    main()
