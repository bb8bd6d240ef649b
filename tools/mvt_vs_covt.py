#!/usr/bin/env python3
"""MVT-vs-COVT decode benchmark (the reference's side-by-side is
parser/js/test/benchmark/decodingPerformance.ts:37-55, and README.md:37-44 publishes COVT/MVT
decode-speed ratios of 2.36x (z4) and 2.74x (z5)).

CPU mode (default; needs the reference's MVT originals, so it runs in the build container):
for every OMT tile with both an MVT original and a committed COVT fixture, one host thread decodes
  * MVT:  protobuf + geometry commands -> feature ids, types, vertices (oracle/mvt_decode.c), and
  * COVT: every Id + Geometry stream (oracle_decode_tiles_mt, the C restatement of DecodingUtils),
the same geometry and ids either way, and the script prints tiles/s, MB/s of tile bytes and the
COVT/MVT speed ratio per zoom and overall.

GPU mode (--gpu N): the committed OMT COVT fixtures replicated to N tiles, one grouped decode launch
(libcovt), timed with HIP events -> tiles/s, for the GPU-vs-CPU side of the same comparison.

usage: mvt_vs_covt.py [--reps R] [--mvt-dir DIR] | mvt_vs_covt.py --gpu N"""
import glob
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
COVT_DIR = os.path.join(ROOT, "tests", "golden", "tiles", "omt")


def _arg(name, default):
    return type(default)(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def _decodable():
    """OMT fixtures the reference decoder decodes (tests/golden/oracle_streams.json; the others fail in
    Java too and are parity cases, not benchmark input)"""
    import json

    rec = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_streams.json")))["tiles"]
    return sorted(os.path.basename(f)[:-5] for f in glob.glob(os.path.join(COVT_DIR, "*.covt"))
                  if rec["omt/" + os.path.basename(f)[:-5]]["decodable"])


def cpu(reps, mvt_dir):
    import oracle

    names = _decodable()
    pairs = [(n, open(os.path.join(mvt_dir, n + ".mvt"), "rb").read(), open(os.path.join(COVT_DIR, n + ".covt"), "rb").read())
             for n in names if os.path.exists(os.path.join(mvt_dir, n + ".mvt"))]
    if not pairs:
        sys.exit("no MVT originals under %s" % mvt_dir)
    by_zoom = {}
    for n, m, c in pairs:
        by_zoom.setdefault(int(n.split("_")[0]), []).append((n, m, c))
    print("MVT vs COVT decode, 1 host thread, %d OMT tiles (ids + geometry; MVT: protobuf + commands -> vertices,"
          " COVT: every Id/Geometry stream), best of %d reps" % (len(pairs), reps))
    print("%5s %6s %10s %10s %12s %12s %9s" % ("zoom", "tiles", "MVT KB", "COVT KB", "MVT ms", "COVT ms", "COVT/MVT"))
    tot = [0, 0, 0.0, 0.0, 0]
    for z in sorted(by_zoom):
        grp = by_zoom[z]
        blob = np.frombuffer(b"".join(c for _, _, c in grp), dtype=np.uint8)
        sizes = np.array([len(c) for _, _, c in grp], dtype=np.uint64)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
        mvts = [m for _, m, _ in grp]
        for m in mvts:  # correctness first: every tile decodes
            assert oracle.mvt_decode(m)[0] == 0
        st = oracle.decode_tiles_mt(blob, offs, sizes, threads=1)[0]
        assert st == 0, st
        t_m = t_c = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            for m in mvts:
                oracle.mvt_decode(m)
            t_m = min(t_m, time.perf_counter() - t0)
            t0 = time.perf_counter()
            oracle.decode_tiles_mt(blob, offs, sizes, threads=1)
            t_c = min(t_c, time.perf_counter() - t0)
        mb, cb = sum(len(m) for m in mvts), int(sizes.sum())
        print("%5d %6d %10.1f %10.1f %12.3f %12.3f %8.2fx" % (z, len(grp), mb / 1e3, cb / 1e3, 1e3 * t_m, 1e3 * t_c, t_m / t_c))
        tot[0] += len(grp); tot[1] += mb; tot[2] += t_m; tot[3] += t_c; tot[4] += cb
    print("%5s %6d %10.1f %10.1f %12.3f %12.3f %8.2fx" % ("all", tot[0], tot[1] / 1e3, tot[4] / 1e3, 1e3 * tot[2],
                                                           1e3 * tot[3], tot[2] / tot[3]))
    print("MVT %.0f tiles/s (%.1f MB/s of MVT bytes); COVT %.0f tiles/s (%.1f MB/s of COVT bytes), 1 thread"
          % (tot[0] / tot[2], tot[1] / tot[2] / 1e6, tot[0] / tot[3], tot[4] / tot[3] / 1e6))


def gpu(n_tiles):
    import torch

    import bench

    covt = bench.load_covt()
    lib = [open(os.path.join(COVT_DIR, n + ".covt"), "rb").read() for n in _decodable()]
    tiles = [lib[i % len(lib)] for i in range(n_tiles)]
    plan = covt.Plan.from_tiles(tiles)
    assert (plan.tile_status == 0).all()
    batch = covt.DeviceBatch(plan, "cuda")
    stream = torch.cuda.current_stream()
    for _ in range(3):
        batch.decode(stream)
    torch.cuda.synchronize()
    _, res = batch.results()
    assert (res[:, 0] == 0).all()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for s, e in ev:
        s.record(stream)
        batch.decode(stream)
        e.record(stream)
    torch.cuda.synchronize()
    per = [s.elapsed_time(e) for s, e in ev]
    print("per-launch ms:", " ".join("%.3f" % t for t in per))
    ms = float(np.median(per))
    print("GPU COVT decode (ids + geometry), %d OMT tiles (%d distinct, %.1f MB): %.3f ms per launch, %.0f tiles/s, %.1f GB/s"
          % (n_tiles, len(lib), plan.in_bytes / 1e6, ms, n_tiles / ms * 1e3, plan.in_bytes / ms / 1e6))


if __name__ == "__main__":
    if "--gpu" in sys.argv:
        gpu(_arg("--gpu", 9200))
    else:
        cpu(_arg("--reps", 5), _arg("--mvt-dir", "/root/reference/test/fixtures/omt/mvt"))
