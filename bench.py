#!/usr/bin/env python3
"""Benchmark: GB/s of raw COVT Id+Geometry stream bytes decoded (+ Mvertices/s) on a z2-z14 tile batch.

BASELINE.json config 5: a 10k-tile mixed-zoom batch sampled with numpy.random.default_rng(20250117),
uniform over the zoom levels that have decodable fixtures, then uniform over that zoom's tiles, from the
90 OMT + 27 Bing decodable fixtures (tests/golden/tiles, byte-identical copies of the reference's
test/fixtures).  A "step" is one decode launch over the whole batch: every Id/Geometry stream of every
tile, inputs (tile bytes + descriptor table) already resident in HBM, outputs written to HBM.

  python bench.py [--gpus N --steps K --warmup W]

N>1: one process per GPU -- either started by torch.distributed.run (WORLD_SIZE/RANK/LOCAL_RANK in the
environment) or, without a launcher, spawned here (one child per GPU, started before anything touches
the GPU; fails if fewer than N GPUs are visible).  Scaling is strong by default, as BASELINE config 5
states it ("10k-tile batch ... sharded across 8xMI355X"): one 10k-tile batch split over the ranks by the
greedy longest-processing-time byte balance of SURVEY §8(e).  At N > 1 the line also carries `weak`: every
rank then decodes a whole 10k-tile batch of its own (seed 20250117 + rank), the per-GPU-work-fixed figure;
`--scaling weak` makes that the headline instead.  Tiles are independent, so there is no collective on
the data path and no RCCL: a gloo group carries the timing barriers and gathers the per-rank numbers.
Besides `value` (config 5) the line carries BASELINE configs 2-4 (`configs`), the PCIe-inclusive and
C-ABI host timings, the device plan (+ decode: `device_plan.plan_plus_decode`), assembly and property legs,
and the CPU baseline.
"""
from __future__ import annotations

import argparse
import glob
import importlib.util
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
METRIC = "GB/s raw COVT bytes decoded + Mvertices/s, z2–z14 tile batch, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md (spec)
SEED = 20250117


def load_covt():
    if "covtiles_amd" in sys.modules:
        return sys.modules["covtiles_amd"]
    path = os.path.join(ROOT, "cov-tiles_amd", "__init__.py")
    spec = importlib.util.spec_from_file_location("covtiles_amd", path,
                                                  submodule_search_locations=[os.path.dirname(path)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["covtiles_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


# sources that decide the decode launch's traffic: the kernels and the plan that lays out their work
KERNEL_SOURCES = ("cov-tiles_amd/csrc/covt_decode.hip", "cov-tiles_amd/csrc/covt_wave.h",
                  "cov-tiles_amd/csrc/covt_internal.h", "cov-tiles_amd/csrc/covt_host.cpp", "include/covt.h")


def kernel_sources_sha256():
    """Fingerprint of KERNEL_SOURCES: profiles/pmc_traffic.json carries the one it was measured on, and
    the bench line reports its traffic only while they match (a kernel change makes it stale, not wrong)."""
    import hashlib

    h = hashlib.sha256()
    for p in KERNEL_SOURCES:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def tile_library():
    """Decodable OMT + Bing fixtures -> {zoom: [(key, bytes)]}."""
    with open(os.path.join(ROOT, "tests", "golden", "oracle_streams.json")) as f:
        rec = json.load(f)["tiles"]
    lib = {}
    for s in ("omt", "bing"):
        for p in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "tiles", s, "*.covt"))):
            key = s + "/" + os.path.basename(p)[:-5]
            if not rec[key]["decodable"]:
                continue
            z = int(os.path.basename(p).replace("-", "_").split("_")[0])
            lib.setdefault(z, []).append((key, open(p, "rb").read()))
    return lib


def sample_batch(lib, n_tiles, seed):
    rng = np.random.default_rng(seed)
    zooms = sorted(lib)
    zs = rng.choice(zooms, size=n_tiles)
    picks = []
    for z in zs:
        cand = lib[int(z)]
        picks.append(cand[int(rng.integers(0, len(cand)))])
    return picks


def lpt_shards(weights, n):
    order = np.argsort(-np.asarray(weights), kind="stable")
    load = np.zeros(n)
    shard = [[] for _ in range(n)]
    for i in order:
        g = int(np.argmin(load))
        shard[g].append(int(i))
        load[g] += weights[i]
    return [sorted(s) for s in shard]


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup-v2 CPU quota."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    n = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return n, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota}


def cpu_baseline(plan, args, config1_tile=None):
    """SURVEY §8(d) "CPU timing": the oracle (C restatement of the Java DecodingUtils semantics; the Java
    decoder cannot run, §8(c)) built -O3 -march=native on this host, over the SAME batch as the GPU run
    (every tile walked + every Id/Geometry stream decoded, one tile per task), all usable host cores:
    median of >= 20 timed iterations after 3 warm-ups; plus a 1-thread figure on the same batch.  At N > 1
    rank 0 runs it over its own batch (every rank's batch has the same size and zoom mix).
    `config1_tile`: BASELINE configs[0] -- that one tile decoded whole (CovtParser.decodeCovt: walk, Id /
    Geometry streams, geometry assembly, property columns) on one thread, and its Id / Geometry part alone."""
    import tempfile

    sys.path.insert(0, ROOT)
    import oracle as O

    bdir = tempfile.mkdtemp(prefix="covt_oracle_native_")
    try:
        L = O.load_native(O.build_native(bdir))
        march = "native"
    except (OSError, subprocess.CalledProcessError):  # no compiler on this host: the portable in-tree build
        L, march = O.lib(), "x86-64-v3"
    threads, cpus = host_cpus()
    threads = args.cpu_threads or threads

    def run(nthr):
        t = time.perf_counter()
        st, ib, ob, vx = O.decode_tiles_mt(plan.blob, plan.offsets, plan.sizes, O.FMT_GENC, args.id_mode, nthr, L)
        el = time.perf_counter() - t
        if st != 0:
            raise RuntimeError("oracle baseline failed: %d" % st)
        return el, ib, vx

    for _ in range(3):
        run(threads)
    times = [run(threads)[0] for _ in range(max(args.cpu_iters, 1))]
    _, ib, vx = run(threads)
    med = float(np.median(times))
    # the same with one thread per CPU the OS reports (os.cpu_count(); on the box 256 while the cgroup
    # quota allows 16 at a time): recorded beside `value`, which uses the usable cores
    nproc = os.cpu_count() or threads
    run(nproc)
    med_np = float(np.median([run(nproc)[0] for _ in range(5)]))
    el1, _, _ = run(1)  # 1 thread: one warm-up-free pass is already seconds long; take the median of 3
    times1 = [el1] + [run(1)[0] for _ in range(2 if el1 < 10 else 0)]
    med1 = float(np.median(times1))
    c1 = None
    if config1_tile is not None:
        st, cnt = O.decode_tile_full(config1_tile, O.FMT_GENC, args.id_mode, L)
        if st != 0:
            raise RuntimeError("oracle full-tile decode failed: %d" % st)
        one = np.frombuffer(config1_tile, dtype=np.uint8)
        o1, s1 = np.zeros(1, dtype=np.uint64), np.array([len(config1_tile)], dtype=np.uint64)

        def idgeom():
            return O.decode_tiles_mt(one, o1, s1, O.FMT_GENC, args.id_mode, 1, L)

        def med_ms(fn, reps=30):
            for _ in range(3):
                fn()
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t)
            return float(np.median(ts)) * 1e3

        c1 = {"cpu_full_ms_1thread": round(med_ms(lambda: O.decode_tile_full(config1_tile, O.FMT_GENC,
                                                                            args.id_mode, L)), 4),
              "cpu_id_geometry_ms_1thread": round(med_ms(idgeom), 4), "cpu_counts": cnt,
              "cpu_note": "oracle/covt_oracle_tile.c (walk + Id/Geometry streams + geometry assembly + property "
                          "columns, as CovtParser.decodeCovt) and the Id/Geometry part alone, one thread, median "
                          "of 30 after 3 warm-ups"}
    return {"value": round(ib / med / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port", "config1": c1,
            "sample": "the full bench batch (%d tiles, %.1f MB stream bytes), median of %d iterations after 3 "
                      "warm-ups (%.1f ms); oracle/covt_oracle.c (C restatement of DecodingUtils + ORC + "
                      "FastPFOR) built -O3 -march=%s here, %d threads, one tile per task" %
                      (plan.n_tiles, ib / 1e6, len(times), med * 1e3, march, threads),
            "mvert_per_s": round(vx / med / 1e6, 3),
            "value_nproc_threads": round(ib / med_np / 1e9, 4), "nproc_threads": nproc,
            "ms_nproc_threads": round(med_np * 1e3, 1),
            "value_1thread": round(ib / med1 / 1e9, 4), "ms_1thread": round(med1 * 1e3, 1),
            "iters_1thread": len(times1),
            "host": dict(cpus, cpu_model=cpu_model())}


def end_to_end(plan, batch, stream, torch, dev, reps):
    """SURVEY §8(d) second timing: pinned host tiles -> H2D -> decode -> D2H of every output (not `value`)."""
    h_in = torch.from_numpy(plan.blob).pin_memory()
    h_desc = torch.from_numpy(plan.descs).pin_memory() if plan.num_streams else None
    h_out = torch.empty(batch.d_out.numel(), dtype=torch.uint8).pin_memory()
    h_res = torch.empty(batch.d_res.numel(), dtype=torch.int32).pin_memory()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tot = [0.0, 0.0, 0.0, 0.0]
    with torch.cuda.stream(stream):
        for i in range(reps + 1):
            ev[0].record(stream)
            batch.d_in.copy_(h_in, non_blocking=True)
            if h_desc is not None:
                batch.d_desc.copy_(h_desc, non_blocking=True)
            ev[1].record(stream)
            batch.decode(stream)
            ev[2].record(stream)
            h_out.copy_(batch.d_out, non_blocking=True)
            h_res.copy_(batch.d_res, non_blocking=True)
            ev[3].record(stream)
            torch.cuda.synchronize(dev)
            if i:  # first rep warms the pinned buffers
                tot[0] += ev[0].elapsed_time(ev[3])
                tot[1] += ev[0].elapsed_time(ev[1])
                tot[2] += ev[1].elapsed_time(ev[2])
                tot[3] += ev[2].elapsed_time(ev[3])
    ms = [t / reps for t in tot]
    return {"value": round(plan.in_bytes / (ms[0] * 1e-3) / 1e9, 3), "unit": "GB/s", "ms": round(ms[0], 3),
            "h2d_ms": round(ms[1], 3), "decode_ms": round(ms[2], 3), "d2h_ms": round(ms[3], 3),
            "h2d_GBps": round(h_in.numel() / (ms[1] * 1e-3) / 1e9, 2),
            "d2h_GBps": round(h_out.numel() / (ms[3] * 1e-3) / 1e9, 2), "reps": reps,
            "note": "pinned host tile bytes + descriptors H2D, one decode launch, all outputs + results D2H"}


def torch_device_index():
    import torch

    return torch.cuda.current_device()


def abi_host_leg(plan, t_plan, reps):
    """The C-ABI host entry a JNI/ctypes caller would use (include/covt.h covt_plan_decode_host): pageable
    tile bytes in, device buffers cached on the plan after the first call, H2D, one decode launch, D2H into
    pageable host memory (fresh buffers each call, so first-touch page faults are included; then reused
    caller buffers, and the same through covt_plan_decode_host_shards with two shards on this device, the
    multi-GPU path's per-shard H2D / launch / D2H).  Not `value`."""
    plan.decode_host()  # warm: HIP context, allocator
    t = time.perf_counter()
    for _ in range(reps):
        out, res = plan.decode_host()
        if (res[:, 0] != 0).any():
            raise RuntimeError("covt_plan_decode_host reported stream errors")
        del out, res
    ms = (time.perf_counter() - t) * 1e3 / reps
    # the same call into caller-owned host buffers reused across calls (already touched: no page faults)
    out, res = plan.decode_host()
    t = time.perf_counter()
    for _ in range(reps):
        plan.decode_host(out=out, res=res)
    ms_reuse = (time.perf_counter() - t) * 1e3 / reps
    dev = torch_device_index()
    plan.decode_host(out=out, res=res, shard_devices=[dev, dev])
    t = time.perf_counter()
    for _ in range(reps):
        plan.decode_host(out=out, res=res, shard_devices=[dev, dev])
    ms_shards = (time.perf_counter() - t) * 1e3 / reps
    return {"ms": round(ms, 3), "value": round(plan.in_bytes / (ms * 1e-3) / 1e9, 3), "unit": "GB/s",
            "ms_reused_buffers": round(ms_reuse, 3), "ms_two_shards_reused": round(ms_shards, 3),
            "raw_tiles_to_host_ms": round(ms + t_plan * 1e3, 1), "reps": reps,
            "note": "covt_plan_decode_host wall clock (pageable bytes, device buffers cached on the plan, H2D + "
                    "decode + D2H) into fresh host buffers; ms_reused_buffers: into caller buffers reused across "
                    "calls; ms_two_shards_reused: covt_plan_decode_host_shards, 2 shards on this device; "
                    "raw_tiles_to_host_ms adds the host metadata walk (covt_plan_create)"}


def device_plan_leg(plan, batch, torch, dev, covt, args, t_plan):
    """covt_device_plan_create on the batch already in HBM (include/covt.h "Device-side plan"): the
    container walk, prefix sums, launch-order sort and descriptor fill on the GPU, wall-clock per
    creation (it synchronises twice: the stream count sizes its arrays), median over --device-plan-reps
    after one warm-up.  Its descriptors must equal the host plan's (nothing splits at this size), and
    the decode launch from them runs at the same speed."""
    offs = torch.from_numpy(plan.offsets.astype(np.int64)).to(dev)
    sizes = torch.from_numpy(plan.sizes.astype(np.int64)).to(dev)
    dp = covt.DevicePlan(batch.d_in, offs, sizes, covt.FORMAT_GENC, args.id_mode)
    _, descs, st = dp.host_copy()
    same = bool(descs.tobytes() == plan.descs.tobytes() and np.array_equal(st, plan.tile_status))
    dp.close()
    times = []
    for k in range(args.device_plan_reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        dp = covt.DevicePlan(batch.d_in, offs, sizes, covt.FORMAT_GENC, args.id_mode)
        times.append(time.perf_counter() - t0)
        if k < args.device_plan_reps - 1:
            dp.close()
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for s_, e_ in ev:
        s_.record(stream)
        dp.decode(batch.d_out, batch.d_res, stream)
        e_.record(stream)
    torch.cuda.synchronize(dev)
    _, res = batch.results()
    out = {"ms_median": round(float(np.median(times)) * 1e3, 3), "ms_min": round(min(times) * 1e3, 3),
           "host_plan_ms": round(t_plan * 1e3, 1), "streams": dp.num_streams,
           "descs_equal_host_plan": same, "decode_ms": round(float(np.mean([a.elapsed_time(b) for a, b in ev])), 4),
           "decode_errors": int((res[:, 0] != 0).sum()), "reps": args.device_plan_reps}
    dp.close()
    # tiles in HBM -> decoded arrays, both halves on the GPU (the figure comparable with
    # cpu_baseline, which walks every tile's metadata too): wall clock of the device plan's creation plus
    # its decode launch, synchronised at the end, median over the reps
    pd = []
    for _ in range(max(args.device_plan_reps, 1)):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        dq = covt.DevicePlan(batch.d_in, offs, sizes, covt.FORMAT_GENC, args.id_mode)
        dq.decode(batch.d_out, batch.d_res, stream)
        torch.cuda.synchronize(dev)
        pd.append(time.perf_counter() - t0)
        dq.close()
    pms = float(np.median(pd)) * 1e3
    out["plan_plus_decode"] = {
        "ms_median": round(pms, 3), "value": round(plan.in_bytes / (pms * 1e-3) / 1e9, 2), "unit": "GB/s",
        "achieved_alg_GBps": round((plan.in_bytes + plan.out_bytes) / (pms * 1e-3) / 1e9, 1),
        "note": "covt_device_plan_create (metadata walk, layout, launch order on the GPU) + its decode launch, "
                "tiles already in HBM, wall clock to the final synchronize; raw stream bytes / time"}
    try:
        out["properties"] = device_plan_props(plan, batch, torch, dev, covt, args, offs, sizes)
    except Exception as e:  # noqa: BLE001 -- reported on the line, never fatal to the headline
        out["properties"] = {"error": repr(e)}
    return out


def device_plan_props(plan, batch, torch, dev, covt, args, offs, sizes):
    """The same batch planned with its property columns (COVT_PLAN_PROPERTIES): the whole decodeCovt plan on
    the GPU, checked against the host plan's records and descriptors."""
    popts = covt.PlanOptions(flags=covt.PLAN_PROPERTIES)
    t0 = time.perf_counter()
    hp = covt.Plan(plan.blob, plan.offsets, plan.sizes, covt.FORMAT_GENC, args.id_mode, options=popts)
    t_hp = time.perf_counter() - t0
    ptimes = []
    for k in range(args.device_plan_reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        pdp = covt.DevicePlan(batch.d_in, offs, sizes, covt.FORMAT_GENC, args.id_mode, options=popts)
        ptimes.append(time.perf_counter() - t0)
        if k < args.device_plan_reps - 1:
            pdp.close()
    info, descs, _ = pdp.host_copy()
    pinfo, pdesc = pdp.property_copy()
    psame = bool(info.tobytes() == hp.streams.tobytes() and descs.tobytes() == hp.descs.tobytes() and
                 pinfo.tobytes() == hp.props.tobytes() and pdesc.tobytes() == hp.pdescs.tobytes())
    res = {"ms_median": round(float(np.median(ptimes)) * 1e3, 3), "ms_min": round(min(ptimes) * 1e3, 3),
           "host_plan_ms": round(t_hp * 1e3, 1), "streams": pdp.num_streams,
           "property_columns": pdp.num_property_columns, "equal_host_plan": psame,
           "note": "covt_device_plan_create_opts with COVT_PLAN_PROPERTIES: Id / Geometry / property "
                   "streams, property records, layout and descriptors on the GPU (wall clock per "
                   "creation, 3 syncs)"}
    pdp.close()
    return res


def assembly_leg(batch, plan, stream, args, dist, torch, dev):
    """GPU geometry assembly (nested offsets + ICE gather) over the decoded batch,
    timed on its own (decode output resident); not part of `value`."""
    batch.decode(stream)
    for _ in range(max(args.warmup, 1)):
        batch.assemble(stream)
    torch.cuda.synchronize(dev)
    _, gres = batch.assembly_results()
    if (gres["status"] != 0).any():
        raise RuntimeError("assembly reported errors on %d columns" % int((gres["status"] != 0).sum()))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    for s, e in ev:
        s.record(stream)
        batch.assemble(stream)
        e.record(stream)
    torch.cuda.synchronize(dev)
    ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    g = plan.geom
    n_feat = int(g["n_features"].sum())
    st = plan.streams
    cnt_elems = 0  # geometryOffsets/partOffsets/ringOffsets/vertexOffsets elements read
    for k in range(1, 5):
        idx = g["stream"][:, k]
        idx = idx[idx >= 0]
        cnt_elems += int(st["out_elems"][idx].sum())
    P, R, V = (int(gres[k].astype(np.int64).sum()) for k in ("num_parts", "num_rings", "num_coords"))
    ncol = plan.num_geometry_columns
    # algorithmic bytes: types 1 B + count/offset streams 4 B + one 8-byte x,y read per coordinate;
    # written: the three offset arrays (4 B, n+1 each) + 8 B per coordinate
    alg = n_feat + 4 * cnt_elems + 8 * V + 4 * (n_feat + P + R + 3 * ncol) + 8 * V
    achieved = alg / (ms * 1e-3) / 1e9
    return {"ms": round(ms, 4), "columns": ncol, "features": n_feat, "parts": P, "rings": R, "coords": V,
            "mcoords_per_s": round(V / (ms * 1e-3) / 1e6, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": alg,
                         "kernel": "covt::assemble_kernel (one wave per geometry column)"}}


def properties_leg(picks, args, dist, torch, dev, covt, stream):
    """property columns of the same batch (a second plan with COVT_PLAN_PROPERTIES).
    Times the decode launch over every stream (Id + Geometry + property streams) and the property
    materialization kernel on its own; not part of `value`."""
    plan = covt.Plan.from_tiles([t for _, t in picks], covt.FORMAT_GENC, args.id_mode, covt.PLAN_PROPERTIES)
    batch = covt.DeviceBatch(plan, dev)

    def timed(fn):
        for _ in range(max(args.warmup, 1)):
            fn()
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)
        for s, e in ev:
            s.record(stream)
            fn()
            e.record(stream)
        torch.cuda.synchronize(dev)
        return float(np.mean([s.elapsed_time(e) for s, e in ev]))

    with torch.cuda.stream(stream):
        ms_dec = timed(lambda: batch.decode(stream))
        ms_mat = timed(lambda: batch.materialize_properties(stream))
    _, pres = batch.property_results()
    if (pres["status"] != 0).any():
        raise RuntimeError("property materialization failed on %d columns" % int((pres["status"] != 0).sum()))
    st = plan.streams
    pst = st[st["column_kind"] == 2]
    P = plan.props
    n = P["n_features"].astype(np.int64)
    nb = (n + 7) // 8
    typ = P["type"]
    vbytes = np.where(typ == covt.PROP_BOOLEAN, nb, np.where(typ == covt.PROP_INT64, 8 * n, 4 * n))
    owner = (plan.pdescs["flags"][P["desc_index"]] & covt.PROP_DICT_OWNER) != 0
    nd = P["n_dict"].astype(np.int64)
    db = P["dict_bytes"].astype(np.int64)
    nv = pres["n_valid"].astype(np.int64)
    dense_elem = np.where(typ == covt.PROP_INT64, 8, np.where(typ == covt.PROP_BOOLEAN, 0, 4))
    # algorithmic bytes of the materialization: present bitmap + dense values read (+ lengths and
    # dictionary bytes read per string sub-column), validity + values written (+ offsets and dictionary
    # bytes by the owner)
    rd = nb.sum() + (nv * dense_elem).sum() + (4 * nd + np.where(owner, db, 0)).sum() * 1
    wr = nb.sum() + vbytes.sum() + np.where(owner, 4 * (nd + 1) + db, 0).sum()
    alg = int(rd + wr)
    achieved = alg / (ms_mat * 1e-3) / 1e9
    return {"ms_decode_all_streams": round(ms_dec, 4), "ms_materialize": round(ms_mat, 4),
            "columns": plan.num_property_columns, "streams_all": plan.num_streams,
            "stream_bytes_all": int(plan.in_bytes),
            "note": "stream_bytes_all = Id + Geometry + property stream bytes (present/data/length decoded, "
                    "float data and dictionary bytes read in place)",
            "gbps_raw_all_streams": round(plan.in_bytes / (ms_dec * 1e-3) / 1e9, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": alg,
                         "kernel": "covt::props_kernel (one wave per property (sub)column)"}}


CONFIG_LEGS = {
    # BASELINE.json configs[1..3]: stream selections of the reference's OMT fixtures
    "config2": ("VertexBuffer Int32 ZigZag-delta-varint decode, one z5 tile (omt/5_16_20): its VERTEX_BUFFER "
                "streams with encoding VARINT_DELTA_ZIG_ZAG (5 ICE_MORTON + 1 PLAIN)"),
    "config3": "Full geometry column (RLE offsets + VertexBuffer), OMT z2-z8 batch: every geometry stream",
    "config4": ("FastPFOR128 topology streams + Id column, OMT z9-z14 batch: FastPFOR non-VertexBuffer geometry "
                "streams + every Id stream"),
}


def config_tiles(lib, name):
    omt = {z: [(k, t) for k, t in tl if k.startswith("omt/")] for z, tl in lib.items()}
    if name == "config2":
        return [(k, t) for k, t in omt[5] if k == "omt/5_16_20"]
    zs = range(2, 9) if name == "config3" else range(9, 15)
    return [kt for z in zs for kt in omt.get(z, [])]


def config_mask(plan, name):
    st = plan.streams
    geom = st["column_kind"] == 1
    if name == "config2":
        return geom & (st["stream_type"] == 9) & (st["encoding"] == 4)
    if name == "config3":
        return geom
    return (geom & (st["encoding"] == 9) & (st["stream_type"] != 9)) | (st["column_kind"] == 0)


CONFIG1_TILE = "omt/5_16_20"  # BASELINE configs[0]: test/fixtures/omt/covt/5_16_20.covt


def config1_tile(lib):
    return dict(lib[5])[CONFIG1_TILE]


def config1_leg(lib, args, torch, dev, covt, stream):
    """BASELINE configs[0] (the reference's single-tile CPU decode, CovtParser.decodeCovt :53-133) on the
    GPU: the z5 tile 5_16_20 decoded whole -- every Id / Geometry / property stream in one decode launch,
    then geometry assembly and property materialization, on one stream -- as one tile's latency (HIP events
    around the three launches, mean of --steps after --warmup), plus the decode launch alone.  The CPU
    figures for the same tile come from the cpu_baseline leg (merged into this object)."""
    tile = config1_tile(lib)
    plan = covt.Plan.from_tiles([tile], covt.FORMAT_GENC, args.id_mode, covt.PLAN_PROPERTIES)
    batch = covt.DeviceBatch(plan, dev)

    def full():
        batch.decode(stream)
        batch.assemble(stream)
        batch.materialize_properties(stream)

    def timed(fn):
        with torch.cuda.stream(stream):
            for _ in range(max(args.warmup, 3)):
                fn()
            torch.cuda.synchronize(dev)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(max(args.steps, 20))]
            for s_, e_ in ev:
                s_.record(stream)
                fn()
                e_.record(stream)
            torch.cuda.synchronize(dev)
        return float(np.mean([a.elapsed_time(b) for a, b in ev]))

    ms_full = timed(full)
    ms_dec = timed(lambda: batch.decode(stream))
    full()
    torch.cuda.synchronize(dev)
    _, res = batch.results()
    _, gres = batch.assembly_results()
    _, pres = batch.property_results()
    idgeom = plan.streams["column_kind"] != 2
    if (res[idgeom][:, 0] != 0).any() or (gres["status"] != 0).any():
        raise RuntimeError("config1: Id/Geometry decode or assembly reported errors")
    return {"workload": "config1: one z5 tile (%s) decoded whole -- Id, Geometry and property streams, "
                        "geometry assembly, property materialization (CovtParser.decodeCovt)" % CONFIG1_TILE,
            "tiles": 1, "tile_bytes": len(tile), "streams": plan.num_streams,
            "id_geometry_stream_bytes": int(plan.streams["byte_length"][idgeom].sum()),
            "gpu_full_ms": round(ms_full, 5), "gpu_decode_ms": round(ms_dec, 5),
            "property_columns": plan.num_property_columns,
            "property_columns_rejected": int((pres["status"] != 0).sum())}


def config_launch(lib, name, covt, dev, id_mode=0):
    """The launch a BASELINE config 2-4 leg times: the config's tiles planned with the default options,
    uploaded, and a DeviceSubset over exactly the config's streams -> (picks, plan, mask, batch, subset).
    tests/test_gpu_configs.py checks this very launch against the oracle digests."""
    picks = config_tiles(lib, name)
    plan = covt.Plan.from_tiles([t for _, t in picks], covt.FORMAT_GENC, id_mode)
    mask = config_mask(plan, name)
    batch = covt.DeviceBatch(plan, dev)
    return picks, plan, mask, batch, batch.subset(mask)


def config_legs(lib, args, torch, dev, covt, stream):
    """BASELINE configs 2-4 on one GPU: kernel-only time of one decode launch over exactly the config's
    streams (inputs + descriptors resident, HIP events on the launch stream, mean of --steps after
    --warmup), bit-exactness of those streams' statuses, and their own roofline.  Not `value`."""
    out = {"config1": config1_leg(lib, args, torch, dev, covt, stream)}
    for name, desc in CONFIG_LEGS.items():
        picks, plan, mask, batch, sub = config_launch(lib, name, covt, dev, args.id_mode)
        with torch.cuda.stream(stream):
            for _ in range(max(args.warmup, 1)):
                sub.decode(stream)
            torch.cuda.synchronize(dev)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.steps)]
            for s, e in ev:
                s.record(stream)
                sub.decode(stream)
                e.record(stream)
            torch.cuda.synchronize(dev)
        ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
        _, res, _ = sub.results()
        if (res[:, 0] != 0).any():
            raise RuntimeError("%s: decode reported errors on %d streams" % (name, int((res[:, 0] != 0).sum())))
        st = plan.streams[mask]
        ib = int(st["byte_length"].sum())
        ob = int((st["out_elems"] * st["elem_bytes"]).sum())
        vb = st[st["stream_type"] == 9]
        vx = int(np.where((vb["column_type"] == 3) | (vb["column_type"] == 4), vb["num_values"],
                          vb["num_values"] // 2).sum())
        ach = (ib + ob) / (ms * 1e-3) / 1e9
        out[name] = {"workload": desc, "tiles": len(picks), "streams": int(mask.sum()), "stream_bytes": ib,
                     "output_bytes": ob, "vertices": vx, "kernel_ms": round(ms, 5),
                     "gbps_raw": round(ib / (ms * 1e-3) / 1e9, 3),
                     "mvert_per_s": round(vx / (ms * 1e-3) / 1e6, 3),
                     "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(ach / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_launch": ib + ob}}
        del sub, batch, plan
    return out


def strong_shards_leg(allp, kern_ms_full, args, torch, dev, covt, stream, ns=(2, 4, 8)):
    """BASELINE config 5 "sharded across 8xMI355X", re-measured on this one GPU at every N = 1 run: the same
    10k-tile batch split over N ranks exactly as `bench.py --gpus N` splits it (LPT byte balance), every
    shard planned with the default options and its decode launch timed alone (HIP events, mean of --steps
    after --warmup).  An N-GPU strong-scaling step lasts as long as its slowest shard, so `projected_value`
    = the batch's stream bytes / that shard's launch and `efficiency` = projected_value / (N x the full
    batch's rate).  A projection (one GPU, no host effects), not the N-GPU run the driver measures."""
    total_in = None
    out = {"note": "per-shard decode launches timed alone on one GPU; an N-GPU step = its slowest shard",
           "full_kernel_ms": round(kern_ms_full, 5)}
    for n in ns:
        shards = lpt_shards([len(t) for _, t in allp], n)
        ms = []
        ins = []
        for sh in shards:
            plan = covt.Plan.from_tiles([allp[i][1] for i in sh], covt.FORMAT_GENC, args.id_mode)
            b = covt.DeviceBatch(plan, dev)
            with torch.cuda.stream(stream):
                for _ in range(max(args.warmup, 2)):
                    b.decode(stream)
                torch.cuda.synchronize(dev)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(max(args.steps // 2, 5))]
                for a, e in ev:
                    a.record(stream)
                    b.decode(stream)
                    e.record(stream)
                torch.cuda.synchronize(dev)
            _, res = b.results()
            if (res[:, 0] != 0).any():
                raise RuntimeError("strong shard decode reported errors")
            ms.append(float(np.mean([a.elapsed_time(e) for a, e in ev])))
            ins.append(int(plan.in_bytes))
            del b, plan
        total_in = sum(ins)
        worst = max(ms)
        proj = total_in / (worst * 1e-3) / 1e9
        full = total_in / (kern_ms_full * 1e-3) / 1e9
        out["n%d" % n] = {"shard_ms": [round(x, 4) for x in ms], "slowest_ms": round(worst, 4),
                          "projected_value": round(proj, 2), "efficiency": round(proj / (n * full), 3)}
    return out


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def timed_steps(batch, stream, steps, torch, dev, barrier):
    """`steps` decode launches bracketed by a barrier + synchronize on both sides -> (wall s, mean HIP-event
    ms of one launch on the launch stream)."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        batch.decode(stream)
        e.record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    wall = time.perf_counter() - t0
    return wall, float(np.mean([s.elapsed_time(e) for s, e in ev]))


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: one child process per GPU (RANK/LOCAL_RANK/WORLD_SIZE set
    before the child touches the GPU), rank 0 prints the line.  This parent never initialises HIP."""
    n = args.gpus
    if not args.dry_run:
        import torch

        have = torch.cuda.device_count()  # does not initialise the GPU on this image
        if have < (1 if args.share_device else n):
            print("bench.py: --gpus %d but only %d GPU(s) visible" % (n, have), file=sys.stderr, flush=True)
            sys.exit(2)
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            c = p.poll()
            if c is None:
                continue
            alive.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in alive:  # a failed rank would leave the others waiting in a barrier
                    q.kill()
        time.sleep(0.05)
    sys.exit(rc if rc >= 0 else 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tiles", type=int, default=10000)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="strong (default): one --tiles batch sharded over the ranks (BASELINE config 5); "
                         "weak: a whole --tiles batch per rank")
    ap.add_argument("--no-weak", action="store_true", help="N > 1 strong runs: skip the extra weak-scaling field")
    ap.add_argument("--cpu-iters", type=int, default=20, help="timed CPU-baseline iterations (after 3 warm-ups)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU-baseline threads (default: all usable CPUs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--id-mode", type=int, default=0)
    ap.add_argument("--no-assemble", action="store_true", help="skip the geometry-assembly leg")
    ap.add_argument("--e2e-reps", type=int, default=3, help="end-to-end (PCIe-inclusive) reps; 0 skips")
    ap.add_argument("--no-props", action="store_true", help="skip the property-column leg")
    ap.add_argument("--no-configs", action="store_true", help="skip the BASELINE config 2-4 legs")
    ap.add_argument("--device-plan-reps", type=int, default=5, help="device-side plan creations timed; 0 skips")
    ap.add_argument("--abi-host-reps", type=int, default=2,
                    help="reps of the C-ABI host entry covt_plan_decode_host (pageable in/out); 0 skips")
    ap.add_argument("--no-strong-shards", action="store_true",
                    help="N = 1: skip the strong-scaling shard projection (per-shard launches for N = 2, 4, 8)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank on cuda:0 (runs the real N-rank path on a one-GPU box; not a scaling figure)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: sample + plan per rank, time an empty step, print the aggregated line "
                         "(tests the rank launch and aggregation on CPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        launch_ranks(args)  # exits
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr, flush=True)
        sys.exit(2)

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        # tiles are independent: no collective on the data path, so no RCCL either --
        # gloo carries the timing barriers and the max/sum of per-rank numbers on the host
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    if not args.dry_run:
        if torch.cuda.device_count() < (1 if args.share_device else world):
            raise SystemExit("bench.py: %d ranks but only %d GPU(s) visible" % (world, torch.cuda.device_count()))
        dev = torch.device("cuda", 0 if args.share_device else local_rank)
        torch.cuda.set_device(dev)
    covt = load_covt()

    lib = tile_library()
    seed = SEED + rank if args.scaling == "weak" else SEED
    if args.scaling == "weak":
        picks = sample_batch(lib, args.tiles, seed)
    else:
        allp = sample_batch(lib, args.tiles, seed)
        shards = lpt_shards([len(t) for _, t in allp], world)
        picks = [allp[i] for i in shards[rank]]

    t_pack = time.perf_counter()
    blob, offs, sizes = covt.pack_tiles([t for _, t in picks])  # test-harness packing (a JNI caller's tiles
    t_pack = time.perf_counter() - t_pack                       # already sit in one direct buffer)
    t_plan = time.perf_counter()
    plan = covt.Plan(blob, offs, sizes, covt.FORMAT_GENC, args.id_mode)
    t_plan = time.perf_counter() - t_plan
    if (plan.tile_status != 0).any():
        raise RuntimeError("tile walk failed")

    def barrier():
        if dist is not None:
            dist.barrier()

    if args.dry_run:
        barrier()
        t0 = time.perf_counter()
        barrier()
        wall = time.perf_counter() - t0
        kern_ms = wall * 1e3 / max(args.steps, 1)
        dev_name = "cpu (dry run)"
    else:
        batch = covt.DeviceBatch(plan, dev)
        stream = torch.cuda.current_stream(dev)
        dev_name = torch.cuda.get_device_name(dev)
        for _ in range(args.warmup):
            batch.decode(stream)
        torch.cuda.synchronize(dev)
        _, res = batch.results()
        if (res[:, 0] != 0).any():
            raise RuntimeError("decode reported errors on %d streams" % int((res[:, 0] != 0).sum()))

        wall, kern_ms = timed_steps(batch, stream, args.steps, torch, dev, barrier)

    legs = {}
    weak = None
    if world > 1 and args.scaling == "strong" and not args.no_weak:
        # the per-GPU-work-fixed figure beside the strong headline: a whole batch per rank
        wpicks = sample_batch(lib, args.tiles, SEED + rank)
        wplan = covt.Plan.from_tiles([t for _, t in wpicks], covt.FORMAT_GENC, args.id_mode)
        if args.dry_run:
            barrier()
            t0 = time.perf_counter()
            barrier()
            wwall = time.perf_counter() - t0
            wms = wwall * 1e3 / max(args.steps, 1)
        else:
            wbatch = covt.DeviceBatch(wplan, dev)
            for _ in range(args.warmup):
                wbatch.decode(stream)
            wwall, wms = timed_steps(wbatch, stream, args.steps, torch, dev, barrier)
            del wbatch
        weak = {"tiles": len(wpicks), "stream_bytes": int(wplan.in_bytes), "wall_s": wwall, "kernel_ms": wms,
                "seed": SEED + rank}
        del wplan
    if not args.dry_run:
        if args.e2e_reps > 0:
            legs["end_to_end"] = end_to_end(plan, batch, stream, torch, dev, args.e2e_reps)
        if args.abi_host_reps > 0 and rank == 0:
            legs["c_abi_host"] = abi_host_leg(plan, t_plan, args.abi_host_reps)
        if args.device_plan_reps > 0:
            legs["device_plan"] = device_plan_leg(plan, batch, torch, dev, covt, args, t_plan)
        if not args.no_assemble and plan.num_geometry_columns:
            legs["assembly"] = assembly_leg(batch, plan, stream, args, dist, torch, dev)
        if not args.no_props:
            legs["properties"] = properties_leg(picks, args, dist, torch, dev, covt, stream)
        if not args.no_configs and rank == 0 and world == 1:
            legs["configs"] = config_legs(lib, args, torch, dev, covt, stream)
        if not args.no_strong_shards and world == 1 and args.scaling == "strong":
            legs["strong_shards"] = strong_shards_leg(allp, kern_ms, args, torch, dev, covt, stream)

    mine = {"rank": rank, "device": dev_name, "local_rank": local_rank, "seed": seed, "tiles": len(picks),
            "streams": int(plan.num_streams), "stream_bytes": int(plan.in_bytes), "output_bytes": int(plan.out_bytes),
            "vertices": int(plan.vertices), "wall_s": wall, "kernel_ms": kern_ms, "weak": weak}
    if dist is not None:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]
    wall = max(r["wall_s"] for r in ranks)
    kern_ms = max(r["kernel_ms"] for r in ranks)
    tot_in = float(sum(r["stream_bytes"] for r in ranks))
    tot_vx = float(sum(r["vertices"] for r in ranks))

    if rank == 0:
        ms_per_step = wall * 1e3 / args.steps
        value = tot_in * args.steps / wall / 1e9
        # stream bytes read + decoded bytes written, per rank over that rank's own launch time.
        # `roofline` is per GPU: at N > 1 the slowest rank's (the minimum of each rank's own bytes over its
        # own kernel time), with the whole job's aggregate (all ranks' bytes over the max time, against N
        # peaks) beside it
        for r in ranks:
            r["alg_bytes"] = r["stream_bytes"] + r["output_bytes"]
            r["achieved"] = r["alg_bytes"] / (r["kernel_ms"] * 1e-3) / 1e9 if r["kernel_ms"] > 0 else 0.0
        slow = min(ranks, key=lambda r: r["achieved"])
        alg_bytes, achieved = slow["alg_bytes"], slow["achieved"]
        agg_bytes = sum(r["alg_bytes"] for r in ranks)
        agg_achieved = agg_bytes / (kern_ms * 1e-3) / 1e9
        traffic, traffic_note = None, "no profiles/pmc_traffic.json"
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                with open(pmc) as f:
                    pm = json.load(f)
                if pm.get("tiles") != args.tiles or len(ranks) > 1:
                    traffic_note = "profiles/pmc_traffic.json measured on another workload"
                elif pm.get("kernel_sources_sha256") != kernel_sources_sha256():
                    traffic_note = "stale: profiles/pmc_traffic.json measured on other decode / plan sources"
                else:
                    traffic = pm.get("hbm_bytes_per_launch")
                    traffic_note = ("rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of the last launch (tools/profile_round.sh), "
                                    "same kernel sources (sha256 %s)" % pm["kernel_sources_sha256"][:12])
            except Exception:  # noqa: BLE001
                traffic = None
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": len(ranks),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "fixture-sampled: seeded sample of the reference's committed OMT+Bing COVT tiles",
            "config": {"workload": ("config5: %d-tile mixed-zoom z2-z14 batch, all Id+Geometry streams" % args.tiles)
                       + (" sharded over %d GPUs (strong scaling, LPT byte balance)" % world if world > 1 and
                          args.scaling == "strong" else " per GPU (weak scaling)" if world > 1 else ", one GPU"),
                       "tiles_per_gpu": len(picks), "streams_per_gpu": plan.num_streams,
                       "stream_bytes_per_gpu": plan.in_bytes, "output_bytes_per_gpu": plan.out_bytes,
                       "vertices_per_gpu": plan.vertices,
                       "per_gpu_note": "*_per_gpu: rank 0's batch; every rank's own in per_rank" if len(ranks) > 1
                       else "one GPU",
                       "tiles_total": sum(r["tiles"] for r in ranks), "streams_total": sum(r["streams"] for r in ranks),
                       "stream_bytes_total": int(tot_in), "output_bytes_total": sum(r["output_bytes"] for r in ranks),
                       "vertices_total": int(tot_vx), "id_mode": "format" if args.id_mode == 0 else "java",
                       "parallelism": "dp%d (tile shards, no collective)" % len(ranks)},
            "mvert_per_s": round(tot_vx * args.steps / wall / 1e6, 2),
            "kernel_ms": round(kern_ms, 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic if len(ranks) == 1 else None, "traffic_note": traffic_note,
                         "kernel": "covt decode launch = decode_family_kernel<RLE|VARINT|FASTPFOR> + "
                                   "decode_lane_kernel run concurrently between fork/join events; "
                                   "duration = HIP events on the launch stream",
                         "per": "GPU: rank %d's own algorithmic bytes over its own mean launch time (the slowest "
                                "rank of %d)" % (slow["rank"], len(ranks)),
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "aggregate": {"achieved": round(agg_achieved, 2), "peak": HBM_PEAK_GBS * len(ranks),
                                       "frac": round(agg_achieved / (HBM_PEAK_GBS * len(ranks)), 4),
                                       "algorithmic_bytes_per_launch": agg_bytes,
                                       "note": "all ranks' bytes over the max-over-ranks launch time, N peaks"}},
            "build": {"library": covt.library_build_id(), "sources": covt.source_build_id(),
                      "match": covt.library_build_id() == covt.source_build_id(),
                      "note": "sha256 prefix of libcovt's sources compiled into the library (Makefile BUILD_ID) "
                              "and of the sources in this tree"},
            "cpu_baseline": None,
            "per_rank": [{"rank": r["rank"], "device": r["device"], "seed": r["seed"], "tiles": r["tiles"],
                          "streams": r["streams"], "stream_bytes": r["stream_bytes"],
                          "output_bytes": r["output_bytes"], "kernel_ms": round(r["kernel_ms"], 4),
                          "roofline_frac": round(r["achieved"] / HBM_PEAK_GBS, 4),
                          "gbps": round(r["stream_bytes"] * args.steps / r["wall_s"] / 1e9, 3)
                          if r["wall_s"] > 0 else None} for r in ranks],
        }
        if ranks[0]["weak"] is not None:
            ww = max(r["weak"]["wall_s"] for r in ranks)
            wb = float(sum(r["weak"]["stream_bytes"] for r in ranks))
            line["weak"] = {"value": round(wb * args.steps / ww / 1e9, 3), "unit": "GB/s",
                            "ms_per_step": round(ww * 1e3 / args.steps, 4),
                            "kernel_ms": round(max(r["weak"]["kernel_ms"] for r in ranks), 4),
                            "tiles_per_gpu": ranks[0]["weak"]["tiles"], "tiles_total": sum(r["weak"]["tiles"] for r in ranks),
                            "stream_bytes_total": int(wb), "seeds": [r["weak"]["seed"] for r in ranks],
                            "note": "weak scaling: every rank decodes its own whole %d-tile batch (seed %d + rank); "
                                    "same step timing as `value`" % (args.tiles, SEED)}
        line.update(legs)
        line["host_plan_ms"] = round(t_plan * 1e3, 1)  # covt_plan_create: metadata walk, descriptors, host
        line["host_pack_ms"] = round(t_pack * 1e3, 1)  # pack_tiles: copying the tiles into one buffer
        if not args.no_cpu:  # rank 0, over its own batch, at every N
            cb = cpu_baseline(plan, args, config1_tile(lib))
            c1 = cb.pop("config1")
            line["cpu_baseline"] = cb
            if c1 is not None and "configs" in line:
                c1["cpu_over_gpu_full"] = round(c1["cpu_full_ms_1thread"] / line["configs"]["config1"]["gpu_full_ms"], 2)
                line["configs"]["config1"].update(c1)
        if args.share_device:
            line["shared_device"] = True  # every rank on cuda:0: the N-rank path exercised, not a scaling figure
        if args.dry_run:
            line["dry_run"] = True
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
