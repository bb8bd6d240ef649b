#!/usr/bin/env python3
"""Benchmark: GB/s of raw COVT Id+Geometry stream bytes decoded (+ Mvertices/s) on a z2-z14 tile batch.

BASELINE.json config 5: a 10k-tile mixed-zoom batch sampled with numpy.random.default_rng(20250117),
uniform over the zoom levels that have decodable fixtures, then uniform over that zoom's tiles, from the
90 OMT + 27 Bing decodable fixtures (tests/golden/tiles, byte-identical copies of the reference's
test/fixtures).  A "step" is one decode launch over the whole batch: every Id/Geometry stream of every
tile, inputs (tile bytes + descriptor table) already resident in HBM, outputs written to HBM.

  python bench.py [--gpus N --steps K --warmup W]     (N>1: torchrun, one rank per GPU)

Scaling is weak by default: each rank decodes its own 10k-tile batch (seed 20250117 + rank), no
collective on the data path (RCCL only for the timing barrier / max).  --scaling strong shards one
10k-tile batch over the ranks with the greedy byte-balanced split of SURVEY §8(e).
"""
from __future__ import annotations

import argparse
import glob
import importlib.util
import json
import os
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


def cpu_baseline(picks, seconds, threads):
    """The oracle (C restatement of the Java DecodingUtils semantics) on host cores: bounded sample."""
    sys.path.insert(0, ROOT)
    import oracle as O

    O.build()
    covt = load_covt()
    sample = picks[: min(len(picks), 400)]
    blob, offs, sizes = covt.pack_tiles([t for _, t in sample])
    st, ib, ob, vx = O.decode_tiles_mt(blob, offs, sizes, O.FMT_GENC, O.ID_FORMAT, threads)
    if st != 0:
        raise RuntimeError("oracle baseline failed: %d" % st)
    def timed(nthr, secs):
        reps, t0 = 0, time.perf_counter()
        while True:
            O.decode_tiles_mt(blob, offs, sizes, O.FMT_GENC, O.ID_FORMAT, nthr)
            reps += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return reps, el

    reps, el = timed(threads, seconds)
    reps1, el1 = timed(1, max(seconds / 3, 1.0))
    return {"value": round(ib * reps / el / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "%d tiles of the same batch (%.1f MB stream bytes) x %d reps in %.1f s; "
                      "C restatement of DecodingUtils (oracle/covt_oracle.c), %d threads" %
                      (len(sample), ib / 1e6, reps, el, threads),
            "mvert_per_s": round(vx * reps / el / 1e6, 3),
            "value_1thread": round(ib * reps1 / el1 / 1e9, 4),
            "host": {"cpu_model": cpu_model(), "nproc": os.cpu_count()}}


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


def abi_host_leg(plan, t_plan, reps):
    """The C-ABI host entry a JNI/ctypes caller would use (include/covt.h covt_plan_decode_host): pageable
    tile bytes in, device buffers allocated per call, H2D, one decode launch, D2H into pageable host memory
    (fresh buffers each call, so first-touch page faults are included).  Not `value`."""
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
    return {"ms": round(ms, 3), "value": round(plan.in_bytes / (ms * 1e-3) / 1e9, 3), "unit": "GB/s",
            "ms_reused_buffers": round(ms_reuse, 3),
            "raw_tiles_to_host_ms": round(ms + t_plan * 1e3, 1), "reps": reps,
            "note": "covt_plan_decode_host wall clock (pageable bytes, per-call device alloc, H2D + decode + "
                    "D2H) into fresh host buffers; ms_reused_buffers: into caller buffers reused across calls; "
                    "raw_tiles_to_host_ms adds the host metadata walk (covt_plan_create)"}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tiles", type=int, default=10000)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--id-mode", type=int, default=0)
    ap.add_argument("--no-assemble", action="store_true", help="skip the geometry-assembly leg")
    ap.add_argument("--e2e-reps", type=int, default=3, help="end-to-end (PCIe-inclusive) reps; 0 skips")
    ap.add_argument("--no-props", action="store_true", help="skip the property-column leg")
    ap.add_argument("--abi-host-reps", type=int, default=2,
                    help="reps of the C-ABI host entry covt_plan_decode_host (pageable in/out); 0 skips")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    covt = load_covt()

    lib = tile_library()
    if args.scaling == "weak":
        picks = sample_batch(lib, args.tiles, SEED + rank)
    else:
        allp = sample_batch(lib, args.tiles, SEED)
        shards = lpt_shards([len(t) for _, t in allp], world)
        picks = [allp[i] for i in shards[rank]]

    t_plan = time.perf_counter()
    plan = covt.Plan.from_tiles([t for _, t in picks], covt.FORMAT_GENC, args.id_mode)
    t_plan = time.perf_counter() - t_plan
    if (plan.tile_status != 0).any():
        raise RuntimeError("tile walk failed")
    batch = covt.DeviceBatch(plan, dev)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        batch.decode(stream)
    torch.cuda.synchronize(dev)
    _, res = batch.results()
    if (res[:, 0] != 0).any():
        raise RuntimeError("decode reported errors on %d streams" % int((res[:, 0] != 0).sum()))

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        batch.decode(stream)
        e.record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))

    e2e = None
    if args.e2e_reps > 0:
        e2e = end_to_end(plan, batch, stream, torch, dev, args.e2e_reps)
    abi = None
    if args.abi_host_reps > 0 and rank == 0:
        abi = abi_host_leg(plan, t_plan, args.abi_host_reps)
    asm_line = None
    if not args.no_assemble and plan.num_geometry_columns:
        asm_line = assembly_leg(batch, plan, stream, args, dist, torch, dev)
    props_line = None
    if not args.no_props:
        props_line = properties_leg(picks, args, dist, torch, dev, covt, stream)

    stats = torch.tensor([wall, float(plan.in_bytes), float(plan.vertices), float(plan.out_bytes), kern_ms],
                         dtype=torch.float64, device=dev)
    if dist is not None:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        wall, kern_ms = float(mx[0]), float(mx[4])
        tot_in, tot_vx = float(sm[1]), float(sm[2])
    else:
        tot_in, tot_vx = float(plan.in_bytes), float(plan.vertices)

    if rank == 0:
        ms_per_step = wall * 1e3 / args.steps
        value = tot_in * args.steps / wall / 1e9
        alg_bytes = plan.in_bytes + plan.out_bytes  # stream bytes read + decoded bytes written
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                with open(pmc) as f:
                    pm = json.load(f)
                if pm.get("tiles") == args.tiles and pm.get("scaling") == args.scaling:
                    traffic = pm.get("hbm_bytes_per_launch")
            except Exception:  # noqa: BLE001
                traffic = None
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "fixture-sampled: seeded sample of the reference's committed OMT+Bing COVT tiles",
            "config": {"workload": "config5: %d-tile mixed-zoom z2-z14 batch per GPU (%s scaling), "
                                   "all Id+Geometry streams" % (len(picks), args.scaling),
                       "tiles_per_gpu": len(picks), "streams_per_gpu": plan.num_streams,
                       "stream_bytes_per_gpu": plan.in_bytes, "output_bytes_per_gpu": plan.out_bytes,
                       "vertices_per_gpu": plan.vertices, "id_mode": "format" if args.id_mode == 0 else "java",
                       "parallelism": "dp%d (tile shards, no collective)" % world},
            "mvert_per_s": round(tot_vx * args.steps / wall / 1e6, 2),
            "kernel_ms": round(kern_ms, 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "covt decode launch = decode_family_kernel<RLE|VARINT|FASTPFOR> + "
                                   "decode_lane_kernel run concurrently between fork/join events; "
                                   "duration = HIP events on the launch stream",
                         "algorithmic_bytes_per_launch": alg_bytes},
            "cpu_baseline": None,
        }
        if asm_line is not None:
            line["assembly"] = asm_line
        if props_line is not None:
            line["properties"] = props_line
        if e2e is not None:
            line["end_to_end"] = e2e
        if abi is not None:
            line["c_abi_host"] = abi
        line["host_plan_ms"] = round(t_plan * 1e3, 1)  # covt_plan_create metadata walk (+ packing), host
        if world == 1 and not args.no_cpu:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(picks, args.cpu_seconds, threads)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
