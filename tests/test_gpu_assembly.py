"""GPU parity of the geometry assembly (covt_assemble.hip) against the CPU oracle, bit-exact, through
the C-ABI (covt_plan_assemble_host, covt_assemble_geometry_device).

The reference contract is CovtParser.convertGeometryColumn (CovtParser.java:135-274): every feature's
parts / rings / vertices in stream order, ICE vertices through vertexOffsets (getICELineString :537-550),
rings closed as JTS LinearRings (getLinearRing :513-516).  The oracle restating it is itself pinned by
the reference's MVT fixtures (tests/test_assembly_oracle.py).
"""
import hashlib

import numpy as np
import pytest

import covt_asm as A
from conftest import tile_key, tile_paths

pytestmark = pytest.mark.gpu


def _digest(geo, part, ring, xy):
    h = hashlib.sha256()
    for a in (geo, part, ring, xy):
        h.update(np.ascontiguousarray(a, dtype=np.int32).tobytes())
        h.update(b"|")
    return h.hexdigest()


def _oracle_digests(oracle, tile):
    return {L: (None if c["asm"] is None else (c["asm"][0], _digest(*c["asm"][1:]) if c["asm"][0] == 0 else None))
            for L, c in A.oracle_tile_columns(oracle, tile).items()}


def test_fixture_tiles_assembly_bitexact(covt, oracle, gpu_available):
    paths = tile_paths()
    tiles = [open(p, "rb").read() for p in paths]
    plan = covt.Plan.from_tiles(tiles)
    asm, gres = plan.assemble_host()
    g = plan.geom
    n_ok = 0
    cache = {}
    for c in range(plan.num_geometry_columns):
        t, L = int(g["tile"][c]), int(g["layer"][c])
        if t not in cache:
            cache[t] = A.oracle_tile_columns(oracle, tiles[t])
        oc = cache[t][L]
        st = int(gres["status"][c])
        if oc["asm"] is None:  # a source stream failed to decode (SURVEY Q4 tiles)
            assert st != 0, (tile_key(paths[t]), L)
            continue
        ost, ogeo, opart, oring, oxy = oc["asm"]
        assert st == ost == 0, (tile_key(paths[t]), L, st, ost)
        col = plan.geometry_arrays(asm, gres, c)
        assert np.array_equal(col.geometry_offsets, ogeo), (tile_key(paths[t]), L)
        assert np.array_equal(col.part_offsets, opart), (tile_key(paths[t]), L)
        assert np.array_equal(col.ring_offsets, oring), (tile_key(paths[t]), L)
        assert np.array_equal(col.coords, oxy), (tile_key(paths[t]), L)
        n_ok += 1
    assert n_ok >= 700


def test_device_batch_assembly_matches_host_path(covt, gpu_available):
    import torch

    tiles = [open(p, "rb").read() for p in tile_paths(("omt",))[:30]]
    plan = covt.Plan.from_tiles(tiles)
    asm_h, gres_h = plan.assemble_host()
    b = covt.DeviceBatch(plan, "cuda:0")
    b.decode()
    b.assemble()
    torch.cuda.synchronize()
    asm_d, gres_d = b.assembly_results()
    assert np.array_equal(gres_h, gres_d)
    for c in range(plan.num_geometry_columns):
        x, y = plan.geometry_arrays(asm_h, gres_h, c), plan.geometry_arrays(asm_d, gres_d, c)
        for f in ("geometry_offsets", "part_offsets", "ring_offsets", "coords"):
            assert np.array_equal(getattr(x, f), getattr(y, f)), (c, f)
    # feature view: a polygon ring is closed
    col = plan.geometry_arrays(asm_h, gres_h, 0)
    assert len(col.feature(0)) >= 1


def _run_kernel(covt, cols, flags_extra=None, in_res=None, dres=None):
    import torch

    dec, desc, asm_bytes, lay = A.pack_columns(covt, cols, flags_extra, in_res)
    dev = torch.device("cuda:0")
    d_dec = torch.from_numpy(dec).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    d_asm = torch.full((asm_bytes,), 0x5A, dtype=torch.uint8, device=dev)
    d_gres = torch.zeros(4 * len(cols), dtype=torch.int32, device=dev)
    dres = np.zeros(2, dtype=np.int32) if dres is None else np.asarray(dres, dtype=np.int32)
    d_res = torch.from_numpy(dres).to(dev)
    s = torch.cuda.current_stream(dev)
    st = covt.lib().covt_assemble_geometry_device(d_dec.data_ptr(), d_res.data_ptr(), d_desc.data_ptr(), len(cols),
                                                  d_asm.data_ptr(), d_gres.data_ptr(), s.cuda_stream)
    assert st == 0
    torch.cuda.synchronize()
    return d_asm.cpu().numpy(), d_gres.cpu().numpy().view(covt.GEOM_RESULT_DTYPE), lay


def _check_vs_oracle(oracle, cols, asm, gres, lay):
    for ci, col in enumerate(cols):
        o = oracle.assemble_geometry(col["types"], col["go"], col["po"], col["ro"], col["vo"], col["vb"],
                                     col["closed"], A.caps(col))
        g = A.unpack_column(asm, lay[ci], col["types"].size, gres[ci])
        assert g[0] == o[0], (ci, g[0], o[0])
        if o[0] == 0:
            for k in range(1, 5):
                assert np.array_equal(g[k], o[k]), (ci, k)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_synthetic_columns(covt, oracle, gpu_available, seed):
    rng = np.random.default_rng(seed)
    cols = []
    for i in range(48):
        big = i % 8 == 7  # up to 300 parts per feature, 40 rings per polygon, 3000 vertices per ring
        n = int(rng.choice([1, 2, 5, 8])) if big else int(rng.choice([0, 1, 5, 63, 64, 65, 200, 1000, 5000]))
        cols.append(A.synth_column(rng, n, ice=bool(i & 1), closed=bool(i & 2), big=big))
    # one-type columns: long runs of empty segments and of 1-vertex rings
    cols.append(A.synth_column(rng, 3000, False, False, probs=[1, 0, 0, 0, 0, 0]))
    cols.append(A.synth_column(rng, 3000, True, False, probs=[0, 0, 0, 1, 0, 0]))
    cols.append(A.synth_column(rng, 6, False, False, big=True, probs=[0, 0, 0, 0, 0, 1]))
    assert all(max(A.caps(c)) <= covt.GEOM_MAX_CAP for c in cols)
    asm, gres, lay = _run_kernel(covt, cols)
    assert (gres["status"] == 0).all()
    _check_vs_oracle(oracle, cols, asm, gres, lay)


def test_assembly_errors(covt, oracle, gpu_available):
    rng = np.random.default_rng(7)
    base = A.synth_column(rng, 300, True, False)
    bad_type = dict(base, types=base["types"].copy())
    bad_type["types"][150] = 6
    go_short = dict(base, types=np.array([4, 4], np.uint8), go=np.array([1], np.int32))
    po_short = dict(base, types=np.array([1, 1], np.uint8), po=np.array([2], np.int32))
    neg = dict(base, types=np.array([2], np.uint8), po=np.array([1], np.int32), ro=np.array([-3], np.int32))
    vo_out = dict(base, vo=base["vo"].copy())
    vo_out["vo"][-1] = base["vb"].size // 2
    too_many = dict(base, types=np.array([1], np.uint8), po=np.array([base["vo"].size + 1], np.int32))
    cols = [bad_type, go_short, po_short, neg, vo_out, too_many]
    for c in cols:
        c["caps"] = A.caps(c)
    asm, gres, lay = _run_kernel(covt, cols)
    assert gres["status"].tolist() == [covt.ERR_BAD_HEADER, covt.ERR_COUNT_MISMATCH, covt.ERR_COUNT_MISMATCH,
                                       covt.ERR_COUNT_MISMATCH, covt.ERR_TRUNCATED, covt.ERR_COUNT_MISMATCH]
    _check_vs_oracle(oracle, cols, asm, gres, lay)
    # a failed source stream fails the column with its status; oversized columns are refused
    ok = A.synth_column(rng, 50, False, False)
    asm, gres, lay = _run_kernel(covt, [ok, ok, ok], flags_extra=[0, 0, 0x80000000],
                                 in_res=[[-1] * 6, [0, -1, -1, -1, -1, 1], [-1] * 6],
                                 dres=[0, 5, covt.ERR_TRUNCATED, 7])
    assert gres["status"].tolist() == [0, covt.ERR_TRUNCATED, covt.ERR_INVALID_ARG]


def test_assembly_errors_cooperative(covt, oracle, gpu_available):
    """The same error checks on columns big enough (>= 8192 items, batches of <= 4096 columns) for the
    workgroup-cooperative path (assemble_coop_kernel): the first failing check's status, as the oracle."""
    rng = np.random.default_rng(8)
    base = A.synth_column(rng, 9000, True, False)
    bad_type = dict(base, types=base["types"].copy())
    bad_type["types"][8700] = 6
    vo_out = dict(base, vo=base["vo"].copy())
    vo_out["vo"][-1] = base["vb"].size // 2
    poly = A.synth_column(rng, 9000, False, False, probs=[0, 0, 1, 0, 0, 0])
    neg = dict(poly, ro=poly["ro"].copy())
    neg["ro"][-5] = -3
    ok_line = A.synth_column(rng, 12000, True, False, probs=[0, 1, 0, 0, 0, 0])
    cols = [bad_type, vo_out, neg, base, poly, ok_line]
    for c in cols:
        c["caps"] = A.caps(c)
        assert max(max(c["caps"]), c["types"].size) >= 8192
    asm, gres, lay = _run_kernel(covt, cols)
    assert gres["status"].tolist() == [covt.ERR_BAD_HEADER, covt.ERR_TRUNCATED, covt.ERR_COUNT_MISMATCH, 0, 0, 0]
    _check_vs_oracle(oracle, cols, asm, gres, lay)


def test_split_columns_multi_chunk(covt, oracle, gpu_available):
    """Columns of many 4,096-item chunks in a small batch go through the split passes (several workgroups
    per column, chunk-to-chunk scans by publish-and-gather, each pass seeding the next one's chunk starts):
    bit-exact against the oracle, including chunks whose expansion takes several steps (runs of empty
    multi-features / parts), ICE and plain, closed and open rings, and a failure in a late chunk."""
    rng = np.random.default_rng(11)
    cols = [A.synth_column(rng, 40000, True, False),
            A.synth_column(rng, 30000, False, True),
            A.synth_column(rng, 20000, False, False, probs=[0, 0, 1, 0, 0, 0]),
            A.synth_column(rng, 25000, True, False, probs=[0, 0, 0, 0.2, 0.4, 0.4]),
            A.synth_column(rng, 2, False, False, big=True, probs=[0, 0, 0, 0, 0, 1])]
    # runs of empty multi-features: 20k MULTILINESTRINGs of which most claim zero parts
    empt = A.synth_column(rng, 20000, False, False, probs=[0, 0, 0, 0, 1, 0])
    go = empt["go"].copy()
    go[rng.random(go.size) < 0.9] = 0
    n = 20000
    types = np.full(n, 4, np.uint8)
    lines = int(go.sum())
    po = rng.integers(2, 5, size=lines).astype(np.int32)
    vb = rng.integers(-(1 << 20), 1 << 20, size=2 * int(po.sum()), dtype=np.int64).astype(np.int32)
    cols.append({"types": types, "go": go.astype(np.int32), "po": po, "ro": np.zeros(0, np.int32), "vo": None,
                 "vb": vb, "closed": False})
    bad = A.synth_column(rng, 30000, False, False, probs=[0, 0, 1, 0, 0, 0])
    bad = dict(bad, ro=bad["ro"].copy())
    bad["ro"][-3] = -1  # a negative ring count in the last chunk of pass 3
    cols.append(bad)
    for c in cols:
        c["caps"] = A.caps(c)
        assert max(c["caps"]) <= covt.GEOM_MAX_CAP
    asm, gres, lay = _run_kernel(covt, cols)
    assert gres["status"].tolist()[:-1] == [0] * (len(cols) - 1)
    assert int(gres["status"][-1]) == covt.ERR_COUNT_MISMATCH
    _check_vs_oracle(oracle, cols, asm, gres, lay)
    assert int(gres["num_coords"][0]) > 8 * 4096  # several chunks in every pass


def _overflow_column(n_multi, parts_each, n_vertices):
    """n_multi MULTIPOINT features each claiming `parts_each` parts over a column of n_vertices point
    vertices: the part total is n_multi * parts_each (2^32 for the cases below), which a wrapping uint32
    scan would see as 0 <= part_cap and accept."""
    return {"types": np.full(n_multi, 3, np.uint8), "go": np.full(n_multi, parts_each, np.int32),
            "po": np.zeros(0, np.int32), "ro": np.zeros(0, np.int32), "vo": None,
            "vb": np.zeros(2 * n_vertices, np.int32), "closed": False}


def test_assembly_part_total_past_2_32(covt, oracle, gpu_available):
    """clamped per-item counts summed over one step reach 2^32.  The scans saturate,
    so the total fails the capacity check (COUNT_MISMATCH, as the oracle's 64-bit count says) instead of
    wrapping to an accepted 0.  Cooperative path: 4096 features x 2^20 parts in one 4096-item step;
    wave path (a batch of more than 4096 columns): 256 features x 2^24 parts in one 256-item step."""
    coop = _overflow_column(4096, 1 << 20, 1 << 20)
    assert A.caps(coop)[0] == 1 << 20  # per-item clamp at pcap + 1 leaves 2^20 each
    asm, gres, lay = _run_kernel(covt, [coop])
    assert gres["status"].tolist() == [covt.ERR_COUNT_MISMATCH]
    o = oracle.assemble_geometry(coop["types"], coop["go"], coop["po"], coop["ro"], coop["vo"], coop["vb"],
                                 coop["closed"], A.caps(coop))
    assert o[0] == covt.ERR_COUNT_MISMATCH
    # the single-wave path: past kCoopMaxColumns columns every column runs on one wave
    wave = _overflow_column(256, 1 << 24, 1 << 24)
    tiny = A.synth_column(np.random.default_rng(9), 1, False, False)
    cols = [wave] + [tiny] * 4096
    asm, gres, lay = _run_kernel(covt, cols)
    assert int(gres["status"][0]) == covt.ERR_COUNT_MISMATCH
    assert (gres["status"][1:] == 0).all()


def test_batch_assembly_properties(covt, oracle, gpu_available):
    """BASELINE config-5 batch (10k sampled tiles): every column equals the oracle's assembly of its source
    tile (goldens reused per source tile), coordinate totals add up."""
    import bench
    import torch

    lib = bench.tile_library()
    picks = bench.sample_batch(lib, 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    b = covt.DeviceBatch(plan, "cuda:0")
    b.decode()
    b.assemble()
    torch.cuda.synchronize()
    asm, gres = b.assembly_results()
    assert (gres["status"] == 0).all()
    ref = {}
    g = plan.geom
    for c in range(plan.num_geometry_columns):
        key, tile = picks[int(g["tile"][c])]
        if key not in ref:
            ref[key] = _oracle_digests(oracle, tile)
        col = plan.geometry_arrays(asm, gres, c)
        d = _digest(col.geometry_offsets, col.part_offsets, col.ring_offsets, col.coords)
        assert ref[key][int(g["layer"][c])] == (0, d), (key, int(g["layer"][c]))
    assert int(gres["num_coords"].sum()) >= plan.vertices  # + closing vertices of PLAIN polygon rings


def _split_cols():
    rng = np.random.default_rng(12)
    cols = [A.synth_column(rng, 30000, True, False), A.synth_column(rng, 20000, False, True),
            A.synth_column(rng, 300, False, False)]
    for c in cols:
        c["caps"] = A.caps(c)
    return cols


def test_split_passes_replay_in_a_hip_graph(covt, oracle, gpu_available):
    """the split passes' look-back records are tagged with an epoch that the launch's
    own prep kernel advances in device memory, so a captured graph replays with a fresh epoch each time
    (a host-side epoch would be frozen into the graph and a replay would accept the previous replay's
    records).  Three replays, output poisoned before each, bit-exact against the oracle."""
    import torch

    cols = _split_cols()
    dec, desc, asm_bytes, lay = A.pack_columns(covt, cols, None, None)
    dev = torch.device("cuda:0")
    d_dec = torch.from_numpy(dec).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    d_asm = torch.full((asm_bytes,), 0x5A, dtype=torch.uint8, device=dev)
    d_gres = torch.zeros(4 * len(cols), dtype=torch.int32, device=dev)
    d_res = torch.zeros(2, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)

    def launch():
        assert covt.lib().covt_assemble_geometry_device(d_dec.data_ptr(), d_res.data_ptr(), d_desc.data_ptr(),
                                                        len(cols), d_asm.data_ptr(), d_gres.data_ptr(),
                                                        s.cuda_stream) == 0

    with torch.cuda.stream(s):
        launch()  # the stream's scratch exists before capture (allocation cannot be captured)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        launch()
    for _ in range(3):
        d_asm.fill_(0x5A)
        d_gres.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        gres = d_gres.cpu().numpy().view(covt.GEOM_RESULT_DTYPE)
        assert (gres["status"] == 0).all()
        _check_vs_oracle(oracle, cols, d_asm.cpu().numpy(), gres, lay)
    del g
    torch.cuda.synchronize()
    assert covt.release_scratch(s) == 0  # pinned by the capture: kept unless asked
    assert covt.release_scratch(s, pinned=True) >= 1


def test_captured_graph_survives_scratch_eviction(covt, oracle, gpu_available):
    """a block used under a graph capture is pinned -- launches on 20 other streams
    after the capture (more than the 16 blocks kept) evict only unpinned blocks, and covt_release_scratch
    without COVT_RELEASE_PINNED keeps it -- so the graph replays into live memory, bit-exact."""
    import torch

    covt.release_scratch(all=True, pinned=True)
    cols = _split_cols()
    dec, desc, asm_bytes, lay = A.pack_columns(covt, cols, None, None)
    dev = torch.device("cuda:0")
    d_dec = torch.from_numpy(dec).to(dev)
    d_desc = torch.from_numpy(desc).to(dev)
    d_asm = torch.full((asm_bytes,), 0x5A, dtype=torch.uint8, device=dev)
    d_gres = torch.zeros(4 * len(cols), dtype=torch.int32, device=dev)
    d_res = torch.zeros(2, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)

    def launch():
        assert covt.lib().covt_assemble_geometry_device(d_dec.data_ptr(), d_res.data_ptr(), d_desc.data_ptr(),
                                                        len(cols), d_asm.data_ptr(), d_gres.data_ptr(),
                                                        s.cuda_stream) == 0

    with torch.cuda.stream(s):
        launch()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        launch()
    streams = [torch.cuda.Stream(dev) for _ in range(20)]
    for o in streams:
        with torch.cuda.stream(o):
            _run_kernel(covt, cols)
        assert covt.scratch_blocks() <= 16
    torch.cuda.synchronize()
    assert covt.release_scratch(all=True) >= 1  # every unpinned block ...
    assert covt.scratch_blocks() == 1           # ... but the graph's
    for _ in range(2):
        d_asm.fill_(0x5A)
        d_gres.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        gres = d_gres.cpu().numpy().view(covt.GEOM_RESULT_DTYPE)
        assert (gres["status"] == 0).all()
        _check_vs_oracle(oracle, cols, d_asm.cpu().numpy(), gres, lay)
    del g
    torch.cuda.synchronize()
    assert covt.release_scratch(all=True, pinned=True) == 1 and covt.scratch_blocks() == 0


def test_scratch_blocks_bounded_and_released(covt, oracle, gpu_available):
    """one scratch block per (device, stream), at most 16 kept (least recently used
    freed), all freed by covt_release_scratch(all); results stay exact on every stream."""
    import torch

    covt.release_scratch(all=True, pinned=True)
    assert covt.scratch_blocks() == 0
    cols = _split_cols()
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(dev) for _ in range(20)]
    for i, s in enumerate(streams):
        with torch.cuda.stream(s):
            asm, gres, lay = _run_kernel(covt, cols)
        if i % 7 == 0:
            _check_vs_oracle(oracle, cols, asm, gres, lay)
        assert covt.scratch_blocks() <= 16
    assert covt.scratch_blocks() == 16
    assert covt.release_scratch(streams[-1]) == 1  # the most recent one is still held
    assert covt.release_scratch(all=True) == 15 and covt.scratch_blocks() == 0
    asm, gres, lay = _run_kernel(covt, cols)  # and a fresh block works
    _check_vs_oracle(oracle, cols, asm, gres, lay)
