"""Device-side plan (covt_device_plan_create, cov-tiles_amd/csrc/covt_plan_device.hip) against the host
plan (covt_plan_create), which the oracle pins (test_capi.py::test_plan_matches_oracle_walk,
test_gpu_parity.py): the GPU's walk of the container metadata (CovtParser.decodeCovt,
CovtParser.java:53-133; decodeLayerMetadata :574-652) must give the host plan's stream records,
tile statuses, output layout, launch order and family counts byte for byte, on Gen C fixtures, Gen D
conversions, malformed tiles and the full BASELINE config-5 batch -- and decoding through it must give
the host plan's outputs.  Both plans are made with the same covt_plan_options: splitting off
(split_min = -1) for the walk tests, and on (the defaults, and forced small chunks) for the split rule,
where decoding through the device plan is also checked against the golden oracle digests."""
import hashlib

import numpy as np
import pytest

import covt_gend_rt as RT
from conftest import tile_paths

pytestmark = pytest.mark.gpu


def _host_plan(covt, tiles, fmt, id_mode, split=False, **kw):
    opts = covt.PlanOptions(**kw) if split else covt.PlanOptions(split_min=-1, **kw)
    return covt.Plan.from_tiles(tiles, fmt, id_mode, options=opts)


def _device_plan(covt, hp, fmt, id_mode):
    import torch

    d_blob = torch.from_numpy(hp.blob).cuda()
    return covt.DevicePlan(d_blob, hp.offsets.astype(np.int64), hp.sizes.astype(np.int64), fmt, id_mode,
                           options=hp.options)


def _assert_same_plan(hp, dp):
    info, descs, st = dp.host_copy()
    assert np.array_equal(st, hp.tile_status)
    assert dp.num_streams == hp.num_streams and dp.num_descs == hp.num_descs
    assert dp.output_bytes == hp.output_bytes
    assert (dp.in_bytes, dp.out_payload, dp.vertices) == (hp.in_bytes, hp.out_bytes, hp.vertices)
    assert np.array_equal(dp.family_counts, hp.family_counts)
    assert info.tobytes() == hp.streams.tobytes()
    assert descs.tobytes() == hp.descs.tobytes()


def _assert_same_geometry(hp, dp):
    """covt_device_plan_geometry: the host plan's geometry records (capacities, flags, 16-byte aligned
    output slices, descriptor index) and launch-ordered geometry descriptors, byte for byte."""
    assert dp.geometry() == hp.num_geometry_columns
    assert dp.assembly_bytes == hp.assembly_bytes
    g, d = dp.geometry_copy()
    assert g.tobytes() == hp.geom.tobytes()
    assert d.tobytes() == hp.gdescs.tobytes()


def _assert_same_assembly(covt, hp, dp):
    """Decode + assembly through the device plan (covt_device_plan_assemble) equal the host path's
    (covt_plan_assemble_host), column by column, statuses included."""
    import torch

    d_out, d_res = dp.alloc()
    d_asm, d_gres = dp.alloc_assembly()
    dp.decode(d_out, d_res)
    dp.assemble(d_out, d_res, d_asm, d_gres)
    torch.cuda.synchronize()
    asm_d = d_asm.cpu().numpy()[:dp.assembly_bytes]
    gres_d = d_gres.cpu().numpy().view(covt.GEOM_RESULT_DTYPE)[:dp.num_geometry_columns]
    if hp.num_geometry_columns:
        gres_d = gres_d[hp.geom["desc_index"]]
    asm_h, gres_h = hp.assemble_host()
    assert np.array_equal(gres_d, gres_h)
    for c in range(hp.num_geometry_columns):
        if int(gres_h["status"][c]) != 0:
            continue
        x, y = hp.geometry_arrays(asm_h, gres_h, c), hp.geometry_arrays(asm_d, gres_d, c)
        for f in ("geometry_offsets", "part_offsets", "ring_offsets", "coords"):
            assert np.array_equal(getattr(x, f), getattr(y, f)), (c, f)


def _assert_same_decode(covt, hp, dp):
    import torch

    d_out, d_res = dp.alloc()
    dp.decode(d_out, d_res)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()[:dp.output_bytes]
    res = d_res.cpu().numpy().reshape(-1, 2)[:dp.num_descs][hp.streams["desc_index"]]
    h_out, h_res = hp.decode_host()
    assert np.array_equal(res, h_res)
    for i in range(hp.num_streams):
        assert np.array_equal(hp.stream_array(out, i), hp.stream_array(h_out, i)), i


@pytest.mark.parametrize("id_mode", [0, 1], ids=["id_format", "id_java"])
def test_fixtures_genc(covt, gpu_available, id_mode):
    """Every committed fixture tile (decodable or not), in one batch."""
    tiles = [open(p, "rb").read() for p in tile_paths()]
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, id_mode)
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, id_mode)
    _assert_same_plan(hp, dp)
    _assert_same_decode(covt, hp, dp)
    _assert_same_geometry(hp, dp)
    _assert_same_assembly(covt, hp, dp)


@pytest.mark.parametrize("optimized", [False, True], ids=["named", "optimized"])
def test_fixtures_gend(covt, gpu_available, decodable_tiles, optimized):
    """Gen D conversions of the decodable fixtures (implicit present streams, TreeMap stream order)."""
    tiles = [RT.genc_to_gend(t, optimized=optimized)[0] for _, t in decodable_tiles[::3]]
    hp = _host_plan(covt, tiles, covt.FORMAT_GEND, 0)
    dp = _device_plan(covt, hp, covt.FORMAT_GEND, 0)
    assert (hp.tile_status == 0).all() and hp.num_streams > 0
    _assert_same_plan(hp, dp)
    _assert_same_decode(covt, hp, dp)
    _assert_same_geometry(hp, dp)
    _assert_same_assembly(covt, hp, dp)


@pytest.mark.parametrize("fmt", [0, 1], ids=["genc", "gend"])
def test_malformed_tiles(covt, gpu_available, decodable_tiles, fmt):
    """Truncations, garbage and bit flips in the metadata: the same status per tile as the host walk
    (first failing check), a failed tile contributing no streams, the rest laid out identically."""
    rng = np.random.default_rng(11 + fmt)
    base = [t for _, t in decodable_tiles[:40]]
    if fmt == 1:
        base = [RT.genc_to_gend(t, optimized=bool(k & 1))[0] for k, t in enumerate(base)]
    tiles = [b"", b"\x01", b"\x01\x05garbage", bytes(rng.integers(0, 256, 500).astype(np.uint8))]
    for t in base:
        tiles.append(t[:int(rng.integers(1, len(t)))])
        b = bytearray(t)
        for _ in range(3):  # flips in the first 256 bytes: mostly metadata
            b[int(rng.integers(0, min(256, len(b))))] ^= 1 << int(rng.integers(0, 8))
        tiles.append(bytes(b))
        tiles.append(t)
    hp = _host_plan(covt, tiles, fmt, 0)
    dp = _device_plan(covt, hp, fmt, 0)
    assert (hp.tile_status != 0).sum() >= 40
    _assert_same_plan(hp, dp)
    _assert_same_geometry(hp, dp)


def test_tile_outside_buffer(covt, gpu_available, decodable_tiles):
    """A tile range past the device buffer gets COVT_ERR_INVALID_ARG and no streams (never read)."""
    import torch

    tiles = [t for _, t in decodable_tiles[:3]]
    blob, offs, sizes = covt.pack_tiles(tiles)
    offs, sizes = offs.astype(np.int64), sizes.astype(np.int64)
    d_blob = torch.from_numpy(blob).cuda()
    offs2, sizes2 = offs.copy(), sizes.copy()
    sizes2[1] = len(blob) + 1
    offs2[2] = len(blob) + 100
    dp = covt.DevicePlan(d_blob, offs2, sizes2)
    _, _, st = dp.host_copy()
    assert st[0] == 0 and st[1] == covt.ERR_INVALID_ARG and st[2] == covt.ERR_INVALID_ARG
    one = covt.Plan.from_tiles(tiles[:1])
    assert dp.num_streams == one.num_streams and dp.output_bytes == one.output_bytes
    empty = covt.DevicePlan(d_blob, offs[:0], sizes[:0])
    assert empty.num_streams == 0 and empty.output_bytes == 0
    assert empty.geometry() == 0 and empty.assembly_bytes == 0


def test_full_batch_plan(covt, gpu_available):
    """BASELINE config 5 (the bench's 10k-tile batch): the host plan splits nothing there, and the device
    plan equals it (records, descriptors, families: the lane family is on at this size)."""
    import bench

    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    hp = _host_plan(covt, [t for _, t in picks], covt.FORMAT_GENC, 0, split=True)
    assert hp.num_descs == hp.num_streams and hp.family_counts[3] > 0  # COVT_FAMILY_LANE
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)
    _assert_same_geometry(hp, dp)


def _genc_layers(t: bytes):
    """Byte ranges [(start, end)] of a Gen C tile's layers (metadata + data, Appendix A.1)."""
    def vu(o):
        r = sh = 0
        while True:
            b = t[o]
            o += 1
            r |= (b & 0x7F) << sh
            sh += 7
            if b < 0x80:
                return r, o

    _, o = vu(0)
    nl, o = vu(o)
    out = []
    for _ in range(nl):
        s = o
        n, o = vu(o)
        o += n
        _, o = vu(o)
        _, o = vu(o)
        nc, o = vu(o)
        tot = 0
        for _ in range(nc):
            n, o = vu(o)
            o += n + 2
            ns, o = vu(o)
            for _ in range(ns):
                n, o = vu(o)
                o += n
                _, o = vu(o)
                bl, o = vu(o)
                o += 1
                tot += bl
        o += tot
        out.append((s, o))
    assert o == len(t)
    return out


def _merge_genc(tiles):
    """One Gen C tile holding every layer of `tiles` (layers are self-contained: metadata, then data)."""
    layers = [t[s:e] for t in tiles for s, e in _genc_layers(t)]
    n = len(layers)
    hdr = bytes([1]) + (bytes([n]) if n < 128 else bytes([0x80 | (n & 0x7F), n >> 7]))
    return hdr + b"".join(layers)


@pytest.mark.parametrize("walk", [0, 1, 4], ids=["slots", "walk_twice", "lanes4"])
@pytest.mark.parametrize("fmt", [0, 1], ids=["genc", "gend"])
def test_tiles_past_slot_capacity(covt, gpu_available, decodable_tiles, walk, fmt):
    """Tiles with more Id / Geometry streams than the count walk's 128 per-tile slots (merged fixture layers:
    164-200+ streams) beside ordinary tiles, in every walk layout (covt_plan_options.device_walk): the slot
    path and the re-walk of the big tiles write one stream array together; it must equal the host plan."""
    omt = [t for k, t in decodable_tiles if k.startswith("omt/")]
    big = [_merge_genc(omt[i:i + 5]) for i in range(0, 20, 5)]
    tiles = []
    for i, b in enumerate(big):
        tiles += omt[20 + 3 * i: 23 + 3 * i] + [b]
    if fmt == 1:
        tiles = [RT.genc_to_gend(t)[0] for t in tiles]
    hp = _host_plan(covt, tiles, fmt, 0, device_walk=walk)
    per_tile = np.bincount(hp.streams["tile"], minlength=len(tiles))
    assert per_tile.max() > 128 and (hp.tile_status == 0).all()
    dp = _device_plan(covt, hp, fmt, 0)
    _assert_same_plan(hp, dp)
    _assert_same_decode(covt, hp, dp)
    _assert_same_geometry(hp, dp)


def test_bound_sized_plan_past_its_bound(covt, gpu_available, decodable_tiles):
    """A plan of more than 2,048 tiles is built without the mid-plan synchronisation, its stream arena sized
    to 128 streams per tile (covt_plan_device.hip, stream_part).  Tiles of merged small fixtures hold more than
    that each, so the bound-sized pass overflows (its writes are clipped) and the plan is redone with the
    counted sizes: it must still equal the host plan and decode to the same outputs."""
    omt = sorted((t for k, t in decodable_tiles if k.startswith("omt/")), key=len)
    merged, i = [], 0
    while True:  # the smallest fixtures merged until the tile holds more than 128 Id / Geometry streams
        merged.append(omt[i])
        i += 1
        hp1 = _host_plan(covt, [_merge_genc(merged)], covt.FORMAT_GENC, 0)
        if hp1.num_streams > 160:
            break
    big = _merge_genc(merged)
    tiles = [big] * 2100
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, 0, split=True)
    assert hp.num_streams > 128 * len(tiles) and hp.num_descs == hp.num_streams
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)  # (descriptors byte-equal: the decode through them is the host plan's)


def test_bound_sized_plan_that_splits(covt, gpu_available, decodable_tiles):
    """A bound-sized plan (more than 2,048 tiles) whose streams stay under split_max_streams and whose largest
    stream passes the split threshold: the split decision, known only at the final synchronisation, redoes the
    stream part as a split plan; it must equal the host plan's (chunks and all) and decode to its outputs."""
    lib = dict(decodable_tiles)
    tiles = [lib["bing/5-8-12"]] * 2100 + [lib["omt/14_8298_10748"]]  # 31 streams each, then the largest tile
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, 0, split=True)
    assert hp.num_streams <= 65536 and hp.num_descs > hp.num_streams
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)
    _assert_same_decode(covt, hp, dp)


def _assert_golden(covt, hp, dp, keys, golden_streams):
    """Decode through the device plan; every stream's status, consumed bytes and output SHA-256 equal
    the oracle's digests of its tile (tests/golden/oracle_streams.json)."""
    import torch

    d_out, d_res = dp.alloc()
    for _ in range(2):  # the split look-back records are reset per launch
        dp.decode(d_out, d_res)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()[:dp.output_bytes]
    res = d_res.cpu().numpy().reshape(-1, 2)[:dp.num_descs][hp.streams["desc_index"]]
    col = golden_streams["columns"]
    ish, ist, ico = col.index("fmt_sha256"), col.index("fmt_status"), col.index("fmt_consumed")
    st = hp.streams
    checked = 0
    for t, key in enumerate(keys):
        rows = golden_streams["tiles"][key]["streams"]
        idx = np.nonzero(st["tile"] == t)[0]
        assert len(idx) == len(rows), key
        for i, row in zip(idx, rows):
            assert int(res[i][0]) == row[ist] and int(res[i][1]) == row[ico], (key, int(i))
            if row[ist] == 0:
                assert hashlib.sha256(hp.stream_array(out, int(i)).tobytes()).hexdigest() == row[ish], (key, int(i))
            checked += 1
    assert checked == hp.num_streams


@pytest.mark.parametrize("n_tiles", [1, 3, 12])
def test_split_default_options(covt, gpu_available, decodable_tiles, golden_streams, n_tiles):
    """Small batches with the default options split their long poles (varint, FastPFOR and RLE chunks):
    the device plan cuts the same chunks (FastPFOR start states included) and decodes to the digests."""
    omt = [(k, t) for k, t in decodable_tiles if k.startswith("omt/")]
    picks = sorted(omt, key=lambda kt: -len(kt[1]))[:n_tiles]
    keys, tiles = [k for k, _ in picks], [t for _, t in picks]
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, 0, split=True)
    fc = hp.family_counts
    assert hp.num_descs > hp.num_streams and fc[covt.FAMILY_SPLIT:].sum() > 0
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)
    _assert_golden(covt, hp, dp, keys, golden_streams)
    _assert_same_assembly(covt, hp, dp)  # split descriptors feed the assembly's stream results


@pytest.mark.parametrize("grow", [0, 1])
def test_split_grow_library(covt, gpu_available, decodable_tiles, golden_streams, grow):
    """The whole fixture library (several MiB of plan cost) split with covt_plan_options.split_grow on and
    off: the device plan grows its chunks by the same factor of the plan's cost (split_grow_factor) and
    cuts the same chunks (FastPFOR start states, RLE group boundaries); decoded to the golden digests."""
    keys, tiles = [k for k, _ in decodable_tiles], [t for _, t in decodable_tiles]
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, 0, split=True, split_min=256, split_ratio=0, split_chunk=1000,
                    split_values=512, split_max_streams=0, split_grow=grow)
    assert (hp.family_counts[covt.FAMILY_SPLIT:] > 0).all(), hp.family_counts
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)
    _assert_golden(covt, hp, dp, keys, golden_streams)


@pytest.mark.parametrize("kw", [dict(split_min=0, split_ratio=0, split_chunk=64, split_values=256),
                                dict(split_min=512, split_ratio=0, split_chunk=300, split_values=512,
                                     fpf_split_weight=3),
                                dict(split_min=0, split_ratio=0, split_chunk=64, split_values=256,
                                     lane_min_streams=0)],
                         ids=["tiny_chunks", "weighted", "lane_and_split"])
def test_split_forced(covt, gpu_available, decodable_tiles, golden_streams, kw):
    """Forced small chunks over a mixed batch: every family splits (all three split families present),
    lane streams beside split ones; the same plan and the golden digests."""
    picks = decodable_tiles[::4][:24]
    keys, tiles = [k for k, _ in picks], [t for _, t in picks]
    id_mode = 1 if "lane_min_streams" in kw else 0
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, id_mode, split=True, **kw)
    fc = hp.family_counts
    assert (fc[covt.FAMILY_SPLIT:] > 0).all(), fc
    if "lane_min_streams" in kw:
        assert fc[covt.FAMILY_LANE] > 0, fc
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, id_mode)
    _assert_same_plan(hp, dp)
    if id_mode == 0:
        _assert_golden(covt, hp, dp, keys, golden_streams)
    else:
        _assert_same_decode(covt, hp, dp)


@pytest.mark.parametrize("optimized", [False, True], ids=["named", "optimized"])
def test_split_forced_gend(covt, gpu_available, decodable_tiles, optimized):
    """Forced small chunks over Gen D conversions (implicit present streams, TreeMap stream order): the
    device walk of the other format feeds the same split rule; the same plan and decode as the host."""
    tiles = [RT.genc_to_gend(t, optimized=optimized)[0] for _, t in decodable_tiles[1::5][:16]]
    hp = _host_plan(covt, tiles, covt.FORMAT_GEND, 0, split=True, split_min=0, split_ratio=0, split_chunk=96,
                    split_values=512)
    assert (hp.family_counts[covt.FAMILY_SPLIT:] > 0).all(), hp.family_counts
    dp = _device_plan(covt, hp, covt.FORMAT_GEND, 0)
    _assert_same_plan(hp, dp)
    _assert_same_decode(covt, hp, dp)


def test_split_malformed_streams(covt, gpu_available, decodable_tiles):
    """Split candidates whose payload bytes are corrupted (metadata intact): the RLE group walk and the
    FastPFOR header walk stop where the host's do -- unframed RLE streams stay whole, FastPFOR chunks
    past the break get no start state -- and decoding reports the host plan's statuses."""
    rng = np.random.default_rng(5)
    tiles = []
    for k, t in decodable_tiles[:30]:
        b = bytearray(t)
        for _ in range(40):  # flips across the tile: mostly stream payloads
            b[int(rng.integers(len(b) // 4, len(b)))] ^= 1 << int(rng.integers(0, 8))
        tiles.append(bytes(b))
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, 0, split=True, split_min=0, split_ratio=0, split_chunk=64,
                    split_values=256)
    assert hp.num_descs > hp.num_streams
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)
    _assert_same_decode(covt, hp, dp)
    _assert_same_assembly(covt, hp, dp)


# ---- property columns (COVT_PLAN_PROPERTIES on the device: covt_plan_device.hip prop_walk ... prop_desc_fill)
def _assert_same_properties(hp, dp):
    """The device plan's property records (covt_prop_info: streams, names, layout) and largest-first
    descriptors equal the host plan's byte for byte."""
    assert dp.num_property_columns == hp.num_property_columns > 0
    assert dp.property_bytes == hp.property_bytes
    pinfo, pdesc = dp.property_copy()
    assert pinfo.tobytes() == hp.props.tobytes()
    assert pdesc.tobytes() == hp.pdescs.tobytes()


def _assert_same_materialization(covt, hp, dp):
    """Decode + materialization through the device plan equal the host path's (covt_plan_properties_host),
    column by column, statuses included."""
    import torch

    d_out, d_res = dp.alloc()
    d_props, d_pres = dp.alloc_properties()
    dp.decode(d_out, d_res)
    dp.materialize(d_out, d_res, d_props, d_pres)
    torch.cuda.synchronize()
    buf_d = d_props.cpu().numpy()[:dp.property_bytes]
    pres_d = d_pres.cpu().numpy().view(covt.PROP_RESULT_DTYPE)[:dp.num_property_columns][hp.props["desc_index"]]
    buf_h, pres_h = hp.properties_host()
    assert np.array_equal(pres_d, pres_h)
    n_ok = 0
    for c in range(hp.num_property_columns):
        if int(pres_h["status"][c]) != 0:
            continue
        x, y = hp.property_column(buf_h, pres_h, c), hp.property_column(buf_d, pres_d, c)
        assert np.array_equal(x.validity, y.validity) and np.array_equal(x.values, y.values), c
        assert (x.dict_offsets is None) == (y.dict_offsets is None), c
        if x.dict_offsets is not None:
            assert np.array_equal(x.dict_offsets, y.dict_offsets) and np.array_equal(x.dict_bytes, y.dict_bytes), c
        n_ok += 1
    return n_ok


@pytest.mark.parametrize("id_mode", [0, 1], ids=["id_format", "id_java"])
def test_properties_genc(covt, gpu_available, id_mode):
    """Every fixture tile with COVT_PLAN_PROPERTIES: Gen C property walk (roles by stream name, localized
    present_<lang> sub-columns sharing their column's dictionary), the property streams after each tile's
    Id / Geometry streams, the same launch order, layout and descriptors as the host plan."""
    tiles = [open(p, "rb").read() for p in tile_paths()]
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, id_mode, flags=covt.PLAN_PROPERTIES)
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, id_mode)
    _assert_same_plan(hp, dp)
    _assert_same_properties(hp, dp)
    assert _assert_same_materialization(covt, hp, dp) > 10000
    _assert_same_decode(covt, hp, dp)


@pytest.mark.parametrize("optimized", [False, True], ids=["named", "optimized"])
def test_properties_gend(covt, gpu_available, decodable_tiles, optimized):
    """Gen D conversions with property columns: the implicit present stream's byte-RLE length walked on the
    device, TreeMap stream order; plan, layout, descriptors and materialization as the host's."""
    tiles = [RT.genc_to_gend(t, optimized=optimized)[0] for _, t in decodable_tiles[::3]]
    hp = _host_plan(covt, tiles, covt.FORMAT_GEND, 0, flags=covt.PLAN_PROPERTIES)
    dp = _device_plan(covt, hp, covt.FORMAT_GEND, 0)
    assert (hp.tile_status == 0).all()
    _assert_same_plan(hp, dp)
    _assert_same_properties(hp, dp)
    _assert_same_materialization(covt, hp, dp)


def test_properties_split(covt, gpu_available, decodable_tiles, golden_streams):
    """Property plans with the split rule forced (long property RLE streams cut into group chunks too):
    the same plan, and the Id / Geometry streams still match the golden digests."""
    picks = decodable_tiles[::4][:24]
    keys, tiles = [k for k, _ in picks], [t for _, t in picks]
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, 0, split=True, split_min=0, split_ratio=0, split_chunk=128,
                    split_values=256, flags=covt.PLAN_PROPERTIES)
    assert (hp.family_counts[covt.FAMILY_SPLIT:] > 0).all(), hp.family_counts
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)
    _assert_same_properties(hp, dp)
    _assert_same_materialization(covt, hp, dp)


def test_properties_full_batch(covt, gpu_available):
    """The bench's 10k-tile batch with COVT_PLAN_PROPERTIES: more than 256 tiles, so both device walks take
    the tiles largest first (a device sort of the sizes) while every record keeps its tile-order place;
    plan, property records and descriptors equal the host plan's."""
    import bench

    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    hp = _host_plan(covt, [t for _, t in picks], covt.FORMAT_GENC, 0, split=True, flags=covt.PLAN_PROPERTIES)
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)
    _assert_same_properties(hp, dp)


def test_bound_sized_plan_redo(covt, gpu_available, decodable_tiles):
    """an Id / Geometry plan of more than split_max_streams / 32 tiles sizes its stream
    arrays to 64 streams per tile before the count is known; a batch of the busiest tiles (more than 64
    streams each) overruns that bound and is redone with the counted size -- still the host plan exactly,
    and it decodes the same."""
    counted = []
    for _, t in decodable_tiles:
        hp1 = _host_plan(covt, [t], covt.FORMAT_GENC, 0)
        counted.append((hp1.num_streams, t))
    counted.sort(key=lambda x: -x[0])
    busy = [t for n, t in counted if n > 64][:1]
    if not busy:
        pytest.skip("no fixture tile with more than 64 Id / Geometry streams")
    tiles = busy * 6
    hp = _host_plan(covt, tiles, covt.FORMAT_GENC, 0, split=True, split_max_streams=64)
    assert hp.num_streams > 64 * len(tiles)
    dp = _device_plan(covt, hp, covt.FORMAT_GENC, 0)
    _assert_same_plan(hp, dp)
    _assert_same_decode(covt, hp, dp)
