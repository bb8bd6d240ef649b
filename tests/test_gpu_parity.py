"""GPU parity: libcovt (HIP, gfx950) vs the CPU oracle, bit-exact, through the C-ABI.

Model: the reference's round-trip contract CovtParserTest.compareTiles
(evaluation/java/src/test/java/com/covt/decoder/CovtParserTest.java:62-90) restated at the stream
level -- every decoded Id / Geometry array must equal the oracle's, and every stream must consume
exactly its byteLength (SURVEY.md §8(c) pin 1).
"""
import hashlib

import numpy as np
import pytest

from conftest import tile_key, tile_paths

pytestmark = pytest.mark.gpu


def _plan_all(covt, id_mode):
    paths = tile_paths()
    tiles = [open(p, "rb").read() for p in paths]
    return [tile_key(p) for p in paths], tiles, covt.Plan.from_tiles(tiles, covt.FORMAT_GENC, id_mode)


@pytest.mark.parametrize("id_mode", [0, 1], ids=["id_format", "id_java"])
def test_fixture_tiles_bitexact(covt, oracle, gpu_available, golden_streams, id_mode):
    keys, tiles, plan = _plan_all(covt, id_mode)
    out, res = plan.decode_host()
    st = plan.streams
    n_ok = n_checked = 0
    for t, key in enumerate(keys):
        ost, oss = oracle.walk_tile(tiles[t])
        assert int(plan.tile_status[t] == 0) == int(ost == 0), key
        idx = np.nonzero(st["tile"] == t)[0]
        assert len(idx) == len(oss), key
        for i, s in zip(idx, oss):
            assert (st["layer"][i], st["stream_type"][i], st["num_values"][i], st["byte_length"][i]) == \
                   (s.layer, s.stream_type, s.num_values, s.byte_length)
            assert st["in_off"][i] == int(plan.offsets[t]) + s.offset
            o_st, o_arr, o_cons = oracle.decode_stream(tiles[t], s, id_mode)
            g_st, g_cons = int(res[i][0]), int(res[i][1])
            n_checked += 1
            if o_st != 0:
                assert g_st != 0, (key, i, o_st)
                continue
            assert g_st == 0, (key, int(i), g_st, s.stream_type, s.encoding, s.column_type)
            got = plan.stream_array(out, int(i))
            assert got.dtype == o_arr.dtype and got.shape == o_arr.shape, (key, i)
            assert np.array_equal(got, o_arr), (key, int(i), s.stream_type, s.encoding, s.column_type)
            assert g_cons == o_cons, (key, i, g_cons, o_cons)
            if id_mode == 1 and s.column_kind == 0 and s.encoding in (1, 4):
                continue  # Java's 4-byte cap / enc-4 label bug misparse these ids
            assert g_cons == s.byte_length, (key, i, g_cons)
            n_ok += 1
    assert n_checked == plan.num_streams
    assert n_ok >= 4400  # all streams of the 126 decodable tiles


def test_golden_sha_pins(covt, gpu_available, golden_streams):
    """GPU output digests equal the committed oracle digests (tests/golden/oracle_streams.json)."""
    keys, tiles, plan = _plan_all(covt, 0)
    out, res = plan.decode_host()
    col = golden_streams["columns"]
    ish = col.index("fmt_sha256")
    for t, key in enumerate(keys):
        rec = golden_streams["tiles"][key]
        if not rec["decodable"]:
            continue
        idx = np.nonzero(plan.streams["tile"] == t)[0]
        for i, row in zip(idx, rec["streams"]):
            assert hashlib.sha256(plan.stream_array(out, int(i)).tobytes()).hexdigest() == row[ish], (key, i)


def test_device_batch_equals_host_path(covt, gpu_available, decodable_tiles):
    import torch

    plan = covt.Plan.from_tiles([t for _, t in decodable_tiles])
    host_out, host_res = plan.decode_host()
    db = covt.DeviceBatch(plan, "cuda")
    for _ in range(2):  # repeated launches are idempotent
        db.decode()
    torch.cuda.synchronize()
    out, res = db.results()
    assert np.array_equal(res, host_res)
    assert (res[:, 0] == 0).all()
    for i in range(plan.num_streams):
        a = plan.stream_array(out, i)
        b = plan.stream_array(host_out, i)
        assert np.array_equal(a, b), i


def test_graph_replay_equals_launch(covt, gpu_available, decodable_tiles):
    """DeviceBatch.decode_graph (the fork/join launch captured once as a HIP graph, then replayed)
    writes exactly what the stream launch writes, replay after replay."""
    import torch

    plan = covt.Plan.from_tiles([t for _, t in decodable_tiles])
    db = covt.DeviceBatch(plan, "cuda")
    db.decode()
    torch.cuda.synchronize()
    ref_out, ref_res = db.d_out.clone(), db.d_res.clone()
    for _ in range(3):
        db.d_out.zero_()
        db.d_res.fill_(-99)
        db.decode_graph()
        torch.cuda.synchronize()
        assert torch.equal(db.d_out, ref_out) and torch.equal(db.d_res, ref_res)


def _slice_mask(plan):
    s = plan.streams
    mask = np.zeros(plan.output_bytes, dtype=bool)
    for off, n in zip(s["out_off"], s["out_elems"].astype(np.int64) * s["elem_bytes"]):
        mask[off:off + n] = True
    return mask


def test_forced_shards_equal_single(covt, gpu_available, decodable_tiles):
    """covt_plan_decode_host_shards with K shards on device 0 runs the multi-GPU shard path (contiguous
    tile ranges, per-shard descriptor tables, one H2D / launch / D2H each, concurrent host threads) on a
    one-GPU box: stream slices and results byte-identical to the single-shard call; covt_plan_decode_host_multi
    (clamped to the visible devices) too."""
    plan = covt.Plan.from_tiles([t for _, t in decodable_tiles])
    o1, r1 = plan.decode_host()
    o1 = o1.copy()
    mask = _slice_mask(plan)
    for k in (2, 3, 7, len(decodable_tiles) + 5):  # more shards than tiles: empty shards are fine
        ok, rk = plan.decode_host(shard_devices=[0] * k)
        assert np.array_equal(rk, r1), k
        assert np.array_equal(ok[mask], o1[mask]), k
    o2, r2 = plan.decode_host(2)
    assert np.array_equal(r2, r1) and np.array_equal(o2[mask], o1[mask])
    plan.release_device()
    o3, r3 = plan.decode_host(shard_devices=[0, 0])  # rebuilt after release
    assert np.array_equal(r3, r1) and np.array_equal(o3[mask], o1[mask])


def test_host_api_failed_tile_and_reused_buffers(covt, gpu_available, decodable_tiles):
    """A plan with a failed tile (no streams, same layout) decodes the rest identically; reused caller
    buffers (dirty on entry) get the same stream slices as fresh ones, call after call."""
    good = [t for _, t in decodable_tiles[:60]]
    whole = covt.Plan.from_tiles(good)
    bad = covt.Plan.from_tiles(good + [b"\x01\x05garbage"])  # failed last tile
    assert bad.tile_status[-1] != 0 and bad.output_bytes == whole.output_bytes
    o1, r1 = whole.decode_host()
    o1 = o1.copy()
    o2, r2 = bad.decode_host()
    assert np.array_equal(r1, r2)
    mask = _slice_mask(whole)  # bytes outside the stream slices are unspecified (include/covt.h)
    assert np.array_equal(o1[mask], o2[mask])
    out = np.full(whole.output_bytes + 64, 0xAB, dtype=np.uint8)
    res = np.full((whole.num_streams, 2), -7, dtype=np.int32)
    for _ in range(3):
        o3, r3 = whole.decode_host(out=out, res=res)
        assert o3.ctypes.data == out.ctypes.data
        assert np.array_equal(o3[mask], o1[mask]) and np.array_equal(r3, r1)
        out[:] = 0xCD
    with pytest.raises(ValueError):
        whole.decode_host(out=np.zeros(1, dtype=np.uint8))


@pytest.mark.parametrize("id_mode", [0, 1], ids=["id_format", "id_java"])
def test_full_batch_digests(covt, gpu_available, golden_streams, id_mode):
    """BASELINE config 5 at full size (the bench's 10k-tile batch, 4.5 GB of output, slices past 4 GiB
    included): every stream's SHA-256 and status equal the oracle's for its source tile
    (tests/golden/oracle_streams.json), decoded by the bench's device-resident launch."""
    import torch

    import bench

    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks], covt.FORMAT_GENC, id_mode)
    assert plan.output_bytes > (1 << 32)
    db = covt.DeviceBatch(plan, "cuda")
    db.decode()
    torch.cuda.synchronize()
    out, res = db.results()
    del db
    col = golden_streams["columns"]
    pre = "fmt_" if id_mode == 0 else "java_"
    ish, ist, ico = col.index(pre + "sha256"), col.index(pre + "status"), col.index(pre + "consumed")
    st = plan.streams
    bounds = np.searchsorted(st["tile"], np.arange(plan.n_tiles + 1))
    n_past_4g = 0
    for t, (key, _) in enumerate(picks):
        rows = golden_streams["tiles"][key]["streams"]
        i0, i1 = int(bounds[t]), int(bounds[t + 1])
        assert i1 - i0 == len(rows), key
        for i, row in zip(range(i0, i1), rows):
            assert int(res[i][0]) == row[ist], (key, i)
            if row[ist] != 0:
                continue
            assert int(res[i][1]) == row[ico], (key, i)
            assert hashlib.sha256(plan.stream_array(out, i).tobytes()).hexdigest() == row[ish], (key, i)
            n_past_4g += int(st["out_off"][i] >= (1 << 32))
    assert n_past_4g > 10000


def test_byte_rle_reencode_advance(covt, oracle, gpu_available):
    """decodeByteRle(byte[], int, IntWrapper) (DecodingUtils.java:290): values as the :275 form, the
    cursor advanced by the ORC writer's re-encoded length (oracle_encode_byte_rle), including streams
    whose own encoding is not the writer's (non-canonical groups) and a partially read last group."""
    D = covt.DecodingUtils
    rng = np.random.default_rng(290)
    for trial in range(60):
        n = int(rng.integers(1, 700))
        kind = trial % 3
        if kind == 0:
            v = rng.integers(0, 3, size=n).astype(np.uint8)
        elif kind == 1:
            v = np.repeat(rng.integers(0, 256, size=n // 7 + 1), 7)[:n].astype(np.uint8)
        else:
            v = rng.integers(0, 256, size=n).astype(np.uint8)
        enc = oracle.encode_byte_rle(v)
        if trial % 5 == 4:  # non-canonical: every value as a 1-literal group (0xff = -1, value)
            enc = bytes(b for x in v for b in (0xFF, int(x)))
        m = n if trial % 4 else max(1, n - int(rng.integers(0, min(n, 50))))  # read fewer than encoded
        buf = b"\x11\x22" + enc + b"\x00" * 8
        p = covt.IntWrapper(2)
        got = D.decodeByteRle(buf, m, p)
        assert np.array_equal(got, v[:m]), trial
        assert p.get() == 2 + len(oracle.encode_byte_rle(v[:m])), trial


def test_decode_covt_layers(covt, gpu_available, oracle):
    """CovtParser mirror returns the GeometryColumn record of CovtParser.java:29-36."""
    t = open(tile_paths(("omt",))[0].replace("10_530_682", "5_16_20"), "rb").read()
    layers = covt.CovtParser.decode_covt(t)
    assert len(layers) == 8
    tr = [lc for lc in layers if lc.geometry.vertexOffsets is not None]
    assert tr, "ICE layers present"
    for lc in layers:
        g = lc.geometry
        assert g.geometryTypes is not None and g.vertexBuffer is not None
        assert g.geometryTypes.max() <= 5
        if g.vertexOffsets is not None:
            assert g.vertexOffsets.max() < g.vertexBuffer.size // 2


# --- stream-level API: every DecodingUtils mirror on every stream of a few tiles ---------------
STREAM_TILES = ("omt/5_16_20", "omt/14_8298_10748", "omt/9_265_341", "bing/4-8-5", "amazon/5_16_11")


@pytest.mark.parametrize("key", STREAM_TILES)
def test_stream_api_matches_oracle_java_semantics(covt, oracle, gpu_available, key):
    D = covt.DecodingUtils
    t = open(tile_paths()[0].rsplit("/tiles/", 1)[0] + "/tiles/" + key + ".covt", "rb").read()
    st, ss = oracle.walk_tile(t)
    assert st == 0
    for s in ss:
        pos = covt.IntWrapper(s.offset)
        off = s.offset
        if s.column_kind == 1 and s.stream_type == covt.GEOMETRY_TYPES:
            got = D.decodeByteRle(t, s.num_values, pos, s.byte_length)
            o = oracle.decode_byte_rle(t, s.num_values, off, s.byte_length)
            assert o[0] == 0 and np.array_equal(got, o[1]) and pos.get() == o[2]
        elif s.encoding == 5:
            got = D.decodeRle(t, s.num_values, pos, False)
            o = oracle.decode_rle(t, s.num_values, off, False)
            assert o[0] == 0 and np.array_equal(got, o[1])
            assert pos.get() == o[2]  # consumed == Java's re-encode advance for writer-made streams
        elif s.encoding == 9:
            if s.stream_type == covt.VERTEX_BUFFER and s.column_type == 4:
                got = D.decodeFastPfor128DeltaMortonCodes(t, s.num_values, s.byte_length, pos, s.num_bits)
                o = oracle.decode_fastpfor_delta_morton_codes(t, s.num_values, s.byte_length, off, s.num_bits)
            elif s.stream_type == covt.VERTEX_BUFFER:
                n = s.num_values * (2 if s.column_type == 3 else 1)
                got = D.decodeFastPfor128DeltaCoordinates(t, n, s.byte_length, pos)
                o = oracle.decode_fastpfor_delta_coordinates(t, n, s.byte_length, off)
            else:
                got = D.decodeFastPfor128ZigZagDelta(t, s.num_values, s.byte_length, pos)
                o = oracle.decode_fastpfor_zigzag_delta(t, s.num_values, s.byte_length, off)
            assert o[0] == 0 and np.array_equal(got, o[1]) and pos.get() == o[2]
        elif s.encoding == 4:
            if s.stream_type == covt.VERTEX_BUFFER and s.column_type == 4:
                got = D.decodeDeltaVarintMortonCodes(t, pos, s.num_values, s.num_bits)
                o = oracle.decode_delta_varint_morton_codes(t, off, s.num_values, s.num_bits)
            elif s.stream_type == covt.VERTEX_BUFFER:
                n = s.num_values * (2 if s.column_type == 3 else 1)
                got = D.decodeZigZagDeltaVarintCoordinates(t, pos, n)
                o = oracle.decode_zigzag_delta_varint_coordinates(t, off, n)
            else:
                got = D.decodeZigZagDeltaVarint(t, pos, s.num_values)
                o = oracle.decode_zigzag_delta_varint(t, off, s.num_values)
            assert o[0] == 0 and np.array_equal(got, o[1]) and pos.get() == o[2]
        elif s.encoding == 1:
            got = D.decodeVarint(t, pos, s.num_values)
            o = oracle.decode_varint(t, off, s.num_values)
            assert o[0] == 0 and np.array_equal(got, o[1]) and pos.get() == o[2]


def test_kats_on_gpu(covt, gpu_available):
    """Known-answer vectors of the reference's TS tests (tests/golden/kats.json)."""
    import json
    import os

    from conftest import GOLDEN

    k = json.load(open(os.path.join(GOLDEN, "kats.json")))
    D = covt.DecodingUtils
    for v in k["varint"]:
        p = covt.IntWrapper(v["pos"])
        assert list(D.decodeVarint(bytes(v["bytes"]), p, 1)) == [v["value"]] and p.get() == v["end"]
    for v in k["varint_java_divergence"]:
        p = covt.IntWrapper(v["pos"])
        assert list(D.decodeVarint(bytes(v["bytes"]), p, 1)) == [v["java_value"]] and p.get() == v["java_end"]
    for v in k["zigzag_varint"]:
        p = covt.IntWrapper(v["pos"])
        assert list(D.decodeZigZagVarint(bytes(v["bytes"]), p, 1)) == [v["value"]] and p.get() == v["end"]
    for v in k["rle"]:
        p = covt.IntWrapper(0)
        assert list(D.decodeRle(bytes(v["bytes"]), v["n"], p, v["signed"])) == v["values"]
        assert p.get() == v["end"]
