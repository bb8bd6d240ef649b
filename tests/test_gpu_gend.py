"""GPU parity on Gen D tiles (the layout CovtParser.decodeCovt reads, CovtParser.java:53-133, :574-652):
every decodable fixture converted by the restated Gen D writer (tests/covt_gend_rt.py, oracle/gend.py),
plus seeded synthetic Gen D layers whose int64 property values need 64-bit varints (the format ops) and
whose strings are multi-byte UTF-8.  Id / Geometry streams and property columns are bit-exact against
the oracle's Gen D decode, statuses included, in both Id modes."""
import numpy as np
import pytest

import covt_gend_rt as RT
from oracle import gend as W

pytestmark = pytest.mark.gpu


def _check_streams(covt, oracle, plan, out, res, tiles, mode):
    st = plan.streams
    n = 0
    for t, gd in enumerate(tiles):
        ost, oss = oracle.walk_tile(gd, oracle.FMT_GEND)
        assert ost == 0
        idx = [i for i in np.nonzero(st["tile"] == t)[0] if st["column_kind"][i] != 2]
        assert len(idx) == len(oss)
        for i, s in zip(idx, oss):
            o_st, o_arr, o_cons = oracle.decode_stream(gd, s, mode)
            assert int(res[i][0]) == o_st, (t, int(i))
            if o_st == 0:
                assert np.array_equal(plan.stream_array(out, int(i)), o_arr), (t, int(i))
                assert int(res[i][1]) == o_cons
            n += 1
    return n


def _check_props(covt, oracle, plan, buf, pres, tiles, mode):
    P = plan.props
    k = 0
    for t, gd in enumerate(tiles):
        ost, props = oracle.walk_properties(gd, oracle.FMT_GEND)
        for q in props:
            o = oracle.decode_property(gd, q, mode)
            assert int(pres["status"][k]) == o[0], (t, k)
            if o[0] == 0:
                col = plan.property_column(buf, pres, k)
                assert col.n_valid == o[5]
                assert np.array_equal(col.validity, o[1]) and np.array_equal(col.values.view(np.uint8),
                                                                             np.asarray(o[2]).view(np.uint8)), (t, k)
                if col.type == covt.PROP_STRING:
                    assert np.array_equal(col.dict_offsets, o[3]) and np.array_equal(col.dict_bytes, o[4])
            k += 1
    assert k == plan.num_property_columns
    return k


@pytest.mark.parametrize("mode", [0, 1], ids=["format", "java"])
def test_converted_fixtures_bitexact(covt, oracle, gpu_available, decodable_tiles, mode):
    tiles = [RT.genc_to_gend(t, optimized=(i % 3 == 1), allow_fpf=(i % 4 != 2))[0]
             for i, (_, t) in enumerate(decodable_tiles)]
    plan = covt.Plan.from_tiles(tiles, covt.FORMAT_GEND, mode, covt.PLAN_PROPERTIES)
    assert (plan.tile_status == 0).all()
    out, res = plan.decode_host()
    assert _check_streams(covt, oracle, plan, out, res, tiles, mode) >= 4000
    buf, pres = plan.properties_host()
    assert _check_props(covt, oracle, plan, buf, pres, tiles, mode) >= 9000


def _synthetic_layer(rng, L):
    n = int(rng.choice([0, 1, 7, 64, 65, 300, 2000]))
    types = np.zeros(n, np.uint8)  # points
    xy = rng.integers(-200, 8400, size=(n, 2))
    cols = [W.id_column(rng.integers(0, 1 << 40, size=n).astype(np.uint64)),
            W.geometry_column(types, vertices=xy, column_type=W.CT_PLAIN, num_bits=14)]
    pres = rng.random(n) < rng.choice([0.0, 0.3, 0.9, 1.0])
    big = [int(v) if p else None for v, p in zip(rng.integers(-(1 << 45), 1 << 45, size=n), pres)]
    small = [int(v) if p else None for v, p in zip(rng.integers(-5, 6, size=n), pres)]
    mono = [int(v) if p else None for v, p in zip(np.cumsum(rng.integers(0, 1 << 20, size=n)), pres)]
    flt = [float(v) if p else None for v, p in zip(rng.normal(size=n) * 1e3, pres)]
    words = ["Straße", "東京", "road", "", "ŻÓŁW", "x" * 40]
    strs = [words[int(i)] if p else None for i, p in zip(rng.integers(0, len(words), size=n), pres)]
    bools = [bool(b) if p else None for b, p in zip(rng.random(n) < 0.5, pres)]
    for name, vals in (("big", big), ("small", small), ("mono", mono), ("f", flt), ("s", strs), ("b", bools)):
        if any(v is not None for v in vals):
            cols.append(W.property_column(name, vals))
    return W.layer("L%d" % L, 8192, n, cols, optimized=bool(L & 1), layer_id=L)


@pytest.mark.parametrize("mode", [0, 1], ids=["format", "java"])
def test_synthetic_gend_layers(covt, oracle, gpu_available, mode):
    rng = np.random.default_rng(2024)
    tiles = [W.tile([_synthetic_layer(rng, L) for L in range(int(rng.integers(1, 5)))]) for _ in range(24)]
    plan = covt.Plan.from_tiles(tiles, covt.FORMAT_GEND, mode, covt.PLAN_PROPERTIES)
    assert (plan.tile_status == 0).all()
    out, res = plan.decode_host()
    _check_streams(covt, oracle, plan, out, res, tiles, mode)
    buf, pres = plan.properties_host()
    _check_props(covt, oracle, plan, buf, pres, tiles, mode)
    # 64-bit property varints: format mode decodes them, Java's 4-byte cap does not
    ops = set(plan.streams["op"][plan.streams["column_kind"] == 2].tolist())
    if mode == 0:
        assert {covt.OP_VARINT_ZZ_S64, covt.OP_BYTE_RLE_RAW, covt.OP_RLE_I32} <= ops
        assert (pres["status"] == 0).all()
