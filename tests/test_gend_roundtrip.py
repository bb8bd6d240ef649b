"""CPU: Gen D round trips.  Every decodable Gen C fixture is decoded by
the oracle and re-encoded as Gen D by the restated converter (oracle/gend.py); the Gen D tile must walk
(CovtParser.decodeLayerMetadata, CovtParser.java:574-652, with the implicit present streams of property
columns) and decode back to the same ids, GeometryColumn arrays and property values -- through the
oracle, and through libcovt's host plan (the product's Gen D walker)."""
import numpy as np
import pytest

import covt_gend_rt as RT


def _check_oracle_decode(oracle, gd, exp):
    st, ss = oracle.walk_tile(gd, oracle.FMT_GEND)
    assert st == 0
    got = {}
    for s in ss:
        st2, arr, cons = oracle.decode_stream(gd, s, oracle.ID_FORMAT)
        assert st2 == 0 and cons == s.byte_length, (s.layer, s.stream_type)
        got.setdefault(s.layer, {})[(s.column_kind, s.stream_type)] = arr
    for L, e in enumerate(exp):
        g = got.get(L, {})
        if e["ids"] is not None:
            assert np.array_equal(g[(0, 1)].astype(np.uint64), e["ids"]), L
        for k, arr in e["geom"].items():
            assert np.array_equal(g[(1, k)], arr), (L, k)
    st, ps = oracle.walk_properties(gd, oracle.FMT_GEND)
    assert st == 0
    by_layer = {}
    for p in ps:
        by_layer.setdefault(p.layer, []).append(p)
    for L, e in enumerate(exp):
        assert len(by_layer.get(L, [])) == len(e["props"]), L
        for p, (name, vals) in zip(by_layer.get(L, []), e["props"]):
            if name is not None:
                assert oracle.prop_name(gd, p) == name
            st2, got_vals = oracle.property_values(gd, p)
            assert st2 == 0 and got_vals == vals, (L, name)


def test_fixture_roundtrip_oracle(oracle, decodable_tiles):
    n = 0
    for key, t in decodable_tiles:
        gd, exp = RT.genc_to_gend(t)
        _check_oracle_decode(oracle, gd, exp)
        n += 1
    assert n == 126


@pytest.mark.parametrize("optimized,allow_fpf,with_ids", [(True, True, True), (False, False, True),
                                                          (True, False, False)])
def test_roundtrip_variants(oracle, decodable_tiles, optimized, allow_fpf, with_ids):
    for key, t in decodable_tiles[::7]:
        gd, exp = RT.genc_to_gend(t, optimized=optimized, allow_fpf=allow_fpf, with_ids=with_ids)
        _check_oracle_decode(oracle, gd, exp)


def test_product_gend_plan_matches_oracle_walk(covt, oracle, decodable_tiles):
    """libcovt's Gen D walker (covt_host.cpp walk_gend) agrees with the oracle's on converted tiles, Id /
    Geometry streams and property records alike."""
    tiles = [RT.genc_to_gend(t)[0] for _, t in decodable_tiles[::3]]
    plan = covt.Plan.from_tiles(tiles, covt.FORMAT_GEND, 0, covt.PLAN_PROPERTIES)
    assert (plan.tile_status == 0).all()
    st = plan.streams
    P = plan.props
    k = 0
    for t, gd in enumerate(tiles):
        ost, oss = oracle.walk_tile(gd, oracle.FMT_GEND)
        idx = [i for i in np.nonzero(st["tile"] == t)[0] if st["column_kind"][i] != 2]
        assert len(idx) == len(oss)
        for i, s in zip(idx, oss):
            assert (st["layer"][i], st["stream_type"][i], st["encoding"][i], st["num_values"][i],
                    st["byte_length"][i]) == (s.layer, s.stream_type, s.encoding, s.num_values, s.byte_length)
            assert st["in_off"][i] == int(plan.offsets[t]) + s.offset
        ost, props = oracle.walk_properties(gd, oracle.FMT_GEND)
        for q in props:
            r = P[k]
            assert (r["tile"], r["layer"], r["column"], r["n_features"]) == (t, q.layer, q.column, q.n_features)
            for role in range(3):
                if r["stream"][role] >= 0:
                    s = st[int(r["stream"][role])]
                    assert s["in_off"] == int(plan.offsets[t]) + q.s_off[role]
                    assert s["byte_length"] == q.s_bl[role]
            k += 1
    assert k == plan.num_property_columns > 1000


def test_gend_present_stream_is_implicit(oracle, decodable_tiles):
    """The writer lists no PRESENT metadata for property columns (CovtConverter.addNamedColumnMetadata
    :452-469) but writes the present bytes first; the walker's present length (consumed bytes) equals
    Java's re-encode advance (DecodingUtils.getByteRleChunkSize, :312-314)."""
    key, t = decodable_tiles[40]
    gd, _ = RT.genc_to_gend(t)
    st, props = oracle.walk_properties(gd, oracle.FMT_GEND)
    n = 0
    for p in props:
        if p.type == oracle.PROP_BOOLEAN:
            assert p.s_off[0] < 0
            continue
        nb = (p.n_features + 7) // 8
        st2, vals, pos, cons = oracle.decode_byte_rle(gd, nb, int(p.s_off[0]), 0)
        assert st2 == 0 and cons == p.s_bl[0] and p.s_off[1] == p.s_off[0] + cons
        n += 1
    assert n > 10
