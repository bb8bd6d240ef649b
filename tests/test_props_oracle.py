"""CPU: the property-column oracle (oracle/covt_oracle_props.c, restating CovtParser.decodePropertyColumn
CovtParser.java:276-354) pinned by the reference's own data -- the property half of
CovtParserTest.compareTiles (CovtParserTest.java:62-90): every decoded property (sub)column of the OMT
fixtures equals the feature properties of the reference's MVT originals (digests committed in
tests/golden/mvt_prop_digests.json by tests/golden/make_golden.py)."""
import collections
import json
import os

import pytest

import covt_props as P
from conftest import GOLDEN, tile_paths


@pytest.fixture(scope="module")
def prop_golden():
    with open(os.path.join(GOLDEN, "mvt_prop_digests.json")) as f:
        return json.load(f)


def test_every_fixture_property_column_decodes(oracle):
    kinds = collections.Counter()
    for p in tile_paths():
        t = open(p, "rb").read()
        st, props = oracle.walk_properties(t)
        assert st == 0, p
        for q in props:
            for mode in (oracle.ID_FORMAT, oracle.ID_JAVA):
                st2, *_ = oracle.decode_property(t, q, mode)
                assert st2 == 0, (p, oracle.prop_name(t, q), mode)
            kinds[(q.type, q.column_type)] += 1
    # dictionary strings, localized strings (Gen C), int64, float (Bing), boolean
    assert kinds[(oracle.PROP_STRING, 1)] >= 1800 and kinds[(oracle.PROP_STRING, 2)] >= 9000
    assert kinds[(oracle.PROP_INT64, 0)] >= 1600 and kinds[(oracle.PROP_FLOAT, 0)] >= 150
    assert kinds[(oracle.PROP_BOOLEAN, 0)] >= 30


def test_property_columns_equal_mvt_originals(oracle, prop_golden):
    """Live: decode every property (sub)column of the OMT tiles and compare its per-feature values with
    the digest of the matching MVT key."""
    n_pass = n_total = 0
    for name, g in sorted(prop_golden.items()):
        t = open(os.path.join(GOLDEN, "tiles", "omt", name + ".covt"), "rb").read()
        names = _names(t)
        st, props = oracle.walk_properties(t)
        assert st == 0 and len(props) == g["n_props"], name
        passed = []
        for p in props:
            st2, vals = oracle.property_values(t, p)
            assert st2 == 0
            col = oracle.prop_name(t, p)
            base, lang = (col.split(":", 1) + [None])[:2] if p.lang >= 0 else (col, None)
            dig = g["mvt"].get(names[p.layer], {})
            d = P.values_digest(vals)
            if any(dig.get(k) == d for k in P.candidate_keys(base, lang)):
                passed.append([p.layer, col])
        assert passed == g["oracle_pass"], name
        n_pass += len(passed)
        n_total += len(props)
    # every property column of every OMT tile with an MVT original matches it
    assert n_total >= 8600 and n_pass == n_total


def test_java_and_format_modes_agree_on_fixtures(oracle):
    """Property varints in the fixtures are <= 3 bytes, so Java's 4-byte cap (DecodingUtils.java:157-186)
    and the 64-bit format reading give the same int64 columns."""
    import numpy as np

    for p in tile_paths(("omt",))[:40]:
        t = open(p, "rb").read()
        for q in oracle.walk_properties(t)[1]:
            if q.type != oracle.PROP_INT64 or q.s_enc[1] == 5:
                continue
            a = oracle.decode_property(t, q, oracle.ID_FORMAT)
            b = oracle.decode_property(t, q, oracle.ID_JAVA)
            assert a[0] == b[0] == 0 and np.array_equal(a[2], b[2])


def test_boolean_semantics(oracle):
    """Gen C boolean columns with a present stream hold only the present values' bits (data numValues =
    present count); without one (Gen D, CovtParser.java:280-291) one bit per feature, all valid."""
    seen = collections.Counter()
    for p in tile_paths(("bing",)):
        t = open(p, "rb").read()
        for q in oracle.walk_properties(t)[1]:
            if q.type != oracle.PROP_BOOLEAN:
                continue
            st, val, vals, _, _, nv = oracle.decode_property(t, q)
            assert st == 0
            if q.s_off[0] >= 0:
                assert q.s_nv[1] == nv
                seen["dense"] += 1
            else:
                assert nv == q.n_features
                seen["per_feature"] += 1
            assert not (vals & ~val).any()  # values only where valid
    assert seen["dense"] >= 15 and seen["per_feature"] >= 10


def _names(t):
    def vu(o):
        r = sh = 0
        while True:
            b = t[o]
            o += 1
            r |= (b & 0x7F) << sh
            sh += 7
            if b < 0x80:
                return r, o

    o = 0
    _, o = vu(o)
    nl, o = vu(o)
    names = []
    for _ in range(nl):
        n, o = vu(o)
        names.append(t[o:o + n].decode())
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
    return names
