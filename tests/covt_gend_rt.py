"""Gen C fixture -> Gen D tile conversion for round-trip tests.

A Gen C fixture is decoded by the oracle (ids, GeometryColumn arrays, property values) and re-encoded
with the restated Gen D writer (oracle/gend.py).  The expected decode of the Gen D tile is then known
exactly: the same ids and GeometryColumn arrays, and per property column the Gen D semantics of
CovtParser.decodePropertyColumn (booleans: one value per feature, absent -> false, all valid;
localized Gen C sub-columns become plain dictionary columns named ``<column>:<lang>``)."""
from __future__ import annotations

import numpy as np

import oracle as O
from oracle import gend as W


def _layer_meta(t: bytes):
    """[(name, extent, n_features)] of a Gen C tile."""
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
    out = []
    for _ in range(nl):
        n, o = vu(o)
        name = t[o:o + n].decode()
        o += n
        ext, o = vu(o)
        nf, o = vu(o)
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
        out.append((name, ext, nf))
    return out


def genc_to_gend(t: bytes, optimized=False, allow_fpf=True, with_ids=True, with_props=True):
    """-> (Gen D tile bytes, expected) ; expected[layer] = {"ids", "geom": {stream_type: array},
    "column_type", "props": [(name or None, values)]}"""
    meta = _layer_meta(t)
    st, ss = O.walk_tile(t)
    assert st == 0
    dec = {}
    for s in ss:
        st2, arr, _ = O.decode_stream(t, s, O.ID_FORMAT)
        assert st2 == 0
        dec.setdefault(s.layer, {})[(s.column_kind, s.stream_type)] = (arr, s)
    props = {}
    if with_props:
        st, ps = O.walk_properties(t)
        assert st == 0
        for p in ps:
            st2, vals = O.property_values(t, p)
            assert st2 == 0
            props.setdefault(p.layer, []).append((O.prop_name(t, p), vals))
    layers, expected = [], []
    for L, (name, extent, nf) in enumerate(meta):
        d = dec.get(L, {})
        cols, exp = [], {"ids": None, "geom": {}, "props": [], "column_type": 0}
        if with_ids and (0, 1) in d:
            ids = d[(0, 1)][0].astype(np.uint64)
            cols.append(W.id_column(ids))
            exp["ids"] = ids
        g = {k[1]: v[0] for k, v in d.items() if k[0] == 1}
        ct = next((v[1].column_type for k, v in d.items() if k[0] == 1 and k[1] == W.VERTEX_BUFFER), 0)
        nb = int(extent).bit_length()  # 32 - Integer.numberOfLeadingZeros(extent), CovtParser.java:77
        vb = g.get(W.VERTEX_BUFFER, np.zeros(0, np.int32)).reshape(-1, 2)
        cols.append(W.geometry_column(g[W.GEOMETRY_TYPES], g.get(W.GEOMETRY_OFFSETS), g.get(W.PART_OFFSETS),
                                      g.get(W.RING_OFFSETS), g.get(W.VERTEX_OFFSETS), vb,
                                      int(ct), nb, allow_fpf, allow_fpf))
        exp["geom"] = g
        exp["column_type"] = int(ct)
        for pname, vals in props.get(L, []):
            if all(v is None for v in vals):
                continue  # a column without a single value carries no type
            cols.append(W.property_column(pname, vals))
            kinds = {type(v) for v in vals if v is not None}
            if kinds <= {bool}:
                vals = [bool(v) if v is not None else False for v in vals]
            elif kinds <= {float, int} and float in kinds:
                vals = [None if v is None else float(np.float32(v)) for v in vals]
            exp["props"].append((None if optimized else pname, vals))
        layers.append(W.layer(name, extent, nf, cols, optimized, L))
        expected.append(exp)
    return W.tile(layers), expected
