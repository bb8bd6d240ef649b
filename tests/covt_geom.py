"""Geometry helpers for the MVT cross-check (the analogue of the reference's
``CovtParserTest.compareTiles``, evaluation/java/src/test/java/com/covt/decoder/CovtParserTest.java:62-90).

* ``mvt_layers``: a minimal protobuf reader for Mapbox Vector Tiles (spec v2), used only by
  ``tests/golden/make_golden.py`` on the reference's MVT fixtures.
* ``assemble``: rebuilds per-feature vertex lists from a decoded GeometryColumn
  (types + count streams + vertex offsets + vertex buffer), i.e. the count semantics of
  ``CovtParser.convertGeometryColumn`` (CovtParser.java:135-274) without its MULTIPOLYGON
  bugs.  Gen C ICE rings carry their closing vertex; it is stripped.
* ``layer_digest``: order-preserving SHA-256 of (geometry class, parts) per feature.
"""
from __future__ import annotations

import hashlib
import struct

POINT, LINESTRING, POLYGON, MULTIPOINT, MULTILINESTRING, MULTIPOLYGON = range(6)


# ---------------------------------------------------------------------------
# protobuf / MVT
# ---------------------------------------------------------------------------
def _varint(b: bytes, o: int):
    r = s = 0
    while True:
        x = b[o]
        o += 1
        r |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return r, o


def _fields(b: bytes):
    o = 0
    while o < len(b):
        key, o = _varint(b, o)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, o = _varint(b, o)
        elif wt == 2:
            n, o = _varint(b, o)
            v = b[o:o + n]
            o += n
        elif wt == 1:
            v = struct.unpack_from("<Q", b, o)[0]
            o += 8
        elif wt == 5:
            v = struct.unpack_from("<I", b, o)[0]
            o += 4
        else:
            raise ValueError("wire type %d" % wt)
        yield f, wt, v


def _packed(b: bytes):
    o, out = 0, []
    while o < len(b):
        v, o = _varint(b, o)
        out.append(v)
    return out


def _zz(v: int) -> int:
    return (v >> 1) ^ -(v & 1)


def _mvt_geometry(gtype: int, cmds):
    """Returns a list of parts (tuples of (x, y)) in MVT order; polygon rings without closing vertex."""
    parts, cur = [], None
    x = y = 0
    i = 0
    while i < len(cmds):
        c = cmds[i]
        i += 1
        cid, cnt = c & 7, c >> 3
        if cid == 1:  # MoveTo
            for _ in range(cnt):
                x += _zz(cmds[i])
                y += _zz(cmds[i + 1])
                i += 2
                if gtype == 1:
                    parts.append(((x, y),))
                else:
                    cur = [(x, y)]
                    parts.append(cur)
        elif cid == 2:  # LineTo
            for _ in range(cnt):
                x += _zz(cmds[i])
                y += _zz(cmds[i + 1])
                i += 2
                cur.append((x, y))
        elif cid == 7:  # ClosePath
            pass
        else:
            raise ValueError("command %d" % cid)
    return [tuple(p) for p in parts]


def mvt_layers(data: bytes):
    """{layer_name: {"extent": e, "features": [(id, geom_class, parts), ...]}}"""
    out = {}
    for f, wt, v in _fields(data):
        if f != 3 or wt != 2:
            continue
        name, extent, feats = None, 4096, []
        for lf, lwt, lv in _fields(v):
            if lf == 1:
                name = lv.decode("utf-8")
            elif lf == 5:
                extent = lv
            elif lf == 2:
                fid, gtype, geom = 0, 0, []
                for ff, fwt, fv in _fields(lv):
                    if ff == 1:
                        fid = fv
                    elif ff == 3:
                        gtype = fv
                    elif ff == 4:
                        geom = _packed(fv) if fwt == 2 else [fv]
                feats.append((fid, gtype, _mvt_geometry(gtype, geom)))
        out[name] = {"extent": extent, "features": feats}
    return out


# ---------------------------------------------------------------------------
# COVT GeometryColumn assembly
# ---------------------------------------------------------------------------
_CLASS = {POINT: 1, MULTIPOINT: 1, LINESTRING: 2, MULTILINESTRING: 2, POLYGON: 3, MULTIPOLYGON: 3}


def assemble(types, geometry_offsets, part_offsets, ring_offsets, vertex_offsets, vertex_buffer,
             ice_closing_vertex: bool):
    """Returns [(geom_class, parts)] per feature.  Count streams hold per-element counts."""
    go = iter(geometry_offsets if geometry_offsets is not None else [])
    po = iter(part_offsets if part_offsets is not None else [])
    ro = iter(ring_offsets if ring_offsets is not None else [])
    vb = vertex_buffer
    state = {"v": 0}

    def take(n):
        pts = []
        for _ in range(n):
            if vertex_offsets is not None:
                k = int(vertex_offsets[state["v"]])
            else:
                k = state["v"]
            state["v"] += 1
            pts.append((int(vb[2 * k]), int(vb[2 * k + 1])))
        return tuple(pts)

    def ring(n):
        r = take(n)
        if ice_closing_vertex and len(r) > 1 and r[0] == r[-1]:
            r = r[:-1]
        return r

    feats = []
    for t in types:
        t = int(t)
        parts = []
        if t == POINT:
            parts.append(take(1))
        elif t == MULTIPOINT:
            for _ in range(int(next(go))):
                parts.append(take(1))
        elif t == LINESTRING:
            parts.append(take(int(next(po))))
        elif t == MULTILINESTRING:
            for _ in range(int(next(go))):
                parts.append(take(int(next(po))))
        elif t == POLYGON:
            for _ in range(int(next(po))):
                parts.append(ring(int(next(ro))))
        elif t == MULTIPOLYGON:
            for _ in range(int(next(go))):
                for _ in range(int(next(po))):
                    parts.append(ring(int(next(ro))))
        else:
            raise ValueError("geometry type %d" % t)
        feats.append((_CLASS[t], parts))
    return feats


def layer_digest(features) -> str:
    """features: [(geom_class, parts)]"""
    h = hashlib.sha256()
    for cls, parts in features:
        h.update(struct.pack("<ii", cls, len(parts)))
        for p in parts:
            h.update(struct.pack("<i", len(p)))
            for x, y in p:
                h.update(struct.pack("<ii", x, y))
    return h.hexdigest()


def ids_digest(ids) -> str:
    h = hashlib.sha256()
    for i in ids:
        h.update(struct.pack("<Q", int(i) & 0xFFFFFFFFFFFFFFFF))
    return h.hexdigest()
