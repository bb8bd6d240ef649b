"""Test helpers for the geometry assembly (include/covt.h "Geometry assembly").

* ``oracle_tile_columns``: every geometry column of a tile decoded and assembled by the CPU oracle
  (oracle_assemble_geometry, the restatement of CovtParser.convertGeometryColumn :135-274);
* ``to_features``: nested offsets -> [(geom_class, parts)] with polygon rings un-closed, the
  representation of ``covt_geom.assemble`` and of the MVT digests;
* ``synth_column`` / ``pack_columns``: seeded synthetic GeometryColumns of every geometry type and the
  device buffers (decoded-stream buffer, covt_geom_desc table, assembly layout) to run the kernel on
  them directly through ``covt_assemble_geometry_device``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

POINT, LINESTRING, POLYGON, MULTIPOINT, MULTILINESTRING, MULTIPOLYGON = range(6)
_CLASS = {POINT: 1, MULTIPOINT: 1, LINESTRING: 2, MULTILINESTRING: 2, POLYGON: 3, MULTIPOLYGON: 3}


def oracle_tile_columns(oracle, tile: bytes, fmt: int = 0):
    """{layer: dict(status, types, column_type, closed, asm=(st, geo, part, ring, coords), streams)}"""
    st, ss = oracle.walk_tile(tile, fmt)
    if st:
        return {}
    cols = {}
    for s in ss:
        if s.column_kind != 1:
            continue
        c = cols.setdefault(s.layer, {"status": 0, "arr": {}, "column_type": s.column_type})
        st2, arr, _ = oracle.decode_stream(tile, s)
        if st2:
            c["status"] = c["status"] or st2
        c["arr"][s.stream_type] = arr
        if s.stream_type == 9:
            c["column_type"] = s.column_type
    for L, c in cols.items():
        c["closed"] = fmt == 0 and c["column_type"] in (3, 4)
        if c["status"]:
            c["asm"] = None
            continue
        a = c["arr"].get
        c["types"] = a(4) if a(4) is not None else np.zeros(0, np.uint8)
        c["asm"] = oracle.assemble_geometry(c["types"], a(5), a(6), a(7), a(8), a(9), c["closed"])
    return cols


def to_features(types, geo, part, ring, coords):
    """[(geom_class, parts)] with the closing vertex of every polygon ring removed."""
    out = []
    for f, t in enumerate(types):
        t = int(t)
        parts = []
        for p in range(int(geo[f]), int(geo[f + 1])):
            for r in range(int(part[p]), int(part[p + 1])):
                pts = [tuple(int(v) for v in xy) for xy in coords[int(ring[r]):int(ring[r + 1])]]
                if t in (POLYGON, MULTIPOLYGON) and pts:
                    pts = pts[:-1]
                parts.append(tuple(pts))
        out.append((_CLASS[t], parts))
    return out


# ---------------------------------------------------------------------------
# synthetic columns
# ---------------------------------------------------------------------------
def synth_column(rng, n, ice, closed, big=False, probs=None):
    """A consistent GeometryColumn of n features: dict(types, go, po, ro, vo, vb, closed)."""
    probs = probs if probs is not None else [0.2, 0.2, 0.2, 0.1, 0.15, 0.15]
    types = rng.choice(6, size=n, p=probs).astype(np.uint8)
    go, po, ro = [], [], []
    nsrc = 0
    hi_parts, hi_rings, hi_verts = (300, 40, 3000) if big else (4, 3, 12)

    def ring_len():
        v = int(rng.integers(0, hi_verts))
        return v

    for t in types:
        t = int(t)
        if t == POINT:
            nsrc += 1
        elif t == MULTIPOINT:
            k = int(rng.integers(0, hi_parts))
            go.append(k)
            nsrc += k
        elif t == LINESTRING:
            v = ring_len()
            po.append(v)
            nsrc += v
        elif t == MULTILINESTRING:
            k = int(rng.integers(0, hi_parts))
            go.append(k)
            for _ in range(k):
                v = ring_len()
                po.append(v)
                nsrc += v
        else:
            k = 1 if t == POLYGON else int(rng.integers(0, hi_parts))
            if t == MULTIPOLYGON:
                go.append(k)
            for _ in range(k):
                r = int(rng.integers(0, hi_rings))
                po.append(r)
                for _ in range(r):
                    v = ring_len()
                    ro.append(v)
                    nsrc += v
    i32 = lambda a: np.asarray(a, dtype=np.int32)  # noqa: E731
    if ice:
        nvb = max(1, nsrc // 2 + 1)
        vo = rng.integers(0, nvb, size=nsrc).astype(np.int32)
    else:
        nvb, vo = nsrc, None
    vb = rng.integers(-(1 << 31), 1 << 31, size=2 * nvb, dtype=np.int64).astype(np.int32)
    return {"types": types, "go": i32(go), "po": i32(po), "ro": i32(ro), "vo": vo, "vb": vb, "closed": closed}


def caps(col):
    n_src = col["vo"].size if col["vo"] is not None else col["vb"].size // 2
    npo, nro = col["po"].size, col["ro"].size
    return n_src + npo, n_src + npo + nro, n_src + (0 if col["closed"] else nro)


def _a16(x):
    return (x + 15) & ~15


def pack_columns(covt, cols, flags_extra=None, in_res=None):
    """-> (decoded uint8 buffer, desc bytes, assembly bytes, layouts) for covt_assemble_geometry_device."""
    parts, off = [], 0
    descs = (covt.GeomDesc * max(len(cols), 1))()
    layouts = []
    aoff = 0
    for ci, col in enumerate(cols):
        d = descs[ci]
        arrs = [col["types"], col["go"], col["po"], col["ro"], col["vo"], col["vb"]]
        for k, a in enumerate(arrs):
            if a is None:
                d.in_off[k], d.in_len[k] = -1, 0
            else:
                b = np.ascontiguousarray(a).tobytes()
                d.in_off[k] = off
                d.in_len[k] = a.size // 2 if k == 5 else a.size
                parts.append((off, b))
                off = _a16(off + len(b))
            d.in_res[k] = -1 if in_res is None else in_res[ci][k]
        pcap, rcap, ccap = col.get("caps") or caps(col)
        d.part_cap, d.ring_cap, d.coord_cap = pcap, rcap, ccap
        d.flags = (1 if col["closed"] else 0) | (flags_extra[ci] if flags_extra else 0)
        if d.flags & 0x80000000:
            d.flags -= 1 << 32
        n = col["types"].size
        sizes = [4 * (n + 1), 4 * (pcap + 1), 4 * (rcap + 1), 8 * ccap, 4 * pcap, 4 * rcap]
        lay = []
        for k in range(6):
            d.out_off[k] = aoff
            lay.append(aoff)
            aoff = _a16(aoff + sizes[k])
        layouts.append(lay)
    dec = np.zeros(max(off, 16) + 64, dtype=np.uint8)
    for o, b in parts:
        dec[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    desc_bytes = np.frombuffer(bytes(descs), dtype=np.uint8)[:len(cols) * C.sizeof(covt.GeomDesc)].copy()
    return dec, desc_bytes, max(aoff, 16), layouts


def unpack_column(asm, lay, n, res):
    st, npart, nring, ncoord = (int(res[k]) for k in ("status", "num_parts", "num_rings", "num_coords"))
    geo = asm[lay[0]:lay[0] + 4 * (n + 1)].view(np.int32)
    part = asm[lay[1]:lay[1] + 4 * (npart + 1)].view(np.int32)
    ring = asm[lay[2]:lay[2] + 4 * (nring + 1)].view(np.int32)
    coords = asm[lay[3]:lay[3] + 8 * ncoord].view(np.int32).reshape(-1, 2)
    return st, geo, part, ring, coords
