"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the COVT Id/Geometry stream decode path.

ctypes binding of ``liboracle_covt.so`` (plain-C restatement of the reference's
``com.covt.decoder.DecodingUtils`` / ``CovtParser`` semantics, see ``covt_oracle.h``).
A pure-Python second restatement lives in ``oracle.pyref`` and is used to cross-check
the C one on small inputs and to generate golden vectors.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package.  The product path (``cov-tiles_amd``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_covt.so")

OK, ERR_UNSUPPORTED, ERR_TRUNCATED, ERR_COUNT, ERR_HEADER, ERR_ARG = 0, -1, -2, -3, -4, -6
FMT_GENC, FMT_GEND = 0, 1
ID_FORMAT, ID_JAVA = 0, 1


class OracleStream(C.Structure):
    _fields_ = [
        ("layer", C.c_int32),
        ("column_kind", C.c_int32),
        ("stream_type", C.c_int32),
        ("encoding", C.c_int32),
        ("column_type", C.c_int32),
        ("num_values", C.c_int32),
        ("byte_length", C.c_int32),
        ("num_bits", C.c_int32),
        ("offset", C.c_int64),
        ("extent", C.c_int32),
        ("num_features", C.c_int32),
    ]


PROP_BOOLEAN, PROP_INT64, PROP_FLOAT, PROP_STRING = 0, 1, 2, 3


class OracleProp(C.Structure):
    """oracle_prop (covt_oracle.h): one property (sub)column; s_* indexed by role
    0 present, 1 data, 2 length, 3 dictionary."""
    _fields_ = [("layer", C.c_int32), ("column", C.c_int32), ("type", C.c_int32), ("column_type", C.c_int32),
                ("n_features", C.c_int32), ("lang", C.c_int32), ("name_len", C.c_int32), ("lang_len", C.c_int32),
                ("name_off", C.c_int64), ("lang_off", C.c_int64), ("s_off", C.c_int64 * 4), ("s_nv", C.c_int32 * 4),
                ("s_bl", C.c_int32 * 4), ("s_enc", C.c_int32 * 4)]


def build(force: bool = False) -> str:
    srcs = ("covt_oracle.c", "covt_oracle_props.c", "mvt_decode.c", "covt_oracle.h")
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < max(os.path.getmtime(os.path.join(_HERE, f)) for f in srcs)
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle_covt.so"])
    return _LIB_PATH


_lib = None


def build_native(out_dir: str) -> str:
    """The same restatement built with -march=native into `out_dir` (bench.py's cpu_baseline leg builds it on
    the GPU box's own host, SURVEY §8(d) "CPU timing"); returns the library path."""
    out = os.path.join(out_dir, "liboracle_covt_native.so")
    srcs = [os.path.join(_HERE, f) for f in ("covt_oracle.c", "covt_oracle_props.c", "covt_oracle_tile.c",
                                             "mvt_decode.c")]
    subprocess.check_call([os.environ.get("CC", "gcc"), "-O3", "-march=native", "-fPIC", "-std=c11", "-shared",
                           "-o", out] + srcs + ["-lpthread"])
    return out


def load_native(path: str):
    """A separately built copy of the restatement (build_native), bound like lib()."""
    return _bind(C.CDLL(path))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = _bind(C.CDLL(_LIB_PATH))
    return _lib


def _bind(L):
    """Set the ctypes signatures of a liboracle_covt CDLL."""
    u8p, i32p, i64p = C.POINTER(C.c_uint8), C.POINTER(C.c_int32), C.POINTER(C.c_int64)
    sz = C.c_size_t
    L.oracle_walk_tile.argtypes = [u8p, sz, C.c_int, C.POINTER(OracleStream), C.c_int32, i32p]
    L.mvt_decode_tile.argtypes = [u8p, C.c_int64, C.c_int, i32p, C.c_int64, i64p, C.POINTER(C.c_uint64)]
    L.oracle_decode_stream.argtypes = [u8p, sz, C.POINTER(OracleStream), C.c_int, C.c_void_p, i32p]
    L.oracle_stream_output.argtypes = [C.POINTER(OracleStream), C.c_int, i32p, i64p]
    L.oracle_decode_tile_full.argtypes = [C.POINTER(C.c_uint8), C.c_size_t, C.c_int, C.c_int,
                                          C.POINTER(C.c_int64)]
    L.oracle_decode_tiles_mt.argtypes = [u8p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int32,
                                         C.c_int, C.c_int, C.c_int32, i64p, i64p, i64p]
    L.oracle_encode_varints_u64.restype = C.c_int64
    L.oracle_encode_varints_u64.argtypes = [C.POINTER(C.c_uint64), C.c_int64, u8p, C.c_int64]
    L.oracle_encode_rle.restype = C.c_int64
    L.oracle_encode_rle.argtypes = [i64p, C.c_int64, C.c_int, u8p, C.c_int64]
    L.oracle_encode_byte_rle.restype = C.c_int64
    L.oracle_encode_byte_rle.argtypes = [u8p, C.c_int64, u8p, C.c_int64]
    L.oracle_encode_fastpfor.restype = C.c_int64
    L.oracle_encode_fastpfor.argtypes = [C.POINTER(C.c_uint32), C.c_int64, u8p, C.c_int64]
    L.oracle_fastpfor_uncompress.argtypes = [u8p, sz, C.c_int32, C.c_int32, C.c_int32,
                                             C.POINTER(C.c_uint32), i32p]
    for name in ("oracle_decode_varint", "oracle_decode_zigzag_varint", "oracle_decode_zigzag_delta_varint",
                 "oracle_decode_zigzag_delta_varint_coordinates"):
        getattr(L, name).argtypes = [u8p, sz, i32p, C.c_int32, i32p]
    L.oracle_decode_varint_u64.argtypes = [u8p, sz, i32p, C.c_int32, C.POINTER(C.c_uint64)]
    L.oracle_decode_rle.argtypes = [u8p, sz, C.c_int32, i32p, C.c_int, i64p, i32p]
    L.oracle_decode_byte_rle.argtypes = [u8p, sz, C.c_int32, i32p, C.c_int32, u8p, i32p]
    L.oracle_decode_fastpfor_zigzag_delta.argtypes = [u8p, sz, C.c_int32, C.c_int32, i32p, i32p]
    L.oracle_decode_fastpfor_delta_coordinates.argtypes = [u8p, sz, C.c_int32, C.c_int32, i32p, i32p]
    L.oracle_decode_delta_varint_morton_codes.argtypes = [u8p, sz, i32p, C.c_int32, C.c_int32, i32p]
    L.oracle_decode_fastpfor_delta_morton_codes.argtypes = [u8p, sz, C.c_int32, C.c_int32, i32p, C.c_int32,
                                                            i32p]
    L.oracle_decode_morton.argtypes = [C.c_int32, C.c_int32, i32p, i32p]
    L.oracle_decode_morton.restype = None
    L.oracle_assemble_geometry.argtypes = [u8p, C.c_int32, i32p, C.c_int32, i32p, C.c_int32, i32p, C.c_int32,
                                           i32p, C.c_int32, i32p, C.c_int32, C.c_int, C.c_int32, C.c_int32,
                                           C.c_int32, i32p, i32p, i32p, i32p, i32p, i32p, i32p]
    L.oracle_walk_properties.argtypes = [u8p, sz, C.c_int, C.POINTER(OracleProp), C.c_int32, i32p]
    L.oracle_property_sizes.argtypes = [C.POINTER(OracleProp), i64p]
    L.oracle_property_sizes.restype = None
    L.oracle_decode_property.argtypes = [u8p, sz, C.POINTER(OracleProp), C.c_int, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, i32p]
    return L


def _u8(buf) -> tuple:
    arr = np.frombuffer(bytes(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    if arr.size == 0:
        arr = np.zeros(1, dtype=np.uint8)[:0]
    return arr, arr.ctypes.data_as(C.POINTER(C.c_uint8))


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


# ---------------------------------------------------------------------------
# stream-level functions (DecodingUtils mirrors).  Each returns (status, values, new_pos)
# ---------------------------------------------------------------------------
def _varint_family(name, buf, pos, n):
    arr, p = _u8(buf)
    out = np.zeros(max(n, 1), dtype=np.int32)
    cpos = C.c_int32(pos)
    st = getattr(lib(), name)(p, arr.size, C.byref(cpos), n, _p(out, C.c_int32))
    return st, out[:n], cpos.value


def decode_varint(buf, pos, n):
    return _varint_family("oracle_decode_varint", buf, pos, n)


def decode_zigzag_varint(buf, pos, n):
    return _varint_family("oracle_decode_zigzag_varint", buf, pos, n)


def decode_zigzag_delta_varint(buf, pos, n):
    return _varint_family("oracle_decode_zigzag_delta_varint", buf, pos, n)


def decode_zigzag_delta_varint_coordinates(buf, pos, n):
    return _varint_family("oracle_decode_zigzag_delta_varint_coordinates", buf, pos, n)


def decode_varint_u64(buf, pos, n):
    arr, p = _u8(buf)
    out = np.zeros(max(n, 1), dtype=np.uint64)
    cpos = C.c_int32(pos)
    st = lib().oracle_decode_varint_u64(p, arr.size, C.byref(cpos), n, _p(out, C.c_uint64))
    return st, out[:n], cpos.value


def decode_rle(buf, n, pos, signed):
    """Returns (status, int64 values, new_pos (Java re-encode advance), consumed bytes)."""
    arr, p = _u8(buf)
    out = np.zeros(max(n, 1), dtype=np.int64)
    cpos, cons = C.c_int32(pos), C.c_int32(0)
    st = lib().oracle_decode_rle(p, arr.size, n, C.byref(cpos), int(signed), _p(out, C.c_int64), C.byref(cons))
    return st, out[:n], cpos.value, cons.value


def decode_byte_rle(buf, n, pos, byte_length):
    arr, p = _u8(buf)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    cpos, cons = C.c_int32(pos), C.c_int32(0)
    st = lib().oracle_decode_byte_rle(p, arr.size, n, C.byref(cpos), byte_length, _p(out, C.c_uint8),
                                      C.byref(cons))
    return st, out[:n], cpos.value, cons.value


def decode_fastpfor_zigzag_delta(buf, n, byte_length, pos):
    arr, p = _u8(buf)
    out = np.zeros(max(n, 1), dtype=np.int32)
    cpos = C.c_int32(pos)
    st = lib().oracle_decode_fastpfor_zigzag_delta(p, arr.size, n, byte_length, C.byref(cpos), _p(out, C.c_int32))
    return st, out[:n], cpos.value


def decode_fastpfor_delta_coordinates(buf, n, byte_length, pos):
    arr, p = _u8(buf)
    out = np.zeros(max(n, 1), dtype=np.int32)
    cpos = C.c_int32(pos)
    st = lib().oracle_decode_fastpfor_delta_coordinates(p, arr.size, n, byte_length, C.byref(cpos),
                                                        _p(out, C.c_int32))
    return st, out[:n], cpos.value


def decode_delta_varint_morton_codes(buf, pos, n_vertices, num_bits):
    arr, p = _u8(buf)
    out = np.zeros(max(2 * n_vertices, 1), dtype=np.int32)
    cpos = C.c_int32(pos)
    st = lib().oracle_decode_delta_varint_morton_codes(p, arr.size, C.byref(cpos), n_vertices, num_bits,
                                                       _p(out, C.c_int32))
    return st, out[:2 * n_vertices], cpos.value


def decode_fastpfor_delta_morton_codes(buf, n_vertices, byte_length, pos, num_bits):
    arr, p = _u8(buf)
    out = np.zeros(max(2 * n_vertices, 1), dtype=np.int32)
    cpos = C.c_int32(pos)
    st = lib().oracle_decode_fastpfor_delta_morton_codes(p, arr.size, n_vertices, byte_length, C.byref(cpos),
                                                         num_bits, _p(out, C.c_int32))
    return st, out[:2 * n_vertices], cpos.value


def fastpfor_uncompress(buf, pos, byte_length, n):
    arr, p = _u8(buf)
    out = np.zeros(max(n, 1), dtype=np.uint32)
    dec = C.c_int32(0)
    st = lib().oracle_fastpfor_uncompress(p, arr.size, pos, byte_length, n, _p(out, C.c_uint32), C.byref(dec))
    return st, out[:n], dec.value


def decode_morton(code, num_bits):
    x, y = C.c_int32(), C.c_int32()
    lib().oracle_decode_morton(code, num_bits, C.byref(x), C.byref(y))
    return x.value, y.value


# ---------------------------------------------------------------------------
# encoders
# ---------------------------------------------------------------------------
def encode_varints(values) -> bytes:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
    n = lib().oracle_encode_varints_u64(_p(v, C.c_uint64), v.size, None, 0)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().oracle_encode_varints_u64(_p(v, C.c_uint64), v.size, _p(out, C.c_uint8), n)
    return out[:n].tobytes()


def encode_rle(values, signed=False) -> bytes:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.int64))
    n = lib().oracle_encode_rle(_p(v, C.c_int64), v.size, int(signed), None, 0)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().oracle_encode_rle(_p(v, C.c_int64), v.size, int(signed), _p(out, C.c_uint8), n)
    return out[:n].tobytes()


def encode_byte_rle(values) -> bytes:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.uint8))
    n = lib().oracle_encode_byte_rle(_p(v, C.c_uint8), v.size, None, 0)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().oracle_encode_byte_rle(_p(v, C.c_uint8), v.size, _p(out, C.c_uint8), n)
    return out[:n].tobytes()


def encode_fastpfor(values) -> bytes:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.uint32))
    cap = v.size * 8 + 65536
    out = np.zeros(cap, dtype=np.uint8)
    n = lib().oracle_encode_fastpfor(_p(v, C.c_uint32), v.size, _p(out, C.c_uint8), cap)
    assert n >= 0, n
    return out[:n].tobytes()


# ---------------------------------------------------------------------------
# tile level
# ---------------------------------------------------------------------------
def walk_tile(tile: bytes, fmt: int = FMT_GENC):
    arr, p = _u8(tile)
    n = C.c_int32(0)
    st = lib().oracle_walk_tile(p, arr.size, fmt, None, 0, C.byref(n))
    if st:
        return st, []
    ss = (OracleStream * max(n.value, 1))()
    st = lib().oracle_walk_tile(p, arr.size, fmt, ss, n.value, C.byref(n))
    return st, list(ss[: n.value])


def walk_properties(tile: bytes, fmt: int = FMT_GENC):
    """(status, [OracleProp]) -- every property (sub)column of a tile (covt_oracle_props.c)."""
    arr, p = _u8(tile)
    n = C.c_int32(0)
    st = lib().oracle_walk_properties(p, arr.size, fmt, None, 0, C.byref(n))
    if st:
        return st, []
    ps = (OracleProp * max(n.value, 1))()
    st = lib().oracle_walk_properties(p, arr.size, fmt, ps, n.value, C.byref(n))
    return st, list(ps[: n.value])


def prop_name(tile: bytes, p: OracleProp) -> str:
    """Column name, plus ':<lang>' for a localized sub-column (Gen C)."""
    name = bytes(tile[p.name_off:p.name_off + p.name_len]).decode("utf-8") if p.name_off >= 0 else ""
    if p.lang >= 0:
        name += ":" + bytes(tile[p.lang_off:p.lang_off + p.lang_len]).decode("utf-8")
    return name


def decode_property(tile: bytes, p: OracleProp, mode: int = ID_FORMAT):
    """(status, validity u8[ceil(n/8)], values, dict_offsets i32[n_dict+1], dict_bytes u8, n_valid) in the
    Arrow-style layout of include/covt.h ("Property columns")."""
    arr, tp = _u8(tile)
    sz = np.zeros(4, dtype=np.int64)
    lib().oracle_property_sizes(C.byref(p), _p(sz, C.c_int64))
    bufs = [np.zeros(max(int(x), 1) + 16, dtype=np.uint8) for x in sz]
    nv = C.c_int32(0)
    st = lib().oracle_decode_property(tp, arr.size, C.byref(p), mode, bufs[0].ctypes.data, bufs[1].ctypes.data,
                                      bufs[2].ctypes.data, bufs[3].ctypes.data, C.byref(nv))
    vdt = {PROP_INT64: np.int64, PROP_FLOAT: np.float32, PROP_STRING: np.int32}.get(p.type)
    vals = bufs[1][:int(sz[1])]
    if vdt is not None:
        vals = vals.view(vdt)
    return (st, bufs[0][:int(sz[0])], vals, bufs[2][:int(sz[2])].view(np.int32), bufs[3][:int(sz[3])],
            nv.value)


def property_values(tile: bytes, p: OracleProp, mode: int = ID_FORMAT):
    """Java-level view (List<Optional>): per feature None or the value (bool / int / float / str)."""
    st, val, vals, doff, dby, _ = decode_property(tile, p, mode)
    if st:
        return st, None
    out = []
    for i in range(p.n_features):
        if not (int(val[i >> 3]) >> (i & 7)) & 1:
            out.append(None)
        elif p.type == PROP_BOOLEAN:
            out.append(bool((int(vals[i >> 3]) >> (i & 7)) & 1))
        elif p.type == PROP_INT64:
            out.append(int(vals[i]))
        elif p.type == PROP_FLOAT:
            out.append(float(vals[i]))
        else:
            k = int(vals[i])
            out.append(bytes(dby[doff[k]:doff[k + 1]]).decode("utf-8"))
    return st, out


def stream_output(s: OracleStream, id_mode: int = ID_FORMAT):
    eb, ne = C.c_int32(), C.c_int64()
    lib().oracle_stream_output(C.byref(s), id_mode, C.byref(eb), C.byref(ne))
    return eb.value, ne.value


_DT = {1: np.uint8, 4: np.int32, 8: np.int64}


def decode_stream(tile: bytes, s: OracleStream, id_mode: int = ID_FORMAT):
    """Returns (status, decoded numpy array, consumed bytes)."""
    arr, p = _u8(tile)
    eb, ne = stream_output(s, id_mode)
    out = np.zeros(max(ne, 1), dtype=_DT[eb])
    cons = C.c_int32(0)
    st = lib().oracle_decode_stream(p, arr.size, C.byref(s), id_mode, out.ctypes.data, C.byref(cons))
    return st, out[:ne], cons.value


def decode_tiles_mt(blob: np.ndarray, offsets, sizes, fmt=FMT_GENC, id_mode=ID_FORMAT, threads=1, L=None):
    """Walk + decode every Id/Geometry stream of every tile on `threads` host threads (the CPU baseline);
    `L` = a library from load_native() (default: lib())."""
    L = L or lib()
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
    szs = np.ascontiguousarray(np.asarray(sizes, dtype=np.uint64))
    ib, ob, vx = C.c_int64(), C.c_int64(), C.c_int64()
    st = L.oracle_decode_tiles_mt(_p(blob, C.c_uint8), _p(offs, C.c_uint64), _p(szs, C.c_uint64), offs.size,
                                      fmt, id_mode, threads, C.byref(ib), C.byref(ob), C.byref(vx))
    return st, ib.value, ob.value, vx.value


# ---------------------------------------------------------------------------
# geometry assembly (CovtParser.convertGeometryColumn, CovtParser.java:135-274)
# ---------------------------------------------------------------------------
def decode_tile_full(tile: bytes, fmt=FMT_GENC, id_mode=ID_FORMAT, L=None):
    """BASELINE configs[0]: one tile decoded the way CovtParser.decodeCovt does (walk, Id / Geometry streams,
    geometry assembly, property columns), one thread -> (status, dict of counts)."""
    L = L or lib()
    buf = (C.c_uint8 * max(len(tile), 1)).from_buffer_copy(tile if tile else b"\0")
    cnt = (C.c_int64 * 4)()
    st = L.oracle_decode_tile_full(buf, len(tile), fmt, id_mode, cnt)
    return st, {"streams": cnt[0], "vertices": cnt[1], "coords": cnt[2], "property_columns": cnt[3]}


def assemble_geometry(types, go, po, ro, vo, vb, closed_in_stream: bool, caps=None):
    """Nested-offset assembly of one decoded GeometryColumn (count arrays may be None).
    vb: int32 x,y interleaved.  Returns (status, geo_off, part_off, ring_off, coords[k,2])."""
    def arr(a):
        return None if a is None else np.ascontiguousarray(np.asarray(a, dtype=np.int32))

    types = np.ascontiguousarray(np.asarray(types if types is not None else [], dtype=np.uint8))
    go, po, ro, vo, vb = arr(go), arr(po), arr(ro), arr(vo), arr(vb if vb is not None else [])
    n_vb = vb.size // 2
    n_src = vo.size if vo is not None else n_vb
    nl = lambda a: 0 if a is None else a.size  # noqa: E731
    if caps is None:  # the plan's data-independent bounds (cov-tiles_amd/csrc/covt_host.cpp plan_geometry)
        caps = (n_src + nl(po), n_src + nl(po) + nl(ro), n_src + (0 if closed_in_stream else nl(ro)))
    pcap, rcap, ccap = caps
    geo = np.zeros(types.size + 1, dtype=np.int32)
    part = np.zeros(pcap + 1, dtype=np.int32)
    ring = np.zeros(rcap + 1, dtype=np.int32)
    coords = np.zeros(2 * max(ccap, 1), dtype=np.int32)
    np_, nr, nc = C.c_int32(), C.c_int32(), C.c_int32()
    ip = lambda a: None if a is None else _p(a, C.c_int32)  # noqa: E731
    st = lib().oracle_assemble_geometry(_p(types, C.c_uint8), types.size, ip(go), nl(go), ip(po), nl(po), ip(ro),
                                        nl(ro), ip(vo), nl(vo), ip(vb), n_vb, int(bool(closed_in_stream)), pcap,
                                        rcap, ccap, _p(geo, C.c_int32), _p(part, C.c_int32), _p(ring, C.c_int32),
                                        _p(coords, C.c_int32), C.byref(np_), C.byref(nr), C.byref(nc))
    return (st, geo, part[:np_.value + 1], ring[:nr.value + 1], coords[:2 * nc.value].reshape(-1, 2))


# ---------------------------------------------------------------------------
# MVT decoder (benchmark infrastructure for the MVT-vs-COVT comparison, oracle/mvt_decode.c)
# ---------------------------------------------------------------------------
def mvt_decode(tile: bytes, with_props: bool = False, cap: int = 1 << 20):
    """Decodes one MVT tile (geometry commands to vertices, ids, types; tags + values with
    with_props).  Returns (status, features, vertices, parts, values, checksum)."""
    arr, p = _u8(tile)
    xy = np.empty(2 * cap, dtype=np.int32)
    o4 = np.zeros(4, dtype=np.int64)
    ck = C.c_uint64(0)
    st = lib().mvt_decode_tile(p, arr.size, int(with_props), xy.ctypes.data_as(C.POINTER(C.c_int32)), cap,
                               o4.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(ck))
    return st, int(o4[0]), int(o4[1]), int(o4[2]), int(o4[3]), ck.value
