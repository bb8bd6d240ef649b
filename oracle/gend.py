"""TEST INFRASTRUCTURE ONLY -- a Gen D COVT writer: the container and stream
encoders of the reference's current converter, restated to produce inputs for the Gen D decode path
(CovtParser.decodeCovt / decodeLayerMetadata, CovtParser.java:53-133, :574-652) and randomised
round-trip tests.  No Gen D fixture exists in the reference.

Restated from evaluation/java/src/main/java/com/covt/converter:
  * layer header + column / stream metadata: CovtConverter.convertLayerMetadata :365-424 and
    convertOptimizedLayerMetadata :300-363, addColumnHeader :471-476, addOptimizedColumnHeader :445-450,
    addOptimizedStreamMetadata :478-483 (u8 streamType << 4 | encoding, varint numValues, byteLength);
    property columns list no PRESENT stream metadata (addNamedColumnMetadata :452-469) although the
    present bytes lead the column payload (convertPropertyColumns :1080-1160);
  * topology streams: convertTopologyStreams :872-897 + addOffsets :899-920 (RLE unless FastPFOR
    zigzag-delta is allowed and not longer);
  * vertex buffers: encodeVertexDictionary :922-937 (zigzag-delta x,y; FastPFOR when shorter),
    Morton codes :939-948 (delta, no zigzag; varint or FastPFOR), vertex offsets :807-813;
  * ids: convertIdColumn :549-569, including its label bug (RLE bytes under VARINT_DELTA_ZIG_ZAG, Q2);
  * properties: encodeBooleans (EncodingUtils.java:213-229), the long-column choice among RLE /
    zigzag-delta varint / zigzag varint (:1087-1110), floats LE, dictionary strings (:1137-1166);
  * EncodingUtils.encodeVarints :39-52 (64-bit LEB128 after delta then zigzag), encodeFastPfor128
    :149-188, encodeZigZagDeltaCoordinates :190-211.
The FastPFOR / ORC writers are the oracle's (oracle/covt_oracle.c).  The converter's MVT reading and
its ICE vertex-dictionary construction are not restated: columns are built from already-decoded
GeometryColumn arrays (e.g. a Gen C fixture decoded by the oracle).
"""
from __future__ import annotations

import numpy as np

from . import decode_morton, encode_byte_rle, encode_fastpfor, encode_rle, encode_varints

# wire enums; Gen D ColumnDataType (converter/ColumnDataType.java)
PLAIN, VARINT, VARINT_ZIG_ZAG, VARINT_DELTA, VARINT_DELTA_ZIG_ZAG, RLE, BOOLEAN_RLE, BYTE_RLE = range(8)
FAST_PFOR_DELTA, FAST_PFOR_DELTA_ZIG_ZAG = 8, 9
PRESENT, DATA, LENGTH, DICTIONARY, GEOMETRY_TYPES, GEOMETRY_OFFSETS, PART_OFFSETS, RING_OFFSETS, \
    VERTEX_OFFSETS, VERTEX_BUFFER = range(10)
DT_BOOLEAN, DT_INT_64, DT_UINT_64, DT_FLOAT, DT_STRING, DT_GEOMETRY = 0, 3, 4, 5, 7, 8
CT_PLAIN, CT_DICTIONARY, CT_ICE, CT_ICE_MORTON = 0, 1, 3, 4
FILE_VERSION = 1


def _zz64(v):
    v = np.asarray(v, dtype=np.int64)
    return ((v << 1) ^ (v >> 63)).astype(np.uint64)


def _zz32(v):
    v = np.asarray(v, dtype=np.int64).astype(np.int32)
    return ((v.astype(np.int64) << 1) ^ (v.astype(np.int64) >> 31)).astype(np.uint32)


def _delta(v):
    v = np.asarray(v, dtype=np.int64)
    return np.diff(v, prepend=0) if v.size else v


def varints(values, zigzag=False, delta=False) -> bytes:
    """EncodingUtils.encodeVarints (64-bit LEB128 after delta, then zigzag)."""
    v = np.asarray(values, dtype=np.int64)
    if delta:
        v = _delta(v)
    return encode_varints(_zz64(v) if zigzag else v.astype(np.uint64))


def fastpfor(values, zigzag=False, delta=False) -> bytes:
    """EncodingUtils.encodeFastPfor128 on int[] (int32 arithmetic)."""
    v = np.asarray(values, dtype=np.int64).astype(np.int32)
    if delta:
        v = (v.astype(np.int64) - np.concatenate([[0], v[:-1].astype(np.int64)])).astype(np.int32) if v.size else v
    u = _zz32(v) if zigzag else v.astype(np.uint32)
    return encode_fastpfor(u)


def string(s: str) -> bytes:
    b = s.encode("utf-8")
    return encode_varints([len(b)]) + b


def booleans(bits) -> bytes:
    """EncodingUtils.encodeBooleans: BitSet bytes (LSB first) padded to ceil(n/8), then byte RLE."""
    bits = np.asarray(bits, dtype=bool)
    packed = np.packbits(bits, bitorder="little") if bits.size else np.zeros(0, np.uint8)
    return encode_byte_rle(packed)


# ---------------------------------------------------------------------------
# columns -> (metadata streams [(type, enc, nv, payload)], dtype, ctype)
# ---------------------------------------------------------------------------
def _offsets(stream_type, counts, allow_fpf):
    counts = np.asarray(counts, dtype=np.int64)
    rle = encode_rle(counts, False)
    if allow_fpf:
        f = fastpfor(counts, zigzag=True, delta=True)
        if len(f) <= len(rle):
            return (stream_type, FAST_PFOR_DELTA_ZIG_ZAG, counts.size, f)
    return (stream_type, RLE, counts.size, rle)


def morton_encode(x, y, num_bits):
    """Inverse of GeometryUtils.decodeMorton (GeometryUtils.java:34-47) on Java ints."""
    hx, hy = decode_morton(0, num_bits)  # decode(0) = (-half, -half)
    ux = (np.asarray(x, dtype=np.int64) - hx).astype(np.uint64)
    uy = (np.asarray(y, dtype=np.int64) - hy).astype(np.uint64)
    code = np.zeros(ux.shape, dtype=np.uint64)
    for i in range(num_bits):
        code |= ((ux >> np.uint64(i)) & np.uint64(1)) << np.uint64(2 * i)
        code |= ((uy >> np.uint64(i)) & np.uint64(1)) << np.uint64(2 * i + 1)
    return code.astype(np.int64)


def geometry_column(types, geometry_offsets=None, part_offsets=None, ring_offsets=None, vertex_offsets=None,
                    vertices=None, column_type=CT_PLAIN, num_bits=13, allow_fpf_topology=True, allow_fpf_vertex=True):
    """GeometryColumn arrays (counts, CovtParser.java:29-36) -> geometry column streams.  vertices: int32
    [n, 2] (PLAIN: in feature order; ICE_MORTON: the vertex dictionary indexed by vertex_offsets)."""
    streams = [(GEOMETRY_TYPES, BYTE_RLE, len(types), encode_byte_rle(np.asarray(types, np.uint8)))]
    for st, arr in ((GEOMETRY_OFFSETS, geometry_offsets), (PART_OFFSETS, part_offsets), (RING_OFFSETS, ring_offsets)):
        if arr is not None and len(arr):
            streams.append(_offsets(st, arr, allow_fpf_topology))
    xy = np.asarray(vertices, dtype=np.int64).reshape(-1, 2)
    if column_type in (CT_ICE, CT_ICE_MORTON):
        vo = np.asarray(vertex_offsets, dtype=np.int64)
        vd = varints(vo, zigzag=True, delta=True)
        vf = fastpfor(vo, zigzag=True, delta=True) if allow_fpf_vertex else None
        if vf is not None and len(vf) <= len(vd):
            streams.append((VERTEX_OFFSETS, FAST_PFOR_DELTA_ZIG_ZAG, vo.size, vf))
        else:
            streams.append((VERTEX_OFFSETS, VARINT_DELTA_ZIG_ZAG, vo.size, vd))
    if column_type == CT_ICE_MORTON:
        codes = morton_encode(xy[:, 0], xy[:, 1], num_bits)
        bd = varints(codes, delta=True)
        bf = fastpfor(codes, delta=True) if allow_fpf_vertex else None
        if bf is not None and len(bf) < len(bd):
            streams.append((VERTEX_BUFFER, FAST_PFOR_DELTA_ZIG_ZAG, xy.shape[0], bf))
        else:
            streams.append((VERTEX_BUFFER, VARINT_DELTA_ZIG_ZAG, xy.shape[0], bd))
    else:
        flat = xy.reshape(-1)
        zd = np.empty(flat.size, dtype=np.int64)  # encodeZigZagDeltaCoordinates (separate x / y sums)
        zd[0::2] = _delta(flat[0::2])
        zd[1::2] = _delta(flat[1::2])
        zdz = _zz32(zd)
        bd = encode_varints(zdz.astype(np.uint64))
        bf = encode_fastpfor(zdz) if allow_fpf_vertex else None
        # ICE: numValues = dictionary vertices although 2 ints each are stored (:779-789); the
        # label follows the bytes actually written (the converter can label varint bytes FastPFOR, :933)
        nv = xy.shape[0] if column_type == CT_ICE else flat.size
        if bf is not None and len(bf) <= len(bd):
            streams.append((VERTEX_BUFFER, FAST_PFOR_DELTA_ZIG_ZAG, nv, bf))
        else:
            streams.append((VERTEX_BUFFER, VARINT_DELTA_ZIG_ZAG, nv, bd))
    return {"name": "geometry", "dtype": DT_GEOMETRY, "ctype": column_type, "streams": streams, "prefix": b""}


def id_column(ids):
    """convertIdColumn (:549-569): the shortest of RLE / delta varint / varint, with the label bug (Q2)."""
    ids = np.asarray(ids, dtype=np.uint64)
    rle = encode_rle(ids.astype(np.int64), False)
    var = encode_varints(ids)
    dvar = varints(ids.astype(np.int64), zigzag=True, delta=True)
    if len(rle) < len(var) and len(rle) < len(dvar):
        s = (DATA, RLE, ids.size, rle)
    elif len(dvar) < len(var):
        s = (DATA, VARINT_DELTA_ZIG_ZAG, ids.size, rle)  # CovtConverter.java:564-566 returns the RLE bytes
    else:
        s = (DATA, VARINT, ids.size, var)
    return {"name": "id", "dtype": DT_UINT_64, "ctype": CT_PLAIN, "streams": [s], "prefix": b""}


def property_column(name, values):
    """One property column from a per-feature value list (None = absent), typed by its values:
    bool -> BOOLEAN, int -> INT_64, float -> FLOAT, str -> STRING (dictionary)."""
    kinds = {type(v) for v in values if v is not None}
    present = np.array([v is not None for v in values], dtype=bool)
    dense = [v for v in values if v is not None]
    if kinds <= {bool} and kinds:
        # convertPropertyColumns :1060-1075: one value per feature, false where absent; no present stream
        data = booleans([bool(v) for v in values])
        return {"name": name, "dtype": DT_BOOLEAN, "ctype": CT_PLAIN, "prefix": b"",
                "streams": [(DATA, BOOLEAN_RLE, len(dense), data)]}
    pre = booleans(present)
    if kinds <= {int}:
        d = np.asarray(dense, dtype=np.int64)
        var = varints(d, zigzag=True)
        dvar = varints(d, zigzag=True, delta=True)
        rle = encode_rle(d, True)
        if len(rle) < len(var) and len(rle) < len(dvar):
            s = (DATA, RLE, d.size, rle)
        elif len(dvar) < len(rle) and len(dvar) < len(var):
            s = (DATA, VARINT_DELTA_ZIG_ZAG, d.size, dvar)
        else:
            s = (DATA, VARINT_ZIG_ZAG, d.size, var)
        return {"name": name, "dtype": DT_INT_64, "ctype": CT_PLAIN, "prefix": pre, "streams": [s]}
    if kinds <= {float, int}:
        f = np.asarray(dense, dtype="<f4").tobytes()
        return {"name": name, "dtype": DT_FLOAT, "ctype": CT_PLAIN, "prefix": pre,
                "streams": [(DATA, PLAIN, len(dense), f)]}
    # strings: dictionary in order of first appearance (convertStringDictionaryColumn :1294-1324)
    dictionary, index = [], {}
    for v in dense:
        if v not in index:
            index[v] = len(dictionary)
            dictionary.append(v)
    idx = np.array([index[v] for v in dense], dtype=np.int64)
    enc = [s.encode("utf-8") for s in dictionary]
    return {"name": name, "dtype": DT_STRING, "ctype": CT_DICTIONARY, "prefix": pre,
            "streams": [(DATA, RLE, idx.size, encode_rle(idx, False)),
                        (LENGTH, RLE, len(enc), encode_rle(np.array([len(b) for b in enc], np.int64), False)),
                        (DICTIONARY, PLAIN, len(enc), b"".join(enc))]}


# ---------------------------------------------------------------------------
# layers and tiles
# ---------------------------------------------------------------------------
def _stream_meta(st, enc, nv, payload):
    return bytes([(st << 4) | enc]) + encode_varints([nv, len(payload)])


def layer(name, extent, n_features, columns, optimized=False, layer_id=0):
    """One Gen D layer: header, column metadata, then the column payloads in column order.  columns[0]
    must be the id or the geometry column (CovtParser.java:66-69)."""
    out = bytearray([(FILE_VERSION << 1) | (1 if optimized else 0)])
    out += encode_varints([layer_id]) if optimized else string(name)
    out += encode_varints([extent, n_features, len(columns)])
    next_id = 2
    for ci, c in enumerate(columns):
        if optimized or ci == 0:  # decodeLayerMetadata reads a column id for column 0 in either mode
            cid = 0 if c["name"] == "id" else 1 if c["name"] == "geometry" else next_id
            if cid >= 2:
                next_id += 1
            out += encode_varints([cid])
        else:
            out += string(c["name"])
        out.append((c["dtype"] << 3) | c["ctype"])
        for st, enc, nv, payload in sorted(c["streams"], key=lambda s: s[0]):  # TreeMap<StreamType>
            out += _stream_meta(st, enc, nv, payload)
    for c in columns:
        out += c["prefix"]
        for st, enc, nv, payload in sorted(c["streams"], key=lambda s: s[0]):
            out += payload
    return bytes(out)


def tile(layers) -> bytes:
    """Gen D tiles have no file header: layers back to back until EOF (CovtParser.java:56)."""
    return b"".join(layers)
