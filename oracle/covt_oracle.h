/*
 * covt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's COVT Id/Geometry stream decode path
 * (springmeyer/cov-tiles, evaluation/java, package com.covt.decoder) and of the
 * third-party arithmetic it calls:
 *   - org.apache.orc:orc-core:1.8.1  RunLengthIntegerReader / RunLengthByteReader
 *     (+ the matching writers, which DecodingUtils.getRleChunkSize uses to find
 *     the stream length, DecodingUtils.java:308-314 -> EncodingUtils.java:123-147)
 *   - me.lemire.integercompression:JavaFastPFOR:0.1.12
 *     Composition(FastPFOR, VariableByte)  (DecodingUtils.java:332,365,427)
 * Neither jar is vendored in the reference; their published algorithms are
 * restated from SURVEY.md Appendix A.3-A.5 and pinned against the reference's
 * committed fixtures (tests/golden, tests/test_oracle_*.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product (cov-tiles_amd/, libcovt.so) never links it.
 *
 * All integer arithmetic follows Java semantics: int32 wraps, `>>>` is a logical
 * shift, shifts are masked to 5 (int) / 6 (long) bits.
 */
#ifndef COVT_ORACLE_H
#define COVT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: identical numbering to include/covt.h */
#define ORC_OK 0
#define ORC_ERR_UNSUPPORTED (-1)
#define ORC_ERR_TRUNCATED (-2)
#define ORC_ERR_COUNT (-3)
#define ORC_ERR_HEADER (-4)
#define ORC_ERR_ARG (-6)

/* ---- DecodingUtils restatement (DecodingUtils.java) ----------------------
 * `avail` = readable bytes of `src` (Java: array length).  pos is the in/out
 * cursor (Java IntWrapper).  Returns a status; on error *pos is unspecified. */
int oracle_decode_varint(const uint8_t* src, size_t avail, int32_t* pos, int32_t n, int32_t* out);                /* :35-44 */
int oracle_decode_zigzag_varint(const uint8_t* src, size_t avail, int32_t* pos, int32_t n, int32_t* out);         /* :46-53 */
int oracle_decode_zigzag_delta_varint(const uint8_t* src, size_t avail, int32_t* pos, int32_t n, int32_t* out);   /* :55-66 */
int oracle_decode_zigzag_delta_varint_coordinates(const uint8_t* src, size_t avail, int32_t* pos, int32_t n,
                                                  int32_t* out);                                                  /* :95-112 */
/* decodeRle :257-272.  *pos advances by the length of the ORC writer's re-encoding of
 * the decoded values (Java behaviour, :268-270); *consumed (optional) receives the bytes
 * the reader actually consumed. */
int oracle_decode_rle(const uint8_t* src, size_t avail, int32_t n, int32_t* pos, int is_signed, int64_t* out,
                      int32_t* consumed);
/* decodeByteRle(buffer, n, pos, byteLength) :275-288 (advance by byteLength) */
int oracle_decode_byte_rle(const uint8_t* src, size_t avail, int32_t n, int32_t* pos, int32_t byte_length,
                           uint8_t* out, int32_t* consumed);
/* decodeFastPfor128ZigZagDelta :316-347 */
int oracle_decode_fastpfor_zigzag_delta(const uint8_t* src, size_t avail, int32_t n, int32_t byte_length,
                                        int32_t* pos, int32_t* out);
/* decodeFastPfor128DeltaCoordinates :349-392 */
int oracle_decode_fastpfor_delta_coordinates(const uint8_t* src, size_t avail, int32_t n, int32_t byte_length,
                                             int32_t* pos, int32_t* out);
/* decodeDeltaVarintMortonCodes :394-409 (out has 2*n ints) */
int oracle_decode_delta_varint_morton_codes(const uint8_t* src, size_t avail, int32_t* pos, int32_t n_vertices,
                                            int32_t num_bits, int32_t* out);
/* decodeFastPfor128DeltaMortonCodes :411-444 (out has 2*n ints) */
int oracle_decode_fastpfor_delta_morton_codes(const uint8_t* src, size_t avail, int32_t n_vertices,
                                              int32_t byte_length, int32_t* pos, int32_t num_bits, int32_t* out);
/* GeometryUtils.decodeMorton, GeometryUtils.java:34-47 */
void oracle_decode_morton(int32_t code, int32_t num_bits, int32_t* x, int32_t* y);

/* Raw Composition(FastPFOR, VariableByte).uncompress of byteLength bytes at pos (BE words,
 * DecodingUtils.java:317-333).  Writes n raw values (zero-filled past the decoded count);
 * *decoded receives how many values the codec produced. */
int oracle_fastpfor_uncompress(const uint8_t* src, size_t avail, int32_t pos, int32_t byte_length, int32_t n,
                               uint32_t* raw, int32_t* decoded);

/* Full 64-bit LEB128 (format truth for Id VARINT streams). */
int oracle_decode_varint_u64(const uint8_t* src, size_t avail, int32_t* pos, int32_t n, uint64_t* out);

/* ---- encoders (EncodingUtils.java:39-230 + orc/JavaFastPFOR writers) -------
 * Used to build synthetic streams for round-trip tests.  Return bytes written
 * (or a negative status if cap is too small). */
int64_t oracle_encode_varints_u64(const uint64_t* v, int64_t n, uint8_t* dst, int64_t cap);
int64_t oracle_encode_rle(const int64_t* v, int64_t n, int is_signed, uint8_t* dst, int64_t cap);
int64_t oracle_encode_byte_rle(const uint8_t* v, int64_t n, uint8_t* dst, int64_t cap);
/* FastPFOR(256-blocks, 65536-pages) + VariableByte tail, emitted as BE bytes like
 * EncodingUtils.encodeFastPfor128 (:149-188) without the delta/zigzag pre-pass. */
int64_t oracle_encode_fastpfor(const uint32_t* v, int64_t n, uint8_t* dst, int64_t cap);

/* ---- container walkers (Gen C: SURVEY Appendix A.1; Gen D: CovtParser.java:574-652) ---- */
#define ORACLE_FMT_GENC 0
#define ORACLE_FMT_GEND 1

typedef struct oracle_stream {
    int32_t layer;        /* layer index within the tile */
    int32_t column_kind;  /* 0 = id column, 1 = geometry column */
    int32_t stream_type;  /* StreamType ordinal (DATA=1 for id) */
    int32_t encoding;     /* StreamEncoding ordinal */
    int32_t column_type;  /* ColumnType ordinal */
    int32_t num_values;   /* wire numValues */
    int32_t byte_length;  /* wire byteLength */
    int32_t num_bits;     /* 32 - nlz(extent), CovtParser.java:77 */
    int64_t offset;       /* payload byte offset within the tile */
    int32_t extent;
    int32_t num_features;
} oracle_stream;

/* Walk one tile; returns status, *n_out = number of Id/Geometry streams found
 * (property columns are skipped by their byte lengths).  max_out may be 0 to count. */
int oracle_walk_tile(const uint8_t* tile, size_t len, int format, oracle_stream* out, int32_t max_out,
                     int32_t* n_out);

/* Id column decode modes */
#define ORACLE_ID_FORMAT 0 /* format truth: VARINT -> 64-bit LEB128, enc 4 -> unsigned RLE */
#define ORACLE_ID_JAVA 1   /* CovtParser.decodedIds verbatim (4-byte varint cap, enc 4 zigzag-delta) */

/* Byte length of the implicit present stream of a Gen D property column starting at tile offset off
 * (Java: re-encoding length of its ceil(n/8) decoded bytes). */
int oracle_gend_present_length(const uint8_t* tile, size_t len, int64_t off, int32_t n_features, int32_t* length);

/* Output element type/count of a stream's decode (1,4,8 bytes) */
int oracle_stream_output(const oracle_stream* s, int id_mode, int32_t* elem_bytes, int64_t* n_elems);
/* Decode one walked stream with CovtParser's dispatch (decodeGeometryColumn :392-511,
 * decodedIds :552-572).  RLE/varint reads are bounded by the stream's byteLength.
 * out must hold n_elems * elem_bytes; *consumed receives bytes consumed. */
int oracle_decode_stream(const uint8_t* tile, size_t len, const oracle_stream* s, int id_mode, void* out,
                         int32_t* consumed);

/* CovtParser.convertGeometryColumn (CovtParser.java:135-274) restated into the nested-offset
 * layout of include/covt.h ("Geometry assembly"): geo_off[n+1], part_off[parts+1],
 * ring_off[rings+1], coords[2*coords].  Count streams may be NULL (absent); vo == NULL means a
 * PLAIN column (vertices read in order), else ICE (vb[2*vo[i]]).  n_vb counts vertices.
 * Deviations from Java (documented in include/covt.h): MULTIPOLYGON without the SURVEY Q7 bugs,
 * MULTIPOINT = geometryOffsets count of points, rings closed once (closed_in_stream: the stream
 * already holds the closing vertex).  Returns 0, ORC_ERR_HEADER (type > 5),
 * ORC_ERR_COUNT (a count stream over-read, a negative count, a capacity exceeded) or
 * ORC_ERR_TRUNCATED (a vertex index outside the vertex buffer). */
int oracle_assemble_geometry(const uint8_t* types, int32_t n, const int32_t* go, int32_t n_go, const int32_t* po,
                             int32_t n_po, const int32_t* ro, int32_t n_ro, const int32_t* vo, int32_t n_vo,
                             const int32_t* vb, int32_t n_vb, int closed_in_stream, int32_t part_cap,
                             int32_t ring_cap, int32_t coord_cap, int32_t* geo_off, int32_t* part_off,
                             int32_t* ring_off, int32_t* coords, int32_t* n_parts, int32_t* n_rings,
                             int32_t* n_coords);

/* ---- property columns (covt_oracle_props.c; CovtParser.decodePropertyColumn :276-354) ----
 * One record per property (sub)column: Gen C LOCALIZED_DICTIONARY columns yield one per language
 * (lang >= 0, sharing the column's length/dictionary streams).  Streams by role:
 * 0 present, 1 data, 2 length, 3 dictionary (s_off = tile-relative payload offset, -1 absent). */
#define ORACLE_PROP_BOOLEAN 0
#define ORACLE_PROP_INT64 1
#define ORACLE_PROP_FLOAT 2
#define ORACLE_PROP_STRING 3
typedef struct oracle_prop {
    int32_t layer, column, type, column_type; /* type: ORACLE_PROP_* or -1 (unsupported data type) */
    int32_t n_features, lang, name_len, lang_len;
    int64_t name_off, lang_off;               /* UTF-8 names inside the tile (-1: none) */
    int64_t s_off[4];
    int32_t s_nv[4], s_bl[4], s_enc[4];
} oracle_prop;
int oracle_walk_properties(const uint8_t* tile, size_t len, int format, oracle_prop* out, int32_t max_out,
                           int32_t* n_out);
/* Output byte sizes: validity, values, dictionary offsets, dictionary bytes */
void oracle_property_sizes(const oracle_prop* p, int64_t sizes[4]);
/* Decode one property (sub)column into the Arrow-style layout of include/covt.h: validity bitmap
 * (LSB first, bits >= n clear), values at feature positions (BOOLEAN: bitmap; INT64: int64;
 * FLOAT: float32 bits; STRING: int32 dictionary index; absent slots 0), dictionary offsets
 * [n_dict + 1] and bytes.  mode: ORACLE_ID_FORMAT (64-bit varints) / ORACLE_ID_JAVA (4-byte cap). */
int oracle_decode_property(const uint8_t* tile, size_t len, const oracle_prop* p, int mode, uint8_t* validity,
                           void* values, int32_t* dict_offsets, uint8_t* dict_bytes, int32_t* n_valid);

/* CPU baseline: walk + decode every Id/Geometry stream of n_tiles tiles (concatenated in
 * `bytes` at `offsets`) on n_threads host threads; output goes to per-thread scratch.
 * Returns status; totals (optional) receive stream bytes, output bytes, vertices. */
int oracle_decode_tiles_mt(const uint8_t* bytes, const uint64_t* offsets, const uint64_t* sizes, int32_t n_tiles,
                           int format, int id_mode, int32_t n_threads, int64_t* in_bytes, int64_t* out_bytes,
                           int64_t* vertices);

/* BASELINE configs[0]: one whole tile as CovtParser.decodeCovt decodes it, single-threaded: walk, every
 * Id / Geometry stream, every geometry column assembled, every property column (covt_oracle_tile.c).
 * counts (optional): streams, vertices, assembled coordinates, property columns. */
int oracle_decode_tile_full(const uint8_t* tile, size_t len, int format, int id_mode, int64_t counts[4]);

#ifdef __cplusplus
}
#endif
#endif
