/*
 * covt.h -- C-ABI of libcovt, the MI355X (gfx950) COVT Id/Geometry stream decoder.
 *
 * Drop-in boundary for the reference's Java decoder API (springmeyer/cov-tiles,
 * evaluation/java, package com.covt.decoder).  Each stream-level entry point
 * replaces one `public static` method of DecodingUtils.java with the same
 * argument order and meaning; the Java `IntWrapper pos` becomes an int32_t*
 * in/out cursor, `byte[]` inputs gain an explicit length, and outputs are
 * caller-provided arrays (the Java methods allocate theirs).  Decoding runs on
 * the GPU in every case: there is no CPU fallback.  A JNI shim
 * (cov-tiles_amd/jni/covt_jni.cc) binds these to
 * com.covt.decoder.gpu.GpuDecodingUtils; see INTEGRATION.md.
 *
 * Status codes map onto the Java exceptions of the reference:
 *   COVT_ERR_UNSUPPORTED_ENCODING -> IllegalArgumentException (CovtParser.java:426,443,460,475,493,508,571)
 *   COVT_ERR_TRUNCATED            -> ArrayIndexOutOfBoundsException / EOFException (ORC readers)
 *   COVT_ERR_COUNT_MISMATCH       -> ArrayIndexOutOfBoundsException (output overrun)
 *   COVT_ERR_BAD_HEADER           -> IllegalArgumentException (malformed FastPFOR / container)
 */
#ifndef COVT_H
#define COVT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COVT_OK 0
#define COVT_ERR_UNSUPPORTED_ENCODING (-1)
#define COVT_ERR_TRUNCATED (-2)
#define COVT_ERR_COUNT_MISMATCH (-3)
#define COVT_ERR_BAD_HEADER (-4)
#define COVT_ERR_DEVICE (-5)
#define COVT_ERR_INVALID_ARG (-6)

/* Device input buffers handed to the *_device entry points must start 16-byte aligned
 * and stay readable for COVT_INPUT_PADDING bytes past the last stream byte. */
#define COVT_INPUT_PADDING 4096

/* Container generations */
#define COVT_FORMAT_GENC 0 /* every committed fixture (test/fixtures/NAME/covt) */
#define COVT_FORMAT_GEND 1 /* what CovtParser.decodeCovt reads, CovtParser.java:574-652 */

/* Id column decode modes */
#define COVT_ID_FORMAT 0 /* format truth: VARINT = 64-bit LEB128, enc 4 = unsigned RLE */
#define COVT_ID_JAVA 1   /* CovtParser.decodedIds verbatim: 4-byte varint cap, enc 4 = zigzag-delta */

/* ---------------------------------------------------------------------------
 * Stream-level API: one function per DecodingUtils method.
 * `buf`/`buf_len` is the Java byte[]; *pos is the IntWrapper.  Host memory in and out.
 * ------------------------------------------------------------------------- */
/* DecodingUtils.decodeVarint(byte[] src, IntWrapper pos, int numValues)          DecodingUtils.java:35 */
int covt_decode_varint(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t num_values, int32_t* out);
/* DecodingUtils.decodeZigZagVarint(byte[], IntWrapper, int)                       DecodingUtils.java:46 */
int covt_decode_zigzag_varint(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t num_values, int32_t* out);
/* DecodingUtils.decodeZigZagDeltaVarint(byte[], IntWrapper, int)                  DecodingUtils.java:55 */
int covt_decode_zigzag_delta_varint(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t num_values,
                                    int32_t* out);
/* DecodingUtils.decodeZigZagDeltaVarintCoordinates(byte[], IntWrapper, int)       DecodingUtils.java:95 */
int covt_decode_zigzag_delta_varint_coordinates(const uint8_t* buf, size_t buf_len, int32_t* pos,
                                                int32_t num_values, int32_t* out);
/* DecodingUtils.decodeRle(byte[], int numValues, IntWrapper, boolean signed)      DecodingUtils.java:257
 * *pos advances by the bytes the RLE reader consumed; for ORC-writer-produced streams this equals
 * the Java advance (the length of the re-encoding, :268-270, :308-310). */
int covt_decode_rle(const uint8_t* buf, size_t buf_len, int32_t num_values, int32_t* pos, int32_t is_signed,
                    int64_t* out);
/* DecodingUtils.decodeByteRle(byte[], int numValues, IntWrapper, int byteLength)  DecodingUtils.java:275 */
int covt_decode_byte_rle(const uint8_t* buf, size_t buf_len, int32_t num_values, int32_t* pos, int32_t byte_length,
                         uint8_t* out);
/* DecodingUtils.decodeByteRle(byte[], int numValues, IntWrapper)                  DecodingUtils.java:290
 * (the form CovtParser.java:295 uses for Gen D present streams): *pos advances by the length of the
 * ORC RunLengthByteWriter re-encoding of the decoded values (getByteRleChunkSize :312-314). */
int covt_decode_byte_rle_reencode(const uint8_t* buf, size_t buf_len, int32_t num_values, int32_t* pos,
                                  uint8_t* out);
/* DecodingUtils.decodeFloatsLE(byte[], IntWrapper, int numValues)                 DecodingUtils.java:446
 * numValues little-endian floats copied out (host memory; no decode arithmetic). */
int covt_decode_floats_le(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t num_values, float* out);
/* DecodingUtils.decodeString(byte[], IntWrapper)                                  DecodingUtils.java:21
 * Reads the 4-byte-capped varint length and returns where the UTF-8 bytes lie (*str_off, *str_len);
 * *pos advances past them.  The JNI shim builds the java.lang.String from them. */
int covt_decode_string(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t* str_off, int32_t* str_len);
/* DecodingUtils.decodeFastPfor128ZigZagDelta(byte[], int, int byteLength, IntWrapper) DecodingUtils.java:316 */
int covt_decode_fastpfor_zigzag_delta(const uint8_t* buf, size_t buf_len, int32_t num_values, int32_t byte_length,
                                      int32_t* pos, int32_t* out);
/* DecodingUtils.decodeFastPfor128DeltaCoordinates(byte[], int, int, IntWrapper)   DecodingUtils.java:349 */
int covt_decode_fastpfor_delta_coordinates(const uint8_t* buf, size_t buf_len, int32_t num_values,
                                           int32_t byte_length, int32_t* pos, int32_t* out);
/* DecodingUtils.decodeDeltaVarintMortonCodes(byte[], IntWrapper, int numVertices, int numBits)
 *                                                                                 DecodingUtils.java:394
 * out holds 2*num_vertices ints (x,y interleaved). */
int covt_decode_delta_varint_morton_codes(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t num_vertices,
                                          int32_t num_bits, int32_t* out);
/* DecodingUtils.decodeFastPfor128DeltaMortonCodes(byte[], int, int, IntWrapper, int numBits)
 *                                                                                 DecodingUtils.java:411 */
int covt_decode_fastpfor_delta_morton_codes(const uint8_t* buf, size_t buf_len, int32_t num_vertices,
                                            int32_t byte_length, int32_t* pos, int32_t num_bits, int32_t* out);

/* ---------------------------------------------------------------------------
 * Batch API: the replacement for the per-tile CovtParser.decodeCovt loop
 * (CovtParser.java:53-133) restricted to the Id and Geometry columns.
 * ------------------------------------------------------------------------- */

/* Device-side decode operations (one per DecodingUtils codec x output type). */
enum covt_op {
    COVT_OP_NONE = 0,
    COVT_OP_BYTE_RLE_U8 = 1,            /* decodeByteRle -> uint8 (GeometryTypes, values <= 5 checked) */
    COVT_OP_RLE_U64 = 2,                /* decodeRle(signed=false) -> int64 (Id) */
    COVT_OP_RLE_I32 = 3,                /* decodeRle(signed=false) then (int) -> int32 (topology counts) */
    COVT_OP_RLE_S64 = 4,                /* decodeRle(signed=true) -> int64 */
    COVT_OP_VARINT_I32 = 5,             /* decodeVarint -> int32 */
    COVT_OP_VARINT_ZZ_I32 = 6,          /* decodeZigZagVarint -> int32 */
    COVT_OP_VARINT_ZZ_DELTA_I32 = 7,    /* decodeZigZagDeltaVarint -> int32 (VertexOffsets) */
    COVT_OP_VARINT_ZZ_DELTA_XY = 8,     /* decodeZigZagDeltaVarintCoordinates -> int32 x,y */
    COVT_OP_VARINT_DELTA_MORTON = 9,    /* decodeDeltaVarintMortonCodes -> int32 x,y per vertex */
    COVT_OP_FPF_ZZ_DELTA_I32 = 10,      /* decodeFastPfor128ZigZagDelta -> int32 */
    COVT_OP_FPF_ZZ_DELTA_XY = 11,       /* decodeFastPfor128DeltaCoordinates -> int32 x,y */
    COVT_OP_FPF_DELTA_MORTON = 12,      /* decodeFastPfor128DeltaMortonCodes -> int32 x,y per vertex */
    COVT_OP_VARINT_U64 = 13,            /* Id VARINT, format truth: 64-bit LEB128 -> int64 */
    COVT_OP_VARINT_I32_AS_I64 = 14,     /* Id VARINT, Java: decodeVarint then (long) */
    COVT_OP_VARINT_ZZ_DELTA_I64 = 15,   /* Id enc 4, Java: decodeZigZagDeltaVarint then (long) */
    COVT_OP_BYTE_RLE_RAW = 16,          /* decodeByteRle -> uint8, no value check (present / boolean bitsets) */
    COVT_OP_VARINT_ZZ_I32_AS_I64 = 17,  /* INT_64 VARINT_ZIG_ZAG, Java: decodeZigZagVarint then (long)
                                           (CovtParser.java:304-307) */
    COVT_OP_VARINT_ZZ_S64 = 18,         /* INT_64 VARINT_ZIG_ZAG, format truth: 64-bit LEB128, zigzag64 */
    COVT_OP_VARINT_ZZ_DELTA_S64 = 19,   /* INT_64 VARINT_DELTA_ZIG_ZAG, format truth: 64-bit, int64 running sum */
    COVT_OP_COUNT = 20
};

/* Codec families: each has its own kernel (register / LDS footprint), launched concurrently. */
#define COVT_FAMILY_RLE 0      /* byte RLE, integer RLE (and COVT_OP_NONE -> unsupported) */
#define COVT_FAMILY_VARINT 1   /* varint / zigzag / delta / Morton ops */
#define COVT_FAMILY_FASTPFOR 2 /* FastPFOR + VariableByte ops */
#define COVT_FAMILY_LANE 3     /* small RLE streams (flag COVT_DESC_LANE): one lane per stream */
#define COVT_FAMILY_SPLIT 4    /* long varint streams cut into chunks decoded by separate waves (COVT_DESC_SPLIT) */
#define COVT_FAMILY_SPLIT_FPF 5 /* long FastPFOR streams cut into chunks (COVT_DESC_SPLIT | COVT_DESC_SPLIT_FPF) */
#define COVT_FAMILY_SPLIT_RLE 6 /* long ORC RLE streams cut at group starts (COVT_DESC_SPLIT | COVT_DESC_SPLIT_RLE) */
#define COVT_NUM_FAMILIES 7

/* covt_stream_desc.flags */
#define COVT_DESC_LANE 0x1u /* decoded by the lane-per-stream kernel (set by the plan for small streams) */
/* Long streams (plan rule: varint ops -- Java-capped and 64-bit LEB128 -- and FastPFOR ops whose cost, bytes
 * + output bytes / 4, exceeds COVT_SPLIT_MIN and the plan's total / COVT_SPLIT_RATIO) are
 * cut into chunks of COVT_SPLIT_CHUNK bytes (varint) or COVT_SPLIT_VALUES values (FastPFOR, whole
 * blocks), each decoded by its own wave; a chunk's value index and running
 * sums come from its predecessors by a decoupled look-back.  A chunk is COVT_SPLIT_SLOTS consecutive
 * descriptors: the chunk descriptor (flags COVT_DESC_SPLIT, avail = chunk index, the other fields those
 * of the stream) and pads (COVT_DESC_SPLIT_PAD; the first carries the chunk's range [in_off, out_off):
 * stream-relative bytes, or values for FastPFOR), whose result entries hold the look-back records.  The stream's result is
 * written to its chunk 0's entry.  Split descriptors need the grouped launch. */
#define COVT_DESC_SPLIT 0x2u
#define COVT_DESC_SPLIT_PAD 0x4u
#define COVT_DESC_SPLIT_FPF 0x8u /* with SPLIT / SPLIT_PAD: a FastPFOR stream's chunk (pads [2..7]: the plan's
                                  * host walk of the headers before it -- int32 slots in every field but
                                  * op / num_bits / flags; all zero = none, the chunk walks them itself) */
#define COVT_DESC_SPLIT_RLE 0x10u /* with SPLIT / SPLIT_PAD: an ORC RLE stream's chunk (whole groups, located by the
                                   * plan; pads [1] bytes [s, e), [2] values (first, count), [3] consumed) */
#define COVT_SPLIT_SLOTS 8
#define COVT_SPLIT_CHUNK 2048 /* default varint / RLE chunk bytes (covt_plan_options.split_chunk) */
#define COVT_SPLIT_VALUES 2048 /* default FastPFOR chunk values, whole blocks (covt_plan_options.split_values) */
#define COVT_SPLIT_MIN 8192   /* default: streams costlier than this are split (covt_plan_options.split_min) */
#define COVT_SPLIT_RATIO 3000 /* ... and than the plan's total cost / this (covt_plan_options.split_ratio) */
#define COVT_LANE_MAX_BYTES 128     /* covt_plan_options.lane_max_bytes 0 (auto): Id / Geometry plans */
#define COVT_LANE_MAX_BYTES_PROPS 512 /* ... plans with COVT_PLAN_PROPERTIES */
#define COVT_LANE_MAX_VALUES 256    /* covt_plan_options.lane_max_values 0 (auto): Id / Geometry plans */
#define COVT_LANE_MAX_VALUES_PROPS 512 /* ... plans with COVT_PLAN_PROPERTIES */
#define COVT_LANE_MIN_STREAMS 65536 /* default covt_plan_options.lane_min_streams */
#define COVT_SPLIT_MAX_STREAMS 65536 /* default covt_plan_options.split_max_streams */

/* Plan-layout options.  Every plan property that used to be steered by the environment is a field
 * here: a library inside a JVM or tile server plans the same way whatever its process inherited.
 * Initialise with covt_plan_options_init (the defaults below), change fields, pass to
 * covt_plan_create_opts / covt_device_plan_create_opts.  Plans made with equal options from equal
 * tiles are byte-identical, host or device. */
typedef struct covt_plan_options {
    uint32_t size;             /* sizeof(covt_plan_options), set by covt_plan_options_init */
    uint32_t flags;            /* COVT_PLAN_PROPERTIES (host plans only) */
    int64_t split_min;         /* split streams whose cost (bytes + output bytes / 4) exceeds this and ... */
    int64_t split_ratio;       /* ... the plan's total cost / split_ratio (0: no batch-relative bound);
                                  split_min < 0: never split */
    int64_t split_chunk;       /* bytes of cost per varint / RLE chunk (>= 64) */
    int64_t split_values;      /* values per FastPFOR chunk (a multiple of 256, >= 256) */
    int32_t fpf_split_weight;  /* a FastPFOR stream's output counted this many times in its split cost (>= 1) */
    int32_t lane_max_bytes;    /* RLE streams of <= this many bytes (<= 65535; 0: auto, COVT_LANE_MAX_BYTES or
                                  _PROPS with property columns) and <= lane_max_values values go to the lane family ... */
    int64_t lane_min_streams;  /* ... when the plan holds at least this many of them (lane_max_bytes < 0: never) */
    int32_t plan_threads;      /* host threads of covt_plan_create (0: min(hardware threads, 16)) */
    int32_t host_prefault;     /* decode_host into pageable memory: fault the output pages in on host threads
                                  while the device works (1, default) or not (0) */
    int32_t prefault_threads;  /* those threads (default 8) */
    int32_t device_walk;       /* covt_device_plan: 0 = a wave per tile with per-tile slots (default),
                                  1 = the same walk twice (no slots), k >= 2: k tiles per workgroup, a lane each */
    int32_t lane_max_values;   /* the lane family's value limit (<= 32767; 0: auto, COVT_LANE_MAX_VALUES or _PROPS with
                                  property columns, whose many small dictionary-index streams favour longer lanes) */
    int64_t split_max_streams; /* plans of more streams than this split nothing (0: no bound).  Enough streams keep
                                  every wave slot busy, and there the chunks' header re-walks and look-back cost
                                  more than the long poles they shorten */
    int32_t split_grow;        /* 1 (default): split_chunk / split_values doubled for plans of >= 4 MiB of cost and
                                  quadrupled from 48 MiB (covt_internal.h split_grow_factor); 0: fixed */
} covt_plan_options;
void covt_plan_options_init(covt_plan_options* opts);

/* One device-resident plan entry (32 bytes). */
typedef struct covt_stream_desc {
    uint64_t in_off;     /* payload byte offset in the batch input buffer */
    uint64_t out_off;    /* output byte offset in the batch output buffer (plans: 128-byte aligned) */
    int32_t avail;       /* readable payload bytes (byteLength for plans; buf_len-pos for stream calls) */
    int32_t num_values;  /* values (vertices for the Morton ops) to produce */
    uint8_t op;          /* enum covt_op */
    uint8_t num_bits;    /* Morton bits, 32 - nlz(extent) (CovtParser.java:77) */
    uint16_t flags;      /* COVT_DESC_* */
    int32_t byte_length; /* wire byteLength (FastPFOR reads byteLength/4 big-endian words) */
} covt_stream_desc;

/* Per-stream result written by the kernel. */
typedef struct covt_stream_result {
    int32_t status;   /* COVT_OK or a negative COVT_ERR_* */
    int32_t consumed; /* payload bytes consumed (FastPFOR / byte RLE: byteLength) */
} covt_stream_result;

/* Host-visible stream record of a plan, in tile order. */
typedef struct covt_stream_info {
    int32_t tile, layer, column_kind, stream_type; /* column_kind: 0 id, 1 geometry */
    int32_t encoding, column_type, num_values, byte_length;
    int32_t num_bits, op, elem_bytes, desc_index; /* desc_index: row in the launch-ordered descs */
    int64_t in_off, out_off, out_elems;
} covt_stream_info;

typedef struct covt_plan covt_plan;

/* Walk the container metadata of n_tiles tiles held back to back in `bytes` (host memory) and
 * build the descriptor table.  Tiles that fail to walk get a negative tile status and no streams. */
int covt_plan_create(const uint8_t* bytes, const uint64_t* tile_offsets, const uint64_t* tile_sizes,
                     int32_t n_tiles, int32_t format, int32_t id_mode, covt_plan** out);
void covt_plan_destroy(covt_plan* plan);
int64_t covt_plan_num_streams(const covt_plan* plan);
int64_t covt_plan_output_bytes(const covt_plan* plan);
/* stream-byte, output-byte and vertex totals over all planned streams */
int covt_plan_totals(const covt_plan* plan, int64_t* in_bytes, int64_t* out_bytes, int64_t* vertices);
int covt_plan_streams(const covt_plan* plan, covt_stream_info* out);    /* num_streams records */
int64_t covt_plan_num_descs(const covt_plan* plan);  /* descriptors (>= streams: split chunks and pads) */
int covt_plan_descs(const covt_plan* plan, covt_stream_desc* out);      /* num_descs, launch order */
/* plan-order stream index of every descriptor (launch order); a stream's result is at its
 * covt_stream_info.desc_index */
int covt_plan_desc_streams(const covt_plan* plan, int64_t* out);
/* Launch order groups descriptors by family (RLE, varint, FastPFOR, lane; largest stream first inside
 * a family, the lane family also by op): counts[f] = descriptors of family f. */
int covt_plan_family_counts(const covt_plan* plan, int64_t counts[COVT_NUM_FAMILIES]);
int covt_plan_tile_status(const covt_plan* plan, int32_t* out);         /* n_tiles */

/* Launch the decode of n_streams descriptors on `hip_stream` (a hipStream_t; NULL = default).
 * d_in: batch bytes on the device (see COVT_INPUT_PADDING); d_desc: descriptors on the device;
 * d_out: output buffer of covt_plan_output_bytes bytes; d_res: n_streams results.  Asynchronous.
 * Split descriptors (COVT_DESC_SPLIT / _PAD) are skipped here: they need the grouped launch. */
int covt_decode_streams_device(const uint8_t* d_in, const covt_stream_desc* d_desc, int64_t n_streams,
                               uint8_t* d_out, covt_stream_result* d_res, void* hip_stream);

/* Same, for descriptors grouped by family (as covt_plan_descs returns them): the family kernels run
 * concurrently on forked streams joined back into `hip_stream`.  d_res holds one entry per
 * descriptor (covt_plan_num_descs); results are at the streams' desc_index entries. */
int covt_decode_streams_device_grouped(const uint8_t* d_in, const covt_stream_desc* d_desc,
                                       const int64_t family_counts[COVT_NUM_FAMILIES], uint8_t* d_out,
                                       covt_stream_result* d_res, void* hip_stream);
/* The same launch with its shape chosen by the caller: COVT_LAUNCH_AUTO (what the call above does: one
 * fused kernel for batches of at most 4096 waves, else the per-family kernels on forked streams),
 * COVT_LAUNCH_FUSED or COVT_LAUNCH_FORKED whatever the batch size (tests pin both code paths; outputs
 * and results are identical). */
#define COVT_LAUNCH_AUTO 0
#define COVT_LAUNCH_FUSED 1
#define COVT_LAUNCH_FORKED 2
/* or-ed into launch_mode: the FastPFOR family's kernel variant in a forked launch.  By default (neither) a
 * family of at least 65,536 streams takes the streamed variant (packed words through an LDS ring, block
 * headers 64 at a time, a batch's exception words gathered at once: the shorter launch for large batches) and
 * smaller ones the per-block pipeline (shorter for strong-scaling shards); both give identical results. */
#define COVT_LAUNCH_FPF_STREAM 0x4
#define COVT_LAUNCH_FPF_CLASSIC 0x8
int covt_decode_streams_device_grouped_mode(const uint8_t* d_in, const covt_stream_desc* d_desc,
                                            const int64_t family_counts[COVT_NUM_FAMILIES], uint8_t* d_out,
                                            covt_stream_result* d_res, void* hip_stream, int32_t launch_mode);

/* Host entry point: H2D + decode + D2H for host tiles on the current device.
 * bytes/n_bytes: the caller's buffer the plan's tile offsets index (every tile must lie inside
 * [0, n_bytes), else COVT_ERR_INVALID_ARG); host_out: covt_plan_output_bytes(plan) bytes, stream i's
 * values at covt_stream_info.out_off; host_res: num_streams results (plan stream order).  Bytes of
 * host_out outside the stream slices (16-byte alignment padding) are unspecified.
 * Device buffers and the descriptor table stay cached on the plan across calls (released by
 * covt_plan_release_device or covt_plan_destroy); calls on one plan are serialised. */
int covt_plan_decode_host(const covt_plan* plan, const uint8_t* bytes, uint64_t n_bytes, uint8_t* host_out,
                          covt_stream_result* host_res);

/* Multi-GPU host entry point: shards the plan's tiles over min(n_gpus, devices) devices (contiguous
 * tile ranges balanced on stream + output bytes, one host thread per device, no collectives); each
 * shard is one H2D, one launch and one D2H into its part of host_out.  Same results as
 * covt_plan_decode_host. */
int covt_plan_decode_host_multi(const covt_plan* plan, const uint8_t* bytes, uint64_t n_bytes, int32_t n_gpus,
                                uint8_t* host_out, covt_stream_result* host_res);

/* The same with an explicit shard -> device map: n_shards shards, shard k on device shard_devices[k]
 * (devices may repeat: several shards of one device run concurrently on their own streams). */
int covt_plan_decode_host_shards(const covt_plan* plan, const uint8_t* bytes, uint64_t n_bytes, int32_t n_shards,
                                 const int32_t* shard_devices, uint8_t* host_out, covt_stream_result* host_res);

/* Free the device buffers the host entry points cached on this plan. */
int covt_plan_release_device(const covt_plan* plan);

/* ---------------------------------------------------------------------------
 * Geometry assembly: the GPU replacement for
 * CovtParser.convertGeometryColumn (CovtParser.java:135-274, getLineString / getLinearRing /
 * getICELineString :513-550).  Java builds one JTS Geometry per feature out of the decoded
 * GeometryColumn; here every geometry column of a plan becomes one GeoArrow-style nested-offset
 * record, computed on the device from the decoded streams (prefix sums of the count streams,
 * ICE vertex gather):
 *
 *   geometry_offsets[n_features + 1]  feature -> parts    (POINT/LINESTRING/POLYGON: 1 part,
 *                                                          MULTI*: geometryOffsets count)
 *   part_offsets[num_parts + 1]       part -> rings       (POLYGON parts: partOffsets count,
 *                                                          point / line parts: 1 ring)
 *   ring_offsets[num_rings + 1]       ring -> coordinates (point: 1, line: partOffsets count,
 *                                                          polygon ring: ringOffsets count, closed)
 *   coords[2 * num_coords]            int32 x,y (ICE: vertexBuffer[2*vertexOffsets[i]], +0/+1)
 *
 * Offsets are absolute within the column and start at 0; types[] of the decoded GeometryTypes
 * stream says how to read a feature.  Polygon rings are closed as JTS LinearRings are
 * (getLinearRing appends the first vertex): a ring whose stream omits the closing vertex gets it
 * appended; Gen C ICE rings already carry it and are copied as they are.
 * Deviations from the Java method, decided for format truth: the MULTIPOLYGON bugs of SURVEY Q7
 * (CovtParser.java:237-259) are not reproduced, and MULTIPOINT (which Java rejects with
 * IllegalArgumentException) reads one geometryOffsets count of points.
 * ------------------------------------------------------------------------- */
#define COVT_GEOM_CLOSED_IN_STREAM 0x1u /* polygon rings carry their closing vertex in the stream */
#define COVT_GEOM_TOO_LARGE 0x80000000u /* over COVT_GEOM_MAX_CAP: not assembled (COVT_ERR_INVALID_ARG) */

/* One device-resident geometry-column entry (160 bytes). */
typedef struct covt_geom_desc {
    int64_t in_off[6];   /* decode-output byte offsets of the GeometryTypes, GeometryOffsets, PartOffsets,
                            RingOffsets, VertexOffsets, VertexBuffer arrays (-1: stream absent) */
    int32_t in_len[6];   /* their element counts (VertexBuffer: vertices) */
    int32_t in_res[6];   /* their row in the decode result array (-1: absent) */
    int64_t out_off[6];  /* assembly-output byte offsets: geometry_offsets, part_offsets, ring_offsets,
                            coords, part scratch, ring scratch (16-byte aligned) */
    int32_t part_cap, ring_cap, coord_cap; /* capacities the output slices were sized for */
    int32_t flags;                         /* COVT_GEOM_* */
} covt_geom_desc;

/* Per-column assembly result written by the kernel. */
typedef struct covt_geom_result {
    int32_t status; /* COVT_OK, a source stream's decode status, or a COVT_ERR_* of the assembly */
    int32_t num_parts, num_rings, num_coords;
} covt_geom_result;

/* Host-visible geometry-column record of a plan, in tile order. */
typedef struct covt_geom_info {
    int32_t tile, layer, column_type, n_features;
    int32_t stream[6]; /* tile-order stream index of each source stream (-1: absent) */
    int32_t part_cap, ring_cap, coord_cap, flags;
    int32_t desc_index, reserved; /* desc_index: row in the launch-ordered geometry descriptors */
    int64_t out_off[6];
} covt_geom_info;

/* Column capacities are bounded so the kernel's 32-bit scans cannot wrap; a larger column
 * (over 2^25 rings or coordinates) is flagged COVT_GEOM_TOO_LARGE and not assembled. */
#define COVT_GEOM_MAX_CAP (1 << 25)

int64_t covt_plan_num_geometry_columns(const covt_plan* plan);
int64_t covt_plan_assembly_bytes(const covt_plan* plan); /* size of the assembly output buffer */
int covt_plan_geometry_columns(const covt_plan* plan, covt_geom_info* out); /* tile order */
int covt_plan_geometry_descs(const covt_plan* plan, covt_geom_desc* out);   /* launch order (largest first) */

/* Assemble every geometry column on `hip_stream` after the decode launch of the same plan:
 * d_decoded / d_res are the decode output and result arrays (launch-order results), d_gdesc the
 * geometry descriptors, d_asm an output buffer of covt_plan_assembly_bytes bytes, d_gres
 * n_columns results (in d_gdesc order).  Asynchronous. */
int covt_assemble_geometry_device(const uint8_t* d_decoded, const covt_stream_result* d_res,
                                  const covt_geom_desc* d_gdesc, int64_t n_columns, uint8_t* d_asm,
                                  covt_geom_result* d_gres, void* hip_stream);

/* Convenience: H2D + decode + assembly + D2H of the whole plan on the current device.
 * host_asm: covt_plan_assembly_bytes bytes; host_gres: one result per column in tile order. */
int covt_plan_assemble_host(const covt_plan* plan, const uint8_t* bytes, uint64_t n_bytes, uint8_t* host_asm,
                            covt_geom_result* host_gres);

/* ---------------------------------------------------------------------------
 * Property columns: the GPU replacement for
 * CovtParser.decodePropertyColumn (CovtParser.java:276-354) and getStringDictionary (:367-377).
 * A plan created with COVT_PLAN_PROPERTIES also plans every property column: its present / data /
 * length streams join the decode launch (column_kind 2 in covt_stream_info, stream_type = the
 * StreamType PRESENT 0 / DATA 1 / LENGTH 2), and covt_materialize_properties_device turns them into
 * Arrow-style columns, one per (sub)column:
 *
 *   validity[ceil(n/8)]   present bits, LSB first (BitSet.valueOf); all set without a present stream
 *   values                BOOLEAN: bitmap[ceil(n/8)];  INT64: int64[n];  FLOAT: float32[n];
 *                         STRING: int32 dictionary index [n]  (absent slots hold 0)
 *   dict_offsets[n_dict+1], dict_bytes   STRING: Arrow string offsets + UTF-8 bytes of the dictionary
 *
 * Java's List<Optional> per feature is validity bit i ? value i : empty.  Localized dictionary
 * columns (Gen C LOCALIZED_DICTIONARY, which Java rejects with IllegalArgumentException) are
 * decoded as format truth: one STRING sub-column per language stream, sharing the column's
 * dictionary (written once, by the sub-column flagged COVT_PROP_DICT_OWNER).  Gen C boolean columns
 * with a present stream store only the present values' bits (data numValues = present count).
 * INT_64 varint columns follow id_mode: COVT_ID_JAVA = the 4-byte-capped int decode widened to long
 * (CovtParser.java:304-312), COVT_ID_FORMAT = 64-bit zigzag varints (what the writer emits).
 * Statuses follow Java's order: a failed source stream first, then the dictionary (negative length
 * -> COUNT_MISMATCH, strings past the dictionary stream -> TRUNCATED), then the feature loop
 * (a present bit without a data value or a dictionary index out of range -> COUNT_MISMATCH).
 * ------------------------------------------------------------------------- */
#define COVT_PLAN_PROPERTIES 0x1u /* covt_plan_create_ex flag */

#define COVT_PROP_BOOLEAN 0
#define COVT_PROP_INT64 1
#define COVT_PROP_FLOAT 2
#define COVT_PROP_STRING 3

#define COVT_PROP_DICT_OWNER 0x1  /* this sub-column writes the dictionary offsets and bytes */
#define COVT_PROP_DENSE_BOOL 0x2  /* BOOLEAN data holds the present values' bits only (Gen C) */
#define COVT_PROP_UNSUPPORTED 0x4 /* data type / missing stream Java rejects: UNSUPPORTED_ENCODING */
#define COVT_PROP_DATA_SHORT 0x8  /* FLOAT data stream shorter than numValues * 4: TRUNCATED */
#define COVT_PROP_UNSUPPORTED_LATE 0x10 /* encoding Java rejects after decoding the present stream */

/* One device-resident property (sub)column entry (96 bytes). */
typedef struct covt_prop_desc {
    int64_t present_off; /* decode-output byte offset of the present bitset (-1: none, all valid) */
    int64_t data_off;    /* decode-output offset of the dense data (BOOLEAN bits, INT64 int64, STRING int32
                            indices); FLOAT: INPUT offset of the little-endian floats */
    int64_t length_off;  /* STRING: decode-output offset of the int32 dictionary lengths */
    int64_t dict_in_off; /* STRING: input offset of the dictionary bytes */
    int64_t out_off[4];  /* validity, values, dictionary offsets, dictionary bytes (16-byte aligned) */
    int32_t res[3];      /* decode-result rows of the present, data, length streams (-1: none) */
    int32_t n_features, n_data, n_dict, dict_bytes;
    int16_t type, flags; /* COVT_PROP_*, COVT_PROP_* flags */
} covt_prop_desc;

typedef struct covt_prop_result {
    int32_t status;  /* COVT_OK, a source stream's status, or a COVT_ERR_* of the materialization */
    int32_t n_valid; /* features with a value */
} covt_prop_result;

/* Host-visible property (sub)column record of a plan, in tile order (112 bytes). */
typedef struct covt_prop_info {
    int32_t tile, layer, column, type;          /* type: COVT_PROP_* or -1 (unsupported data type) */
    int32_t column_type, n_features, n_data, n_dict;
    int32_t lang, name_len, lang_len, dict_bytes; /* lang: language index of a localized sub-column, -1 */
    int32_t stream[3];                          /* tile-order stream index of present, data, length (-1) */
    int32_t desc_index;                         /* row in the launch-ordered property descriptors */
    int64_t name_off, lang_off;                 /* UTF-8 column / language names in the batch input (-1) */
    int64_t out_off[4];
} covt_prop_info;

/* covt_plan_create plus flags (COVT_PLAN_PROPERTIES), default options otherwise. */
int covt_plan_create_ex(const uint8_t* bytes, const uint64_t* tile_offsets, const uint64_t* tile_sizes,
                        int32_t n_tiles, int32_t format, int32_t id_mode, uint32_t flags, covt_plan** out);
/* covt_plan_create with explicit options (NULL: the defaults).  COVT_ERR_INVALID_ARG for an
 * options struct of the wrong size or out-of-range fields. */
int covt_plan_create_opts(const uint8_t* bytes, const uint64_t* tile_offsets, const uint64_t* tile_sizes,
                          int32_t n_tiles, int32_t format, int32_t id_mode, const covt_plan_options* opts,
                          covt_plan** out);
int64_t covt_plan_num_property_columns(const covt_plan* plan);
int64_t covt_plan_property_bytes(const covt_plan* plan); /* size of the property output buffer */
int covt_plan_property_columns(const covt_plan* plan, covt_prop_info* out); /* tile order */
int covt_plan_property_descs(const covt_plan* plan, covt_prop_desc* out);   /* launch order (largest first) */

/* Materialize every property column on `hip_stream` after the decode launch of the same plan:
 * d_in the batch input (dictionary bytes and floats are read from it), d_decoded / d_res the decode
 * output and launch-order results, d_pdesc the property descriptors, d_props an output buffer of
 * covt_plan_property_bytes bytes, d_pres n_columns results (in d_pdesc order).  Asynchronous. */
int covt_materialize_properties_device(const uint8_t* d_in, const uint8_t* d_decoded, const covt_stream_result* d_res,
                                       const covt_prop_desc* d_pdesc, int64_t n_columns, uint8_t* d_props,
                                       covt_prop_result* d_pres, void* hip_stream);

/* Scratch of the small-batch paths.  For batches of at most 4,096 columns covt_assemble_geometry_device
 * and covt_materialize_properties_device keep one device scratch block per (device, HIP stream) (about
 * 8.4 MB for assembly, 0.6 MB for properties), allocated and zeroed on the stream's first use and reused
 * by every later launch on it.  Each launch tags its look-back records with an epoch its own first kernel
 * advances in device memory, so launches captured in a HIP graph replay correctly -- under two rules: a
 * graph is replayed on its capture stream (or on streams ordered with it: replays of graphs that share a
 * capture stream must not overlap, they share one block's tickets and epoch), and the stream has run one
 * such launch before the capture (a block cannot be allocated while capturing: the launch then fails with
 * COVT_ERR_DEVICE).  A block used under a capture is pinned for the graph: it is never evicted and
 * covt_release_scratch frees it only with COVT_RELEASE_PINNED.  At most 16 unpinned blocks of each kind
 * are kept; beyond that the least recently used unpinned one is freed.  covt_release_scratch frees the
 * unpinned block of (current device, hip_stream), or every unpinned block when bit 0 of `all` is set, plus
 * the pinned ones matched the same way with COVT_RELEASE_PINNED (the caller promises that no graph
 * captured on them replays again), and returns how many it freed.  hipFree waits for the device, so no
 * launch still in flight uses a freed block; a caller that creates a stream per batch should release its
 * blocks before destroying the stream. */
#define COVT_RELEASE_PINNED 0x2
int covt_release_scratch(void* hip_stream, int all);
/* blocks currently held (assembly + properties) */
int64_t covt_scratch_blocks(void);

/* Convenience: H2D + decode + property materialization + D2H of the whole plan on the current device.
 * host_props: covt_plan_property_bytes bytes; host_pres: one result per (sub)column in tile order. */
int covt_plan_properties_host(const covt_plan* plan, const uint8_t* bytes, uint64_t n_bytes, uint8_t* host_props,
                              covt_prop_result* host_pres);

/* ---- Device-side plan ------------------------------------------------------------------------
 * covt_plan_create's Id / Geometry walk run on the GPU, for tiles already resident in HBM (the host
 * half of CovtParser.decodeCovt, CovtParser.java:53-133 / :574-652, without the round trip through
 * host memory).  d_bytes / n_bytes: the batch on the current device; d_tile_offsets / d_tile_sizes:
 * n_tiles uint64 each, on the device (a tile outside [0, n_bytes) gets COVT_ERR_INVALID_ARG as its
 * status).  The result is the host plan's layout exactly: streams in tile order with the same
 * covt_stream_info fields and 128-byte aligned output slices, descriptors in the same launch order
 * and families, including the split rule: with the same options, the long poles of a small batch are
 * cut into the same chunks (varint byte chunks, FastPFOR value chunks with their start states, ORC RLE
 * group chunks); geometry-column planning on request (covt_device_plan_geometry); property columns
 * with COVT_PLAN_PROPERTIES in opts->flags.  Multi-GPU shards stay with the host plan.
 * Runs on `hip_stream` and synchronises it: once for an Id / Geometry plan of more than
 * split_max_streams / 32 tiles (nothing splits there; the stream arrays are sized to 64 streams per tile
 * and the count is checked at the end -- a batch averaging more is redone with its counted size: three
 * syncs), otherwise twice (three times when it splits: the stream count and the descriptor count size the
 * arrays); COVT_PLAN_PROPERTIES adds one more (the property record count).  COVT_ERR_BAD_HEADER if the property walk fails a tile the Id / Geometry walk accepted (the
 * walkers diverged: never on well-formed or corrupted input that the host plan rejects the same way).
 * Limits and memory: a tile of 0x7ff00000 bytes or more gets COVT_ERR_INVALID_ARG as its status
 * (32-bit cursors; the host plan walks such tiles); besides the stream arrays the plan holds ~5 KiB
 * of per-tile walk slots on the device (128 stream records of 40 bytes per tile: ~0.5 GB at 100k
 * tiles) unless opts->device_walk != 0.  The arenas come from a per-device stream-ordered memory pool
 * that keeps up to 1 GiB of freed plan memory for the next plan (PyTorch's allocator does not see it);
 * covt_device_plan_pool_trim(device, keep_bytes) releases all but keep_bytes of it. */
typedef struct covt_device_plan covt_device_plan;
int covt_device_plan_create(const uint8_t* d_bytes, uint64_t n_bytes, const uint64_t* d_tile_offsets,
                            const uint64_t* d_tile_sizes, int32_t n_tiles, int32_t format, int32_t id_mode,
                            void* hip_stream, covt_device_plan** out);
/* the same with explicit options (NULL: the defaults; flags: 0 or COVT_PLAN_PROPERTIES) */
int covt_device_plan_create_opts(const uint8_t* d_bytes, uint64_t n_bytes, const uint64_t* d_tile_offsets,
                                 const uint64_t* d_tile_sizes, int32_t n_tiles, int32_t format, int32_t id_mode,
                                 const covt_plan_options* opts, void* hip_stream, covt_device_plan** out);
void covt_device_plan_destroy(covt_device_plan* plan);
int covt_device_plan_pool_trim(int device, uint64_t keep_bytes);
int64_t covt_device_plan_num_streams(const covt_device_plan* plan);
int64_t covt_device_plan_num_descs(const covt_device_plan* plan); /* = num_streams unless it splits */
int64_t covt_device_plan_output_bytes(const covt_device_plan* plan);
int covt_device_plan_totals(const covt_device_plan* plan, int64_t* in_bytes, int64_t* out_bytes, int64_t* vertices);
int covt_device_plan_family_counts(const covt_device_plan* plan, int64_t counts[COVT_NUM_FAMILIES]);
/* device arrays owned by the plan: num_descs descriptors (launch order), num_streams stream records
 * (tile order, desc_index = the stream's first descriptor), n_tiles statuses, and the stream index of
 * each descriptor (num_descs) */
const covt_stream_desc* covt_device_plan_descs_device(const covt_device_plan* plan);
const covt_stream_info* covt_device_plan_streams_device(const covt_device_plan* plan);
const int32_t* covt_device_plan_tile_status_device(const covt_device_plan* plan);
const uint32_t* covt_device_plan_order_device(const covt_device_plan* plan);
/* copies of the device arrays into host memory (any pointer may be NULL) */
int covt_device_plan_copy(const covt_device_plan* plan, covt_stream_info* streams, covt_stream_desc* descs,
                          int32_t* tile_status);
/* Geometry assembly from a device plan (covt_plan_geometry_columns / covt_plan_geometry_descs built on
 * the device, CovtParser.convertGeometryColumn's input): the first call of covt_device_plan_geometry
 * (or covt_device_plan_assemble) builds the geometry-column records and launch-ordered descriptors on
 * `hip_stream` -- the host plan's exactly -- and synchronises it; later calls return at once. */
int covt_device_plan_geometry(covt_device_plan* plan, void* hip_stream);
int64_t covt_device_plan_num_geometry_columns(const covt_device_plan* plan); /* 0 before geometry() */
int64_t covt_device_plan_assembly_bytes(const covt_device_plan* plan);
const covt_geom_desc* covt_device_plan_geometry_descs_device(const covt_device_plan* plan);
int covt_device_plan_geometry_copy(const covt_device_plan* plan, covt_geom_info* infos, covt_geom_desc* descs);
/* covt_assemble_geometry_device over the plan's geometry descriptors (built first if needed), after
 * covt_device_plan_decode on the same stream: d_asm covt_device_plan_assembly_bytes bytes, d_gres one
 * result per column in launch order (column c's at its covt_geom_info.desc_index). */
int covt_device_plan_assemble(covt_device_plan* plan, const uint8_t* d_decoded, const covt_stream_result* d_res,
                              uint8_t* d_asm, covt_geom_result* d_gres, void* hip_stream);
/* Property columns from a device plan made with COVT_PLAN_PROPERTIES in opts->flags: the records,
 * output layout and largest-first descriptors of covt_plan_property_columns / covt_plan_property_descs,
 * built on the device with the plan (the host plan's exactly); a plan without the flag has none. */
int64_t covt_device_plan_num_property_columns(const covt_device_plan* plan);
int64_t covt_device_plan_property_bytes(const covt_device_plan* plan);
const covt_prop_desc* covt_device_plan_property_descs_device(const covt_device_plan* plan);
int covt_device_plan_property_copy(const covt_device_plan* plan, covt_prop_info* infos, covt_prop_desc* descs);
/* covt_materialize_properties_device over the plan's property descriptors, after covt_device_plan_decode
 * on the same stream: d_props covt_device_plan_property_bytes bytes, d_pres one result per (sub)column in
 * descriptor order (column c's at its covt_prop_info.desc_index). */
int covt_device_plan_materialize(const covt_device_plan* plan, const uint8_t* d_in, const uint8_t* d_decoded,
                                 const covt_stream_result* d_res, uint8_t* d_props, covt_prop_result* d_pres,
                                 void* hip_stream);
/* the grouped decode launch over the plan's descriptors (covt_decode_streams_device_grouped):
 * d_out covt_device_plan_output_bytes bytes, d_res num_descs results (stream i's at its desc_index).
 * Asynchronous. */
int covt_device_plan_decode(const covt_device_plan* plan, const uint8_t* d_in, uint8_t* d_out,
                            covt_stream_result* d_res, void* hip_stream);

/* Library info */
const char* covt_version(void);
int covt_device_count(int32_t* n);

#ifdef __cplusplus
}
#endif
#endif /* COVT_H */
