// covt_props_plan.h -- the property-column planning rule (CovtParser.decodePropertyColumn,
// CovtParser.java:276-367), shared by the host plan (covt_host.cpp) and the device plan
// (covt_plan_device.hip), so both give a (sub)column the same decode streams, ops and flags.
#ifndef COVT_PROPS_PLAN_H
#define COVT_PROPS_PLAN_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"
#include "covt_walk.h"

// One property (sub)column found by a walker.  Streams by role 0 present, 1 data, 2 length,
// 3 dictionary; offsets tile-relative (-1: absent).
struct PropRaw {
    int32_t layer, column, type, ctype, nf, lang, name_len, lang_len;
    int64_t name_off, lang_off;  // tile-relative UTF-8 names (-1: none)
    int64_t s_off[4];
    int32_t s_nv[4], s_bl[4], s_enc[4];
};
__host__ __device__ inline PropRaw prop_init(int32_t layer, int32_t column, int32_t nf) {
    PropRaw p{};
    p.layer = layer;
    p.column = column;
    p.nf = nf;
    p.lang = -1;
    p.name_off = p.lang_off = -1;
    for (int r = 0; r < 4; ++r) p.s_off[r] = -1;
    return p;
}
// (constant indices only: a record indexed by a run-time role lives in scratch on the GPU, where the
// property walk kept its record -- 144 bytes per lane of private memory)
__host__ __device__ inline void prop_stream(PropRaw& p, int role, int64_t off, int32_t nv, int32_t bl, int32_t enc) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (r != role) continue;
        p.s_off[r] = off;
        p.s_nv[r] = nv;
        p.s_bl[r] = bl;
        p.s_enc[r] = enc;
    }
}
// Gen C ColumnDataType (evaluation/file/ColumnDataType.java) / Gen D (converter/ColumnDataType.java)
__host__ __device__ inline int genc_prop_type(int dt) {
    return dt == 0 ? COVT_PROP_STRING : dt == 1 ? COVT_PROP_FLOAT : dt == 3 ? COVT_PROP_INT64 : dt == 5 ? COVT_PROP_BOOLEAN : -1;
}
__host__ __device__ inline int gend_prop_type(int dt) {
    return dt == 0 ? COVT_PROP_BOOLEAN : dt == 3 ? COVT_PROP_INT64 : dt == 5 ? COVT_PROP_FLOAT : dt == 7 ? COVT_PROP_STRING : -1;
}

// The decode streams of a (sub)column and its flags.  Unsupported shapes get a flag instead of
// streams, in the order Java would throw: before anything (type, missing streams) or after the present
// stream was decoded (data encodings, non-dictionary strings).
struct PropStreams {
    uint16_t flags;
    int32_t n;                            // streams
    uint32_t has;                         // bit r: a stream of role r (0 present, 1 data, 2 length)
    int32_t op[3], elem[3];               // by role; the streams go in role order
    int64_t count[3];                     // output elements of each
    int64_t in_bytes;                     // stream bytes + bytes read in place (floats, the owner's dictionary)
};
__host__ __device__ inline void prop_streams(const PropRaw& q, int id_mode, PropStreams& ps) {
    uint16_t fl = 0;
    const int32_t nf = q.nf > 0 ? q.nf : 0, nb = (int32_t)(((int64_t)nf + 7) / 8);
    const bool early_unsup = q.type < 0 || q.s_off[1] < 0 || (q.type != COVT_PROP_BOOLEAN && q.s_off[0] < 0) ||
                             q.nf < 0 || q.s_nv[1] < 0;
    int data_op = COVT_OP_NONE, data_elem = 0;
    int64_t data_n = 0;
    bool late_unsup = false;
    if (!early_unsup) {
        switch (q.type) {
        case COVT_PROP_BOOLEAN:
            if (q.s_off[0] >= 0) fl |= COVT_PROP_DENSE_BOOL;
            data_op = COVT_OP_BYTE_RLE_RAW;
            data_elem = 1;
            data_n = (q.s_off[0] >= 0) ? ((int64_t)q.s_nv[1] + 7) / 8 : nb;
            break;
        case COVT_PROP_INT64:
            data_elem = 8;
            data_n = q.s_nv[1];
            if (q.s_enc[1] == ENC_RLE) data_op = COVT_OP_RLE_S64;
            else if (q.s_enc[1] == 2) data_op = id_mode == COVT_ID_JAVA ? COVT_OP_VARINT_ZZ_I32_AS_I64 : COVT_OP_VARINT_ZZ_S64;
            else if (q.s_enc[1] == ENC_VARINT_DELTA_ZZ)
                data_op = id_mode == COVT_ID_JAVA ? COVT_OP_VARINT_ZZ_DELTA_I64 : COVT_OP_VARINT_ZZ_DELTA_S64;
            else late_unsup = true;
            break;
        case COVT_PROP_FLOAT:  // no decode: the kernel reads the little-endian words from the input
            if ((int64_t)q.s_nv[1] * 4 > q.s_bl[1]) fl |= COVT_PROP_DATA_SHORT;
            break;
        default:  // STRING
            if ((q.ctype != 1 && q.ctype != 2) || q.s_off[2] < 0 || q.s_off[3] < 0 || q.s_enc[1] != ENC_RLE ||
                q.s_nv[3] < 0) {
                late_unsup = true;
            } else {
                data_op = COVT_OP_RLE_I32;  // (int) data[dataCounter++]
                data_elem = 4;
                data_n = q.s_nv[1];
                if (q.lang <= 0) fl |= COVT_PROP_DICT_OWNER;
            }
            break;
        }
    }
    if (early_unsup) fl |= COVT_PROP_UNSUPPORTED;
    if (late_unsup) fl |= COVT_PROP_UNSUPPORTED_LATE;
    ps.flags = fl;
    ps.n = 0;
    ps.in_bytes = 0;
    ps.has = 0;
    // (indexed by the role, a constant at every call: a slot index would put the arrays in scratch)
    auto add = [&](int role, int op, int64_t n, int elem) {
        ps.has |= 1u << role;
        ps.op[role] = op;
        ps.count[role] = n;
        ps.elem[role] = elem;
        ps.in_bytes += q.s_bl[role];
        ++ps.n;
    };
    if (!early_unsup) {
        if (q.s_off[0] >= 0) add(0, COVT_OP_BYTE_RLE_RAW, nb, 1);  // decodeByteRle(numBytes), :296
        if (!late_unsup && data_op != COVT_OP_NONE) add(1, data_op, data_n, data_elem);
        if (!late_unsup && q.type == COVT_PROP_STRING) add(2, COVT_OP_RLE_I32, q.s_nv[3], 4);  // lengths: n_dict
        if (q.type == COVT_PROP_FLOAT) ps.in_bytes += q.s_bl[1];  // read in place
        if (fl & COVT_PROP_DICT_OWNER) ps.in_bytes += q.s_bl[3];
    }
}

// covt_prop_info of a (sub)column before the layout (stream indices, output offsets filled later; the
// FLOAT data and STRING dictionary input offsets parked in out_off[1] / out_off[3])
__host__ __device__ inline covt_prop_info prop_info_of(const PropRaw& q, int32_t t, int64_t tile_off) {
    covt_prop_info pi{};
    pi.tile = t;
    pi.layer = q.layer;
    pi.column = q.column;
    pi.type = q.type;
    pi.column_type = q.ctype;
    pi.n_features = q.nf;
    pi.n_data = q.s_nv[1];
    pi.n_dict = q.s_off[3] >= 0 ? (q.s_nv[3] > 0 ? q.s_nv[3] : 0) : 0;
    pi.lang = q.lang;
    pi.name_len = q.name_len;
    pi.lang_len = q.lang_len;
    pi.dict_bytes = q.s_off[3] >= 0 ? (q.s_bl[3] > 0 ? q.s_bl[3] : 0) : 0;
    pi.name_off = q.name_off >= 0 ? tile_off + q.name_off : -1;
    pi.lang_off = q.lang_off >= 0 ? tile_off + q.lang_off : -1;
    for (int k = 0; k < 3; ++k) pi.stream[k] = -1;
    pi.desc_index = 0;
    // temporarily (as values: two conditional stores were merged into one at a computed index, in scratch)
    pi.out_off[0] = pi.out_off[2] = 0;
    pi.out_off[1] = (q.type == COVT_PROP_FLOAT && q.s_off[1] >= 0) ? tile_off + q.s_off[1] : 0;
    pi.out_off[3] = (q.type == COVT_PROP_STRING && q.s_off[3] >= 0) ? tile_off + q.s_off[3] : 0;
    return pi;
}

// the property output layout: bytes of a (sub)column's validity, values and (the owner's) dictionary
__host__ __device__ inline int64_t prop_align16(int64_t x) { return (x + 15) & ~(int64_t)15; }
__host__ __device__ inline void prop_layout_sizes(const covt_prop_info& pi, bool owner, int64_t (&sz)[4]) {
    const int64_t n = pi.n_features > 0 ? pi.n_features : 0, nb = (n + 7) / 8;
    const int64_t vbytes = pi.type == COVT_PROP_BOOLEAN ? nb : pi.type == COVT_PROP_INT64 ? 8 * n : 4 * n;
    sz[0] = prop_align16(nb);
    sz[1] = prop_align16(vbytes);
    const bool own = pi.type == COVT_PROP_STRING && owner;
    sz[2] = own ? prop_align16(4 * ((int64_t)pi.n_dict + 1)) : 0;
    sz[3] = own ? prop_align16(pi.dict_bytes) : 0;
}
// the largest-first materialization order key (features + dictionary entries; ties in tile order)
__host__ __device__ inline uint64_t prop_order_key(const covt_prop_info& pi) {
    return (1ull << 40) - (uint64_t)((int64_t)pi.n_features + pi.n_dict);
}

#endif
