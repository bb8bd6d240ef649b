// covt_walk.h -- wire enums and the CovtParser stream dispatch, shared by the host plan (covt_host.cpp)
// and the device-side metadata walk (covt_plan_device.hip), so both plans choose the same op for a stream.
#ifndef COVT_WALK_H
#define COVT_WALK_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"

// ---- wire enums --------------------------------------------------
enum StreamType { ST_PRESENT = 0, ST_DATA = 1, ST_LENGTH = 2, ST_DICTIONARY = 3, ST_GEOMETRY_TYPES = 4,
                  ST_GEOMETRY_OFFSETS = 5, ST_PART_OFFSETS = 6, ST_RING_OFFSETS = 7, ST_VERTEX_OFFSETS = 8,
                  ST_VERTEX_BUFFER = 9, ST_Z = 10, ST_M = 11 };
enum Encoding { ENC_PLAIN = 0, ENC_VARINT = 1, ENC_VARINT_DELTA_ZZ = 4, ENC_RLE = 5, ENC_FPF_DELTA_ZZ = 9 };
enum ColumnType { CT_PLAIN = 0, CT_ICE = 3, CT_ICE_MORTON = 4 };

struct RawStream {
    int32_t layer, kind, type, enc, ctype, nv, bl, nb;
    int64_t off;  // tile-relative payload offset
};

// 32 - Integer.numberOfLeadingZeros(extent), CovtParser.java:77
__host__ __device__ inline int nbits_of_extent(uint64_t extent) {
    const uint32_t e = (uint32_t)extent;
    return e ? 32 - __builtin_clz(e) : 0;
}

// CovtParser dispatch: decodeGeometryColumn (:392-511) and decodedIds (:552-572)
__host__ __device__ inline void choose_op(const RawStream& s, int id_mode, int& op, int64_t& nvals, int& elem, int64_t& out_elems) {
    op = COVT_OP_NONE;
    nvals = s.nv;
    elem = 4;
    out_elems = s.nv;
    if (s.kind == 0) {
        elem = 8;
        if (s.enc == ENC_RLE) op = COVT_OP_RLE_U64;
        else if (s.enc == ENC_VARINT) op = id_mode == COVT_ID_JAVA ? COVT_OP_VARINT_I32_AS_I64 : COVT_OP_VARINT_U64;
        else if (s.enc == ENC_VARINT_DELTA_ZZ)
            op = id_mode == COVT_ID_JAVA ? COVT_OP_VARINT_ZZ_DELTA_I64 : COVT_OP_RLE_U64;
        return;
    }
    switch (s.type) {
    case ST_GEOMETRY_TYPES: op = COVT_OP_BYTE_RLE_U8; elem = 1; return;
    case ST_GEOMETRY_OFFSETS:
    case ST_PART_OFFSETS:
    case ST_RING_OFFSETS:
        if (s.enc == ENC_RLE) op = COVT_OP_RLE_I32;
        else if (s.enc == ENC_FPF_DELTA_ZZ) op = COVT_OP_FPF_ZZ_DELTA_I32;
        return;
    case ST_VERTEX_OFFSETS:
        if (s.enc == ENC_VARINT_DELTA_ZZ) op = COVT_OP_VARINT_ZZ_DELTA_I32;
        else if (s.enc == ENC_FPF_DELTA_ZZ) op = COVT_OP_FPF_ZZ_DELTA_I32;
        return;
    case ST_VERTEX_BUFFER:
        if (s.ctype == CT_ICE_MORTON) {
            out_elems = 2 * (int64_t)s.nv;
            if (s.enc == ENC_VARINT_DELTA_ZZ) op = COVT_OP_VARINT_DELTA_MORTON;
            else if (s.enc == ENC_FPF_DELTA_ZZ) op = COVT_OP_FPF_DELTA_MORTON;
        } else {
            if (s.ctype == CT_ICE) nvals = out_elems = 2 * (int64_t)s.nv;  // SURVEY Q4 build rule
            if (s.enc == ENC_VARINT_DELTA_ZZ) op = COVT_OP_VARINT_ZZ_DELTA_XY;
            else if (s.enc == ENC_FPF_DELTA_ZZ) op = COVT_OP_FPF_ZZ_DELTA_XY;
        }
        return;
    default: return;
    }
}

// decode kernel family of an op (launch grouping of both plans)
__host__ __device__ constexpr int covt_op_family(int op) {
    return (op >= COVT_OP_FPF_ZZ_DELTA_I32 && op <= COVT_OP_FPF_DELTA_MORTON) ? COVT_FAMILY_FASTPFOR
           : ((op >= COVT_OP_VARINT_I32 && op <= COVT_OP_VARINT_DELTA_MORTON) ||
              (op >= COVT_OP_VARINT_U64 && op <= COVT_OP_VARINT_ZZ_DELTA_I64) ||
              (op >= COVT_OP_VARINT_ZZ_I32_AS_I64 && op <= COVT_OP_VARINT_ZZ_DELTA_S64))
               ? COVT_FAMILY_VARINT
               : COVT_FAMILY_RLE;  // RLE ops and COVT_OP_NONE / unknown ops (reported as unsupported)
}

#endif
