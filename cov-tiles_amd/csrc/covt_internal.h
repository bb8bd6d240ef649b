// covt_internal.h -- declarations shared by the kernel and host translation units of libcovt.
#ifndef COVT_INTERNAL_H
#define COVT_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"

extern "C" {
// Enqueues the decode kernel of one family (covt_decode.hip) on `stream` over descriptors
// [0, n_streams); descriptors of other families are skipped.
int covt_launch_family(int fam, const uint8_t* d_in, const covt_stream_desc* d_desc, int64_t n_streams,
                       uint8_t* d_out, covt_stream_result* d_res, hipStream_t stream);
// Split chunks (descriptors d_split[0, n_split), their results / look-back records at d_split_res) of
// kind fam (VARINT: COVT_FAMILY_SPLIT, RLE: COVT_FAMILY_SPLIT_RLE, FASTPFOR: COVT_FAMILY_SPLIT_FPF),
// then family fam over d_desc[0, n_streams) on the same stream.
int covt_launch_family_split(int fam, const uint8_t* d_in, const covt_stream_desc* d_desc, int64_t n_streams,
                             uint8_t* d_out, covt_stream_result* d_res, const covt_stream_desc* d_split,
                             int64_t n_split, covt_stream_result* d_split_res, hipStream_t stream);
// The same with the FastPFOR family's variant chosen by the caller: 0 auto (run_fastpfor_stream for at least
// kFpfStreamMinStreams descriptors, run_fastpfor below), COVT_LAUNCH_FPF_STREAM or COVT_LAUNCH_FPF_CLASSIC.
int covt_launch_family_split_mode(int fam, const uint8_t* d_in, const covt_stream_desc* d_desc, int64_t n_streams,
                                  uint8_t* d_out, covt_stream_result* d_res, const covt_stream_desc* d_split,
                                  int64_t n_split, covt_stream_result* d_split_res, hipStream_t stream, int fpf_mode);
int covt_op_family_of(int op);
// Every family of a grouped descriptor table (family f at offset sum(counts[0..f))) in ONE kernel launch
// on `stream` (small batches; split regions' records zeroed beforehand).
int covt_launch_fused(const uint8_t* d_in, const covt_stream_desc* d_desc, const int64_t counts[COVT_NUM_FAMILIES],
                      uint8_t* d_out, covt_stream_result* d_res, hipStream_t stream);
}
// A FastPFOR family launch of at least this many streams takes run_fastpfor_stream (8 times the chip's 8,192
// wave slots: the bench batch's 77k; a strong-scaling shard of it, 9.7k-39k, keeps run_fastpfor)
constexpr int64_t kFpfStreamMinStreams = 65536;
// Batches of at most this many waves (split chunks + wave-per-stream descriptors + lane streams /
// kFusedLaneStreams) decode in one fused launch instead of the forked per-family launches
constexpr int64_t kFusedMaxWaves = 4096;
// The decode kernels' workgroup: kWavesPerBlock independent waves (covt_decode.hip); the fused launch's
// lane segment gives every thread of a workgroup one lane stream
#ifndef COVT_WAVES_PER_BLOCK
#define COVT_WAVES_PER_BLOCK 2  // A/B: 1 -> +8 %, 4 -> +1 % on the bench launch
#endif
constexpr int kWavesPerBlock = COVT_WAVES_PER_BLOCK;
constexpr int64_t kFusedLaneStreams = 64 * kWavesPerBlock;

// Output slices of the decode launch (host and device plans): every stream's slice starts on a 128-byte
// line.  A family's 1 KiB (or 2 KiB) wave stores then cover whole lines instead of straddling two partial
// ones per store: the config-5 launch 1.602 -> 1.558 ms with the same kernels (tools/probe/layout_ab.py,
// profiles/r04/layout_ab.txt; 16-byte slices, the round-3 layout, cost ~24 MB less buffer).
constexpr int64_t kOutAlign = 128;
__host__ __device__ inline int64_t align_out(int64_t x) { return (x + kOutAlign - 1) & ~(kOutAlign - 1); }

// Launch order (covt_plan_create step 3; the device plan's stream_keys): a 16-bit key, family-major
// (3 bits), then -- for the lane family -- the op and the exact cost (bytes + output bytes / 4 <= 1023 for
// a lane stream), largest first, so each 64-stream wave gets streams of one op and near-equal length;
// for every other family the cost in 1/128 octaves, largest first, so the long poles start early.  A
// stable sort keeps tile order inside a key.  (The rounds 1-4 key was a 60-bit exact cost: a 40-bit
// radix sort on the device, ~18 launches, 0.16 ms of the 10k-tile plan; this one is two 8-bit
// counting-sort passes.)
constexpr int kLaunchFamShift = 13;
__host__ __device__ inline uint32_t lane_op_index(int32_t op) {  // the lane ops in op order
    return op == COVT_OP_BYTE_RLE_U8 ? 0u : op == COVT_OP_RLE_U64 ? 1u : op == COVT_OP_RLE_I32 ? 2u
         : op == COVT_OP_RLE_S64 ? 3u : 4u;
}
__host__ __device__ inline uint32_t launch_key(uint32_t fam, bool lane, int32_t op, int64_t cost) {
    const uint64_t c = cost > 0 ? (uint64_t)cost : 0;
    uint32_t sub;
    if (lane) {
        sub = (lane_op_index(op) << 10) | (1023u - (uint32_t)(c < 1023 ? c : 1023));
    } else {
        uint32_t h = 0;  // 0: no cost; else 1 + e * 128 + the 7 bits below the top one, e = floor(log2 c)
        if (c) {
            const int e = 63 - __builtin_clzll(c);
            const uint32_t mant = e >= 7 ? (uint32_t)(c >> (e - 7)) & 127u : (uint32_t)(c << (7 - e)) & 127u;
            h = ((uint32_t)e << 7) + mant + 1u;
        }
        sub = 8191u - (h < 8191u ? h : 8191u);
    }
    return (fam << kLaunchFamShift) | sub;
}

// Plan rule for the lane-per-stream kernel: RLE streams of at most max_values values and max_bytes bytes
// (a lane decodes serially; larger streams amortise a wave's window setup).  The two limits travel
// packed as one int32 (values << 16 | bytes; < 0: no lane family), see lane_limits.
constexpr int64_t kLaneMinStreams = COVT_LANE_MIN_STREAMS;  // plans with fewer lane-eligible streams use no lane kernel

// The caller's plan options checked and completed (NULL: the defaults; auto lane limits resolved from the
// flags); false for a wrong struct size or out-of-range fields.  Shared by the host and the device plan.
bool covt_resolve_options(const covt_plan_options* in, covt_plan_options& out);
__host__ __device__ inline int32_t lane_limits(int32_t max_bytes, int32_t max_values) {
    return max_bytes < 0 ? -1 : (int32_t)(((uint32_t)max_values << 16) | (uint32_t)max_bytes);
}
__host__ __device__ inline bool lane_stream(int op, int32_t num_values, int32_t byte_length, int32_t limits) {
    return limits >= 0 &&
           (op == COVT_OP_BYTE_RLE_U8 || op == COVT_OP_BYTE_RLE_RAW || op == COVT_OP_RLE_U64 || op == COVT_OP_RLE_S64 ||
            op == COVT_OP_RLE_I32) &&
           num_values >= 0 && num_values <= (limits >> 16) && byte_length >= 0 && byte_length <= (limits & 0xffff);
}
inline int desc_family(const covt_stream_desc& d) {
    if (d.flags & (COVT_DESC_SPLIT | COVT_DESC_SPLIT_PAD))
        return (d.flags & COVT_DESC_SPLIT_FPF)   ? COVT_FAMILY_SPLIT_FPF
               : (d.flags & COVT_DESC_SPLIT_RLE) ? COVT_FAMILY_SPLIT_RLE
                                                 : COVT_FAMILY_SPLIT;
    return (d.flags & COVT_DESC_LANE) ? COVT_FAMILY_LANE : covt_op_family_of(d.op);
}
// Plan rule for split streams: the Java-capped int32 varint ops (value ends are local: every byte
// with bit 7 clear ends a value, DecodingUtils.java:157-186), longer than split_min bytes.
__host__ __device__ inline bool split_op(int op) {
    return op == COVT_OP_VARINT_I32 || op == COVT_OP_VARINT_ZZ_I32 || op == COVT_OP_VARINT_ZZ_DELTA_I32 ||
           op == COVT_OP_VARINT_ZZ_DELTA_XY || op == COVT_OP_VARINT_DELTA_MORTON || op == COVT_OP_VARINT_I32_AS_I64 ||
           op == COVT_OP_VARINT_ZZ_I32_AS_I64 || op == COVT_OP_VARINT_ZZ_DELTA_I64 || op == COVT_OP_VARINT_U64 ||
           op == COVT_OP_VARINT_ZZ_S64;
}
// FastPFOR ops whose long streams split into value chunks.  The chunk kernel (covt_decode.hip
// run_fastpfor_chunk) adds a chunk's carry in place for the linear int32 ops (ZZ_DELTA_I32, ZZ_DELTA_XY) and
// decodes Morton twice; an op added here needs a carry rule there (static_asserts guard it).
__host__ __device__ inline bool split_fpf_op(int op) {
    return op == COVT_OP_FPF_ZZ_DELTA_I32 || op == COVT_OP_FPF_ZZ_DELTA_XY || op == COVT_OP_FPF_DELTA_MORTON;
}
__host__ __device__ inline bool split_rle_op(int op) {
    return op == COVT_OP_RLE_U64 || op == COVT_OP_RLE_I32 || op == COVT_OP_RLE_S64 || op == COVT_OP_BYTE_RLE_U8 ||
           op == COVT_OP_BYTE_RLE_RAW;
}
// FastPFOR streams split by values into chunks of whole blocks (their own headers and page directories
// locate every block), at least two chunks
// cost: the stream's bytes + output bytes / 4 (covt_plan_create's launch-order key)
__host__ __device__ inline bool split_stream(int op, int32_t num_values, int64_t cost, int64_t split_min, int64_t split_values) {
    if (split_min < 0 || num_values <= 0 || cost <= split_min) return false;
    if (split_fpf_op(op)) return num_values > split_values && !(op == COVT_OP_FPF_ZZ_DELTA_XY && (num_values & 1));
    return split_op(op) && !(op == COVT_OP_VARINT_ZZ_DELTA_XY && (num_values & 1));
}

// covt_plan_options.split_grow: chunks (split_chunk bytes, split_values values) doubled for plans of >= 4 MiB of
// cost and quadrupled from 48 MiB.  In a plan whose streams fill the chip a chunk wave shares its SIMD with
// the crowd, and its fixed costs (start state, look-back) weigh more than a longer body
// (profiles/r05/shard_sizes.txt: 2 KiB chunks best for one tile, 4 KiB for 8-30 MiB plans, 8 KiB above)
__host__ __device__ inline int64_t split_grow_factor(int64_t total_cost, int32_t grow) {
    if (!grow) return 1;
    return total_cost >= (48ll << 20) ? 4 : total_cost >= (4ll << 20) ? 2 : 1;
}

// FastPFOR split chunks: the host-walked start state in pads [2..7] of the chunk (covt_host.cpp
// fpf_chunk_states): seven int32 slots per pad, every field but op / num_bits / flags
constexpr int kFpfStateSlots = 42;
__host__ __device__ constexpr int covt_fpf_state_byte(int k) { return k < 6 ? 4 * k : 28; }

#endif
