// covt_wave.h -- wave64 primitives shared by the gfx950 kernels of libcovt (decode, assembly):
// wave-uniform reads, lane broadcast, DPP inclusive scan / max without LDS traffic.
#ifndef COVT_WAVE_H
#define COVT_WAVE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace covt {

// --------------------------------------------------------------------------------------------
// wave primitives
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t uniu(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ int64_t uni64(int64_t x) {
    const uint32_t lo = uniu((uint32_t)x), hi = uniu((uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t lane_bcast(uint32_t x, int src) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, src);
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
// inclusive prefix sum over the 64 lanes (wrapping uint32): DPP row shifts within 16-lane rows,
// then row broadcasts 15 and 31 across rows (the GFX9 wave64 scan sequence, no LDS traffic)
__device__ __forceinline__ uint32_t incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// unsigned add saturating at 0xffffffff (v_add_u32 with clamp)
__device__ __forceinline__ uint32_t add_sat(uint32_t a, uint32_t b) { return __builtin_elementwise_add_sat(a, b); }
// inclusive prefix sum over the 64 lanes saturating at 0xffffffff (same DPP sequence as incl_scan):
// a sum that passes 2^32 - 1 stays there instead of wrapping, so a bound check on it cannot be fooled
__device__ __forceinline__ uint32_t incl_scan_sat(uint32_t x) {
    x = add_sat(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = add_sat(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = add_sat(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = add_sat(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
    x = add_sat(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast:15
    x = add_sat(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return x;
}

// inclusive prefix sum of 64-bit values over the 64 lanes (same DPP sequence, carry by hand)
__device__ __forceinline__ uint64_t incl_scan64(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
#define COVT_SCAN64_STEP(ctrl, rmask)                                                             \
    {                                                                                             \
        const uint32_t l2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, ctrl, rmask, 0xf, false); \
        const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, ctrl, rmask, 0xf, false); \
        const uint32_t s = lo + l2;                                                               \
        hi = hi + h2 + (s < lo ? 1u : 0u);                                                        \
        lo = s;                                                                                   \
    }
    COVT_SCAN64_STEP(0x111, 0xf)  // row_shr:1
    COVT_SCAN64_STEP(0x112, 0xf)  // row_shr:2
    COVT_SCAN64_STEP(0x114, 0xf)  // row_shr:4
    COVT_SCAN64_STEP(0x118, 0xf)  // row_shr:8
    COVT_SCAN64_STEP(0x142, 0xa)  // row_bcast:15
    COVT_SCAN64_STEP(0x143, 0xc)  // row_bcast:31
#undef COVT_SCAN64_STEP
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t lane_bcast64(uint64_t x, int src) {
    return ((uint64_t)lane_bcast((uint32_t)(x >> 32), src) << 32) | lane_bcast((uint32_t)x, src);
}

// inclusive running maximum over the 64 lanes (same DPP sequence as incl_scan)
__device__ __forceinline__ uint32_t incl_max_scan(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast:15
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return x;
}

// maximum over the 64 lanes (DPP row shifts, then row broadcasts), returned uniform
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast:15
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return lane_bcast(x, 63);
}

// bitwise OR over the 64 lanes of a 64-bit value (DPP on both halves), returned uniform
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#define COVT_OR64_STEP(ctrl, rmask)                                                    \
    lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, ctrl, rmask, 0xf, false); \
    hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, ctrl, rmask, 0xf, false);
    COVT_OR64_STEP(0x111, 0xf)  // row_shr:1
    COVT_OR64_STEP(0x112, 0xf)  // row_shr:2
    COVT_OR64_STEP(0x114, 0xf)  // row_shr:4
    COVT_OR64_STEP(0x118, 0xf)  // row_shr:8
    COVT_OR64_STEP(0x142, 0xa)  // row_bcast:15
    COVT_OR64_STEP(0x143, 0xc)  // row_bcast:31
#undef COVT_OR64_STEP
    return ((uint64_t)lane_bcast(hi, 63) << 32) | lane_bcast(lo, 63);
}

// lane l + 1's value (lane 63: `tail`, which must be wave-uniform): DPP wave_shl:1, no LDS traffic.
// The DPP source lane has no successor for lane 63, which then keeps the `old` operand; keeping the
// select inside the DPP matters: a separate `l == 63 ? tail : dpp(x)` can be turned into an
// exec-masked branch, and a DPP move reading from a lane masked off returns the old value instead.
__device__ __forceinline__ uint32_t lane_next(uint32_t x, uint32_t tail = 0) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)tail, (int)x, 0x130, 0xf, 0xf, false);
}
// set bits of the 64-bit lane mask m below this lane (v_mbcnt_lo / _hi: two VALU, no 64-bit shifts)
__device__ __forceinline__ int32_t bits_below(uint64_t m) {
    return (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// value of lane `src` (any lane index 0..63 per lane): ds_bpermute, no LDS allocation
__device__ __forceinline__ int32_t lane_get(int32_t x, int32_t src) {
    return __builtin_amdgcn_ds_bpermute(src << 2, x);
}

}  // namespace covt

#endif
