// covt_assemble.hip -- gfx950 geometry assembly: decoded GeometryColumn streams -> GeoArrow-style
// nested offsets + flat coordinates (include/covt.h, "Geometry assembly").
//
// Reference: CovtParser.convertGeometryColumn (CovtParser.java:135-274) walks the features of a
// column once, consuming the count streams (geometryOffsets / partOffsets / ringOffsets) and the
// vertex stream (vertexBuffer, or vertexBuffer[2*vertexOffsets[i]] for ICE columns through
// getICELineString :537-550) in order, and builds JTS objects.  Here one wave64 assembles one
// column in four streaming passes, each a wave-wide segmented expansion with carried bases:
//
//   1. features: P_f = multi ? geometryOffsets[rank of f among MULTI*] : 1
//                -> geometry_offsets = exclusive scan of P_f
//   2. parts:    feature of each part by expanding geometry_offsets; R_p = polygon part ?
//                partOffsets[rank among po-consuming parts] : 1  -> part_offsets; a per-part scratch
//                word keeps the vertex count of a point / line part
//   3. rings:    part of each ring by expanding part_offsets; V_r = polygon ring ?
//                ringOffsets[rank among polygon rings] (+1 closing vertex unless the stream has it)
//                : scratch count -> ring_offsets; a per-ring scratch word keeps the ring's first
//                source-vertex index and its closing flag
//   4. vertices: ring of each coordinate by expanding ring_offsets; source vertex = first + rank
//                (the closing coordinate repeats the first); ICE: through vertexOffsets; gather
//                the x,y pair.
//
// The expansion (`Expand`): output items are processed 256 at a time, four consecutive ones per
// lane; the 256 segment ends after the carried segment base are loaded (four per lane) into LDS,
// each end marks its position in a 256-slot LDS table (the last of equal ends wins), and a running
// max over the table (in-lane over four slots, then a DPP wave scan) gives each item the number of
// segments that end at or before it -- its segment index; the segment's start and end come from
// the LDS copy of the ends.  Empty segments cost nothing extra; a step consumes 256 items or 256
// segments, so every wave reaches its exit.  Four items per lane give each wave four independent
// gathers in flight per dependent step (the passes are latency-bound chains of gathers).
// Pass 4 skips the expansion when the column inserts no closing vertex (ICE rings of Gen C, line
// and point layers): coordinate v is then source vertex v.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"
#include "covt_internal.h"
#include "covt_scratch.h"
#include "covt_wave.h"

namespace covt {

#ifndef COVT_ASM_WAVES
#define COVT_ASM_WAVES 1
#endif
constexpr int kAsmWaves = COVT_ASM_WAVES;  // independent waves (columns) per workgroup
// Small batches (at most kCoopMaxColumns columns: one tile's latency, BASELINE config 1): a column's
// passes are chains of dependent gathers, one step per 256 items on one wave (the config-1 tile's
// 35k-feature, 72k-coordinate line column: ~700 steps, 0.78 ms).  Columns of at least kSplitMinItems
// features / parts / rings / coordinates are cut into chunks of one 4 x 64 x kCoopWaves-item step each,
// run by as many workgroups at once (the split passes below); the rest by single waves as in a batch.
constexpr int kCoopWaves = 16;
constexpr int kCoopMaxColumns = 4096;
constexpr int32_t kSplitMinItems = 512;

typedef __attribute__((address_space(1))) const int32_t g_i32;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const uint8_t g_u8;
typedef __attribute__((address_space(1))) const uint64_t g_u64;
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const i32x4 g_i32x4;

template <int NW, int IPL = 4>
struct __attribute__((aligned(16))) AsmSmemT {
    int32_t slot[IPL * 64 * NW];  // expansion: segment-end marks of the current step
    int32_t ends[IPL * 64 * NW];  // expansion: the step's segment ends
    uint32_t red[2][NW];          // cooperative scans / reductions: per-wave totals (two buffers)
};
// Items of a step per thread.  A single wave holds its items LANE-MAJOR (item k of lane l is step item
// 64 k + l): every load and store instruction of the passes then covers 64 consecutive items (256 bytes
// of int32), where four consecutive items per lane spread each instruction over 1 KiB -- the batch
// assembly is bound by the texture address unit's per-line work (TA busy 87 % of the kernel, issue
// stalls 31 % of wave time; 8 consecutive items per lane: 2 KiB per instruction, 3.82 -> 5.35 ms).
// A cooperative group (NW > 1, the split passes) keeps IPL consecutive items per thread.
#ifndef COVT_ASM_IPL
#define COVT_ASM_IPL 8
#endif
// single waves: the step's count window (the next K PartOffsets / RingOffsets entries from the rank
// base) loaded with the step's own loads and picked from LDS by rank, instead of a load that waits on
// the rank scan
#ifndef COVT_ASM_WIN
#define COVT_ASM_WIN 1
#endif
#ifndef COVT_ASM_NT  // pass 4: single-use loads (vertexOffsets, a plain column's vertices) nontemporal
#define COVT_ASM_NT 1
#endif
constexpr int kAsmIpl = COVT_ASM_IPL;
typedef AsmSmemT<1, kAsmIpl> AsmSmem;

// The threads assembling one column: a wave (NW = 1: lane_id, wave primitives, no barrier) or a whole
// workgroup of NW waves (thread index, per-wave partials through LDS and workgroup barriers).  Items
// of a step: IPL consecutive per thread, K = 64 IPL NW per step.
template <int NW, int IPL = 4>
struct Coop {
    static constexpr int K = IPL * 64 * NW;
    __device__ __forceinline__ static int tid() { return NW == 1 ? lane_id() : (int)threadIdx.x; }
    __device__ __forceinline__ static int wid() { return NW == 1 ? 0 : (int)(threadIdx.x >> 6); }
    __device__ __forceinline__ static void sync() {
        if (NW == 1) wave_sync();
        else __syncthreads();
    }
    __device__ __forceinline__ static bool any(bool p) { return NW == 1 ? __ballot(p) != 0ull : __syncthreads_or(p) != 0; }
    // exclusive prefix of a per-thread value over the group (wave inclusive `inc` given, saturating),
    // group total.  Sums saturate at 0xffffffff: every count is checked against a capacity below 2^31, so
    // a saturated total fails the check, where a wrapped one could pass it (a 4096-item cooperative step
    // of clamped counts can reach 2^32).  A saturated prefix is only ever stored for a failing column.
    template <int I>
    __device__ __forceinline__ static uint32_t group_prefix(AsmSmemT<NW, I>& sm, uint32_t inc, uint32_t own,
                                                           uint32_t& tot, int buf) {
        if (NW == 1) {
            tot = lane_bcast(inc, 63);
            return inc - own;
        }
        if (lane_id() == 63) sm.red[buf][wid()] = inc;
        __syncthreads();
        uint32_t pre = 0, all = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const uint32_t t = sm.red[buf][i];
            pre = add_sat(pre, i < wid() ? t : 0u);
            all = add_sat(all, t);
        }
        tot = all;
        return add_sat(pre, inc - own);
    }
};

__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) {  // lane l - 1's value (lane 0: 0), DPP wave_shr:1
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);
}

// exclusive scan of the step's items held IPL per thread (items IPL t .. IPL t + IPL - 1); `tot` gets the
// uniform total.  Cooperative groups alternate the two partial buffers (each buffer is rewritten only after
// a barrier that follows every read of its previous contents).
template <int NW, int IPL>
__device__ __forceinline__ void excl_scan4(AsmSmemT<NW, IPL>& sm, int& buf, const uint32_t (&x)[IPL], uint32_t (&ex)[IPL],
                                           uint32_t& tot) {
    if (NW == 1) {  // lane-major items: a wave scan per row of 64, rows carried in order
        uint32_t carry = 0;
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            const uint32_t inc = incl_scan_sat(x[k]);
            ex[k] = add_sat(carry, inc - x[k]);
            carry = add_sat(carry, lane_bcast(inc, 63));
        }
        tot = carry;
        buf ^= 1;
        return;
    }
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < IPL; ++k) s = add_sat(s, x[k]);  // saturating: see group_prefix
    const uint32_t inc = incl_scan_sat(s);
    uint32_t run = Coop<NW, IPL>::group_prefix(sm, inc, s, tot, buf);
    buf ^= 1;
#pragma unroll
    for (int k = 0; k < IPL; ++k) {
        ex[k] = run;
        run = add_sat(run, x[k]);
    }
}

// items q + IPL l + k (k < IPL) of a step of L: 16-byte stores when the lane's items are valid and
// aligned (arrays are 16-byte aligned; aligned when q % 4 == 0), else element stores
template <int NW, int IPL>
__device__ __forceinline__ void store4(int32_t* a, int32_t q, int32_t L, const uint32_t (&v)[IPL]) {
    if (NW == 1) {  // lane-major: each store 64 consecutive items
#pragma unroll
        for (int k = 0; k < IPL; ++k)
            if (64 * k + lane_id() < L) a[q + 64 * k + lane_id()] = (int32_t)v[k];
        return;
    }
    const int32_t i0 = IPL * Coop<NW, IPL>::tid();
    if ((q & 3) == 0 && i0 + IPL <= L) {
#pragma unroll
        for (int k = 0; k < IPL; k += 4)
            *(i32x4*)(a + q + i0 + k) = i32x4{(int32_t)v[k], (int32_t)v[k + 1], (int32_t)v[k + 2], (int32_t)v[k + 3]};
    } else {
#pragma unroll
        for (int k = 0; k < IPL; ++k)
            if (i0 + k < L) a[q + i0 + k] = (int32_t)v[k];
    }
}
// coordinates (8 bytes each): 16-byte nontemporal stores for aligned valid items
template <int NW, int IPL>
__device__ __forceinline__ void store4_xy(uint64_t* a, int32_t q, int32_t L, const uint64_t (&v)[IPL]) {
    if (NW == 1) {  // lane-major: each store 64 consecutive coordinates (512 bytes)
#pragma unroll
        for (int k = 0; k < IPL; ++k)
            if (64 * k + lane_id() < L) __builtin_nontemporal_store(v[k], a + q + 64 * k + lane_id());
        return;
    }
    const int32_t i0 = IPL * Coop<NW, IPL>::tid();
    if ((q & 3) == 0 && i0 + IPL <= L) {
        i32x4* p = (i32x4*)(a + q + i0);
#pragma unroll
        for (int k = 0; k < IPL; k += 2)
            __builtin_nontemporal_store(
                i32x4{(int32_t)v[k], (int32_t)(v[k] >> 32), (int32_t)v[k + 1], (int32_t)(v[k + 1] >> 32)}, p + k / 2);
    } else {
#pragma unroll
        for (int k = 0; k < IPL; ++k)
            if (i0 + k < L) a[q + i0 + k] = v[k];
    }
}

// Segmented expansion cursor over O[0..S] (nondecreasing, O[0] = 0, O[S] = total), uniform over the
// group.  A step covers up to K items, thread t the IPL items q + IPL t + k.
template <int NW, int IPL = 4>
struct Expand {
    static constexpr int K = Coop<NW, IPL>::K;
    const int32_t* O;
    int32_t S, total;
    int32_t base;   // segment index with O[base] <= q
    int32_t obase;  // O[base]
    int32_t q;      // first item of the next step

    // one step: L items (uniform); item k of the thread (valid if IPL t + k < L) gets its segment, the
    // segment's start and end
    __device__ __forceinline__ int32_t step(AsmSmemT<NW, IPL>& sm, int& buf, int32_t (&seg)[IPL], int32_t (&start)[IPL],
                                            int32_t (&end)[IPL]) {
        if (NW == 1) return step_lm(sm, seg, start, end);
        const int t = Coop<NW, IPL>::tid();
        int32_t e[IPL];
        const int32_t j0 = base + 1 + IPL * t;  // ends of segments base + 1 + IPL t + k
        if (j0 + IPL - 1 <= S) {  // 16-byte loads (4-byte aligned)
            typedef int32_t i32x4u __attribute__((ext_vector_type(4), aligned(4)));
#pragma unroll
            for (int k = 0; k < IPL; k += 4) {
                const i32x4u w = *(const __attribute__((address_space(1))) i32x4u*)(O + j0 + k);
                e[k] = w.x, e[k + 1] = w.y, e[k + 2] = w.z, e[k + 3] = w.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < IPL; ++k) e[k] = j0 + k <= S ? ((const g_i32*)O)[j0 + k] : 0x7fffffff;
        }
#pragma unroll
        for (int k = 0; k < IPL; k += 4) {
            *(i32x4*)&sm.ends[IPL * t + k] = i32x4{e[k], e[k + 1], e[k + 2], e[k + 3]};
            *(i32x4*)&sm.slot[IPL * t + k] = i32x4{0, 0, 0, 0};
        }
        Coop<NW, IPL>::sync();
        int32_t r[IPL + 1];
#pragma unroll
        for (int k = 0; k < IPL; ++k) r[k] = max(e[k] - q, 0);  // item offset where segment base+2+IPL t+k starts
        if (NW == 1) r[IPL] = (int32_t)lane_next((uint32_t)r[0], 0x7fffffffu);
        else r[IPL] = IPL * t + IPL < K ? max(sm.ends[IPL * t + IPL] - q, 0) : 0x7fffffff;
#pragma unroll
        for (int k = 0; k < IPL; ++k)
            if (r[k] < K && r[k + 1] != r[k]) sm.slot[r[k]] = IPL * t + k + 1;  // the last of equal ends wins
        Coop<NW, IPL>::sync();
        uint32_t m[IPL];
#pragma unroll
        for (int k = 0; k < IPL; k += 4) {
            const i32x4 sl = *(const i32x4*)&sm.slot[IPL * t + k];
            m[k] = k ? max(m[k - 1], (uint32_t)sl.x) : (uint32_t)sl.x;
            m[k + 1] = max(m[k], (uint32_t)sl.y);
            m[k + 2] = max(m[k + 1], (uint32_t)sl.z);
            m[k + 3] = max(m[k + 2], (uint32_t)sl.w);
        }
        const uint32_t wincl = incl_max_scan(m[IPL - 1]);
        uint32_t prev = wave_shr1(wincl);
        if (NW > 1) {  // the maximum over the lower waves' marks
            if (lane_id() == 63) sm.red[buf][Coop<NW, IPL>::wid()] = wincl;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NW; ++i)
                if (i < Coop<NW, IPL>::wid()) prev = max(prev, sm.red[buf][i]);
            buf ^= 1;
        }
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            const int32_t cnt = (int32_t)max(prev, m[k]);  // segment ends <= q + IPL t + k
            start[k] = cnt == 0 ? obase : sm.ends[cnt - 1];
            end[k] = sm.ends[min(cnt, K - 1)];
            seg[k] = base + cnt;
        }
        // items this step: at most K, the rest of the column, and what the K loaded ends cover
        int32_t L = min(K, total - q);
        if (base + K < S) L = min(L, (NW == 1 ? (int32_t)lane_bcast((uint32_t)e[IPL - 1], 63) : sm.ends[K - 1]) - q);
        L = max(L, 0);
        int adv = 0;  // segments ending at or before the next q
#pragma unroll
        for (int k = 0; k < IPL; ++k) adv += __popcll(__ballot(e[k] <= q + L));
        if (NW > 1) {
            uint32_t tot;
            (void)Coop<NW, IPL>::group_prefix(sm, lane_id() == 63 ? (uint32_t)adv : 0u, 0u, tot, buf);
            buf ^= 1;
            adv = (int)tot;
        }
        const int32_t nob = adv > 0 ? uni(sm.ends[adv - 1]) : obase;
        Coop<NW, IPL>::sync();
        obase = nob;
        base += adv;
        q += L;
        return L;
    }

    // the single-wave step, items lane-major (item k of lane l: step item 64 k + l; segment base + 1 + 64 k + l
    // ends at ends[64 k + l])
    __device__ __forceinline__ int32_t step_lm(AsmSmemT<NW, IPL>& sm, int32_t (&seg)[IPL], int32_t (&start)[IPL],
                                               int32_t (&end)[IPL]) {
        const int l = lane_id();
        int32_t e[IPL], r[IPL];
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            const int32_t j = base + 1 + 64 * k + l;
            e[k] = j <= S ? ((const g_i32*)O)[j] : 0x7fffffff;
        }
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            sm.ends[64 * k + l] = e[k];
            sm.slot[64 * k + l] = 0;
            r[k] = max(e[k] - q, 0);  // item offset where segment base + 2 + 64 k + l starts
        }
        wave_sync();
#pragma unroll
        for (int k = 0; k < IPL; ++k) {  // the last of equal ends marks (the next segment's end: lane l + 1)
            const uint32_t tail = k + 1 < IPL ? lane_bcast((uint32_t)r[k + 1 < IPL ? k + 1 : k], 0) : 0x7fffffffu;
            const int32_t rn = (int32_t)lane_next((uint32_t)r[k], tail);
            if (r[k] < K && rn != r[k]) sm.slot[r[k]] = 64 * k + l + 1;
        }
        wave_sync();
        uint32_t carry = 0;
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            const uint32_t m = max(incl_max_scan((uint32_t)sm.slot[64 * k + l]), carry);  // segment ends <= item
            carry = lane_bcast(m, 63);
            const int32_t cnt = (int32_t)m;
            start[k] = cnt == 0 ? obase : sm.ends[cnt - 1];
            end[k] = sm.ends[min(cnt, K - 1)];
            seg[k] = base + cnt;
        }
        int32_t L = min(K, total - q);
        if (base + K < S) L = min(L, (int32_t)lane_bcast((uint32_t)e[IPL - 1], 63) - q);
        L = max(L, 0);
        int adv = 0;
#pragma unroll
        for (int k = 0; k < IPL; ++k) adv += __popcll(__ballot(e[k] <= q + L));
        const int32_t nob = adv > 0 ? uni(sm.ends[adv - 1]) : obase;
        wave_sync();
        obase = nob;
        base += adv;
        q += L;
        return L;
    }
};

template <int NW>
__device__ __forceinline__ void mem_publish() {  // the group's global stores visible to its own loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (NW > 1) __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int NW, int IPL = 4>
__device__ void assemble_column(const uint8_t* __restrict__ dec, const covt_stream_result* __restrict__ dres,
                                const covt_geom_desc& d, uint8_t* __restrict__ outb, covt_geom_result& res,
                                AsmSmemT<NW, IPL>& sm) {
    constexpr int K = Coop<NW, IPL>::K;
    const int l = Coop<NW, IPL>::tid();
    // step item of this thread's k-th item: lane-major for a wave, IPL consecutive per thread for a group
    auto ioff = [&](int k) { return NW == 1 ? 64 * k + l : IPL * l + k; };
    int buf = 0;  // cooperative partials buffer (see excl_scan4)
    res.num_parts = res.num_rings = res.num_coords = 0;
    if ((uint32_t)d.flags & COVT_GEOM_TOO_LARGE) { res.status = COVT_ERR_INVALID_ARG; return; }
    for (int k = 0; k < 6; ++k) {  // a failed source stream fails the column
        const int32_t ri = d.in_res[k];
        if (ri >= 0) {
            const int32_t st = uni(dres[ri].status);
            if (st) { res.status = st; return; }
        }
    }
    const uint8_t* types = dec + d.in_off[0];
    const int32_t* go = (const int32_t*)(dec + d.in_off[1]);
    const int32_t* po = (const int32_t*)(dec + d.in_off[2]);
    const int32_t* ro = (const int32_t*)(dec + d.in_off[3]);
    const int32_t* vo = (const int32_t*)(dec + d.in_off[4]);
    const uint64_t* vb = (const uint64_t*)(dec + d.in_off[5]);  // x,y pairs
    const int32_t n = d.in_off[0] >= 0 ? d.in_len[0] : 0;
    const int32_t n_go = d.in_off[1] >= 0 ? d.in_len[1] : 0;
    const int32_t n_po = d.in_off[2] >= 0 ? d.in_len[2] : 0;
    const int32_t n_ro = d.in_off[3] >= 0 ? d.in_len[3] : 0;
    const bool ice = d.in_off[4] >= 0;
    const int32_t n_vo = ice ? d.in_len[4] : 0;
    const int32_t n_vb = d.in_off[5] >= 0 ? d.in_len[5] : 0;
    const int32_t n_src = ice ? n_vo : n_vb;  // source vertices the rings can consume
    const bool closed = d.flags & COVT_GEOM_CLOSED_IN_STREAM;
    int32_t* geo_off = (int32_t*)(outb + d.out_off[0]);
    int32_t* part_off = (int32_t*)(outb + d.out_off[1]);
    int32_t* ring_off = (int32_t*)(outb + d.out_off[2]);
    uint64_t* coords = (uint64_t*)(outb + d.out_off[3]);
    int32_t* part_scr = (int32_t*)(outb + d.out_off[4]);
    int32_t* ring_scr = (int32_t*)(outb + d.out_off[5]);
    const uint32_t pcap = (uint32_t)d.part_cap, rcap = (uint32_t)d.ring_cap, ccap = (uint32_t)d.coord_cap;
    bool bad_type = false, bad_cnt = false;

    // ---- pass 1: features -> parts (items: features) ----
    uint32_t go_base = 0, P = 0;
    bool multi_n = false;   // some feature's part count is not 1
    bool has_poly = false;  // some feature is a polygon or multi-polygon
    for (int32_t f0 = 0; f0 < n; f0 += K) {
        uint32_t t[IPL], multi[IPL], gi[IPL], pf[IPL], ex[IPL], nm, tot;
        if (NW == 1) {  // lane-major: one byte per item
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const bool valid = f0 + ioff(k) < n;
                t[k] = valid ? (uint32_t)((const g_u8*)types)[f0 + ioff(k)] : 0u;
                bad_type |= t[k] > 5u;
                has_poly |= t[k] == 2u || t[k] == 5u;
                multi[k] = (valid && t[k] >= 3u && t[k] <= 5u) ? 1u : 0u;
                pf[k] = valid ? 1u : 0u;
            }
        } else {
            const int32_t fl = f0 + IPL * l;  // this thread's first feature; types are 16-byte aligned
            const uint32_t tw = fl < n ? ((const g_u32*)types)[fl >> 2] : 0u;
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const bool valid = fl + k < n;
                t[k] = valid ? (tw >> (8 * k)) & 0xffu : 0u;
                bad_type |= t[k] > 5u;
                has_poly |= t[k] == 2u || t[k] == 5u;
                multi[k] = (valid && t[k] >= 3u && t[k] <= 5u) ? 1u : 0u;
                pf[k] = valid ? 1u : 0u;
            }
        }
        excl_scan4(sm, buf, multi, gi, nm);
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            if (multi[k]) {
                const uint32_t i = go_base + gi[k];
                if (i < (uint32_t)n_go) {
                    const int32_t c = ((const g_i32*)go)[i];
                    bad_cnt |= c < 0;
                    pf[k] = min((uint32_t)max(c, 0), pcap + 1u);  // clamped, and the scans saturate (group_prefix)
                } else {
                    bad_cnt = true;
                }
            }
        }
        excl_scan4(sm, buf, pf, ex, tot);
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            ex[k] += P;
            multi_n |= multi[k] && pf[k] != 1u;
        }
        store4<NW>(geo_off, f0, n - f0, ex);
        go_base += nm;
        P = add_sat(P, tot);
        if (Coop<NW>::any(bad_type || bad_cnt) || P > pcap) break;
    }
    if (Coop<NW>::any(bad_type)) { res.status = COVT_ERR_BAD_HEADER; return; }  // GeometryType.values()[b]
    if (Coop<NW>::any(bad_cnt) || P > pcap) { res.status = COVT_ERR_COUNT_MISMATCH; return; }
    if (l == 0) geo_off[n] = (int32_t)P;
    mem_publish<NW>();

#if defined(COVT_ASM_PASSES) && COVT_ASM_PASSES < 2  // ablation build: stop here
    res.status = COVT_OK;
    return;
#endif
    // a pass whose segments all hold one item: item i is segment i
    auto ident_step = [&](Expand<NW, IPL>& x, int32_t (&sg)[IPL]) {
        const int32_t L = min(K, x.total - x.q);
#pragma unroll
        for (int k = 0; k < IPL; ++k) sg[k] = x.q + ioff(k);
        x.q += L;
        return L;
    };
    const bool ident2 = !Coop<NW>::any(multi_n);
    // no polygon: every part is one ring (rings = parts), so pass 2 also writes the ring offsets (the
    // exclusive scan of the parts' vertex counts) and pass 3, with both scratch arrays, is skipped
    const bool nopoly = !Coop<NW>::any(has_poly);
    uint32_t V = 0, VS = 0;
    // ---- pass 2: parts -> rings (items: parts, segments: features) ----
    uint32_t po_base = 0, R = 0;
    bool poly_n = false;  // some part's ring count is not 1
    {
        Expand<NW, IPL> x{geo_off, n, (int32_t)P, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t p0 = x.q;
            int32_t f[IPL], fs[IPL], fe[IPL], pw[IPL];
            constexpr bool kWin = NW == 1 && COVT_ASM_WIN;
            if (kWin) {
#pragma unroll
                for (int k = 0; k < IPL; ++k) {
                    const uint32_t i = po_base + (uint32_t)ioff(k);
                    pw[k] = i < (uint32_t)n_po ? ((const g_i32*)po)[i] : 0;
                }
            }
            // one part per feature (no multi-geometry with a count other than 1): part p is feature p, no
            // expansion (most columns; the step's loads, marks and scans are half of the pass)
            const int32_t L = ident2 ? ident_step(x, f) : x.step(sm, buf, f, fs, fe);
            uint32_t t[IPL], usep[IPL], pi[IPL], rp[IPL], scr[IPL], ex[IPL], npo, tot;
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const bool valid = ioff(k) < L;
                t[k] = valid ? (uint32_t)((const g_u8*)types)[f[k]] : 0u;
                usep[k] = (valid && t[k] != 0u && t[k] != 3u) ? 1u : 0u;  // line and polygon parts
            }
            excl_scan4(sm, buf, usep, pi, npo);
            if (kWin) {  // (the step's expansion is done with the LDS tables)
                wave_sync();
#pragma unroll
                for (int k = 0; k < IPL; ++k) sm.slot[ioff(k)] = pw[k];
                wave_sync();
            }
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const bool valid = ioff(k) < L;
                uint32_t c = 0;
                if (usep[k]) {
                    const uint32_t i = po_base + pi[k];
                    if (i < (uint32_t)n_po) {
                        const int32_t v = kWin ? sm.slot[pi[k]] : ((const g_i32*)po)[i];
                        bad_cnt |= v < 0;
                        c = min((uint32_t)max(v, 0), rcap + 1u);
                    } else {
                        bad_cnt = true;
                    }
                }
                const bool poly = t[k] == 2u || t[k] == 5u;
                rp[k] = valid ? (poly ? c : 1u) : 0u;
                const uint32_t vcount = (t[k] == 1u || t[k] == 4u) ? c : 1u;  // vertices of a line / point part
                scr[k] = poly ? 1u : (min(vcount, ccap + 1u) << 1);
            }
            excl_scan4(sm, buf, rp, ex, tot);
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                ex[k] += R;
                poly_n |= ioff(k) < L && rp[k] != 1u;
            }
            store4<NW>(part_off, p0, L, ex);
            if (nopoly) {  // ring p = part p: its coordinates start at the scan of the vertex counts
                uint32_t vc[IPL], vex[IPL], vt;
#pragma unroll
                for (int k = 0; k < IPL; ++k) vc[k] = ioff(k) < L ? scr[k] >> 1 : 0u;
                excl_scan4(sm, buf, vc, vex, vt);
#pragma unroll
                for (int k = 0; k < IPL; ++k) vex[k] += V;
                store4<NW>(ring_off, p0, L, vex);
                V = add_sat(V, vt);
            } else {
                store4<NW>(part_scr, p0, L, scr);
            }
            po_base += npo;
            R = add_sat(R, tot);
            if (Coop<NW>::any(bad_cnt) || R > rcap || (nopoly && V > ccap)) break;
        }
    }
    if (Coop<NW>::any(bad_cnt) || R > rcap) { res.status = COVT_ERR_COUNT_MISMATCH; return; }
    if (l == 0) part_off[P] = (int32_t)R;
    mem_publish<NW>();

#if defined(COVT_ASM_PASSES) && COVT_ASM_PASSES < 3  // ablation build: stop here
    res.status = COVT_OK;
    return;
#endif
    const bool ident3 = !Coop<NW>::any(poly_n);
    // ---- pass 3: rings -> coordinates (items: rings, segments: parts) ----
    uint32_t ro_base = 0;
    if (nopoly) {
        VS = V;  // (no closing vertex; the checks of pass 3's end)
    } else {
        Expand<NW, IPL> x{part_off, (int32_t)P, (int32_t)R, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t r0 = x.q;
            int32_t p[IPL], ps[IPL], pe[IPL], rw[IPL];
            constexpr bool kWin = NW == 1 && COVT_ASM_WIN;
            if (kWin) {
#pragma unroll
                for (int k = 0; k < IPL; ++k) {
                    const uint32_t i = ro_base + (uint32_t)ioff(k);
                    rw[k] = i < (uint32_t)n_ro ? ((const g_i32*)ro)[i] : 0;
                }
            }
            const int32_t L = ident3 ? ident_step(x, p) : x.step(sm, buf, p, ps, pe);  // (one ring per part)
            uint32_t poly[IPL], ri[IPL], vs[IPL], vo_[IPL], ex[IPL], src[IPL], nr, tv, ts;
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const bool valid = ioff(k) < L;
                const int32_t sp = valid ? ((const g_i32*)part_scr)[p[k]] : 0;
                poly[k] = (valid && (sp & 1)) ? 1u : 0u;
                vs[k] = valid ? (uint32_t)sp >> 1 : 0u;
            }
            excl_scan4(sm, buf, poly, ri, nr);
            if (kWin) {
                wave_sync();
#pragma unroll
                for (int k = 0; k < IPL; ++k) sm.slot[ioff(k)] = rw[k];
                wave_sync();
            }
            uint32_t closing[IPL];
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                if (poly[k]) {
                    const uint32_t i = ro_base + ri[k];
                    if (i < (uint32_t)n_ro) {
                        const int32_t v = kWin ? sm.slot[ri[k]] : ((const g_i32*)ro)[i];
                        bad_cnt |= v < 0;
                        vs[k] = min((uint32_t)max(v, 0), ccap + 1u);
                    } else {
                        bad_cnt = true;
                    }
                }
                closing[k] = (poly[k] && !closed && vs[k] > 0u) ? 1u : 0u;
                vo_[k] = vs[k] + closing[k];
            }
            excl_scan4(sm, buf, vo_, ex, tv);
            excl_scan4(sm, buf, vs, src, ts);
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                ex[k] += V;
                src[k] = (VS + src[k]) | (closing[k] << 31);
            }
            store4<NW>(ring_off, r0, L, ex);
            if (!closed) store4<NW>(ring_scr, r0, L, src);  // (read by pass 4 only when rings get a closing vertex)
            ro_base += nr;
            V = add_sat(V, tv);
            VS = add_sat(VS, ts);
            if (Coop<NW>::any(bad_cnt) || V > ccap || VS > (uint32_t)n_src) break;
        }
    }
    if (Coop<NW>::any(bad_cnt) || V > ccap || VS > (uint32_t)n_src) { res.status = COVT_ERR_COUNT_MISMATCH; return; }
    if (l == 0) ring_off[R] = (int32_t)V;
    mem_publish<NW>();

#if defined(COVT_ASM_PASSES) && COVT_ASM_PASSES < 4  // ablation build: stop here
    res.status = COVT_OK;
    return;
#endif
    // ---- pass 4: coordinates (ICE gather) ----
    bool bad_idx = false;
    if (V == VS) {
        // no closing vertex to insert: coordinate v is source vertex v (a straight copy / gather).  Two
        // steps per iteration, their index loads and gathers issued before any store (stores may alias
        // the loads as far as the compiler knows, so a one-step loop waits out every chain in turn)
        auto idx4 = [&](int32_t i0, int32_t (&idx)[IPL]) {
            if (ice && i0 + IPL <= (int32_t)V) {  // vertexOffsets are 16-byte aligned, i0 % 4 == 0
#pragma unroll
                for (int k = 0; k < IPL; k += 4) {
                    const i32x4 w = *(const g_i32x4*)(vo + i0 + k);
                    idx[k] = w.x; idx[k + 1] = w.y; idx[k + 2] = w.z; idx[k + 3] = w.w;
                }
            } else {
#pragma unroll
                for (int k = 0; k < IPL; ++k)
                    idx[k] = i0 + k < (int32_t)V ? (ice ? ((const g_i32*)vo)[i0 + k] : i0 + k) : 0;
            }
        };
        auto gather4 = [&](int32_t i0, const int32_t (&idx)[IPL], uint64_t (&xy)[IPL]) {
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const bool valid = i0 + k < (int32_t)V;
                const bool inr = (uint32_t)idx[k] < (uint32_t)n_vb;
                bad_idx |= valid && !inr;
                xy[k] = (valid && inr) ? ((const g_u64*)vb)[idx[k]] : 0ull;
            }
        };
        if (NW == 1) {  // lane-major: two steps per iteration, every instruction 64 consecutive coordinates
            for (int32_t v0 = 0; v0 < (int32_t)V; v0 += 2 * K) {
                int32_t ia[2 * IPL];
#pragma unroll
                for (int k = 0; k < 2 * IPL; ++k) {
                    const int32_t i = v0 + 64 * k + l;
                    // (vertexOffsets are read once: streamed past L2, which keeps the dictionary the gathers reuse)
                    ia[k] = i < (int32_t)V ? (ice ? (COVT_ASM_NT ? __builtin_nontemporal_load(vo + i) : ((const g_i32*)vo)[i]) : i) : 0;
                }
                uint64_t xa[2 * IPL];
#pragma unroll
                for (int k = 0; k < 2 * IPL; ++k) {
                    const bool valid = v0 + 64 * k + l < (int32_t)V;
                    const bool inr = (uint32_t)ia[k] < (uint32_t)n_vb;
                    bad_idx |= valid && !inr;
                    // (a plain column's vertices are copied once: streamed too; an ICE dictionary is gathered ~2.7
                    // times per vertex and stays cached)
                    xa[k] = (valid && inr) ? ((COVT_ASM_NT && !ice) ? __builtin_nontemporal_load(vb + ia[k]) : ((const g_u64*)vb)[ia[k]]) : 0ull;
                }
#pragma unroll
                for (int k = 0; k < 2 * IPL; ++k)
                    if (v0 + 64 * k + l < (int32_t)V) __builtin_nontemporal_store(xa[k], coords + v0 + 64 * k + l);
            }
        } else {
            for (int32_t v0 = 0; v0 < (int32_t)V; v0 += 2 * K) {
                const int32_t i0 = v0 + IPL * l, i1 = i0 + K;
                int32_t ia[IPL], ib[IPL];
                idx4(i0, ia);
                idx4(i1, ib);
                uint64_t xa[IPL], xb[IPL];
                gather4(i0, ia, xa);
                gather4(i1, ib, xb);
                store4_xy<NW>(coords, v0, (int32_t)V - v0, xa);
                if (v0 + K < (int32_t)V) store4_xy<NW>(coords, v0 + K, (int32_t)V - v0 - K, xb);
            }
        }
    } else {
        Expand<NW, IPL> x{ring_off, (int32_t)R, (int32_t)V, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t v0 = x.q;
            int32_t r[IPL], rs[IPL], re[IPL];
            const int32_t L = x.step(sm, buf, r, rs, re);
            uint64_t xy[IPL];
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const int32_t v = v0 + ioff(k);
                const bool valid = ioff(k) < L;
                const uint32_t sr = valid ? (uint32_t)((const g_i32*)ring_scr)[r[k]] : 0u;
                const int32_t first = (int32_t)(sr & 0x7fffffffu);
                const int32_t src = ((sr >> 31) && v == re[k] - 1) ? first : first + (v - rs[k]);
                const int32_t idx = valid ? (ice ? ((const g_i32*)vo)[src] : src) : 0;
                const bool inr = (uint32_t)idx < (uint32_t)n_vb;
                bad_idx |= valid && !inr;  // vertexBuffer[offset] out of range (ArrayIndexOutOfBounds)
                xy[k] = (valid && inr) ? ((const g_u64*)vb)[idx] : 0ull;
            }
            store4_xy<NW>(coords, v0, L, xy);
        }
    }
    if (Coop<NW>::any(bad_idx)) { res.status = COVT_ERR_TRUNCATED; return; }
    res.status = COVT_OK;
    res.num_parts = (int32_t)P;
    res.num_rings = (int32_t)R;
    res.num_coords = (int32_t)V;
}

// the items a column's passes step over (features, parts, rings, coordinates): its capacities
__device__ __forceinline__ int32_t column_items(const covt_geom_desc& d) {
    const int32_t n = d.in_off[0] >= 0 ? d.in_len[0] : 0;
    return max(max(n, d.part_cap), max(d.ring_cap, d.coord_cap));
}

// one wave per column (large batches: every wave has a column, the batch keeps the chip busy)
__global__ __launch_bounds__(64 * kAsmWaves) void assemble_kernel(const uint8_t* __restrict__ dec,
                                                                  const covt_stream_result* __restrict__ dres,
                                                                  const covt_geom_desc* __restrict__ descs,
                                                                  int64_t n_cols, uint8_t* __restrict__ outb,
                                                                  covt_geom_result* __restrict__ gres) {
    __shared__ AsmSmem smem[kAsmWaves];
    const int w = threadIdx.x >> 6;
    const int64_t c = uni64((int64_t)blockIdx.x * kAsmWaves + w);
    if (c >= n_cols) return;
    const covt_geom_desc d = descs[c];
    covt_geom_result r{COVT_OK, 0, 0, 0};
    assemble_column<1, kAsmIpl>(dec, dres, d, outb, r, smem[w]);
    if (lane_id() == 0) gres[c] = r;
}

// ---- multi-workgroup columns (small batches: one tile's latency, BASELINE config 1) -------------------
// A whole workgroup still walks a big column's passes one 4,096-item step at a time (the config-1 tile's
// 35k-feature line column: ~45 dependent steps, ~190 us).  Here each pass is a kernel of its own and the
// column's items are cut into chunks of kSplitK (one workgroup step each) that run on different
// workgroups at once:
//   * the scans that carry state from one chunk to the next (rank among MULTI* features / polygon parts /
//     polygon rings, and the parts / rings / coordinates before the chunk) are a publish-and-gather: a
//     chunk publishes its own total, then sums its predecessors' published totals (one load per
//     predecessor, all in flight together; chunks take tickets in order, so a chunk only waits on chunks
//     that started before it);
//   * each pass leaves, for every chunk of the next pass, the segment that chunk's first item falls in
//     (a segment -- a feature / part / ring -- containing a chunk boundary writes it), so the next pass's
//     expansion starts mid-column without a search;
//   * a check that fails marks the column with the lowest (pass, chunk) that failed, as the single-
//     workgroup walk stops at its first failing step (same step size, same status); later passes skip a
//     marked column.
// The last chunk of pass 4 to finish writes the column's result.
constexpr int kSplitK = Coop<kCoopWaves>::K;  // items per chunk: one cooperative step
constexpr int kSplitMaxChunks = 65536;         // per pass over all split columns (past it: single waves)
constexpr int kSplitGrid = 256;                // persistent workgroups per pass kernel (tickets)
constexpr uint32_t kSplitMaxSpins = 1u << 22;  // look-back polls (~seconds) before a column is failed

struct SplitCol {
    unsigned long long fail;  // min over failures of (stage << 56 | chunk << 32 | -status); ~0: none
    uint32_t P, R, V, VS;     // totals, written by the last chunk of passes 1 (P), 2 (R), 3 (V, VS)
    uint32_t done4;           // pass-4 chunks finished
    uint32_t pad;
};
// Per (device, stream) scratch of the split passes.  The look-back records carry the launch's epoch in
// their high half (a record of an earlier launch reads as "not yet"), so nothing is cleared per launch.
struct SplitScratch {
    uint32_t ticket[4];                       // next ticket of pass p
    int32_t n_split, n_small;                 // split columns; columns left to single waves
    uint32_t epoch;                           // this launch's record tag, advanced by split_prep (never 0)
    int32_t pad;
    int32_t pre[4][kCoopMaxColumns + 1];      // pass p: chunks of split columns before column k
    int32_t col[kCoopMaxColumns];             // split column k -> batch column
    int32_t small[kCoopMaxColumns];           // the other columns (single waves, pass 1's workgroups)
    SplitCol st[kCoopMaxColumns];
    int2 base[4][kSplitMaxChunks];            // pass p (1..3) chunk: (segment, segment start) of its first item
    unsigned long long rec[4][3][kSplitMaxChunks];  // pass p, scan s, chunk: (epoch << 32 | total)
};

// chunks per pass of a column: ceil(capacity / kSplitK) (chunks past the pass's real item count exit)
__device__ __forceinline__ void split_chunks(const covt_geom_desc& d, int32_t (&c)[4]) {
    const int32_t n = d.in_off[0] >= 0 ? d.in_len[0] : 0;
    c[0] = max(1, (n + kSplitK - 1) / kSplitK);  // at least one chunk: chunk 0 writes the terminal offset
    c[1] = max(1, (d.part_cap + kSplitK - 1) / kSplitK);
    c[2] = max(1, (d.ring_cap + kSplitK - 1) / kSplitK);
    c[3] = max(1, (d.coord_cap + kSplitK - 1) / kSplitK);
}

// exclusive prefix over a 1024-thread workgroup of NV int32 values per thread (DPP wave scans, the 16
// wave totals through LDS); tot gets the workgroup totals
template <int NV>
__device__ __forceinline__ void wg_excl_scan(int32_t (&x)[NV], int32_t (&tot)[NV], int32_t (*lds)[16]) {
    const int w = threadIdx.x >> 6;
    uint32_t inc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        inc[v] = incl_scan((uint32_t)x[v]);
        if (lane_id() == 63) lds[v][w] = (int32_t)inc[v];
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        int32_t pre = 0, all = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int32_t t = lds[v][i];
            pre += i < w ? t : 0;
            all += t;
        }
        x[v] = pre + (int32_t)inc[v] - x[v];
        tot[v] = all;
    }
    __syncthreads();
}

// One workgroup: the columns of at least split_min items (not too large) become split columns, in batch
// order while every pass keeps within kSplitMaxChunks; the others go to the small list (single waves)
__global__ __launch_bounds__(1024) void split_prep(const covt_geom_desc* __restrict__ descs, int64_t n_cols,
                                                   int32_t split_min, SplitScratch* __restrict__ sc) {
    __shared__ int32_t lds[6][16];
    const int t = threadIdx.x;
    int32_t ch[4][4] = {};
    bool want[4] = {}, live[4] = {};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t c = 4 * t + k;
        live[k] = c < n_cols;
        if (live[k]) {
            const covt_geom_desc d = descs[c];
            if (column_items(d) >= split_min && !((uint32_t)d.flags & COVT_GEOM_TOO_LARGE)) {
                split_chunks(d, ch[k]);
                want[k] = true;
            }
        }
    }
    // the budget: a thread whose running chunk totals pass kSplitMaxChunks splits none of its columns
    int32_t x[6], tot[6];
#pragma unroll
    for (int p = 0; p < 4; ++p) x[p] = ch[0][p] + ch[1][p] + ch[2][p] + ch[3][p];
    x[4] = x[5] = 0;
    int32_t own[4] = {x[0], x[1], x[2], x[3]};
    wg_excl_scan<6>(x, tot, lds);
    bool fits = true;
#pragma unroll
    for (int p = 0; p < 4; ++p) fits = fits && x[p] + own[p] <= kSplitMaxChunks;
    bool keep[4];
    int32_t nsplit = 0, nsmall = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        keep[k] = fits && want[k];
        nsplit += keep[k] ? 1 : 0;
        nsmall += (live[k] && !keep[k]) ? 1 : 0;
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) x[p] = keep[0] * ch[0][p] + keep[1] * ch[1][p] + keep[2] * ch[2][p] + keep[3] * ch[3][p];
    x[4] = nsplit;
    x[5] = nsmall;
    wg_excl_scan<6>(x, tot, lds);
    int32_t run[4] = {x[0], x[1], x[2], x[3]}, idx = x[4], sidx = x[5];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t c = 4 * t + k;
        if (!live[k]) continue;
        if (!keep[k]) {
            sc->small[sidx++] = (int32_t)c;
            continue;
        }
        sc->col[idx] = (int32_t)c;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            sc->pre[p][idx] = run[p];
            run[p] += ch[k][p];
        }
        sc->st[idx] = SplitCol{~0ull, 0, 0, 0, 0, 0, 0};
        ++idx;
    }
    if (t == 0) {
        sc->n_split = tot[4];
        sc->n_small = tot[5];
        // a new tag for this launch's look-back records, kept in device memory so that a captured graph
        // replays with a fresh one (epoch 0, the zeroed scratch's, is never used)
        const uint32_t e = sc->epoch + 1u;
        sc->epoch = e ? e : 1u;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            sc->pre[p][tot[4]] = tot[p];
            sc->ticket[p] = 0;
        }
    }
}

__device__ __forceinline__ unsigned long long ld_acq(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// publish this chunk's totals of NS scans (records rec[s][j]), then the sums of chunks [0, j) of each
// (saturating; every thread gets them).  Chunks of a column are consecutive record slots from `g0`.
template <int NS>
__device__ __forceinline__ void split_gather(AsmSmemT<kCoopWaves>& sm, unsigned long long (*rec)[kSplitMaxChunks],
                                             int32_t g0, int32_t j, const uint32_t (&own)[NS], uint32_t (&pre)[NS],
                                             uint32_t epoch) {
    if (threadIdx.x == 0)
        for (int s = 0; s < NS; ++s) st_rel(&rec[s][g0 + j], ((unsigned long long)epoch << 32) | own[s]);
    uint32_t acc[NS];
    for (int s = 0; s < NS; ++s) acc[s] = 0;
    bool lost = false;
    for (int32_t i = threadIdx.x; i < j; i += 1024) {
        for (int s = 0; s < NS; ++s) {
            unsigned long long v;
            // bounded wait: a predecessor that never publishes (a bug, not an input property) fails the
            // column instead of hanging the launch
            uint32_t spins = 0;
            while ((uint32_t)((v = ld_acq(&rec[s][g0 + i])) >> 32) != epoch && ++spins < kSplitMaxSpins)
                __builtin_amdgcn_s_sleep(2);
            lost |= (uint32_t)(v >> 32) != epoch;
            acc[s] = add_sat(acc[s], (uint32_t)v);
        }
    }
    if (__syncthreads_or(lost)) {
        for (int s = 0; s < NS; ++s) acc[s] = 0xffffffffu;  // saturated: every capacity check fails
    }
    // workgroup sums: DPP wave sums, then the 16 wave partials through LDS (one buffer per scan)
    __syncthreads();
    for (int s = 0; s < NS; ++s) {
        const uint32_t w = lane_bcast(incl_scan_sat(acc[s]), 63);
        if (lane_id() == 0) sm.slot[16 * s + (threadIdx.x >> 6)] = (int32_t)w;
    }
    __syncthreads();
    for (int s = 0; s < NS; ++s) {
        uint32_t tot = 0;
#pragma unroll
        for (int i = 0; i < kCoopWaves; ++i) tot = add_sat(tot, (uint32_t)sm.slot[16 * s + i]);
        pre[s] = tot;
    }
    __syncthreads();
}

// the column's first failure wins (stage = pass, then chunk); status < 0
__device__ __forceinline__ void split_fail(SplitCol& st, int stage, int32_t chunk, int32_t status) {
    const unsigned long long key = ((unsigned long long)stage << 56) | ((unsigned long long)(uint32_t)chunk << 32) |
                                   (uint32_t)(-status);
    atomicMin(&st.fail, key);
}
// failed in an earlier pass (a failure of this pass is only acted on by the chunk that found it: a later
// chunk that skipped its gather would leave the chunks after it waiting)
__device__ __forceinline__ bool split_failed_before(const SplitCol& st, int pass) {
    return (ld_acq(&st.fail) >> 56) < (unsigned long long)pass;
}

// segments whose item range [s, s + len) contains chunk boundaries b * kSplitK (b < nch) record
// themselves for those chunks of the next pass
__device__ __forceinline__ void split_bases(int2* __restrict__ base, int32_t nch, int32_t seg, uint32_t s, uint32_t len) {
    if (len == 0) return;
    const uint32_t e = s + len;  // (no wrap: checked against the capacity before this is called)
    for (uint32_t b = (s + kSplitK - 1) / kSplitK; b * (uint32_t)kSplitK < e && (int32_t)b < nch; ++b)
        base[b] = make_int2(seg, (int32_t)s);
}

// one chunk of one pass of split column k (global chunk g of the pass)
template <int PASS>
__device__ void split_chunk(const uint8_t* __restrict__ dec, const covt_stream_result* __restrict__ dres,
                            const covt_geom_desc& d, uint8_t* __restrict__ outb, SplitScratch* __restrict__ sc,
                            int32_t k, int32_t j, AsmSmemT<kCoopWaves>& sm, covt_geom_result* __restrict__ gres,
                            int32_t c, uint32_t epoch) {
    constexpr int NW = kCoopWaves, K = kSplitK;
    const int l = threadIdx.x;
    int buf = 0;
    SplitCol& st = sc->st[k];
    const int32_t g0 = sc->pre[PASS - 1][k];  // this column's first chunk slot in the pass
    const uint8_t* types = dec + d.in_off[0];
    const int32_t* go = (const int32_t*)(dec + d.in_off[1]);
    const int32_t* po = (const int32_t*)(dec + d.in_off[2]);
    const int32_t* ro = (const int32_t*)(dec + d.in_off[3]);
    const int32_t* vo = (const int32_t*)(dec + d.in_off[4]);
    const uint64_t* vb = (const uint64_t*)(dec + d.in_off[5]);
    const int32_t n = d.in_off[0] >= 0 ? d.in_len[0] : 0;
    const int32_t n_go = d.in_off[1] >= 0 ? d.in_len[1] : 0;
    const int32_t n_po = d.in_off[2] >= 0 ? d.in_len[2] : 0;
    const int32_t n_ro = d.in_off[3] >= 0 ? d.in_len[3] : 0;
    const bool ice = d.in_off[4] >= 0;
    const int32_t n_vo = ice ? d.in_len[4] : 0;
    const int32_t n_vb = d.in_off[5] >= 0 ? d.in_len[5] : 0;
    const int32_t n_src = ice ? n_vo : n_vb;
    const bool closed = d.flags & COVT_GEOM_CLOSED_IN_STREAM;
    int32_t* geo_off = (int32_t*)(outb + d.out_off[0]);
    int32_t* part_off = (int32_t*)(outb + d.out_off[1]);
    int32_t* ring_off = (int32_t*)(outb + d.out_off[2]);
    uint64_t* coords = (uint64_t*)(outb + d.out_off[3]);
    int32_t* part_scr = (int32_t*)(outb + d.out_off[4]);
    int32_t* ring_scr = (int32_t*)(outb + d.out_off[5]);
    const uint32_t pcap = (uint32_t)d.part_cap, rcap = (uint32_t)d.ring_cap, ccap = (uint32_t)d.coord_cap;
    int32_t nch[4];
    split_chunks(d, nch);
    const int32_t q0 = j * K;

    if constexpr (PASS == 1) {
        if (j == 0) {  // a failed source stream fails the column (assemble_column's first check)
            for (int s = 0; s < 6; ++s) {
                const int32_t ri = d.in_res[s];
                const int32_t stt = ri >= 0 ? dres[ri].status : 0;
                if (stt) {
                    if (l == 0) split_fail(st, 0, 0, stt);
                    break;
                }
            }
        }
        bool src_bad = false;
        for (int s = 0; s < 6; ++s) src_bad |= d.in_res[s] >= 0 && dres[d.in_res[s]].status != 0;
        if (src_bad) return;  // (uniform)
        if (q0 >= n) {  // no features (n == 0, chunk 0): no parts
            if (l == 0) geo_off[0] = 0;
            return;
        }
        const int32_t fl = q0 + 4 * l;
        const uint32_t tw = fl < n ? ((const g_u32*)types)[fl >> 2] : 0u;
        uint32_t t[4], multi[4], gi[4], pf[4], ex[4], nm, tot;
        bool bad_type = false, bad_cnt = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool valid = fl + q < n;
            t[q] = valid ? (tw >> (8 * q)) & 0xffu : 0u;
            bad_type |= t[q] > 5u;
            multi[q] = (valid && t[q] >= 3u && t[q] <= 5u) ? 1u : 0u;
            pf[q] = valid ? 1u : 0u;
        }
        excl_scan4(sm, buf, multi, gi, nm);
        uint32_t own1[1] = {nm}, pre1[1];
        split_gather<1>(sm, sc->rec[0], g0, j, own1, pre1, epoch);
        const uint32_t go_base = pre1[0];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (multi[q]) {
                const uint32_t i = add_sat(go_base, gi[q]);
                if (i < (uint32_t)n_go) {
                    const int32_t cc = ((const g_i32*)go)[i];
                    bad_cnt |= cc < 0;
                    pf[q] = min((uint32_t)max(cc, 0), pcap + 1u);
                } else {
                    bad_cnt = true;
                }
            }
        }
        excl_scan4(sm, buf, pf, ex, tot);
        uint32_t own2[1] = {tot}, pre2[1];
        split_gather<1>(sm, sc->rec[0] + 1, g0, j, own2, pre2, epoch);
        const uint32_t P0 = pre2[0], P1 = add_sat(P0, tot);
        const bool any_type = __syncthreads_or(bad_type), any_cnt = __syncthreads_or(bad_cnt);
        if (any_type || any_cnt || P1 > pcap) {
            if (l == 0) split_fail(st, 1, j, any_type ? COVT_ERR_BAD_HEADER : COVT_ERR_COUNT_MISMATCH);
            return;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) ex[q] += P0;
        store4<NW>(geo_off, q0, n - q0, ex);
        int2* base = sc->base[1] + sc->pre[1][k];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (fl + q < n) split_bases(base, nch[1], fl + q, ex[q], pf[q]);
        if (q0 + K >= n && l == 0) {  // the last chunk: the column's part count
            geo_off[n] = (int32_t)P1;
            st.P = P1;
        }
    } else if constexpr (PASS == 2) {
        if (split_failed_before(st, 2)) return;
        const uint32_t P = st.P;
        if ((uint32_t)q0 >= P) {
            if (j == 0 && l == 0) part_off[0] = 0;  // no parts: no rings
            return;
        }
        const int32_t q1 = (int32_t)min((uint32_t)(q0 + K), P);
        const int2 b0 = sc->base[1][sc->pre[1][k] + j];
        // sweep A: the features of the chunk's parts -> the chunk's count of partOffsets-consuming parts
        Expand<NW> x{geo_off, n, q1, b0.x, b0.y, q0};
        const Expand<NW> x0 = x;
        uint32_t usep_all = 0;
        int32_t f[4], fs[4], fe[4], L = 0;
        bool one_step = true;
        uint32_t t[4], usep[4], pi[4], npo = 0;
        while (x.q < q1) {
            L = x.step(sm, buf, f, fs, fe);
            one_step = one_step && x.q >= q1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool valid = 4 * l + q < L;
                t[q] = valid ? (uint32_t)((const g_u8*)types)[f[q]] : 0u;
                usep[q] = (valid && t[q] != 0u && t[q] != 3u) ? 1u : 0u;
            }
            uint32_t stot;
            excl_scan4(sm, buf, usep, pi, stot);
            usep_all = add_sat(usep_all, stot);
        }
        npo = usep_all;
        uint32_t own1[1] = {npo}, pre1[1];
        split_gather<1>(sm, sc->rec[1], g0, j, own1, pre1, epoch);
        uint32_t po_base = pre1[0];
        // sweep B: the ring counts (re-expanding only if the chunk took more than one step)
        uint32_t R0 = 0, Rrun = 0;
        bool bad_cnt = false;
        int2* base = sc->base[2] + sc->pre[2][k];
        // pass 2 has a second chained scan (rings before the chunk): gather it from the first sweep's ring
        // totals is not possible (ring counts need po_base), so sweep B computes the totals, publishes,
        // and stores after the gather (registers hold a single step; longer chunks redo the expansion)
        uint32_t rp[4], scr[4], ex[4], tot = 0, rtot = 0;
        auto ring_counts = [&](const uint32_t (&tt)[4], const uint32_t (&us)[4], const uint32_t (&pix)[4], int32_t LL,
                               uint32_t pob) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool valid = 4 * l + q < LL;
                uint32_t cc = 0;
                if (us[q]) {
                    const uint32_t i = add_sat(pob, pix[q]);
                    if (i < (uint32_t)n_po) {
                        const int32_t v = ((const g_i32*)po)[i];
                        bad_cnt |= v < 0;
                        cc = min((uint32_t)max(v, 0), rcap + 1u);
                    } else {
                        bad_cnt = true;
                    }
                }
                const bool poly = tt[q] == 2u || tt[q] == 5u;
                rp[q] = valid ? (poly ? cc : 1u) : 0u;
                const uint32_t vcount = (tt[q] == 1u || tt[q] == 4u) ? cc : 1u;
                scr[q] = poly ? 1u : (min(vcount, ccap + 1u) << 1);
            }
        };
        if (one_step) {
            ring_counts(t, usep, pi, L, po_base);
            excl_scan4(sm, buf, rp, ex, tot);
            uint32_t own2[1] = {tot}, pre2[1];
            split_gather<1>(sm, sc->rec[1] + 1, g0, j, own2, pre2, epoch);
            R0 = pre2[0];
            Rrun = add_sat(R0, tot);
            const bool any_cnt = __syncthreads_or(bad_cnt);
            if (any_cnt || Rrun > rcap) {
                if (l == 0) split_fail(st, 2, j, COVT_ERR_COUNT_MISMATCH);
                return;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) ex[q] += R0;
            store4<NW>(part_off, q0, L, ex);
            store4<NW>(part_scr, q0, L, scr);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (4 * l + q < L) split_bases(base, nch[2], q0 + 4 * l + q, ex[q], rp[q]);
        } else {
            // several steps: first their ring totals (no stores), then the gather, then the stores
            x = x0;
            uint32_t pob = po_base;
            while (x.q < q1) {
                L = x.step(sm, buf, f, fs, fe);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool valid = 4 * l + q < L;
                    t[q] = valid ? (uint32_t)((const g_u8*)types)[f[q]] : 0u;
                    usep[q] = (valid && t[q] != 0u && t[q] != 3u) ? 1u : 0u;
                }
                uint32_t stot;
                excl_scan4(sm, buf, usep, pi, stot);
                ring_counts(t, usep, pi, L, pob);
                excl_scan4(sm, buf, rp, ex, tot);
                rtot = add_sat(rtot, tot);
                pob = add_sat(pob, stot);
            }
            uint32_t own2[1] = {rtot}, pre2[1];
            split_gather<1>(sm, sc->rec[1] + 1, g0, j, own2, pre2, epoch);
            R0 = pre2[0];
            Rrun = add_sat(R0, rtot);
            const bool any_cnt = __syncthreads_or(bad_cnt);
            if (any_cnt || Rrun > rcap) {
                if (l == 0) split_fail(st, 2, j, COVT_ERR_COUNT_MISMATCH);
                return;
            }
            x = x0;
            pob = po_base;
            uint32_t R = R0;
            while (x.q < q1) {
                const int32_t p0 = x.q;
                L = x.step(sm, buf, f, fs, fe);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool valid = 4 * l + q < L;
                    t[q] = valid ? (uint32_t)((const g_u8*)types)[f[q]] : 0u;
                    usep[q] = (valid && t[q] != 0u && t[q] != 3u) ? 1u : 0u;
                }
                uint32_t stot;
                excl_scan4(sm, buf, usep, pi, stot);
                ring_counts(t, usep, pi, L, pob);
                excl_scan4(sm, buf, rp, ex, tot);
#pragma unroll
                for (int q = 0; q < 4; ++q) ex[q] += R;
                store4<NW>(part_off, p0, L, ex);
                store4<NW>(part_scr, p0, L, scr);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (4 * l + q < L) split_bases(base, nch[2], p0 + 4 * l + q, ex[q], rp[q]);
                R = add_sat(R, tot);
                pob = add_sat(pob, stot);
            }
        }
        if (q1 == (int32_t)P && l == 0) {  // the last chunk: the column's ring count
            part_off[P] = (int32_t)Rrun;
            st.R = Rrun;
        }
    } else if constexpr (PASS == 3) {
        if (split_failed_before(st, 3)) return;
        const uint32_t P = st.P, R = st.R;
        if ((uint32_t)q0 >= R) {
            if (j == 0 && l == 0) ring_off[0] = 0;  // no rings: no coordinates
            return;
        }
        const int32_t q1 = (int32_t)min((uint32_t)(q0 + K), R);
        const int2 b0 = sc->base[2][sc->pre[2][k] + j];
        Expand<NW> x{part_off, (int32_t)P, q1, b0.x, b0.y, q0};
        const Expand<NW> x0 = x;
        // sweep A: polygon rings of the chunk (the ringOffsets rank)
        uint32_t npoly = 0;
        int32_t p[4], ps[4], pe[4], L = 0;
        uint32_t poly[4], ri[4], vs[4];
        bool one_step = true;
        while (x.q < q1) {
            L = x.step(sm, buf, p, ps, pe);
            one_step = one_step && x.q >= q1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool valid = 4 * l + q < L;
                const int32_t sp = valid ? ((const g_i32*)part_scr)[p[q]] : 0;
                poly[q] = (valid && (sp & 1)) ? 1u : 0u;
                vs[q] = valid ? (uint32_t)sp >> 1 : 0u;
            }
            uint32_t stot;
            excl_scan4(sm, buf, poly, ri, stot);
            npoly = add_sat(npoly, stot);
        }
        uint32_t own1[1] = {npoly}, pre1[1];
        split_gather<1>(sm, sc->rec[2], g0, j, own1, pre1, epoch);
        const uint32_t ro_base = pre1[0];
        bool bad_cnt = false;
        uint32_t closing[4], vo_[4], ex[4], src[4], tv = 0, ts = 0;
        auto vertex_counts = [&](uint32_t rob) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (poly[q]) {
                    const uint32_t i = add_sat(rob, ri[q]);
                    if (i < (uint32_t)n_ro) {
                        const int32_t v = ((const g_i32*)ro)[i];
                        bad_cnt |= v < 0;
                        vs[q] = min((uint32_t)max(v, 0), ccap + 1u);
                    } else {
                        bad_cnt = true;
                    }
                }
                closing[q] = (poly[q] && !closed && vs[q] > 0u) ? 1u : 0u;
                vo_[q] = vs[q] + closing[q];
            }
        };
        auto reload = [&](int32_t LL) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool valid = 4 * l + q < LL;
                const int32_t sp = valid ? ((const g_i32*)part_scr)[p[q]] : 0;
                poly[q] = (valid && (sp & 1)) ? 1u : 0u;
                vs[q] = valid ? (uint32_t)sp >> 1 : 0u;
            }
        };
        int2* base = sc->base[3] + sc->pre[3][k];
        uint32_t V0, VS0, V1, VS1;
        if (one_step) {
            vertex_counts(ro_base);
            excl_scan4(sm, buf, vo_, ex, tv);
            excl_scan4(sm, buf, vs, src, ts);
        } else {
            x = x0;
            uint32_t rob = ro_base;
            while (x.q < q1) {
                L = x.step(sm, buf, p, ps, pe);
                reload(L);
                uint32_t stot;
                excl_scan4(sm, buf, poly, ri, stot);
                vertex_counts(rob);
                uint32_t a, b;
                excl_scan4(sm, buf, vo_, ex, a);
                excl_scan4(sm, buf, vs, src, b);
                tv = add_sat(tv, a);
                ts = add_sat(ts, b);
                rob = add_sat(rob, stot);
            }
        }
        uint32_t own2[2] = {tv, ts}, pre2[2];
        split_gather<2>(sm, sc->rec[2] + 1, g0, j, own2, pre2, epoch);
        V0 = pre2[0];
        VS0 = pre2[1];
        V1 = add_sat(V0, tv);
        VS1 = add_sat(VS0, ts);
        const bool any_cnt = __syncthreads_or(bad_cnt);
        if (any_cnt || V1 > ccap || VS1 > (uint32_t)n_src) {
            if (l == 0) split_fail(st, 3, j, COVT_ERR_COUNT_MISMATCH);
            return;
        }
        auto store_rings = [&](int32_t r0, int32_t LL, uint32_t Vb, uint32_t VSb) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                ex[q] += Vb;
                src[q] = (VSb + src[q]) | (closing[q] << 31);
            }
            store4<NW>(ring_off, r0, LL, ex);
            store4<NW>(ring_scr, r0, LL, src);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (4 * l + q < LL) split_bases(base, nch[3], r0 + 4 * l + q, ex[q], vo_[q]);
        };
        if (one_step) {
            store_rings(q0, L, V0, VS0);
        } else {
            x = x0;
            uint32_t rob = ro_base, Vb = V0, VSb = VS0;
            while (x.q < q1) {
                const int32_t r0 = x.q;
                L = x.step(sm, buf, p, ps, pe);
                reload(L);
                uint32_t stot;
                excl_scan4(sm, buf, poly, ri, stot);
                vertex_counts(rob);
                uint32_t a, b;
                excl_scan4(sm, buf, vo_, ex, a);
                excl_scan4(sm, buf, vs, src, b);
                store_rings(r0, L, Vb, VSb);
                Vb = add_sat(Vb, a);
                VSb = add_sat(VSb, b);
                rob = add_sat(rob, stot);
            }
        }
        if (q1 == (int32_t)R && l == 0) {  // the last chunk: the column's coordinate counts
            ring_off[R] = (int32_t)V1;
            st.V = V1;
            st.VS = VS1;
        }
    } else {  // PASS 4: coordinates
        bool bad_idx = false;
        if (!split_failed_before(st, 4)) {
            const uint32_t R = st.R, V = st.V, VS = st.VS;
            if ((uint32_t)q0 < V) {
                const int32_t q1 = (int32_t)min((uint32_t)(q0 + K), V);
                if (V == VS) {  // straight gather: coordinate v is source vertex v
                    const int32_t i0 = q0 + 4 * l;
                    int32_t idx[4];
                    if (ice && i0 + 4 <= q1) {
                        const i32x4 w = *(const g_i32x4*)(vo + i0);
                        idx[0] = w.x; idx[1] = w.y; idx[2] = w.z; idx[3] = w.w;
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; ++q) idx[q] = i0 + q < q1 ? (ice ? ((const g_i32*)vo)[i0 + q] : i0 + q) : 0;
                    }
                    uint64_t xy[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const bool valid = i0 + q < q1;
                        const bool inr = (uint32_t)idx[q] < (uint32_t)n_vb;
                        bad_idx |= valid && !inr;
                        xy[q] = (valid && inr) ? ((const g_u64*)vb)[idx[q]] : 0ull;
                    }
                    store4_xy<NW>(coords, q0, q1 - q0, xy);
                } else {
                    const int2 b0 = sc->base[3][sc->pre[3][k] + j];
                    Expand<NW> x{ring_off, (int32_t)R, q1, b0.x, b0.y, q0};
                    while (x.q < q1) {
                        const int32_t v0 = x.q;
                        int32_t r[4], rs[4], re[4];
                        const int32_t L = x.step(sm, buf, r, rs, re);
                        uint64_t xy[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int32_t v = v0 + 4 * l + q;
                            const bool valid = 4 * l + q < L;
                            const uint32_t sr = valid ? (uint32_t)((const g_i32*)ring_scr)[r[q]] : 0u;
                            const int32_t first = (int32_t)(sr & 0x7fffffffu);
                            const int32_t s = ((sr >> 31) && v == re[q] - 1) ? first : first + (v - rs[q]);
                            const int32_t idx = valid ? (ice ? ((const g_i32*)vo)[s] : s) : 0;
                            const bool inr = (uint32_t)idx < (uint32_t)n_vb;
                            bad_idx |= valid && !inr;
                            xy[q] = (valid && inr) ? ((const g_u64*)vb)[idx] : 0ull;
                        }
                        store4_xy<NW>(coords, v0, L, xy);
                    }
                }
            }
        }
        if (__syncthreads_or(bad_idx) && l == 0) split_fail(st, 4, j, COVT_ERR_TRUNCATED);
        // the column's last pass-4 chunk to finish writes its result
        __syncthreads();
        if (l == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const uint32_t done = atomicAdd(&st.done4, 1u) + 1u;
            if (done == (uint32_t)nch[3]) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                const unsigned long long fk = ld_acq(&st.fail);
                covt_geom_result r{COVT_OK, 0, 0, 0};
                if (fk != ~0ull) {
                    r.status = -(int32_t)(uint32_t)(fk & 0xffffffffu);
                } else {
                    r.num_parts = (int32_t)st.P;
                    r.num_rings = (int32_t)st.R;
                    r.num_coords = (int32_t)st.V;
                }
                gres[c] = r;
            }
        }
    }
}

// pass PASS over every split column: workgroups take chunks by ticket (a chunk waits only on chunks of
// its column with lower tickets, all already running) until the pass has none left; pass 1's workgroups
// then take the small columns, sixteen per ticket, one wave each (their four passes on that wave)
template <int PASS>
__global__ __launch_bounds__(64 * kCoopWaves) void split_pass_kernel(const uint8_t* __restrict__ dec,
                                                                     const covt_stream_result* __restrict__ dres,
                                                                     const covt_geom_desc* __restrict__ descs,
                                                                     uint8_t* __restrict__ outb,
                                                                     covt_geom_result* __restrict__ gres,
                                                                     SplitScratch* __restrict__ sc) {
    __shared__ union U {
        AsmSmemT<kCoopWaves> coop;
        AsmSmem wave[kCoopWaves];
    } smem;
    __shared__ int32_t lpre[kCoopMaxColumns + 1];  // the pass's chunk prefixes (binary search in LDS)
    __shared__ int32_t tk;
    const int32_t ns = sc->n_split;
    const int32_t total = sc->pre[PASS - 1][ns];
    const uint32_t epoch = sc->epoch;  // (split_prep, earlier on this stream)
    const int32_t small_groups = PASS == 1 ? (sc->n_small + kCoopWaves - 1) / kCoopWaves : 0;
    for (int32_t i = threadIdx.x; i <= ns; i += 64 * kCoopWaves) lpre[i] = sc->pre[PASS - 1][i];
    __syncthreads();
    for (;;) {
        if (threadIdx.x == 0) tk = (int32_t)atomicAdd(&sc->ticket[PASS - 1], 1u);
        __syncthreads();
        const int32_t g = tk;
        __syncthreads();
        if (g >= total) {
            if (PASS != 1 || g >= total + small_groups) return;
            const int w = threadIdx.x >> 6;
            const int32_t si = (g - total) * kCoopWaves + w;
            if (si < sc->n_small) {  // (wave-uniform)
                const int32_t c = uni(sc->small[si]);
                const covt_geom_desc d = descs[c];
                covt_geom_result r{COVT_OK, 0, 0, 0};
                assemble_column<1>(dec, dres, d, outb, r, smem.wave[w]);
                if (lane_id() == 0) gres[c] = r;
            }
            __syncthreads();
            continue;
        }
        // the split column holding chunk g: the last k with lpre[k] <= g
        int32_t lo = 0, hi = ns;  // lpre[lo] <= g < lpre[hi]
        while (hi - lo > 1) {
            const int32_t mid = (lo + hi) >> 1;
            if (lpre[mid] <= g) lo = mid;
            else hi = mid;
        }
        const int32_t k = lo, j = g - lpre[k], c = sc->col[k];
        const covt_geom_desc d = descs[c];
        split_chunk<PASS>(dec, dres, d, outb, sc, k, j, smem.coop, gres, c, epoch);
        __syncthreads();
    }
}

}  // namespace covt

namespace covt {
// split-pass scratch, one per (device, stream) (covt_scratch.h)
StreamScratch& assembly_scratch() {
    static StreamScratch m(sizeof(SplitScratch));
    return m;
}
}  // namespace covt

extern "C" int covt_assemble_geometry_device(const uint8_t* d_decoded, const covt_stream_result* d_res,
                                             const covt_geom_desc* d_gdesc, int64_t n_columns, uint8_t* d_asm,
                                             covt_geom_result* d_gres, void* hip_stream) {
    if (n_columns < 0 || (n_columns && (!d_decoded || !d_res || !d_gdesc || !d_asm || !d_gres)))
        return COVT_ERR_INVALID_ARG;
    if (n_columns == 0) return COVT_OK;
    const int64_t blocks = (n_columns + covt::kAsmWaves - 1) / covt::kAsmWaves;
    if (blocks > 0x7fffffff) return COVT_ERR_INVALID_ARG;
    hipStream_t s = (hipStream_t)hip_stream;
    // small batches (one tile's latency): big columns by many workgroups at once (the split passes);
    // large batches: a wave per column
    const bool coop = n_columns <= covt::kCoopMaxColumns;
    if (coop) {
        // every column in the split passes' kernels: big ones chunked, the rest on single waves in pass 1
        covt::SplitScratch* sc = (covt::SplitScratch*)covt::assembly_scratch().get(s);
        if (!sc) return COVT_ERR_DEVICE;
        const dim3 wg(64 * covt::kCoopWaves);
        hipLaunchKernelGGL(covt::split_prep, dim3(1), dim3(1024), 0, s, d_gdesc, n_columns, covt::kSplitMinItems, sc);
        hipLaunchKernelGGL(covt::split_pass_kernel<1>, dim3(covt::kSplitGrid), wg, 0, s, d_decoded, d_res, d_gdesc,
                           d_asm, d_gres, sc);
        hipLaunchKernelGGL(covt::split_pass_kernel<2>, dim3(covt::kSplitGrid), wg, 0, s, d_decoded, d_res, d_gdesc,
                           d_asm, d_gres, sc);
        hipLaunchKernelGGL(covt::split_pass_kernel<3>, dim3(covt::kSplitGrid), wg, 0, s, d_decoded, d_res, d_gdesc,
                           d_asm, d_gres, sc);
        hipLaunchKernelGGL(covt::split_pass_kernel<4>, dim3(covt::kSplitGrid), wg, 0, s, d_decoded, d_res, d_gdesc,
                           d_asm, d_gres, sc);
    } else {
        hipLaunchKernelGGL(covt::assemble_kernel, dim3((unsigned)blocks), dim3(64 * covt::kAsmWaves), 0, s, d_decoded,
                           d_res, d_gdesc, n_columns, d_asm, d_gres);
    }
    return hipGetLastError() == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
}
