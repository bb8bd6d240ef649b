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
#include "covt_wave.h"

namespace covt {

#ifndef COVT_ASM_WAVES
#define COVT_ASM_WAVES 4
#endif
constexpr int kAsmWaves = COVT_ASM_WAVES;  // independent waves (columns) per workgroup
// Small batches (at most kCoopMaxColumns columns: one tile's latency, BASELINE config 1): columns with
// at least kCoopMinItems features / parts / rings / coordinates are assembled by a whole workgroup of
// kCoopWaves waves (4 x 64 x kCoopWaves items per step), the rest by single waves as in a batch.  A
// column's passes are chains of dependent gathers, one step per 256 items on one wave (the config-1
// tile's 35k-feature, 72k-coordinate line column: ~700 steps, 0.78 ms); sixteen waves take 16x fewer.
constexpr int kCoopWaves = 16;
constexpr int kCoopMaxColumns = 4096;
constexpr int32_t kCoopMinItems = 8192;

typedef __attribute__((address_space(1))) const int32_t g_i32;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const uint8_t g_u8;
typedef __attribute__((address_space(1))) const uint64_t g_u64;
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const i32x4 g_i32x4;

template <int NW>
struct __attribute__((aligned(16))) AsmSmemT {
    int32_t slot[4 * 64 * NW];  // expansion: segment-end marks of the current step
    int32_t ends[4 * 64 * NW];  // expansion: the step's segment ends
    uint32_t red[2][NW];        // cooperative scans / reductions: per-wave totals (two buffers)
};
typedef AsmSmemT<1> AsmSmem;

// The threads assembling one column: a wave (NW = 1: lane_id, wave primitives, no barrier) or a whole
// workgroup of NW waves (thread index, per-wave partials through LDS and workgroup barriers).  Items
// of a step: 4 consecutive per thread, K = 256 NW per step.
template <int NW>
struct Coop {
    static constexpr int K = 4 * 64 * NW;
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
    __device__ __forceinline__ static uint32_t group_prefix(AsmSmemT<NW>& sm, uint32_t inc, uint32_t own,
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

// exclusive scan of the step's items held 4 per thread (items 4t .. 4t+3); `tot` gets the uniform total.
// Cooperative groups alternate the two partial buffers (each buffer is rewritten only after a barrier
// that follows every read of its previous contents).
template <int NW>
__device__ __forceinline__ void excl_scan4(AsmSmemT<NW>& sm, int& buf, const uint32_t x[4], uint32_t ex[4], uint32_t& tot) {
    const uint32_t s = add_sat(add_sat(x[0], x[1]), add_sat(x[2], x[3]));  // saturating: see group_prefix
    const uint32_t inc = incl_scan_sat(s);
    uint32_t run = Coop<NW>::group_prefix(sm, inc, s, tot, buf);
    buf ^= 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        ex[k] = run;
        run = add_sat(run, x[k]);
    }
}

// items q + 4l + k (k < 4) of a step of L: one 16-byte store when the lane's four are valid and
// aligned (arrays are 16-byte aligned; aligned when q % 4 == 0), else element stores
template <int NW>
__device__ __forceinline__ void store4(int32_t* a, int32_t q, int32_t L, const uint32_t v[4]) {
    const int32_t i0 = 4 * Coop<NW>::tid();
    if ((q & 3) == 0 && i0 + 4 <= L) {
        *(i32x4*)(a + q + i0) = i32x4{(int32_t)v[0], (int32_t)v[1], (int32_t)v[2], (int32_t)v[3]};
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i0 + k < L) a[q + i0 + k] = (int32_t)v[k];
    }
}
// coordinates (8 bytes each): two 16-byte nontemporal stores for four aligned valid items
template <int NW>
__device__ __forceinline__ void store4_xy(uint64_t* a, int32_t q, int32_t L, const uint64_t v[4]) {
    const int32_t i0 = 4 * Coop<NW>::tid();
    if ((q & 3) == 0 && i0 + 4 <= L) {
        i32x4* p = (i32x4*)(a + q + i0);
        __builtin_nontemporal_store(i32x4{(int32_t)v[0], (int32_t)(v[0] >> 32), (int32_t)v[1], (int32_t)(v[1] >> 32)}, p);
        __builtin_nontemporal_store(i32x4{(int32_t)v[2], (int32_t)(v[2] >> 32), (int32_t)v[3], (int32_t)(v[3] >> 32)},
                                    p + 1);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i0 + k < L) a[q + i0 + k] = v[k];
    }
}

// Segmented expansion cursor over O[0..S] (nondecreasing, O[0] = 0, O[S] = total), uniform over the
// group.  A step covers up to K items, thread t the four items q + 4t + k.
template <int NW>
struct Expand {
    static constexpr int K = Coop<NW>::K;
    const int32_t* O;
    int32_t S, total;
    int32_t base;   // segment index with O[base] <= q
    int32_t obase;  // O[base]
    int32_t q;      // first item of the next step

    // one step: L items (uniform); item k of the thread (valid if 4t + k < L) gets its segment, the
    // segment's start and end
    __device__ __forceinline__ int32_t step(AsmSmemT<NW>& sm, int& buf, int32_t seg[4], int32_t start[4],
                                            int32_t end[4]) {
        const int t = Coop<NW>::tid();
        int32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // end of segment base + 1 + 4t + k
            const int32_t j = base + 1 + 4 * t + k;
            e[k] = j <= S ? ((const g_i32*)O)[j] : 0x7fffffff;
        }
        *(i32x4*)&sm.ends[4 * t] = i32x4{e[0], e[1], e[2], e[3]};
        *(i32x4*)&sm.slot[4 * t] = i32x4{0, 0, 0, 0};
        Coop<NW>::sync();
        int32_t r[5];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = max(e[k] - q, 0);  // item offset where segment base+2+4t+k starts
        if (NW == 1) r[4] = (int32_t)lane_next((uint32_t)r[0], 0x7fffffffu);
        else r[4] = 4 * t + 4 < K ? max(sm.ends[4 * t + 4] - q, 0) : 0x7fffffff;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (r[k] < K && r[k + 1] != r[k]) sm.slot[r[k]] = 4 * t + k + 1;  // the last of equal ends wins
        Coop<NW>::sync();
        const i32x4 sl = *(const i32x4*)&sm.slot[4 * t];
        uint32_t m[4];
        m[0] = (uint32_t)sl.x;
        m[1] = max(m[0], (uint32_t)sl.y);
        m[2] = max(m[1], (uint32_t)sl.z);
        m[3] = max(m[2], (uint32_t)sl.w);
        const uint32_t wincl = incl_max_scan(m[3]);
        uint32_t prev = wave_shr1(wincl);
        if (NW > 1) {  // the maximum over the lower waves' marks
            if (lane_id() == 63) sm.red[buf][Coop<NW>::wid()] = wincl;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NW; ++i)
                if (i < Coop<NW>::wid()) prev = max(prev, sm.red[buf][i]);
            buf ^= 1;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int32_t cnt = (int32_t)max(prev, m[k]);  // segment ends <= q + 4t + k
            start[k] = cnt == 0 ? obase : sm.ends[cnt - 1];
            end[k] = sm.ends[min(cnt, K - 1)];
            seg[k] = base + cnt;
        }
        // items this step: at most K, the rest of the column, and what the K loaded ends cover
        int32_t L = min(K, total - q);
        if (base + K < S) L = min(L, (NW == 1 ? (int32_t)lane_bcast((uint32_t)e[3], 63) : sm.ends[K - 1]) - q);
        L = max(L, 0);
        int adv = 0;  // segments ending at or before the next q
#pragma unroll
        for (int k = 0; k < 4; ++k) adv += __popcll(__ballot(e[k] <= q + L));
        if (NW > 1) {
            uint32_t tot;
            (void)Coop<NW>::group_prefix(sm, lane_id() == 63 ? (uint32_t)adv : 0u, 0u, tot, buf);
            buf ^= 1;
            adv = (int)tot;
        }
        const int32_t nob = adv > 0 ? uni(sm.ends[adv - 1]) : obase;
        Coop<NW>::sync();
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

template <int NW>
__device__ void assemble_column(const uint8_t* __restrict__ dec, const covt_stream_result* __restrict__ dres,
                                const covt_geom_desc& d, uint8_t* __restrict__ outb, covt_geom_result& res,
                                AsmSmemT<NW>& sm) {
    constexpr int K = Coop<NW>::K;
    const int l = Coop<NW>::tid();
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
    for (int32_t f0 = 0; f0 < n; f0 += K) {
        const int32_t fl = f0 + 4 * l;  // this lane's first feature; types are 16-byte aligned
        const uint32_t tw = fl < n ? ((const g_u32*)types)[fl >> 2] : 0u;
        uint32_t t[4], multi[4], gi[4], pf[4], ex[4], nm, tot;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool valid = fl + k < n;
            t[k] = valid ? (tw >> (8 * k)) & 0xffu : 0u;
            bad_type |= t[k] > 5u;
            multi[k] = (valid && t[k] >= 3u && t[k] <= 5u) ? 1u : 0u;
            pf[k] = valid ? 1u : 0u;
        }
        excl_scan4(sm, buf, multi, gi, nm);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
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
        for (int k = 0; k < 4; ++k) ex[k] += P;
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
    // ---- pass 2: parts -> rings (items: parts, segments: features) ----
    uint32_t po_base = 0, R = 0;
    {
        Expand<NW> x{geo_off, n, (int32_t)P, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t p0 = x.q;
            int32_t f[4], fs[4], fe[4];
            const int32_t L = x.step(sm, buf, f, fs, fe);
            uint32_t t[4], usep[4], pi[4], rp[4], scr[4], ex[4], npo, tot;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool valid = 4 * l + k < L;
                t[k] = valid ? (uint32_t)((const g_u8*)types)[f[k]] : 0u;
                usep[k] = (valid && t[k] != 0u && t[k] != 3u) ? 1u : 0u;  // line and polygon parts
            }
            excl_scan4(sm, buf, usep, pi, npo);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool valid = 4 * l + k < L;
                uint32_t c = 0;
                if (usep[k]) {
                    const uint32_t i = po_base + pi[k];
                    if (i < (uint32_t)n_po) {
                        const int32_t v = ((const g_i32*)po)[i];
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
            for (int k = 0; k < 4; ++k) ex[k] += R;
            store4<NW>(part_off, p0, L, ex);
            store4<NW>(part_scr, p0, L, scr);
            po_base += npo;
            R = add_sat(R, tot);
            if (Coop<NW>::any(bad_cnt) || R > rcap) break;
        }
    }
    if (Coop<NW>::any(bad_cnt) || R > rcap) { res.status = COVT_ERR_COUNT_MISMATCH; return; }
    if (l == 0) part_off[P] = (int32_t)R;
    mem_publish<NW>();

#if defined(COVT_ASM_PASSES) && COVT_ASM_PASSES < 3  // ablation build: stop here
    res.status = COVT_OK;
    return;
#endif
    // ---- pass 3: rings -> coordinates (items: rings, segments: parts) ----
    uint32_t ro_base = 0, V = 0, VS = 0;
    {
        Expand<NW> x{part_off, (int32_t)P, (int32_t)R, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t r0 = x.q;
            int32_t p[4], ps[4], pe[4];
            const int32_t L = x.step(sm, buf, p, ps, pe);
            uint32_t poly[4], ri[4], vs[4], vo_[4], ex[4], src[4], nr, tv, ts;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool valid = 4 * l + k < L;
                const int32_t sp = valid ? ((const g_i32*)part_scr)[p[k]] : 0;
                poly[k] = (valid && (sp & 1)) ? 1u : 0u;
                vs[k] = valid ? (uint32_t)sp >> 1 : 0u;
            }
            excl_scan4(sm, buf, poly, ri, nr);
            uint32_t closing[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (poly[k]) {
                    const uint32_t i = ro_base + ri[k];
                    if (i < (uint32_t)n_ro) {
                        const int32_t v = ((const g_i32*)ro)[i];
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
            for (int k = 0; k < 4; ++k) {
                ex[k] += V;
                src[k] = (VS + src[k]) | (closing[k] << 31);
            }
            store4<NW>(ring_off, r0, L, ex);
            store4<NW>(ring_scr, r0, L, src);
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
        auto idx4 = [&](int32_t i0, int32_t (&idx)[4]) {
            if (ice && i0 + 4 <= (int32_t)V) {  // vertexOffsets are 16-byte aligned, i0 % 4 == 0
                const i32x4 w = *(const g_i32x4*)(vo + i0);
                idx[0] = w.x; idx[1] = w.y; idx[2] = w.z; idx[3] = w.w;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    idx[k] = i0 + k < (int32_t)V ? (ice ? ((const g_i32*)vo)[i0 + k] : i0 + k) : 0;
            }
        };
        auto gather4 = [&](int32_t i0, const int32_t (&idx)[4], uint64_t (&xy)[4]) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool valid = i0 + k < (int32_t)V;
                const bool inr = (uint32_t)idx[k] < (uint32_t)n_vb;
                bad_idx |= valid && !inr;
                xy[k] = (valid && inr) ? ((const g_u64*)vb)[idx[k]] : 0ull;
            }
        };
        for (int32_t v0 = 0; v0 < (int32_t)V; v0 += 2 * K) {
            const int32_t i0 = v0 + 4 * l, i1 = i0 + K;
            int32_t ia[4], ib[4];
            idx4(i0, ia);
            idx4(i1, ib);
            uint64_t xa[4], xb[4];
            gather4(i0, ia, xa);
            gather4(i1, ib, xb);
            store4_xy<NW>(coords, v0, (int32_t)V - v0, xa);
            if (v0 + K < (int32_t)V) store4_xy<NW>(coords, v0 + K, (int32_t)V - v0 - K, xb);
        }
    } else {
        Expand<NW> x{ring_off, (int32_t)R, (int32_t)V, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t v0 = x.q;
            int32_t r[4], rs[4], re[4];
            const int32_t L = x.step(sm, buf, r, rs, re);
            uint64_t xy[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int32_t v = v0 + 4 * l + k;
                const bool valid = 4 * l + k < L;
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

// one wave per column; columns of at least `coop_min` items are left to assemble_coop_kernel
__global__ __launch_bounds__(64 * kAsmWaves) void assemble_kernel(const uint8_t* __restrict__ dec,
                                                                  const covt_stream_result* __restrict__ dres,
                                                                  const covt_geom_desc* __restrict__ descs,
                                                                  int64_t n_cols, uint8_t* __restrict__ outb,
                                                                  covt_geom_result* __restrict__ gres, int32_t coop_min) {
    __shared__ AsmSmem smem[kAsmWaves];
    const int w = threadIdx.x >> 6;
    const int64_t c = uni64((int64_t)blockIdx.x * kAsmWaves + w);
    if (c >= n_cols) return;
    const covt_geom_desc d = descs[c];
    if (uni(column_items(d)) >= coop_min && !((uint32_t)d.flags & COVT_GEOM_TOO_LARGE)) return;
    covt_geom_result r{COVT_OK, 0, 0, 0};
    assemble_column<1>(dec, dres, d, outb, r, smem[w]);
    if (lane_id() == 0) gres[c] = r;
}

// one workgroup of kCoopWaves waves per column of at least `coop_min` items (small batches only: the
// grid is one workgroup per column, the others return at once)
__global__ __launch_bounds__(64 * kCoopWaves) void assemble_coop_kernel(const uint8_t* __restrict__ dec,
                                                                        const covt_stream_result* __restrict__ dres,
                                                                        const covt_geom_desc* __restrict__ descs,
                                                                        int64_t n_cols, uint8_t* __restrict__ outb,
                                                                        covt_geom_result* __restrict__ gres,
                                                                        int32_t coop_min) {
    __shared__ AsmSmemT<kCoopWaves> smem;
    const int64_t c = blockIdx.x;
    if (c >= n_cols) return;
    const covt_geom_desc d = descs[c];
    if (column_items(d) < coop_min || ((uint32_t)d.flags & COVT_GEOM_TOO_LARGE)) return;  // (uniform)
    covt_geom_result r{COVT_OK, 0, 0, 0};
    assemble_column<kCoopWaves>(dec, dres, d, outb, r, smem);
    if (threadIdx.x == 0) gres[c] = r;
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
    // small batches: big columns by whole workgroups (launched first: they are the critical path)
    const bool coop = n_columns <= covt::kCoopMaxColumns;
    const int32_t coop_min = coop ? covt::kCoopMinItems : 0x7fffffff;
    if (coop)
        hipLaunchKernelGGL(covt::assemble_coop_kernel, dim3((unsigned)n_columns), dim3(64 * covt::kCoopWaves), 0,
                           (hipStream_t)hip_stream, d_decoded, d_res, d_gdesc, n_columns, d_asm, d_gres, coop_min);
    hipLaunchKernelGGL(covt::assemble_kernel, dim3((unsigned)blocks), dim3(64 * covt::kAsmWaves), 0,
                       (hipStream_t)hip_stream, d_decoded, d_res, d_gdesc, n_columns, d_asm, d_gres, coop_min);
    return hipGetLastError() == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
}
