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
// The expansion (`Expand`): output items are processed 64 at a time; the 64 segment ends after the
// carried segment base are loaded one per lane, each segment end marks its position in a 64-slot
// LDS table (the last of equal ends wins), and an inclusive running max over the table gives each
// lane the number of segments that end at or before its item -- its segment index, with the
// segment start fetched by ds_bpermute.  Empty segments cost nothing extra; a step consumes 64
// items or 64 segments, so every wave reaches its exit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"
#include "covt_internal.h"
#include "covt_wave.h"

namespace covt {

constexpr int kAsmWaves = 4;  // independent waves (columns) per workgroup

typedef __attribute__((address_space(1))) const int32_t g_i32;
typedef __attribute__((address_space(1))) const uint8_t g_u8;
typedef __attribute__((address_space(1))) const uint64_t g_u64;

struct AsmSmem {
    int32_t slot[64];
};

// Segmented expansion cursor over O[0..S] (nondecreasing, O[0] = 0, O[S] = total), wave-uniform.
struct Expand {
    const int32_t* O;
    int32_t S, total;
    int32_t base;   // segment index with O[base] <= q
    int32_t obase;  // O[base]
    int32_t q;      // first item of the next step

    // one step: L items (uniform) from q; lane l < L gets its segment, rank in it and segment end
    __device__ __forceinline__ int32_t step(AsmSmem& sm, int32_t& seg, int32_t& rank, int32_t& seg_end) {
        const int l = lane_id();
        const int32_t j = base + 1 + l;
        const int32_t e = j <= S ? ((const g_i32*)O)[j] : 0x7fffffff;
        const int32_t r0 = max(e - q, 0);  // item offset (in this step) where segment base+l+1 starts
        const int32_t r1 = (int32_t)lane_next((uint32_t)r0, 0x7fffffffu);
        sm.slot[l] = 0;
        wave_sync();
        if (r0 < 64 && r1 != r0) sm.slot[r0] = l + 1;  // the last of equal ends wins
        wave_sync();
        const int32_t cnt = (int32_t)incl_max_scan((uint32_t)sm.slot[l]);  // segment ends <= q + l
        wave_sync();
        const int32_t e_prev = lane_get(e, max(cnt - 1, 0));
        seg_end = lane_get(e, min(cnt, 63));
        const int32_t start = cnt == 0 ? obase : e_prev;
        seg = base + cnt;
        rank = q + l - start;
        // items this step: at most 64, the rest of the column, and what the 64 loaded ends cover
        int32_t L = min(64, total - q);
        if (base + 64 < S) L = min(L, (int32_t)lane_bcast((uint32_t)e, 63) - q);
        L = max(L, 0);
        const uint64_t done = __ballot(e <= q + L);
        const int k = __popcll(done);  // segments ending at or before the next q (a prefix of lanes)
        if (k > 0) obase = (int32_t)lane_bcast((uint32_t)e, k - 1);
        base += k;
        q += L;
        return L;
    }
};

__device__ __forceinline__ void mem_publish() {  // this wave's global stores visible to its own loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// exclusive scan of x over the lanes (uint32); `tot` gets the uniform total
__device__ __forceinline__ uint32_t excl_scan(uint32_t x, uint32_t& tot) {
    const uint32_t inc = incl_scan(x);
    tot = lane_bcast(inc, 63);
    return inc - x;
}

__device__ void assemble_column(const uint8_t* __restrict__ dec, const covt_stream_result* __restrict__ dres,
                                const covt_geom_desc& d, uint8_t* __restrict__ outb, covt_geom_result& res,
                                AsmSmem& sm) {
    const int l = lane_id();
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

    // ---- pass 1: features -> parts ----
    uint32_t go_base = 0, P = 0;
    bool bad_type = false, bad_cnt = false;
    for (int32_t f0 = 0; f0 < n; f0 += 64) {
        const int32_t f = f0 + l;
        const bool valid = f < n;
        const uint32_t t = valid ? (uint32_t)((const g_u8*)types)[f] : 0u;
        bad_type |= t > 5u;
        const bool multi = valid && t >= 3u && t <= 5u;
        uint32_t nm;
        const uint32_t gi = go_base + excl_scan(multi ? 1u : 0u, nm);
        uint32_t pf = valid ? 1u : 0u;
        if (multi) {
            if (gi < (uint32_t)n_go) {
                const int32_t c = ((const g_i32*)go)[gi];
                bad_cnt |= c < 0;
                pf = min((uint32_t)max(c, 0), pcap + 1u);  // clamped: the scan below cannot wrap
            } else {
                bad_cnt = true;
            }
        }
        uint32_t tot;
        const uint32_t ex = P + excl_scan(pf, tot);
        if (valid) geo_off[f] = (int32_t)ex;
        go_base += nm;
        P += tot;
        if (__ballot(bad_type || bad_cnt) || P > pcap) break;
    }
    if (__ballot(bad_type)) { res.status = COVT_ERR_BAD_HEADER; return; }  // GeometryType.values()[b]
    if (__ballot(bad_cnt) || P > pcap) { res.status = COVT_ERR_COUNT_MISMATCH; return; }
    if (l == 0) geo_off[n] = (int32_t)P;
    mem_publish();

    // ---- pass 2: parts -> rings ----
    uint32_t po_base = 0, R = 0;
    {
        Expand x{geo_off, n, (int32_t)P, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t p0 = x.q;
            int32_t f, rank, fend;
            const int32_t L = x.step(sm, f, rank, fend);
            const bool valid = l < L;
            const uint32_t t = valid ? (uint32_t)((const g_u8*)types)[f] : 0u;
            const bool uses_po = valid && t != 0u && t != 3u;  // line and polygon parts
            uint32_t npo;
            const uint32_t pi = po_base + excl_scan(uses_po ? 1u : 0u, npo);
            uint32_t c = 0;
            if (uses_po) {
                if (pi < (uint32_t)n_po) {
                    const int32_t v = ((const g_i32*)po)[pi];
                    bad_cnt |= v < 0;
                    c = min((uint32_t)max(v, 0), rcap + 1u);
                } else {
                    bad_cnt = true;
                }
            }
            const bool poly = t == 2u || t == 5u;
            const uint32_t rp = valid ? (poly ? c : 1u) : 0u;
            const uint32_t vcount = (t == 1u || t == 4u) ? c : 1u;  // vertices of a line / point part
            uint32_t tot;
            const uint32_t ex = R + excl_scan(rp, tot);
            if (valid) {
                part_off[p0 + l] = (int32_t)ex;
                part_scr[p0 + l] = poly ? 1 : (int32_t)(min(vcount, ccap + 1u) << 1);
            }
            po_base += npo;
            R += tot;
            if (__ballot(bad_cnt) || R > rcap) break;
        }
    }
    if (__ballot(bad_cnt) || R > rcap) { res.status = COVT_ERR_COUNT_MISMATCH; return; }
    if (l == 0) part_off[P] = (int32_t)R;
    mem_publish();

    // ---- pass 3: rings -> coordinates ----
    uint32_t ro_base = 0, V = 0, VS = 0;
    {
        Expand x{part_off, (int32_t)P, (int32_t)R, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t r0i = x.q;
            int32_t p, rank, pend;
            const int32_t L = x.step(sm, p, rank, pend);
            const bool valid = l < L;
            const int32_t sp = valid ? ((const g_i32*)part_scr)[p] : 0;
            const bool poly = valid && (sp & 1);
            uint32_t nr;
            const uint32_t ri = ro_base + excl_scan(poly ? 1u : 0u, nr);
            uint32_t vs = valid ? (uint32_t)sp >> 1 : 0u;
            if (poly) {
                if (ri < (uint32_t)n_ro) {
                    const int32_t v = ((const g_i32*)ro)[ri];
                    bad_cnt |= v < 0;
                    vs = min((uint32_t)max(v, 0), ccap + 1u);
                } else {
                    bad_cnt = true;
                }
            }
            const uint32_t closing = (poly && !closed && vs > 0u) ? 1u : 0u;
            uint32_t tv, ts;
            const uint32_t ex = V + excl_scan(vs + closing, tv);
            const uint32_t src = VS + excl_scan(vs, ts);
            if (valid) {
                ring_off[r0i + l] = (int32_t)ex;
                ring_scr[r0i + l] = (int32_t)(src | (closing << 31));
            }
            ro_base += nr;
            V += tv;
            VS += ts;
            if (__ballot(bad_cnt) || V > ccap || VS > (uint32_t)n_src) break;
        }
    }
    if (__ballot(bad_cnt) || V > ccap || VS > (uint32_t)n_src) { res.status = COVT_ERR_COUNT_MISMATCH; return; }
    if (l == 0) ring_off[R] = (int32_t)V;
    mem_publish();

    // ---- pass 4: coordinates (ICE gather) ----
    bool bad_idx = false;
    {
        Expand x{ring_off, (int32_t)R, (int32_t)V, 0, 0, 0};
        while (x.q < x.total) {
            const int32_t v0 = x.q;
            int32_t r, rank, rend;
            const int32_t L = x.step(sm, r, rank, rend);
            if (l < L) {
                const uint32_t sr = (uint32_t)((const g_i32*)ring_scr)[r];
                const int32_t first = (int32_t)(sr & 0x7fffffffu);
                const bool last = (int32_t)(v0 + l) == rend - 1;
                const int32_t src = (sr >> 31) && last ? first : first + rank;
                const int32_t idx = ice ? ((const g_i32*)vo)[src] : src;
                if ((uint32_t)idx < (uint32_t)n_vb) {
                    coords[v0 + l] = ((const g_u64*)vb)[idx];
                } else {
                    bad_idx = true;  // vertexBuffer[offset] out of range (ArrayIndexOutOfBounds)
                    coords[v0 + l] = 0;
                }
            }
        }
    }
    if (__ballot(bad_idx)) { res.status = COVT_ERR_TRUNCATED; return; }
    res.status = COVT_OK;
    res.num_parts = (int32_t)P;
    res.num_rings = (int32_t)R;
    res.num_coords = (int32_t)V;
}

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
    assemble_column(dec, dres, d, outb, r, smem[w]);
    if (lane_id() == 0) gres[c] = r;
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
    hipLaunchKernelGGL(covt::assemble_kernel, dim3((unsigned)blocks), dim3(64 * covt::kAsmWaves), 0,
                       (hipStream_t)hip_stream, d_decoded, d_res, d_gdesc, n_columns, d_asm, d_gres);
    return hipGetLastError() == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
}
