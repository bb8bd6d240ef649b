// covt_props.hip -- gfx950 property-column materialization (include/covt.h "Property columns";
// SURVEY.md §8(f) row 3): the decoded present / data / length streams of a property column become
// an Arrow-style column (validity bitmap, values at feature positions, dictionary offsets + bytes).
//
// Reference: CovtParser.decodePropertyColumn (CovtParser.java:276-354) walks the features of a layer
// once and takes the next decoded data value (j++) for every feature whose present bit is set;
// string columns look the value up in the dictionary built by getStringDictionary (:367-377).  Here
// one wave64 materializes one (sub)column, 256 features per step, four consecutive features per
// lane: the lane's four validity bits give it a count, a DPP wave prefix sum (plus the carried total
// of the earlier steps) gives every present feature its rank j in the dense data stream, and the
// value is gathered from there.  A dictionary owner first turns the decoded length stream into Arrow
// offsets (exclusive scan, 256 per step) and copies the dictionary bytes (16 bytes per lane).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"
#include "covt_internal.h"
#include "covt_scratch.h"
#include "covt_wave.h"

namespace covt {

#ifndef COVT_PROP_WAVES
#define COVT_PROP_WAVES 2  // A/B: 4 -> +2 %
#endif
constexpr int kPropWaves = COVT_PROP_WAVES;  // independent waves (columns) per workgroup
// Small batches (at most kPropCoopMaxColumns columns, e.g. one tile: BASELINE config 1): columns of at
// least kPropSplitMinFeatures features are cut into chunks of 4 x 64 x kPropCoopWaves features (one step
// of a whole workgroup; a step is a chain of dependent loads: the validity nibbles, then the gathers at
// the scanned ranks) run by as many workgroups at once (prop_split_kernel below), the rest by single waves.
constexpr int kPropCoopWaves = 16;
constexpr int kPropCoopMaxColumns = 4096;
constexpr int32_t kPropSplitMinFeatures = 512;

struct PropSmem {
    uint32_t red[2][kPropCoopWaves];  // per-wave partials (two buffers, alternating)
    int32_t st;                       // the dictionary's status (wave 0 checks / writes it)
};

typedef __attribute__((address_space(1))) const uint8_t gp_u8;
typedef __attribute__((address_space(1))) const uint32_t gp_u32;
typedef __attribute__((address_space(1))) const int32_t gp_i32;
typedef __attribute__((address_space(1))) const int64_t gp_i64;
typedef int32_t pi32x4 __attribute__((ext_vector_type(4)));

// 4 bytes at any address of the input (the batch input is padded past its last byte)
__device__ __forceinline__ uint32_t pld_le32(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const gp_u32* q = (const gp_u32*)(a & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}

// bits f .. f+3 (f % 4 == 0) of an LSB-first bitmap, clipped to n
__device__ __forceinline__ uint32_t nibble(const uint8_t* bm, int32_t f, int32_t n) {
    if (f >= n) return 0u;
    const uint32_t v = (((const gp_u8*)bm)[f >> 3] >> (f & 4)) & 0xfu;
    return n - f >= 4 ? v : (v & ((1u << (n - f)) - 1u));
}
__device__ __forceinline__ uint32_t all_valid(int32_t f, int32_t n) {
    return f >= n ? 0u : (n - f >= 4 ? 0xfu : ((1u << (n - f)) - 1u));
}

// Arrow offsets of the dictionary (exclusive scan of the int32 lengths) and its bytes.  Returns a status.
__device__ int32_t dictionary(const uint8_t* in, const uint8_t* dec, const covt_prop_desc& d, uint8_t* outb,
                              bool write) {
    const int l = lane_id();
    const int32_t nd = d.n_dict;
    const gp_i32* lens = (const gp_i32*)(dec + d.length_off);
    int32_t* offs = (int32_t*)(outb + d.out_off[2]);
    if (!write) {
        // sub-columns that share the owner's dictionary only check it: the lengths are summed and
        // tested for negatives in one strided pass, 16 independent loads per lane per iteration
        bool neg = false;
        uint64_t s = 0;
        for (int32_t q = 0; q < nd; q += 1024) {
            int32_t x[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int32_t j = q + 256 * (k >> 2) + 4 * l + (k & 3);
                x[k] = j < nd ? lens[j] : 0;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                neg |= x[k] < 0;
                s += (uint64_t)(uint32_t)x[k];
            }
        }
        if (__ballot(neg)) return COVT_ERR_COUNT_MISMATCH;  // decodeString with a negative length
        const uint64_t run = lane_bcast64(incl_scan64(s), 63);
        return run > (uint64_t)d.dict_bytes ? COVT_ERR_TRUNCATED : COVT_OK;
    }
    // the owner: offsets (exclusive scan, 256 per step, four steps' loads in flight) and the bytes; a
    // negative length anywhere fails the column (decodeString) whatever was written
    bool neg = false;
    uint64_t run = 0;  // uniform: bytes before this step
    for (int32_t q0 = 0; q0 < nd; q0 += 1024) {
        int32_t xs[4][4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int32_t j = q0 + 256 * t + 4 * l + k;
                xs[t][k] = j < nd ? lens[j] : 0;
            }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int32_t q = q0 + 256 * t;
            if (q >= nd) break;
            uint64_t x[4], s = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                neg |= xs[t][k] < 0;
                x[k] = (uint64_t)(uint32_t)xs[t][k];
                s += x[k];
            }
            const uint64_t inc = incl_scan64(s);
            uint64_t e = run + inc - s;
            int32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                o[k] = (int32_t)e;
                e += x[k];
            }
            const int32_t i0 = q + 4 * l;
            if (i0 + 4 <= nd) {
                *(pi32x4*)(offs + i0) = pi32x4{o[0], o[1], o[2], o[3]};
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (i0 + k < nd) offs[i0 + k] = o[k];
            }
            run += lane_bcast64(inc, 63);
        }
    }
    if (__ballot(neg)) return COVT_ERR_COUNT_MISMATCH;
    if (run > (uint64_t)d.dict_bytes) return COVT_ERR_TRUNCATED;  // strings past the dictionary stream
    if (l == 0) offs[nd] = (int32_t)run;
    const uint8_t* src = in + d.dict_in_off;
    uint8_t* dst = outb + d.out_off[3];
    for (int32_t b = 16 * l; b < d.dict_bytes; b += 1024) {
        if (b + 16 <= d.dict_bytes) {
            *(pi32x4*)(dst + b) = pi32x4{(int32_t)pld_le32(src + b), (int32_t)pld_le32(src + b + 4),
                                         (int32_t)pld_le32(src + b + 8), (int32_t)pld_le32(src + b + 12)};
        } else {
            for (int32_t i = b; i < d.dict_bytes; ++i) dst[i] = ((const gp_u8*)src)[i];
        }
    }
    return COVT_OK;
}

// NW = 1: one wave (lane_id, wave primitives); NW > 1: the workgroup's NW waves cooperate on the column
template <int NW>
__device__ void materialize(const uint8_t* in, const uint8_t* dec, const covt_stream_result* dres,
                            const covt_prop_desc& d, uint8_t* outb, covt_prop_result& res, PropSmem* smp) {
    const int l = NW == 1 ? lane_id() : (int)threadIdx.x;
    const int wv = NW == 1 ? 0 : (int)(threadIdx.x >> 6);
    int buf = 0;
    res.status = COVT_OK;
    res.n_valid = 0;
    // Java's order: unsupported shapes, the present stream, encodings rejected after it, the data and
    // length streams, a short float stream, the dictionary, then the feature loop
    if (d.flags & COVT_PROP_UNSUPPORTED) { res.status = COVT_ERR_UNSUPPORTED_ENCODING; return; }
    int32_t st[3];
    for (int k = 0; k < 3; ++k) st[k] = d.res[k] >= 0 ? uni(((const gp_i32*)dres)[2 * d.res[k]]) : COVT_OK;
    // every sub-column checks its dictionary lengths; the owner also writes the dictionary, whatever
    // its own present / data streams hold (the other languages of a localized column share it)
    int32_t dst = COVT_OK;
    if (d.type == COVT_PROP_STRING && d.res[2] >= 0 && st[2] == COVT_OK) {
        if (NW == 1) {
            dst = dictionary(in, dec, d, outb, (d.flags & COVT_PROP_DICT_OWNER) != 0);
        } else {  // wave 0 (the dictionary is the owner's, whatever its size), then its status to all
            if (wv == 0) {
                const int32_t x = dictionary(in, dec, d, outb, (d.flags & COVT_PROP_DICT_OWNER) != 0);
                if (lane_id() == 0) smp->st = x;
            }
            __syncthreads();
            dst = smp->st;
        }
    }
    for (int k = 0; k < 3; ++k) {
        if (st[k]) { res.status = st[k]; return; }
        if (k == 0 && (d.flags & COVT_PROP_UNSUPPORTED_LATE)) { res.status = COVT_ERR_UNSUPPORTED_ENCODING; return; }
    }
    if (d.flags & COVT_PROP_DATA_SHORT) { res.status = COVT_ERR_TRUNCATED; return; }
    if (dst) { res.status = dst; return; }
    const int32_t n = d.n_features, dn = d.n_data;
    const uint8_t* pres = d.present_off >= 0 ? dec + d.present_off : nullptr;
    uint8_t* vout = outb + d.out_off[0];
    uint8_t* xout = outb + d.out_off[1];
    const bool dense_bool = (d.flags & COVT_PROP_DENSE_BOOL) != 0;
    uint32_t carry = 0;  // present features before this step (uniform)
    bool bad = false;
    for (int32_t f0 = 0; f0 < n; f0 += 4 * 64 * NW) {
        const int32_t f = f0 + 4 * l;
        const uint32_t vb = pres ? nibble(pres, f, n) : all_valid(f, n);
        const uint32_t cnt = (uint32_t)__popc(vb);
        const uint32_t inc = incl_scan(cnt);
        uint32_t pre = inc - cnt, tot;  // present features of the step before this thread's, and in all
        if (NW == 1) {
            tot = lane_bcast(inc, 63);
        } else {  // + the lower waves' counts (LDS partials; a buffer is rewritten two barriers later)
            if (lane_id() == 63) smp->red[buf][wv] = inc;
            __syncthreads();
            tot = 0;
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const uint32_t t = smp->red[buf][i];
                pre += i < wv ? t : 0u;
                tot += t;
            }
            buf ^= 1;
        }
        uint32_t j = carry + pre;  // rank of this thread's first present feature
        carry += tot;
        // lanes 2m and 2m+1 hold the two nibbles of byte m of the step
        const uint32_t vhi = lane_next(vb);
        if (!(l & 1) && f < n) vout[f >> 3] = (uint8_t)(vb | (vhi << 4));
        if (d.type == COVT_PROP_BOOLEAN) {
            uint32_t xb;
            if (dense_bool) {  // Gen C: the bitset holds the present values only
                xb = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const bool p = (vb >> k) & 1u;
                    const bool ok = p && j < (uint32_t)dn;
                    bad |= p && !ok;
                    if (ok) xb |= ((((const gp_u8*)(dec + d.data_off))[j >> 3] >> (j & 7u)) & 1u) << k;
                    j += p ? 1u : 0u;
                }
            } else {  // one bit per feature (CovtParser.java:280-291)
                xb = nibble(dec + d.data_off, f, n) & vb;
            }
            const uint32_t xhi = lane_next(xb);
            if (!(l & 1) && f < n) xout[f >> 3] = (uint8_t)(xb | (xhi << 4));
        } else if (d.type == COVT_PROP_INT64) {
            int64_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool p = (vb >> k) & 1u;
                const bool ok = p && j < (uint32_t)dn;
                bad |= p && !ok;
                v[k] = ok ? ((const gp_i64*)(dec + d.data_off))[j] : 0;
                j += p ? 1u : 0u;
            }
            int64_t* o = (int64_t*)xout + f;
            if (f + 4 <= n) {
                *(pi32x4*)o = pi32x4{(int32_t)v[0], (int32_t)(v[0] >> 32), (int32_t)v[1], (int32_t)(v[1] >> 32)};
                *(pi32x4*)(o + 2) = pi32x4{(int32_t)v[2], (int32_t)(v[2] >> 32), (int32_t)v[3], (int32_t)(v[3] >> 32)};
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (f + k < n) o[k] = v[k];
            }
        } else {  // FLOAT (little-endian words of the input) or STRING (int32 dictionary indices)
            const bool flt = d.type == COVT_PROP_FLOAT;
            int32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool p = (vb >> k) & 1u;
                const bool ok = p && j < (uint32_t)dn;
                bad |= p && !ok;
                int32_t x = 0;
                if (ok) x = flt ? (int32_t)pld_le32(in + d.data_off + 4 * (int64_t)j) : ((const gp_i32*)(dec + d.data_off))[j];
                bad |= ok && !flt && (uint32_t)x >= (uint32_t)d.n_dict;  // dictionaryData[index]
                v[k] = x;
                j += p ? 1u : 0u;
            }
            int32_t* o = (int32_t*)xout + f;
            if (f + 4 <= n) {
                *(pi32x4*)o = pi32x4{v[0], v[1], v[2], v[3]};
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (f + k < n) o[k] = v[k];
            }
        }
    }
    if (NW == 1 ? __ballot(bad) != 0ull : __syncthreads_or(bad) != 0) { res.status = COVT_ERR_COUNT_MISMATCH; return; }
    res.n_valid = (int32_t)carry;
}

// one wave per column (large batches)
__global__ __launch_bounds__(64 * kPropWaves) void props_kernel(const uint8_t* __restrict__ in,
                                                                const uint8_t* __restrict__ dec,
                                                                const covt_stream_result* __restrict__ dres,
                                                                const covt_prop_desc* __restrict__ descs,
                                                                int64_t n_cols, uint8_t* __restrict__ outb,
                                                                covt_prop_result* __restrict__ pres) {
    const int w = threadIdx.x >> 6;
    const int64_t c = uni64((int64_t)blockIdx.x * kPropWaves + w);
    if (c >= n_cols) return;
    const covt_prop_desc d = descs[c];
    covt_prop_result r;
    materialize<1>(in, dec, dres, d, outb, r, nullptr);
    if (lane_id() == 0) pres[c] = r;
}

// ---- multi-workgroup columns (small batches: one tile's latency, BASELINE config 1) -------------------
// A whole workgroup still steps through a big column 4,096 features at a time, each step a chain of
// dependent loads (validity nibbles -> scan -> gathers at the ranks).  The steps only share the count of
// present features before them, so here every step is a chunk on a workgroup of its own: a chunk
// publishes its present count and sums its predecessors' published counts (one load each, all in
// flight; chunks take tickets in order, so a chunk only waits on chunks already running), then writes
// its validity bits and values.  Chunk 0 also builds (or checks) the dictionary; the last chunk of a
// column to finish writes the column's result in Java's status order.
constexpr int kPropSplitK = 4 * 64 * kPropCoopWaves;  // features per chunk
constexpr int kPropSplitMaxChunks = 65536;          // over all split columns (past it: single waves)
constexpr int kPropSplitGrid = 256;                 // persistent workgroups (tickets)
constexpr uint32_t kPropSplitMaxSpins = 1u << 22;   // look-back polls before a column is failed

struct PropSplitCol {
    int32_t dst;           // the dictionary's status (chunk 0)
    uint32_t bad;          // any chunk saw an out-of-range rank / index
    uint32_t done;         // chunks finished
    uint32_t n_valid;      // present features (the last chunk)
};
// Per (device, stream) scratch; records carry the launch's epoch in their high half (nothing is cleared
// per launch)
struct PropSplitScratch {
    uint32_t ticket;
    int32_t n_split, n_small;
    uint32_t epoch;  // this launch's record tag, advanced by prop_split_prep (never 0)
    int32_t pre[kPropCoopMaxColumns + 1];  // chunks of split columns before column k
    int32_t col[kPropCoopMaxColumns];      // split column k -> batch column
    int32_t small[kPropCoopMaxColumns];    // the other columns (single waves)
    PropSplitCol st[kPropCoopMaxColumns];
    unsigned long long rec[kPropSplitMaxChunks];  // chunk: (epoch << 32 | present count)
};

__device__ __forceinline__ bool prop_split_wanted(const covt_prop_desc& d, int32_t split_min) {
    return d.n_features >= split_min && !(d.flags & COVT_PROP_UNSUPPORTED);
}

// exclusive prefix of NV int32 per thread over a 1024-thread workgroup (DPP wave scans + 16 wave totals)
template <int NV>
__device__ __forceinline__ void pwg_excl_scan(int32_t (&x)[NV], int32_t (&tot)[NV], int32_t (*lds)[16]) {
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

// one workgroup: the split columns and their chunk prefixes (batch order while within the budget), and
// the small list (every other column)
__global__ __launch_bounds__(1024) void prop_split_prep(const covt_prop_desc* __restrict__ descs, int64_t n_cols,
                                                        int32_t split_min, PropSplitScratch* __restrict__ sc) {
    __shared__ int32_t lds[3][16];
    const int t = threadIdx.x;
    int32_t ch[4] = {};
    bool live[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t c = 4 * t + k;
        live[k] = c < n_cols;
        if (live[k]) {
            const covt_prop_desc d = descs[c];
            if (prop_split_wanted(d, split_min)) ch[k] = (d.n_features + kPropSplitK - 1) / kPropSplitK;
        }
    }
    int32_t x[3], tot[3];
    x[0] = ch[0] + ch[1] + ch[2] + ch[3];
    x[1] = x[2] = 0;
    const int32_t own = x[0];
    pwg_excl_scan<3>(x, tot, lds);
    const bool fits = x[0] + own <= kPropSplitMaxChunks;  // (the prefix only grows: the budget cuts a tail)
    int32_t keep = 0, nk = 0, nsm = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool sp = fits && ch[k] > 0;
        keep += sp ? ch[k] : 0;
        nk += sp ? 1 : 0;
        nsm += (live[k] && !sp) ? 1 : 0;
    }
    x[0] = keep;
    x[1] = nk;
    x[2] = nsm;
    pwg_excl_scan<3>(x, tot, lds);
    int32_t run = x[0], idx = x[1], sidx = x[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t c = 4 * t + k;
        if (!live[k]) continue;
        if (!(fits && ch[k] > 0)) {
            sc->small[sidx++] = (int32_t)c;
            continue;
        }
        sc->col[idx] = (int32_t)c;
        sc->pre[idx] = run;
        sc->st[idx] = PropSplitCol{COVT_OK, 0u, 0u, 0u};
        run += ch[k];
        ++idx;
    }
    if (t == 0) {
        sc->n_split = tot[1];
        sc->n_small = tot[2];
        sc->pre[tot[1]] = tot[0];
        sc->ticket = 0;
        // a new tag for this launch's look-back records, kept in device memory so that a captured graph
        // replays with a fresh one (epoch 0, the zeroed scratch's, is never used)
        const uint32_t e = sc->epoch + 1u;
        sc->epoch = e ? e : 1u;
    }
}

__device__ __forceinline__ unsigned long long pld_rlx(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// chunk j of split column k (batch column c)
__device__ void prop_split_chunk(const uint8_t* in, const uint8_t* dec, const covt_stream_result* dres,
                                 const covt_prop_desc& d, uint8_t* outb, covt_prop_result* pres, PropSplitScratch* sc,
                                 int32_t k, int32_t j, int32_t c, PropSmem* smp, uint32_t epoch) {
    constexpr int NW = kPropCoopWaves;
    const int l = (int)threadIdx.x, wv = (int)(threadIdx.x >> 6);
    PropSplitCol& cs = sc->st[k];
    const int32_t g0 = sc->pre[k], nch = sc->pre[k + 1] - g0;
    int32_t st[3];
    for (int q = 0; q < 3; ++q) st[q] = d.res[q] >= 0 ? ((const gp_i32*)dres)[2 * d.res[q]] : COVT_OK;
    bool early = st[0] || st[1] || st[2] || (d.flags & (COVT_PROP_UNSUPPORTED_LATE | COVT_PROP_DATA_SHORT));
    const int32_t n = d.n_features, dn = d.n_data;
    const int32_t f0 = j * kPropSplitK;
    bool bad = false;
    uint32_t carry = 0, tot = 0;
    if (!early) {
        const uint8_t* prs = d.present_off >= 0 ? dec + d.present_off : nullptr;
        uint8_t* vout = outb + d.out_off[0];
        uint8_t* xout = outb + d.out_off[1];
        const bool dense_bool = (d.flags & COVT_PROP_DENSE_BOOL) != 0;
        const int32_t f = f0 + 4 * l;
        const uint32_t vb = prs ? nibble(prs, f, n) : all_valid(f, n);
        const uint32_t cnt = (uint32_t)__popc(vb);
        const uint32_t inc = incl_scan(cnt);
        uint32_t pre = inc - cnt;
        if (lane_id() == 63) smp->red[0][wv] = inc;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const uint32_t t = smp->red[0][i];
            pre += i < wv ? t : 0u;
            tot += t;
        }
        // publish this chunk's count, sum the predecessors' (bounded wait: a lost record fails the column)
        if (l == 0)
            __hip_atomic_store(&sc->rec[g0 + j], ((unsigned long long)epoch << 32) | tot, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        uint32_t acc = 0;
        bool lost = false;
        for (int32_t i = l; i < j; i += 1024) {
            unsigned long long v;
            uint32_t spins = 0;
            while ((uint32_t)((v = pld_rlx(&sc->rec[g0 + i])) >> 32) != epoch && ++spins < kPropSplitMaxSpins)
                __builtin_amdgcn_s_sleep(2);
            lost |= (uint32_t)(v >> 32) != epoch;
            acc += (uint32_t)v;
        }
        const uint32_t wsum = lane_bcast(incl_scan(acc), 63);
        __syncthreads();
        if (lane_id() == 0) smp->red[1][wv] = wsum;
        __syncthreads();
        for (int i = 0; i < NW; ++i) carry += smp->red[1][i];
        bad |= __syncthreads_or(lost);
        uint32_t jr = carry + pre;  // rank of this thread's first present feature
        const uint32_t vhi = lane_next(vb);
        if (!(l & 1) && f < n) vout[f >> 3] = (uint8_t)(vb | (vhi << 4));
        if (d.type == COVT_PROP_BOOLEAN) {
            uint32_t xb;
            if (dense_bool) {
                xb = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool p = (vb >> q) & 1u;
                    const bool ok = p && jr < (uint32_t)dn;
                    bad |= p && !ok;
                    if (ok) xb |= ((((const gp_u8*)(dec + d.data_off))[jr >> 3] >> (jr & 7u)) & 1u) << q;
                    jr += p ? 1u : 0u;
                }
            } else {
                xb = nibble(dec + d.data_off, f, n) & vb;
            }
            const uint32_t xhi = lane_next(xb);
            if (!(l & 1) && f < n) xout[f >> 3] = (uint8_t)(xb | (xhi << 4));
        } else if (d.type == COVT_PROP_INT64) {
            int64_t v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool p = (vb >> q) & 1u;
                const bool ok = p && jr < (uint32_t)dn;
                bad |= p && !ok;
                v[q] = ok ? ((const gp_i64*)(dec + d.data_off))[jr] : 0;
                jr += p ? 1u : 0u;
            }
            int64_t* o = (int64_t*)xout + f;
            if (f + 4 <= n) {
                *(pi32x4*)o = pi32x4{(int32_t)v[0], (int32_t)(v[0] >> 32), (int32_t)v[1], (int32_t)(v[1] >> 32)};
                *(pi32x4*)(o + 2) = pi32x4{(int32_t)v[2], (int32_t)(v[2] >> 32), (int32_t)v[3], (int32_t)(v[3] >> 32)};
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (f + q < n) o[q] = v[q];
            }
        } else {
            const bool flt = d.type == COVT_PROP_FLOAT;
            int32_t v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool p = (vb >> q) & 1u;
                const bool ok = p && jr < (uint32_t)dn;
                bad |= p && !ok;
                int32_t x = 0;
                if (ok) x = flt ? (int32_t)pld_le32(in + d.data_off + 4 * (int64_t)jr) : ((const gp_i32*)(dec + d.data_off))[jr];
                bad |= ok && !flt && (uint32_t)x >= (uint32_t)d.n_dict;
                v[q] = x;
                jr += p ? 1u : 0u;
            }
            int32_t* o = (int32_t*)xout + f;
            if (f + 4 <= n) {
                *(pi32x4*)o = pi32x4{v[0], v[1], v[2], v[3]};
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (f + q < n) o[q] = v[q];
            }
        }
        bad = __syncthreads_or(bad) != 0;
    }
    // the dictionary (chunk 0, wave 0): written by the owner whatever this sub-column's other streams hold.
    // Built after the chunk has published its present count, so the column's later chunks never wait in
    // their look-back for a long dictionary (cs.dst is read only by the column's last chunk to finish)
    if (j == 0 && d.type == COVT_PROP_STRING && d.res[2] >= 0 && st[2] == COVT_OK) {
        if (wv == 0) {
            const int32_t x = dictionary(in, dec, d, outb, (d.flags & COVT_PROP_DICT_OWNER) != 0);
            if (lane_id() == 0) cs.dst = x;
        }
    }
    __syncthreads();
    if (l == 0) {
        if (bad) atomicOr(&cs.bad, 1u);
        if (!early && f0 + kPropSplitK >= n) cs.n_valid = carry + tot;  // the last chunk: the column's count
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t done = atomicAdd(&cs.done, 1u) + 1u;
        if (done == (uint32_t)nch) {  // the column's last chunk to finish: its result, in Java's order
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            covt_prop_result r{COVT_OK, 0};
            const int32_t dst = __hip_atomic_load(&cs.dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int q = 0; q < 3 && !r.status; ++q) {
                if (st[q]) r.status = st[q];
                else if (q == 0 && (d.flags & COVT_PROP_UNSUPPORTED_LATE)) r.status = COVT_ERR_UNSUPPORTED_ENCODING;
            }
            if (!r.status && (d.flags & COVT_PROP_DATA_SHORT)) r.status = COVT_ERR_TRUNCATED;
            if (!r.status && dst) r.status = dst;
            if (!r.status && __hip_atomic_load(&cs.bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                r.status = COVT_ERR_COUNT_MISMATCH;
            if (!r.status) r.n_valid = (int32_t)__hip_atomic_load(&cs.n_valid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pres[c] = r;
        }
    }
}

// workgroups take chunks by ticket (a chunk waits only on chunks of its column already running) until
// none are left, then the small columns, sixteen per ticket, one wave each
__global__ __launch_bounds__(64 * kPropCoopWaves) void prop_split_kernel(const uint8_t* __restrict__ in,
                                                                         const uint8_t* __restrict__ dec,
                                                                         const covt_stream_result* __restrict__ dres,
                                                                         const covt_prop_desc* __restrict__ descs,
                                                                         uint8_t* __restrict__ outb,
                                                                         covt_prop_result* __restrict__ pres,
                                                                         PropSplitScratch* __restrict__ sc) {
    __shared__ PropSmem smem;
    __shared__ int32_t lpre[kPropCoopMaxColumns + 1];
    __shared__ int32_t tk;
    const int32_t ns = sc->n_split, total = sc->pre[ns];
    const uint32_t epoch = sc->epoch;  // (prop_split_prep, earlier on this stream)
    const int32_t small_groups = (sc->n_small + kPropCoopWaves - 1) / kPropCoopWaves;
    for (int32_t i = threadIdx.x; i <= ns; i += 64 * kPropCoopWaves) lpre[i] = sc->pre[i];
    __syncthreads();
    for (;;) {
        if (threadIdx.x == 0) tk = (int32_t)atomicAdd(&sc->ticket, 1u);
        __syncthreads();
        const int32_t g = tk;
        __syncthreads();
        if (g >= total) {
            if (g >= total + small_groups) return;
            const int32_t si = (g - total) * kPropCoopWaves + (int32_t)(threadIdx.x >> 6);
            if (si < sc->n_small) {  // (wave-uniform)
                const int32_t c = uni(sc->small[si]);
                const covt_prop_desc d = descs[c];
                covt_prop_result r;
                materialize<1>(in, dec, dres, d, outb, r, nullptr);
                if (lane_id() == 0) pres[c] = r;
            }
            __syncthreads();
            continue;
        }
        int32_t lo = 0, hi = ns;  // lpre[lo] <= g < lpre[hi]
        while (hi - lo > 1) {
            const int32_t mid = (lo + hi) >> 1;
            if (lpre[mid] <= g) lo = mid;
            else hi = mid;
        }
        const int32_t c = sc->col[lo];
        const covt_prop_desc d = descs[c];
        prop_split_chunk(in, dec, dres, d, outb, pres, sc, lo, g - lpre[lo], c, &smem, epoch);
        __syncthreads();
    }
}

}  // namespace covt

namespace covt {
// split scratch, one per (device, stream) (covt_scratch.h)
StreamScratch& property_scratch() {
    static StreamScratch m(sizeof(PropSplitScratch));
    return m;
}
}  // namespace covt

extern "C" int covt_materialize_properties_device(const uint8_t* d_in, const uint8_t* d_decoded,
                                                  const covt_stream_result* d_res, const covt_prop_desc* d_pdesc,
                                                  int64_t n_columns, uint8_t* d_props, covt_prop_result* d_pres,
                                                  void* hip_stream) {
    if (n_columns < 0 || (n_columns && (!d_in || !d_decoded || !d_res || !d_pdesc || !d_props || !d_pres)))
        return COVT_ERR_INVALID_ARG;
    if (n_columns == 0) return COVT_OK;
    const int64_t blocks = (n_columns + covt::kPropWaves - 1) / covt::kPropWaves;
    if (blocks > 0x7fffffff) return COVT_ERR_INVALID_ARG;
    hipStream_t s = (hipStream_t)hip_stream;
    if (n_columns <= covt::kPropCoopMaxColumns) {
        // small batches: columns of kPropSplitMinFeatures or more in chunks on many workgroups, the rest
        // on single waves of the same kernel
        covt::PropSplitScratch* sc = (covt::PropSplitScratch*)covt::property_scratch().get(s);
        if (!sc) return COVT_ERR_DEVICE;
        hipLaunchKernelGGL(covt::prop_split_prep, dim3(1), dim3(1024), 0, s, d_pdesc, n_columns,
                           covt::kPropSplitMinFeatures, sc);
        hipLaunchKernelGGL(covt::prop_split_kernel, dim3(covt::kPropSplitGrid), dim3(64 * covt::kPropCoopWaves), 0, s,
                           d_in, d_decoded, d_res, d_pdesc, d_props, d_pres, sc);
    } else {
        hipLaunchKernelGGL(covt::props_kernel, dim3((unsigned)blocks), dim3(64 * covt::kPropWaves), 0, s, d_in,
                           d_decoded, d_res, d_pdesc, n_columns, d_props, d_pres);
    }
    return hipGetLastError() == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
}

extern "C" int covt_release_scratch(void* hip_stream, int all) {
    const hipStream_t s = (hipStream_t)hip_stream;
    const bool every = (all & 1) != 0, pinned = (all & COVT_RELEASE_PINNED) != 0;
    return covt::assembly_scratch().release(s, every, pinned) + covt::property_scratch().release(s, every, pinned);
}

extern "C" int64_t covt_scratch_blocks(void) {
    return (int64_t)(covt::assembly_scratch().size() + covt::property_scratch().size());
}
