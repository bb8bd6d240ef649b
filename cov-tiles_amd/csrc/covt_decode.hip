// covt_decode.hip -- gfx950 (MI355X) kernels for the COVT Id/Geometry stream codecs.
//
// One wave64 decodes one stream (a covt_stream_desc); a 256-thread workgroup runs four
// independent waves with no workgroup barrier, so a wave retires as soon as its stream is done.
// All decode state is wave-uniform except the per-lane data; cross-lane work goes through
// ballot/prefix-scan primitives and a per-wave LDS scratch area.
//
// Codecs (reference semantics, evaluation/java/src/main/java/com/covt/decoder/DecodingUtils.java):
//   * varint family (:35-112, :394-409): 1 KiB windows of the stream are loaded with one
//     16-byte load per lane (coalesced), a per-byte terminator bitmask is built in registers,
//     a wave prefix-sum of popcounts turns it into a list of value end positions in LDS, then
//     each lane assembles one value and zigzag / delta / Morton run as a wave scan with a
//     carried running sum.  The Java 4-byte cap (:157-186) is exact: a run of 4 continuation
//     bytes in a window sends that window through a lane-serial parse.
//   * ORC RLE v1 integer/byte (orc-core RunLengthIntegerReader/RunLengthByteReader, called at
//     :257-306): the group headers are walked wave-uniformly out of the LDS window; runs are
//     expanded lane-parallel, literal groups reuse the varint machinery.
//   * FastPFOR(256-blocks, 65536-pages) + VariableByte (JavaFastPFOR 0.1.12 via :316-444):
//     per page the exception-array directory is read, the byte container is walked in batches
//     of 64 blocks, each block's 8*b packed words are staged in LDS and every lane unpacks four
//     consecutive values, exceptions are patched through LDS, and the VariableByte tail reuses
//     the varint machinery on the word-reversed byte order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"
#include "covt_internal.h"
#include "covt_wave.h"
#include "covt_walk.h"

namespace covt {

constexpr int kWin = 1024;  // window bytes (64 lanes x 16 B)
// kWavesPerBlock (covt_internal.h): independent waves (streams) per workgroup
constexpr int kFpfBlock = 256;
constexpr int kFpfPage = 65536;
constexpr int kFpfBcCap = 3 * kFpfPage / kFpfBlock + kFpfPage;  // JavaFastPFOR byteContainer size

#ifndef COVT_LONG_STREAM
#define COVT_LONG_STREAM 16384
#endif
#ifndef COVT_LONG_PRIO
#define COVT_LONG_PRIO 2
#endif
#ifndef COVT_RLE_SHORT_SPAN  // int RLE windows with at most this many live bytes build next[] position-major
#define COVT_RLE_SHORT_SPAN 448
#endif
#ifndef COVT_CHUNK_PRIO
#define COVT_CHUNK_PRIO 2
#endif
constexpr int kLongStream = COVT_LONG_STREAM;  // bytes or values: raised wave priority
#ifdef COVT_TIMING
constexpr int kPhases = 8;            // profiling build: per-stream phase clocks
__device__ uint32_t* covt_phase_buf;  // [n_streams][kPhases], set by covt_debug_set_phase_buffer
__device__ const covt_stream_desc* covt_phase_desc0;  // descriptor 0 of the launch (row index base)
#endif

typedef __attribute__((address_space(3))) const uint16_t lds_cu16;

// Per-wave LDS scratch.  The small fields come first so each codec family's kernel allocates only
// the prefix it uses (kFamSmem below): varint windows, RLE windows + group tables, or FastPFOR
// staging + byte container.
struct __attribute__((aligned(16))) WaveSmem {
    int32_t misc[4];
    uint16_t cpre[64];   // window index: terminators before each 16-byte chunk
    uint16_t cmask[64];  // window index: terminator mask of each chunk
    union alignas(16) {  // 16-byte aligned: uint4 (ds_*_b128) accesses
        struct {
            uint32_t win[kWin / 4 + 4];    // window bytes (+16 B slack for 12-byte reads)
            uint16_t list[kWin];           // terminator positions (window-relative)
            uint16_t next[kWin + 8];       // RLE: start of the next group if a header sat at j (+sentinel)
            uint16_t grec[64];             // RLE: the chain walk's successor of each step (int RLE)
        } v;
        struct {
            union {
                uint32_t stage[324];  // split chunks: packed words of one FastPFOR block (<= 1024 + 15 B)
                uint32_t ring[512];   // whole streams: two 1 KiB windows of the page's packed words
            };
            uint32_t patch[256];  // exception patches of one block
            uint32_t cbuf[260];   // 1 KiB chunk of the page's byte container
            union {
                uint8_t posx[2][192];  // split chunks: positions of exceptions 64..255 of the next two blocks
                uint32_t xw[224];      // whole streams: a block batch's exception words (kFpfXw)
            };
        } f;
    } u;
};
constexpr int kSmemHdr = 272;  // offsetof(WaveSmem, u), checked below
constexpr int kFamSmemRle = kSmemHdr + (kWin / 4 + 4) * 4 + kWin * 2 + (kWin + 8) * 2 + 64 * 2;
constexpr int kFamSmemVarint = kSmemHdr + (kWin / 4 + 4) * 4 + kWin * 2;
constexpr int kFamSmemFpf = kSmemHdr + (512 + 256 + 260 + 224) * 4 > kFamSmemVarint
                                ? kSmemHdr + (512 + 256 + 260 + 224) * 4
                                : kFamSmemVarint;
constexpr int kFpfXw = 224;  // LDS words of a FastPFOR block batch's gathered exception words
static_assert(kFamSmemFpf >= kSmemHdr + (int)sizeof(((WaveSmem*)nullptr)->u.f), "FastPFOR scratch stride");
static_assert(kFamSmemVarint >= kSmemHdr + (int)sizeof(((WaveSmem*)nullptr)->u.v.win) +
                                    (int)sizeof(((WaveSmem*)nullptr)->u.v.list), "varint scratch stride");
static_assert(__builtin_offsetof(WaveSmem, u) == kSmemHdr, "WaveSmem header size");
static_assert(kFamSmemRle == (int)sizeof(WaveSmem), "RLE uses the whole scratch");
static_assert(kFamSmemRle % 16 == 0 && kFamSmemVarint % 16 == 0 && kFamSmemFpf % 16 == 0, "16-B strides");

// --------------------------------------------------------------------------------------------
// byte helpers
// --------------------------------------------------------------------------------------------
// Loads go through explicit global (address-space 1) pointers: an integer->pointer cast would
// otherwise yield flat_load, which counts on both vmcnt and lgkmcnt and forces full drains
// (vmcnt(0) & lgkmcnt(0)) at every LDS wait, serialising the wave's memory traffic.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const u32x4 g_v4;
__device__ __forceinline__ const g_u32* g32(uintptr_t a) { return (const g_u32*)a; }
// 16-byte load from a 16-byte aligned global address
__device__ __forceinline__ uint4 ld128(uintptr_t a16) {
    const u32x4 v = *(const g_v4*)a16;
    return make_uint4(v.x, v.y, v.z, v.w);
}
// the same from a uniform base and a 32-bit per-lane offset (global_load ... v_off, s[base])
typedef __attribute__((address_space(1))) const uint8_t g_u8;
__device__ __forceinline__ uint4 ld128_off(const g_u8* base, uint32_t off) {
    const u32x4 v = *(const g_v4*)(base + off);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {  // any alignment (input is padded)
    const uintptr_t a = (uintptr_t)p;
    const g_u32* q = g32(a & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}
__device__ __forceinline__ uint32_t ld_be32(const uint8_t* p) { return __builtin_bswap32(ld_le32(p)); }
// v_perm_b32 selector of "bytes [sh, sh + 4) of {hi:lo}, byte-swapped": the big-endian word that starts
// sh bytes into lo, in one instruction (alignbyte + bswap would be two)
__host__ __device__ constexpr uint32_t be_sel(uint32_t sh) {
    return (sh + 3u) | ((sh + 2u) << 8) | ((sh + 1u) << 16) | (sh << 24);
}
__device__ __forceinline__ uint32_t be_word(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
// loads from a wave-uniform address through the scalar data cache (constant address space)
typedef __attribute__((address_space(4))) const uint32_t c_u32;
typedef __attribute__((address_space(4))) const u32x4 c_v4;
__device__ __forceinline__ uint32_t sld_le32(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const c_u32* q = (const c_u32*)(a & ~(uintptr_t)3);
    const uint64_t v = ((uint64_t)q[1] << 32) | q[0];
    return (uint32_t)(v >> (8u * (uint32_t)(a & 3u)));
}
__device__ __forceinline__ uint32_t sld_be32(const uint8_t* p) { return uniu(__builtin_bswap32(sld_le32(p))); }
__device__ __forceinline__ uint4 sld128(uintptr_t a16) {
    const u32x4 v = *(const c_v4*)a16;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// bits 7,15,23,31 of each dword -> 16-bit mask of "high bit set" bytes
__device__ __forceinline__ uint32_t hibits4(uint32_t x) {
    x &= 0x80808080u;
    return ((x >> 7) & 1u) | ((x >> 14) & 2u) | ((x >> 21) & 4u) | ((x >> 28) & 8u);
}
__device__ __forceinline__ uint32_t hibits16(uint4 d) {
    return hibits4(d.x) | (hibits4(d.y) << 4) | (hibits4(d.z) << 8) | (hibits4(d.w) << 12);
}
// mask of byte slots [s, e) within 16 (clamped)
__device__ __forceinline__ uint32_t range16(int32_t s, int32_t e) {
    s = s < 0 ? 0 : (s > 16 ? 16 : s);
    e = e < 0 ? 0 : (e > 16 ? 16 : e);
    if (e <= s) return 0u;
    return ((1u << e) - 1u) & ~((1u << s) - 1u);
}
// 7-bit groups of up to four LEB128 bytes (little-endian in x): the byte pairs of each 16-bit half joined
// by one packed 16-bit shift (no bits cross the halves), then the two 14-bit halves -- five VALU with the
// caller's mask folded into the first (four shifts and masks took eight)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pext7(uint32_t x) {
    x &= 0x7f7f7f7fu;
    const uint32_t y = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, x) >> (u16x2){1, 1});  // v_pk_lshrrev_b16
    const uint32_t t = (x & 0x007f007fu) | (y & ~0x007f007fu);  // b0 | b1 << 7 at bit 0, b2 | b3 << 7 at bit 16
    return (t & 0x3fffu) | ((t >> 2) & ~0x3fffu);
}
__device__ __forceinline__ uint32_t bytemask(int n) {  // low n bytes, clamped to [0,4]
    return n >= 4 ? 0xffffffffu : (n <= 0 ? 0u : ((1u << (8 * n)) - 1u));
}
__device__ __forceinline__ int32_t zz32(uint32_t e) { return (int32_t)((e >> 1) ^ (0u - (e & 1u))); }
__device__ __forceinline__ int64_t zz64(uint64_t e) { return (int64_t)((e >> 1) ^ (0ull - (e & 1ull))); }

// GeometryUtils.decodeMorton (GeometryUtils.java:34-47) with Java int/long semantics, both axes at
// once: four delta swaps move the even bits of the code to the low half and the odd bits (the even
// bits of code >> 1) to the high half.
__host__ __device__ __forceinline__ void morton_xy(int32_t code, int nb, uint32_t& x, uint32_t& y) {
    uint32_t v = (uint32_t)code, t;
    t = (v ^ (v >> 1)) & 0x22222222u; v ^= t ^ (t << 1);
    t = (v ^ (v >> 2)) & 0x0c0c0c0cu; v ^= t ^ (t << 2);
    t = (v ^ (v >> 4)) & 0x00f000f0u; v ^= t ^ (t << 4);
    t = (v ^ (v >> 8)) & 0x0000ff00u; v ^= t ^ (t << 8);
    const uint32_t low = nb >= 16 ? 0xffffu : (nb <= 0 ? 0u : ((1u << nb) - 1u));
    // bits 2i >= 32 of the sign-extended long are the sign bit (both axes: code >> 1 keeps the sign)
    const uint32_t top = nb <= 16 ? 0u : ((nb >= 32 ? 0xffffffffu : ((1u << nb) - 1u)) & ~0xffffu);
    const uint32_t hi = code < 0 ? top : 0u;
    x = (v & low) | hi;
    y = ((v >> 16) & low) | hi;
}
__device__ __forceinline__ int32_t morton_half(int nb) {
    const int32_t te = (int32_t)(2u << ((uint32_t)(nb - 2) & 31u));
    return te / 2;
}

// --------------------------------------------------------------------------------------------
// sinks: per-op output transforms for K consecutive values per lane (value index base+lane*K+k)
// --------------------------------------------------------------------------------------------
struct Carry {
    uint32_t x, y;
};

// Full 16-byte-per-lane output stores (1 KiB per wave instruction) are nontemporal: decoded columns
// are written once, and streaming whole lines past L2 keeps thousands of concurrent per-stream
// write fronts from thrashing it (FastPFOR family 1.12 -> 0.94 ms on the config-5 batch).  Narrower
// stores stay cached: nontemporal partial lines measured 1.8x slower for RLE, 1.2x for varint.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_out16(int32_t* p, int4 v) {
    const i32x4 w = {v.x, v.y, v.z, v.w};
#if defined(COVT_ABL_NOSTORE)  // ablation build: wide stores land on the first KiB of their 64 KiB
    p = (int32_t*)(((uintptr_t)p & ~(uintptr_t)65535) | ((uintptr_t)p & 1023));
#endif
#if defined(COVT_ST16_CACHED)  // experiment build: 16-byte output stores through L2 like the narrow ones
    *(i32x4*)p = w;
#else
    __builtin_nontemporal_store(w, (i32x4*)p);
#endif
}
template <class T>
__device__ __forceinline__ void st_out(T* p, T v) {
#if defined(COVT_ABL_NOSTORE)  // ablation build: narrow stores all land on one address
    *(T*)((uintptr_t)p & ~(uintptr_t)1023) = v;
#else
    *p = v;
#endif
}
__device__ __forceinline__ int64_t pack_xy(int32_t x, int32_t y) {
    return (int64_t)(((uint64_t)(uint32_t)y << 32) | (uint32_t)x);
}

// An arithmetic run v(i) = base + i * delta, i in [0, n), written at element index o of an E-byte
// array (E = 1, 4 or 8; the array is 16-byte aligned): the 16-byte-aligned body with one 16-byte
// nontemporal store per lane (lanes past the end repeat the last chunk), the unaligned head and
// tail element by element.  Wave-uniform arguments.
template <int E>
__device__ __forceinline__ void store_run(uint8_t* arr, int32_t o, int32_t n, int64_t base, int32_t delta) {
    constexpr int K = 16 / E;
    const int l = lane_id();
    auto val = [&](int32_t i) -> int64_t { return (int64_t)((uint64_t)base + (uint64_t)(int64_t)(int32_t)(i * delta)); };
    const int32_t a0 = (o + K - 1) & ~(K - 1);  // first aligned element
    const int32_t head = min(a0 - o, n);
    const int32_t nch = (n - head) / K;         // whole 16-byte chunks
    const int32_t body_end = head + nch * K;
    // head and tail: at most 2 (K - 1) elements, one lane each
    const int32_t ti = l < head ? l : body_end + (l - head);
    if (l < head || (l - head < n - body_end && l >= head)) {
        const int64_t v = val(ti);
        if (E == 8) st_out((int64_t*)arr + o + ti, v);
        else if (E == 4) st_out((int32_t*)arr + o + ti, (int32_t)v);
        else st_out(arr + o + ti, (uint8_t)v);
    }
    for (int32_t c0 = 0; c0 < nch; c0 += 64) {
        const int32_t ch = c0 + l < nch ? c0 + l : nch - 1;
        const int32_t i = head + K * ch;  // run index of the chunk's first element
        int4 w;
        if (E == 8) {
            const int64_t v0 = val(i), v1 = val(i + 1);
            w = make_int4((int)v0, (int)(v0 >> 32), (int)v1, (int)(v1 >> 32));
        } else if (E == 4) {
            w = make_int4((int)val(i), (int)val(i + 1), (int)val(i + 2), (int)val(i + 3));
        } else {  // byte runs: delta 0 (ORC byte runs repeat one value)
            const uint32_t b = (uint32_t)base & 0xffu, q = b * 0x01010101u;
            w = make_int4((int)q, (int)q, (int)q, (int)q);
        }
        st_out16((int32_t*)(arr + (int64_t)(o + i) * E), w);
    }
}

// The same for four runs at once, one per 16-lane quarter of the wave (o, n, base, delta uniform within a
// quarter; a quarter with n <= 0 stores nothing).  The long runs of an ORC RLE batch went through store_run
// one at a time, each iteration a chain of lane broadcasts and one store (RLE_U64 streams of long runs --
// 6 KB of bytes, 31.5k values -- were the longest single waves of small batches).
template <int E>
__device__ __forceinline__ void store_run_q(uint8_t* arr, int32_t o, int32_t n, int64_t base, int32_t delta) {
    constexpr int K = 16 / E;
    static_assert(2 * (K - 1) <= 16, "head and tail elements fit a quarter");
    const int q = lane_id() & 15;
    auto val = [&](int32_t i) -> int64_t { return (int64_t)((uint64_t)base + (uint64_t)(int64_t)(int32_t)(i * delta)); };
    const int32_t a0 = (o + K - 1) & ~(K - 1);
    const int32_t head = n > 0 ? min(a0 - o, n) : 0;
    const int32_t nch = n > 0 ? (n - head) / K : 0;
    const int32_t body_end = head + nch * K;
    const int32_t tailn = n > 0 ? n - body_end : 0;
    if (q < head + tailn) {  // head and tail: one element per lane
        const int32_t ti = q < head ? q : body_end + (q - head);
        const int64_t v = val(ti);
        if (E == 8) st_out((int64_t*)arr + o + ti, v);
        else st_out((int32_t*)arr + o + ti, (int32_t)v);
    }
    const int32_t steps = (int32_t)wave_max((uint32_t)((nch + 15) >> 4));
    for (int32_t c0 = 0; c0 < 16 * steps; c0 += 16) {
        const int32_t ch = c0 + q;
        if (ch < nch) {
            const int32_t i = head + K * ch;
            int4 w;
            if (E == 8) {
                const int64_t v0 = val(i), v1 = val(i + 1);
                w = make_int4((int)v0, (int)(v0 >> 32), (int)v1, (int)(v1 >> 32));
            } else {
                w = make_int4((int)val(i), (int)val(i + 1), (int)val(i + 2), (int)val(i + 3));
            }
            st_out16((int32_t*)(arr + (int64_t)(o + i) * E), w);
        }
    }
}

// Per-op output transform, specialised at compile time.  Lane l holds slots base + K l .. + K - 1;
// slots [first, first + count) of the group are values (uniform; `first` < K skips leading slots so
// that `base` can stay a multiple of K and 16-byte stores stay aligned).  A full group takes the
// branch-free path; otherwise lanes whose K slots are all values still store 16 bytes at once and
// only the boundary lanes store element by element.  Invalid slots enter the delta scans as 0.
template <int OP, int K>
__device__ __forceinline__ void sink_values(const uint32_t (&vin)[K], int64_t base, int32_t first, int32_t count,
                                            int nb, uint8_t* __restrict__ out, Carry& c) {
    const int l = lane_id();
    const bool full = first == 0 && count >= 64 * K;
    const int32_t s0 = l * K - first;  // value index of this lane's slot 0
    const bool lfull = full || (s0 >= 0 && s0 + K <= count);
    const int64_t i0 = base + (int64_t)l * K;
    bool ok[K];
    uint32_t v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        ok[k] = full || (s0 + k >= 0 && s0 + k < count);
        v[k] = ok[k] ? vin[k] : 0u;
    }
    auto st32 = [&](const int32_t (&r)[K]) {
        int32_t* o = (int32_t*)out + i0;
        if (K == 4 && lfull) {
            st_out16(o, make_int4(r[0], r[K > 1 ? 1 : 0], r[K > 2 ? 2 : 0], r[K > 3 ? 3 : 0]));
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (ok[k]) st_out(o + k, r[k]);
        }
    };
    auto st64 = [&](const int64_t (&r)[K]) {
        int64_t* o = (int64_t*)out + i0;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (ok[k]) st_out(o + k, r[k]);
    };
    if constexpr (OP == COVT_OP_VARINT_I32 || OP == COVT_OP_VARINT_ZZ_I32) {
        int32_t r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = OP == COVT_OP_VARINT_I32 ? (int32_t)v[k] : zz32(v[k]);
        st32(r);
    } else if constexpr (OP == COVT_OP_VARINT_I32_AS_I64 || OP == COVT_OP_VARINT_ZZ_I32_AS_I64) {
        int64_t r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = OP == COVT_OP_VARINT_I32_AS_I64 ? (int64_t)(int32_t)v[k] : (int64_t)zz32(v[k]);
        st64(r);
    } else if constexpr (OP == COVT_OP_VARINT_ZZ_DELTA_I32 || OP == COVT_OP_FPF_ZZ_DELTA_I32 ||
                         OP == COVT_OP_VARINT_ZZ_DELTA_I64) {
        uint32_t sacc[K];
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc += (uint32_t)zz32(v[k]);  // invalid slots hold 0 -> zz 0
            sacc[k] = acc;
        }
        const uint32_t inc = incl_scan(acc);
        const uint32_t pre = c.x + inc - acc;
        if constexpr (OP == COVT_OP_VARINT_ZZ_DELTA_I64) {
            int64_t r[K];
#pragma unroll
            for (int k = 0; k < K; ++k) r[k] = (int64_t)(int32_t)(pre + sacc[k]);
            st64(r);
        } else {
            int32_t r[K];
#pragma unroll
            for (int k = 0; k < K; ++k) r[k] = (int32_t)(pre + sacc[k]);
            st32(r);
        }
        c.x += lane_bcast(inc, 63);
    } else if constexpr (OP == COVT_OP_VARINT_ZZ_DELTA_XY || OP == COVT_OP_FPF_ZZ_DELTA_XY) {
        uint32_t sx[K], sy[K];
        uint32_t ax = 0, ay = 0;
        const uint32_t par0 = (uint32_t)(i0 & 1);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t z = (uint32_t)zz32(v[k]);
            const bool isx = ((par0 + k) & 1u) == 0;
            ax += isx ? z : 0u;
            ay += isx ? 0u : z;
            sx[k] = ax;
            sy[k] = ay;
        }
        const uint32_t incx = incl_scan(ax), incy = incl_scan(ay);
        const uint32_t prex = c.x + incx - ax, prey = c.y + incy - ay;
        int32_t r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = (int32_t)((((par0 + k) & 1u) == 0) ? (prex + sx[k]) : (prey + sy[k]));
        st32(r);
        c.x += lane_bcast(incx, 63);
        c.y += lane_bcast(incy, 63);
    } else if constexpr (OP == COVT_OP_VARINT_DELTA_MORTON || OP == COVT_OP_FPF_DELTA_MORTON) {
        uint32_t sacc[K];
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc += v[k];  // no zigzag (DecodingUtils.java:398-399, :435)
            sacc[k] = acc;
        }
        const uint32_t inc = incl_scan(acc);
        const uint32_t pre = c.x + inc - acc;
        const int32_t half = morton_half(nb);
        int32_t* o = (int32_t*)out + 2 * i0;
        int32_t xy[2 * K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint32_t mx, my;
            morton_xy((int32_t)(pre + sacc[k]), nb, mx, my);
            xy[2 * k] = (int32_t)(mx - (uint32_t)half);
            xy[2 * k + 1] = (int32_t)(my - (uint32_t)half);
        }
        if (K == 4 && lfull) {
            st_out16(o, make_int4(xy[0], xy[1], xy[K > 1 ? 2 : 0], xy[K > 1 ? 3 : 0]));
            st_out16(o + 4, make_int4(xy[K > 2 ? 4 : 0], xy[K > 2 ? 5 : 0], xy[K > 3 ? 6 : 0], xy[K > 3 ? 7 : 0]));
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (ok[k]) st_out((int64_t*)(o + 2 * k), pack_xy(xy[2 * k], xy[2 * k + 1]));
        }
        c.x += lane_bcast(inc, 63);
    }
}

// --------------------------------------------------------------------------------------------
// the 1 KiB indexed window and the varint machinery
// --------------------------------------------------------------------------------------------
enum { MODE_RAW = 0, MODE_WORDREV = 1 };                           // byte order of the window
enum { VAL_J4 = 0, VAL_VB = 1, VAL_U64 = 2, VAL_U64_STRICT = 3, VAL_NONE = 4 };  // value grammar (NONE: bytes only)

// A window holds 1 KiB of the stream in LDS (and each lane's 16 bytes in registers) plus an index
// of its value terminators: list[] = window-relative positions of every terminator byte in the
// valid range, cpre/cmask = per-16-byte-chunk prefix counts and masks, so rank(q) (terminators
// before q) is O(1) and a run of values starting at any value boundary is list[rank(q) ...].
// RAW: window byte j = stream byte woff + j, woff = ((sb + p) & ~15) - sb.
// WORDREV: window byte j = logical byte woff + j of the VariableByte sequence, i.e. the LE bytes of
// the big-endian words W[i] (DecodingUtils.java:319-327); woff is a multiple of 16.
__device__ __forceinline__ uint32_t win_byte(const WaveSmem& sm, int32_t j) {
    return ((const uint8_t*)sm.u.v.win)[j];  // ds_read_u8 (a dword read needed a shift and a mask)
}
// bytes [j, j+12) of the window as three little-endian dwords
__device__ __forceinline__ void win_bytes12(const WaveSmem& sm, int32_t j, uint32_t& x0, uint32_t& x1,
                                            uint32_t& x2) {
    const int32_t d = j >> 2;
    const uint32_t sh = (uint32_t)(j & 3);
    const uint32_t w0 = sm.u.v.win[d], w1 = sm.u.v.win[d + 1], w2 = sm.u.v.win[d + 2], w3 = sm.u.v.win[d + 3];
    x0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
    x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    x2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
}

struct Win {
    int32_t woff;  // stream-relative position of window byte 0
    int32_t K;     // terminators indexed
    int32_t p0;    // J4 serial windows: list[] starts at value boundary p0 (rank(p0) = 0)
    bool valid, serial;
    uint4 d;             // this lane's 16 window bytes
    uint32_t cpre, cmsk; // this lane's chunk: terminators before it, terminator mask
};

// lsrc (MODE_WORDREV only): the stream words already staged in LDS, lsrc[i] = W(lw0 + i) for the words the
// window needs (those before `end`), so the window costs no HBM round trip (FastPFOR's VariableByte tail
// inside the page's meta window).  lsrc must not overlap the window or its index (win, list).
template <int MODE, int VAL>
__device__ void win_load(WaveSmem& sm, const uint8_t* sb, Win& w, int32_t p, int32_t end, const uint32_t* lsrc = nullptr,
                         int32_t lw0 = 0) {
    const int l = lane_id();
    uint4 d;
    int32_t woff;
    // lanes whose 16 bytes start at or past `end` load nothing: a short stream's window would otherwise
    // fetch up to 1 KiB of its neighbours (bytes past `end` are never used)
    if (MODE == MODE_RAW) {
        const uintptr_t a = ((uintptr_t)(sb + p)) & ~(uintptr_t)15;
        woff = uni((int32_t)((intptr_t)a - (intptr_t)sb));
        d = woff + 16 * l < end ? ld128(a + 16 * (uintptr_t)l) : make_uint4(0, 0, 0, 0);
    } else {
        woff = p & ~15;
        const uint8_t* q = sb + woff + 16 * l;
        d = make_uint4(0, 0, 0, 0);
        if (woff + 16 * l < end) {
            if (lsrc) {
                const uint32_t* ws = lsrc + ((woff + 16 * l) >> 2) - lw0;
                d = make_uint4(ws[0], ws[1], ws[2], ws[3]);
            } else {
                d.x = ld_be32(q);
                d.y = ld_be32(q + 4);
                d.z = ld_be32(q + 8);
                d.w = ld_be32(q + 12);
            }
        }
        wave_sync();  // (every lane's LDS reads before the window's writes)
    }
    ((uint4*)sm.u.v.win)[l] = d;
    if (VAL == VAL_NONE) {  // byte-oriented readers: no terminator index
        wave_sync();
        w.d = d;
        w.woff = woff;
        w.K = 0;
        w.p0 = p;
        w.valid = true;
        w.serial = false;
        return;
    }
    const int32_t q0 = woff + 16 * l;
    const uint32_t V = range16((VAL == VAL_J4 ? p : 0) - q0, end - q0);  // J4 indexes from p only
    const uint32_t H = hibits16(d);
    uint32_t T = (VAL == VAL_VB) ? (V & H) : (V & ~H);
    bool serial = false;
    if (VAL == VAL_J4) {
        // a run of four continuation bytes changes the capped grammar: parse serially
        const uint32_t N = V & ~T;
        uint32_t prevN = (uint32_t)__shfl_up((int)N, 1, 64);
        if (l == 0) prevN = 0;
        const uint32_t ext = (N << 3) | ((prevN >> 13) & 7u);
        serial = __any((ext & (ext >> 1) & (ext >> 2) & (ext >> 3)) != 0);
    }
    int32_t K;
    if (!serial) {
        const uint32_t cnt = __popc(T);
        const uint32_t inc = incl_scan(cnt);
        uint32_t idx = inc - cnt;
        sm.cpre[l] = (uint16_t)idx;
        sm.cmask[l] = (uint16_t)T;
        w.cpre = idx;
        w.cmsk = T;
        while (T) {
            const int k = __ffs(T) - 1;
            T &= T - 1;
            sm.u.v.list[idx++] = (uint16_t)(16 * l + k);
        }
        K = (int32_t)lane_bcast(inc, 63);
    } else {
        wave_sync();
        if (l == 0) {  // DecodingUtils.java:157-186, one value at a time from p
            const int32_t lim = (end < woff + kWin ? end : woff + kWin) - woff;
            int32_t j = p - woff, k = 0;
            while (j < lim) {
                int32_t len = 0;
                bool done = false;
                for (int b = 0; b < 4; ++b) {
                    if (j + b >= lim) break;
                    ++len;
                    if (b == 3 || (win_byte(sm, j + b) & 0x80u) == 0) { done = true; break; }
                }
                if (!done) break;
                sm.u.v.list[k++] = (uint16_t)(j + len - 1);
                j += len;
            }
            sm.misc[0] = k;
        }
        wave_sync();
        K = uni(sm.misc[0]);
    }
    wave_sync();
    w.d = d;
    w.woff = woff;
    w.K = K;
    w.p0 = p;
    w.valid = true;
    w.serial = serial || VAL == VAL_J4;
}

// terminators of the window before stream position q (q inside the window)
__device__ __forceinline__ int32_t win_rank(const WaveSmem& sm, const Win& w, int32_t q) {
    const int32_t j = q - w.woff;
    if (j <= 0) return 0;
    if (j >= kWin) return w.K;
    const int32_t c = j >> 4;
    return (int32_t)uniu((uint32_t)sm.cpre[c] + __popc((uint32_t)sm.cmask[c] & ((1u << (j & 15)) - 1u)));
}

// Decode up to `want` values starting at stream position `pos` (a value boundary; updated) with
// bytes valid in [pos, end).  emit(lo, hi, base, count) is called per group of <=64 values, one per
// lane.  Returns the number of values decoded.  With `until_end` (VariableByte tail) the region is
// decoded to its end, a trailing partial value is dropped and more than `want` values is an error.
// one value whose bytes are window bytes [sj, ej] (ej = its terminator) in grammar VAL
template <int VAL>
__device__ __forceinline__ void win_value(const WaveSmem& sm, int32_t sj, int32_t ej, uint32_t& lo, uint32_t& hi,
                                          bool& lerr) {
    const int32_t len = ej - sj + 1;
    uint32_t x0, x1, x2;
    win_bytes12(sm, sj, x0, x1, x2);
    lo = 0;
    hi = 0;
    if (VAL == VAL_J4) {
        lo = pext7(x0 & bytemask(len));
    } else if (VAL == VAL_VB) {
        if (len <= 5) {
            lo = pext7(x0 & bytemask(len));
            if (len == 5) lo += (x1 & 0x7fu) << 28;
        } else {  // VariableByte.uncompress: v += (c & 127) << shift, shift masked to 5 bits
            uint32_t vv = 0;
            for (int b = 0; b < len; ++b) vv += (win_byte(sm, sj + b) & 0x7fu) << ((7 * b) & 31);
            lo = vv;
        }
    } else {
        uint64_t rv;
        if (len <= 10) {
            const uint32_t m0 = x0 & bytemask(len), m1 = x1 & bytemask(len - 4), m2 = x2 & bytemask(len - 8);
            rv = (uint64_t)pext7(m0) | ((uint64_t)pext7(m1) << 28) | ((uint64_t)(m2 & 0x7fu) << 56) |
                 ((uint64_t)((m2 >> 8) & 0x7fu) << 63);
        } else {  // orc readVulong: shift masked to 6 bits
            rv = 0;
            for (int b = 0; b < len; ++b) rv |= (uint64_t)(win_byte(sm, sj + b) & 0x7fu) << ((7 * b) & 63);
            lerr = true;
        }
        lo = (uint32_t)rv;
        hi = (uint32_t)(rv >> 32);
    }
}

// Decode up to `want` values starting at stream position `pos` (a value boundary; updated) with
// bytes valid in [pos, end).  emit(lo[K], hi[K], base, first, count) is called per group of 64 K
// slots, lane l holding slots base + K l .. base + K l + K - 1 (base counted from this call's first
// value, which is output index out0: groups are aligned so that out0 + base is a multiple of K);
// slots [first, first + count) are values.  Returns the number of values decoded.  With `until_end`
// (VariableByte tail) the region is decoded to its end, a trailing partial value is dropped and
// more than `want` values is an error.  VAL_U64_STRICT with `first_bad`: the index (from this call's
// first value) of the first over-long value is stored there when one stops the call.
// `line` (values per 128-byte output line, a power of two; 0: off): a window's values end on an output
// line unless they are the call's last -- the tail of a line is decoded from the next window, which
// starts at it -- so no output line is written in two parts by consecutive windows (varint WRITE_SIZE
// was 1.10x the output bytes, profiles/r03/pmc_traffic.txt)
#ifndef COVT_VARINT_LINES
#define COVT_VARINT_LINES 1
#endif
template <int MODE, int VAL, int K = 1, class Emit>
__device__ int32_t varint_take(WaveSmem& sm, const uint8_t* sb, Win& w, int32_t& pos, int32_t end, int32_t want,
                               bool until_end, int32_t& err, Emit&& emit, int32_t out0 = 0,
                               int32_t* first_bad = nullptr, int32_t line = 0, const uint32_t* lsrc = nullptr,
                               int32_t lw0 = 0) {
    const int l = lane_id();
    int32_t got = 0;
    while (until_end ? (pos < end) : (got < want)) {
        if (!w.valid || pos < w.woff || pos >= w.woff + kWin || (w.serial && pos != w.p0)) {
            win_load<MODE, VAL>(sm, sb, w, pos, end, lsrc, lw0);
            lsrc = nullptr;  // (the first window's index overwrites the staged words)
        }
        const int32_t r = w.serial ? 0 : win_rank(sm, w, pos);
        const int32_t have = w.K - r;
        if (have <= 0) {
            const int32_t aligned = (MODE == MODE_RAW) ? (int32_t)(((uintptr_t)(sb + pos) & ~(uintptr_t)15) -
                                                                   (uintptr_t)sb)
                                                       : (pos & ~15);
            if (w.woff != aligned) {  // the value straddles the window end: reload at pos
                win_load<MODE, VAL>(sm, sb, w, pos, end);
                continue;
            }
            if (until_end) break;  // VariableByte: trailing partial value is dropped
            err = (w.woff + kWin >= end) ? COVT_ERR_TRUNCATED : COVT_ERR_BAD_HEADER;
            break;
        }
        int32_t take = have;
        if (until_end) {
            if (got + have > want) { err = COVT_ERR_COUNT_MISMATCH; take = want - got; }
        } else if (take > want - got) {
            take = want - got;
        }
        if (take <= 0) break;
        if (COVT_VARINT_LINES && MODE == MODE_RAW && line && !until_end && got + take < want) {
            const int32_t cut = (out0 + got + take) & (line - 1);  // values past the window's last whole line
            if (cut < take) {
                take -= cut;
            } else {
                const int32_t aligned = (int32_t)(((uintptr_t)(sb + pos) & ~(uintptr_t)15) - (uintptr_t)sb);
                if (w.woff != aligned) {  // only a line's tail left here: restart the window at it
                    win_load<MODE, VAL>(sm, sb, w, pos, end);
                    continue;
                }
            }
        }
        bool lerr = false;
        int32_t fb = INT32_MAX;  // first over-long value (VAL_U64_STRICT, first_bad)
        const int32_t s0 = pos - w.woff;
        const int32_t lead = (K > 1) ? ((out0 + got) & (K - 1)) : 0;  // slots before the first value
        for (int32_t g = -lead; g < take; g += 64 * K) {
            uint32_t lo[K], hi[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                int32_t vi = g + K * l + k;
                vi = vi < 0 ? 0 : (vi < take ? vi : take - 1);  // slots outside repeat an edge value (not emitted)
                const int32_t li = r + vi - 1;
                const int32_t pv = (int32_t)sm.u.v.list[li < 0 ? 0 : li] + 1;
                const int32_t sj = vi == 0 ? s0 : pv;  // the value starts after the previous terminator
                if constexpr (VAL == VAL_J4) {
                    // Java's 4-byte-capped varint: its bytes end at the first terminator among the 4 at
                    // sj (or all 4): mask = bits up to that terminator's bit 7, no length needed
                    const int32_t dq = sj >> 2;
                    const uint32_t x = __builtin_amdgcn_alignbyte(sm.u.v.win[dq + 1], sm.u.v.win[dq], (uint32_t)sj & 3u);
                    const uint32_t u = ~x & 0x80808080u;
                    lo[k] = pext7(x & (u ^ (u - 1u)));
                    hi[k] = 0;
                } else {
                    bool lk = false;
                    win_value<VAL>(sm, sj, sm.u.v.list[r + vi], lo[k], hi[k], lk);
                    if (VAL == VAL_U64_STRICT && first_bad && lk) fb = min(fb, got + vi);
                    lerr = lerr || lk;
                }
            }
            const int32_t first = g < 0 ? -g : 0;
            const int32_t cnt = (take - g < 64 * K ? take - g : 64 * K) - first;
            emit(lo, hi, got + g, first, cnt);
        }
        if (VAL == VAL_U64_STRICT && __any(lerr) && !err) {
            err = COVT_ERR_BAD_HEADER;
            if (first_bad) *first_bad = (int32_t)~wave_max(~(uint32_t)fb);
        }
        pos = w.woff + (int32_t)uniu(sm.u.v.list[r + take - 1]) + 1;
        if (w.serial) { w.p0 = pos; w.valid = false; }  // serial lists are only valid from p0
        got += take;
        if (err) break;
    }
    return got;
}

// --------------------------------------------------------------------------------------------
// per-op drivers
// --------------------------------------------------------------------------------------------
struct Ctx {
    WaveSmem* sm;
    const uint8_t* sb;  // stream payload
    uint8_t* out;       // stream output
    int32_t avail, n, nb, op, byte_length;
    int32_t err, consumed;
#ifdef COVT_TIMING
    uint64_t ph_last;
    uint32_t ph[kPhases];
#endif
};
// profiling build only: shader clocks spent per phase of a stream's decode
#ifdef COVT_TIMING
#define COVT_PHASE(c, k)                                          \
    do {                                                          \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();         \
        (c).ph[k] += (uint32_t)(t_ - (c).ph_last);                \
        (c).ph_last = t_;                                         \
    } while (0)
#else
#define COVT_PHASE(c, k) \
    do {                 \
    } while (0)
#endif

// byte q of the stream through the window (loaded on demand so that [q, q + need) is inside
// the window unless the stream ends first); wave-uniform
template <int VAL>
__device__ __forceinline__ uint32_t rd_byte(Ctx& c, Win& w, int32_t q, int32_t need = 1) {
    if (!w.valid || q < w.woff || (q + need > w.woff + kWin && w.woff + kWin < c.avail))
        win_load<MODE_RAW, VAL>(*c.sm, c.sb, w, q, c.avail);
    return uniu(win_byte(*c.sm, q - w.woff));
}

// 64-bit LEB128 values (ids; INT_64 property columns in format mode: zigzag64, + running sum `acc`,
// carried across groups, uniform) for slots base + 4 lane .. + 3 of the group, values [first, first + count)
template <int OP>
__device__ __forceinline__ void sink_u64(const uint32_t (&lo)[4], const uint32_t (&hi)[4], int64_t base, int32_t first,
                                         int32_t count, int64_t* o, uint64_t& acc) {
    const int32_t s0 = 4 * lane_id() - first;
    int64_t* p = o + base + 4 * lane_id();
    uint64_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool ok = s0 + k >= 0 && s0 + k < count;
        v[k] = ok ? (((uint64_t)hi[k] << 32) | lo[k]) : 0ull;
        if constexpr (OP != COVT_OP_VARINT_U64) v[k] = (uint64_t)zz64(v[k]);  // zz(0) = 0
    }
    if constexpr (OP == COVT_OP_VARINT_ZZ_DELTA_S64) {
        uint64_t sacc = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            sacc += v[k];
            v[k] = sacc;
        }
        const uint64_t inc = incl_scan64(sacc);
        const uint64_t pre = acc + inc - sacc;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += pre;
        acc += lane_bcast64(inc, 63);
    }
    if (s0 >= 0 && s0 + 4 <= count) {
        st_out16((int32_t*)p, make_int4((int)v[0], (int)(v[0] >> 32), (int)v[1], (int)(v[1] >> 32)));
        st_out16((int32_t*)(p + 2), make_int4((int)v[2], (int)(v[2] >> 32), (int)v[3], (int)(v[3] >> 32)));
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (s0 + k >= 0 && s0 + k < count) st_out(p + k, (int64_t)v[k]);
    }
}

template <int OP>
__device__ __forceinline__ void run_varint_stream(Ctx& c) {
    // values per 128-byte output line: 8-byte outputs (ids as int64, Morton x,y pairs) 16, else 32
    constexpr int32_t kLine = (OP == COVT_OP_VARINT_I32_AS_I64 || OP == COVT_OP_VARINT_ZZ_I32_AS_I64 ||
                               OP == COVT_OP_VARINT_ZZ_DELTA_I64 || OP == COVT_OP_VARINT_DELTA_MORTON) ? 16 : 32;
    int32_t pos = 0;
    Carry cr{0, 0};
    Win w;
    w.valid = false;
    auto sink4 = [&](const uint32_t (&lo)[4], const uint32_t (&hi)[4], int32_t base, int32_t first, int32_t count) {
        sink_values<OP, 4>(lo, base, first, count, c.nb, c.out, cr);
    };
    if constexpr (OP == COVT_OP_VARINT_U64 || OP == COVT_OP_VARINT_ZZ_S64 || OP == COVT_OP_VARINT_ZZ_DELTA_S64) {
        uint64_t acc = 0;
        varint_take<MODE_RAW, VAL_U64_STRICT, 4>(
            *c.sm, c.sb, w, pos, c.avail, c.n, false, c.err,
            [&](const uint32_t (&lo)[4], const uint32_t (&hi)[4], int32_t base, int32_t first, int32_t count) {
                sink_u64<OP>(lo, hi, base, first, count, (int64_t*)c.out, acc);
            },
            0, nullptr, 16);
    } else {
        if ((OP == COVT_OP_VARINT_ZZ_DELTA_XY) && (c.n & 1)) {
            // Java decodes the x,y pair and then overruns values[] (ArrayIndexOutOfBounds)
            varint_take<MODE_RAW, VAL_J4, 4>(*c.sm, c.sb, w, pos, c.avail, c.n - 1, false, c.err, sink4, 0, nullptr,
                                             kLine);
            if (!c.err) c.err = COVT_ERR_COUNT_MISMATCH;
        } else {
            varint_take<MODE_RAW, VAL_J4, 4>(*c.sm, c.sb, w, pos, c.avail, c.n, false, c.err, sink4, 0, nullptr, kLine);
        }
    }
    c.consumed = pos;
}

// terminators before window-relative position j (per lane, j in [0, kWin])
__device__ __forceinline__ int32_t rank_rel(const WaveSmem& sm, int32_t j, int32_t K) {
    if (j >= kWin) return K;
    const int32_t c = j >> 4;
    return (int32_t)sm.cpre[c] + __popc((uint32_t)sm.cmask[c] & ((1u << (j & 15)) - 1u));
}
// 64-bit LEB128 value in window bytes [sj, ej] (orc SerializationUtils.readVulong)
__device__ __forceinline__ uint64_t win_vulong(const WaveSmem& sm, int32_t sj, int32_t ej) {
    const int32_t len = ej - sj + 1;
    if (len <= 10) {
        uint32_t x0, x1, x2;
        win_bytes12(sm, sj, x0, x1, x2);
        const uint32_t m0 = x0 & bytemask(len), m1 = x1 & bytemask(len - 4), m2 = x2 & bytemask(len - 8);
        return (uint64_t)pext7(m0) | ((uint64_t)pext7(m1) << 28) | ((uint64_t)(m2 & 0x7fu) << 56) |
               ((uint64_t)((m2 >> 8) & 0x7fu) << 63);
    }
    uint64_t r = 0;  // shift masked to 6 bits
    for (int b = 0; b < len; ++b) r |= (uint64_t)(win_byte(sm, sj + b) & 0x7fu) << ((7 * b) & 63);
    return r;
}
// its low 32 bits (the (int) of RLE_I32): bytes 5..9 only reach bits >= 35, so up to 10 bytes the
// first five decide; longer (malformed) varints wrap their shifts and take the full path
__device__ __forceinline__ uint32_t win_vulong_lo32(const WaveSmem& sm, int32_t sj, int32_t ej) {
    const int32_t len = ej - sj + 1;
    if (len > 10) return (uint32_t)win_vulong(sm, sj, ej);
    const int32_t d = sj >> 2;
    const uint32_t sh = (uint32_t)(sj & 3);
    const uint32_t w0 = sm.u.v.win[d], w1 = sm.u.v.win[d + 1], w2 = sm.u.v.win[d + 2];
    const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, sh), x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    return pext7(x0 & bytemask(len)) | (len >= 5 ? (x1 & 0x7fu) << 28 : 0u);
}

// ORC RLE v1 integer reader (RunLengthIntegerReader.readValues / next).
// Per 1 KiB window: (1) every byte position j computes, from the terminator index, where the next
// group would start if a header sat at j (run: after the base varint at j+2; literal: after the
// (256-c)-th varint from j+1) -- fully lane-parallel; (2) one wave-uniform walk follows that chain
// (one LDS read per group) and records the group starts; (3) groups expand lane-parallel: small
// groups one per lane, groups of more than 8 values with the whole wave.
// o0: output index of the first value (a split chunk of a stream: its stream bytes start at c.sb, its
// values are [o0, c.n) of the stream's output at c.out)
__device__ __forceinline__ void run_rle_int(Ctx& c, int32_t o0 = 0) {
    WaveSmem& sm = *c.sm;
    const int l = lane_id();
    const bool is_signed = c.op == COVT_OP_RLE_S64;
    const bool to_i32 = c.op == COVT_OP_RLE_I32;
    Win w;
    w.valid = false;
    int32_t pos = 0, done = o0;
    auto store = [&](int64_t i, uint64_t raw) {
        const int64_t v = is_signed ? zz64(raw) : (int64_t)raw;
        if (to_i32) st_out((int32_t*)c.out + i, (int32_t)v);
        else st_out((int64_t*)c.out + i, v);
    };
    while (done < c.n && !c.err) {
        if (pos >= c.avail) { c.err = COVT_ERR_TRUNCATED; break; }
        COVT_PHASE(c, 7);
        win_load<MODE_RAW, VAL_U64>(sm, c.sb, w, pos, c.avail);
        COVT_PHASE(c, 0);
        const int32_t woff = w.woff, K = w.K;
        const int32_t jlo = pos - woff;  // (positions at or past the valid end rank K: no group there)
        // (1) next[] for this lane's 16 positions, branch-free: the terminator rank of position
        // 16l + k is R[k] (incremental popcounts of this lane's chunk mask, then the next lane's).
        // Entries hold the LDS byte address of next[target] (the walk's read -> read chain then needs
        // no arithmetic); "no group completes here" is the sentinel next[kWin], which points at itself.
        const uint32_t nb = (uint32_t)(uintptr_t)(lds_cu16*)&sm.u.v.next[0];
        const uint32_t sent = nb + 2u * (uint32_t)kWin;
        // live positions: [jlo, vlen) (the walk starts at jlo; a group ends at most at vlen)
        const int32_t vlen = min(kWin, c.avail - woff);
        if (vlen - jlo <= COVT_RLE_SHORT_SPAN) {
            // a short window (a stream's last, or a short stream): position-major, one position per lane and
            // step -- ceil(live / 64) steps instead of every lane's 16 positions; each position's terminator
            // rank from the window index (cpre / cmask).  Positions outside [jlo, vlen] are never visited.
            if (l == 0) {
                if (vlen < kWin) sm.u.v.next[vlen] = (uint16_t)sent;
                sm.u.v.next[kWin] = (uint16_t)sent;
            }
            const int32_t its = uni((vlen - jlo + 63) >> 6);
            for (int32_t i = 0; i < its; ++i) {
                const int32_t j = jlo + 64 * i + l;
                uint32_t nx = sent;
                if (j < vlen) {
                    const uint32_t cb = win_byte(sm, j);
                    const int32_t x = j + (cb < 0x80u ? 2 : 1);  // run: rank of j + 2; literal: of j + 1
                    uint32_t rk = (uint32_t)K;
                    if (x < kWin) {
                        const int32_t ch = x >> 4;
                        rk = (uint32_t)sm.cpre[ch] + __popc((uint32_t)sm.cmask[ch] & ((1u << (x & 15)) - 1u));
                    }
                    const uint32_t ridx = cb < 0x80u ? rk : rk + (0xffu - cb);
                    if (ridx < (uint32_t)K) nx = nb + 2u * ((uint32_t)sm.u.v.list[ridx] + 1u);
                }
                if (j < kWin) sm.u.v.next[j] = (uint16_t)nx;
            }
        } else {
            const uint32_t ncmsk = lane_next(w.cmsk);
            uint32_t R[18];
            R[0] = w.cpre;
#pragma unroll
            for (int k = 0; k < 16; ++k) R[k + 1] = R[k] + ((w.cmsk >> k) & 1u);
            R[17] = R[16] + (ncmsk & 1u);
            const uint32_t dw[4] = {w.d.x, w.d.y, w.d.z, w.d.w};
            uint32_t nx2[8];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int32_t j = 16 * l + k;
                const uint32_t cb = (dw[k >> 2] >> (8 * (k & 3))) & 0xffu;
                // run: the base varint ends at terminator R[k+2]; literals: the (256-cb)-th from R[k+1]
                const uint32_t ridx = cb < 0x80u ? R[k + 2] : R[k + 1] + (0xffu - cb);
                const uint32_t e = (uint32_t)sm.u.v.list[ridx < (uint32_t)kWin ? ridx : (uint32_t)kWin - 1] + 1u;
                const uint32_t nx = (j >= jlo && ridx < (uint32_t)K) ? nb + 2u * e : sent;
                if (k & 1) nx2[k >> 1] |= nx << 16;
                else nx2[k >> 1] = nx;
            }
            ((uint4*)sm.u.v.next)[2 * l] = make_uint4(nx2[0], nx2[1], nx2[2], nx2[3]);
            ((uint4*)sm.u.v.next)[2 * l + 1] = make_uint4(nx2[4], nx2[5], nx2[6], nx2[7]);
            if (l == 0) sm.u.v.next[kWin] = (uint16_t)sent;  // a group ending at the window end
        }
        wave_sync();
        COVT_PHASE(c, 1);
        // (2) chain walk, 64 groups at a time (lane g of `gs` = start of group g), (3) each batch
        // expanded right away: small groups one per lane, groups of more than 8 values by the wave
        int32_t pj = jlo, out = done;
        bool first = true;
        while (true) {
            // the walk only follows next[]: value counts (and the stop at n) come from the batch scan
            int32_t G = 0;
            uint32_t gs = 0;
            const int32_t out0 = out;
            {
                // Eight steps per scalar test, branch-free: the chain's critical path is one LDS read
                // whose result is the next read's address.  Steps past the end are no-ops (the sentinel
                // points at itself); lanes left at ~0 hold no group.
                auto rd = [](uint32_t a) -> uint32_t { return *(lds_cu16*)(uintptr_t)a; };
                uint16_t* const rec = sm.u.v.grec;
                const uint32_t c0 = nb + 2u * (uint32_t)pj;
                uint32_t nx = rd(c0);
                int32_t steps = 64;
                for (int32_t g0 = 0; g0 < 64; g0 += 8) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        rec[g0 + k] = (uint16_t)nx;
                        nx = rd(nx);
                    }
                    if (uniu(nx) == sent) {
                        steps = g0 + 8;
                        break;
                    }
                }
                wave_sync();
                const uint32_t mine = l < steps ? (uint32_t)rec[l] : sent;
                const uint32_t prev = l == 0 ? c0 : (l <= steps ? (uint32_t)rec[l - 1] : sent);
                const bool gv0 = mine != sent;
                G = __popcll(__ballot(gv0));
                gs = gv0 ? (prev - nb) >> 1 : ~0u;  // positions
                pj = G > 0 ? (int32_t)((lane_bcast(mine, G - 1) - nb) >> 1) : pj;
                wave_sync();
            }
            COVT_PHASE(c, 2);
            if (G == 0) {
                if (!first) break;
                // the group at pos does not complete inside this window
                const uint32_t cb = uniu(win_byte(sm, jlo));
                const int32_t aligned = (int32_t)(((uintptr_t)(c.sb + pos) & ~(uintptr_t)15) - (uintptr_t)c.sb);
                // (<=: a literal ending exactly at the window end has next[] = next[kWin], the sentinel)
                if (cb >= 0x80u && woff == aligned && woff + kWin <= c.avail) {
                    // a literal group longer than a window (up to 128 x 10 B): multi-window varint path
                    const int32_t cnt = 0x100 - (int32_t)cb, lim = c.n - done, d0 = done;
                    int32_t p1 = pos + 1;
                    varint_take<MODE_RAW, VAL_U64>(
                        sm, c.sb, w, p1, c.avail, cnt, false, c.err,
                        [&](const uint32_t (&lo)[1], const uint32_t (&hi)[1], int32_t base, int32_t, int32_t count) {
                            const int32_t k = base + l;
                            if (l < count && k < lim) store(d0 + k, ((uint64_t)hi[0] << 32) | lo[0]);
                        });
                    out = done + (cnt < lim ? cnt : lim);
                    pj = p1 - woff;
                    COVT_PHASE(c, 5);
                    break;
                }
                c.err = (woff + kWin >= c.avail) ? COVT_ERR_TRUNCATED : COVT_ERR_BAD_HEADER;
                break;
            }
            first = false;
            {
                const bool gv = l < G;
                const int32_t pg = gv ? (int32_t)gs : 0;
                const uint32_t cb = gv ? win_byte(sm, pg) : 0u;
                const int32_t cnt = !gv ? 0 : (cb < 0x80u ? (int32_t)cb + 3 : 0x100 - (int32_t)cb);
                const uint32_t inc = incl_scan((uint32_t)cnt);
                const int32_t goff = out0 + (int32_t)(inc - (uint32_t)cnt);
                int32_t take = c.n - goff;
                take = take < 0 ? 0 : (take > cnt ? cnt : take);
                out = out0 + (int32_t)lane_bcast(inc, 63);
                if (out >= c.n) {  // the batch reaches n: stop after the group that does (Java reads no further)
                    const uint64_t fin = __ballot(gv && goff + cnt >= c.n);
                    const int gl = __ffsll((long long)fin) - 1;
                    const uint32_t nxt = lane_bcast(gs, gl + 1 < 64 ? gl + 1 : 63);
                    pj = gl + 1 < G ? (int32_t)nxt : pj;
                }
                // runs, base + i * delta: one lane per run of at most 8 values (a wave-uniform trip
                // count; lanes past their run's end repeat its last value, same address and data),
                // the whole wave per longer run
                const bool isrun = cb < 0x80u;
                const int32_t rr = gv ? rank_rel(sm, pg + (isrun ? 2 : 1), K) : 0;
                const bool rv = gv && isrun && take > 0;
                int64_t b64 = 0;
                int32_t delta = 0;
                if (rv) {
                    delta = (int32_t)(int8_t)win_byte(sm, pg + 1);
                    if (to_i32) {  // (int): the low 32 bits of the base, 32-bit arithmetic from here on
                        b64 = (int64_t)(int32_t)win_vulong_lo32(sm, pg + 2, sm.u.v.list[rr]);
                    } else {
                        const uint64_t raw = win_vulong(sm, pg + 2, sm.u.v.list[rr]);
                        b64 = is_signed ? zz64(raw) : (int64_t)raw;
                    }
                }
#if defined(COVT_ABL_RLE_NORUN)  // ablation build: runs not expanded (outputs wrong)
                const bool small = false;
#else
                const bool small = rv && take <= 8;
#endif
                const int32_t tmax = (int32_t)wave_max((uint32_t)(small ? take : 0));
                if (small && to_i32) {
                    int32_t* const o = (int32_t*)c.out + goff;
                    const uint32_t b32 = (uint32_t)b64;
                    for (int32_t i0 = 0; i0 < tmax; ++i0) {
                        const int32_t i = i0 < take ? i0 : take - 1;
                        st_out(o + i, (int32_t)(b32 + (uint32_t)(i * delta)));
                    }
                } else if (small) {
                    for (int32_t i0 = 0; i0 < tmax; ++i0) {
                        const int32_t i = i0 < take ? i0 : take - 1;
                        const int64_t v = (int64_t)((uint64_t)b64 + (uint64_t)(int64_t)(int32_t)(i * delta));
                        st_out((int64_t*)c.out + goff + i, v);
                    }
                }
                const bool big = rv && take > 8;
                const uint64_t bigm = __ballot(big);
                if (bigm) {  // the batch's long runs, compacted to lanes 0..nbig-1, four at a time
                    const int32_t nbig = __popcll(bigm);
                    const uint64_t below = (1ull << l) - 1ull;
                    const int32_t dst = big ? __popcll(bigm & below) : nbig + __popcll(~bigm & below);
                    const int32_t co = __builtin_amdgcn_ds_permute(dst << 2, goff);
                    const int32_t ct = __builtin_amdgcn_ds_permute(dst << 2, big ? take : 0);
                    const int32_t cd = __builtin_amdgcn_ds_permute(dst << 2, delta);
                    const int32_t cbl = __builtin_amdgcn_ds_permute(dst << 2, (int32_t)(uint32_t)b64);
                    const int32_t cbh = __builtin_amdgcn_ds_permute(dst << 2, (int32_t)(uint32_t)((uint64_t)b64 >> 32));
                    for (int32_t r0 = 0; r0 < nbig; r0 += 4) {
                        const int32_t src = r0 + (l >> 4);  // this quarter's run
                        // (every lane_get with the whole wave active: a bpermute under a select can become a
                        // branch, and a source lane off in EXEC reads 0)
                        const int32_t o2 = lane_get(co, src & 63);
                        const int32_t tk = lane_get(ct, src & 63);
                        const int32_t t2 = src < nbig ? tk : 0;
                        const int32_t d2 = lane_get(cd, src & 63);
                        const int64_t bb = (int64_t)(((uint64_t)(uint32_t)lane_get(cbh, src & 63) << 32) |
                                                     (uint32_t)lane_get(cbl, src & 63));
                        if (to_i32) store_run_q<4>(c.out, o2, t2, bb, d2);  // literals[0] + used * delta
                        else store_run_q<8>(c.out, o2, t2, bb, d2);
                    }
                }
                COVT_PHASE(c, 3);
                // literals: every literal value of the batch, 64 per step whatever the group sizes.
                // Literal groups are compacted to lanes 0..nl-1 (ds_permute); value u's group is the
                // number of group starts at or before u (ballot over the starts <= u0, then a 64-bit
                // mask of the starts inside the step), and its varint is terminator rank rr + (u - ust).
                const bool lv = gv && !isrun && take > 0;
                const uint32_t lc = lv ? (uint32_t)take : 0u;
                const uint32_t linc = incl_scan(lc);
#if defined(COVT_ABL_RLE_NOLIT)  // ablation build: literals not expanded (outputs wrong)
                const int32_t U = 0 * (int32_t)lane_bcast(linc, 63);
#else
                const int32_t U = (int32_t)lane_bcast(linc, 63);
#endif
                // Dictionary-index columns are mostly literal groups of one-byte varints (values < 128):
                // when every literal value of the batch is one byte (a group's `take` values end on
                // `take` consecutive terminators right after its header), value u is the window byte
                // u + (its group's first value byte - the group's first u), no varint parse.
                const bool one = !lv || (int32_t)sm.u.v.list[lv ? rr + take - 1 : 0] == pg + take;
                if (U > 0 && __ballot(!one) == 0) {
                    const uint64_t lm = __ballot(lv), below = (1ull << l) - 1ull;
                    const int32_t nl = __popcll(lm);
                    const int32_t dst = lv ? __popcll(lm & below) : nl + __popcll(~lm & below);
                    const int32_t ust = (int32_t)(linc - lc);
                    // byte and output offsets relative to u, 15 + 17 bits (pg < 1024, ust and goff - out0 < 2^14)
                    const uint32_t pk = (uint32_t)(pg + 1 - ust + 16384) | ((uint32_t)(goff - out0 - ust) << 15);
                    const int32_t cust = __builtin_amdgcn_ds_permute(dst << 2, lv ? ust : 0x3fffffff);
                    const uint32_t cpk = (uint32_t)__builtin_amdgcn_ds_permute(dst << 2, (int32_t)pk);
                    for (int32_t u0 = 0; u0 < U; u0 += 64) {
                        const int32_t s = cust - u0;
                        const int32_t gb = __popcll(__ballot(cust <= u0)) - 1;  // group holding value u0
                        // the groups starting inside the step mark their first value's lane (ds_permute: a lane
                        // no one writes to reads 0, the instruction's defined result; groups without a start
                        // inside send 0 to lane 0, which no start inside the step reaches); a value's group is
                        // gb + the marks at or below its lane: one ballot and a v_mbcnt (was: a DPP running
                        // max over the marking lanes, before that a 64-bit OR reduction)
                        const bool in = s > 0 && s < 64;
                        const int32_t mk = __builtin_amdgcn_ds_permute(in ? s << 2 : 0, in ? 1 : 0);
                        const int32_t gk = gb + bits_below(__ballot(mk != 0)) + mk;
                        const uint32_t info = (uint32_t)lane_get((int32_t)cpk, gk);
                        const int32_t u = u0 + l;
                        if (u < U) {
                            const uint32_t b = win_byte(sm, u + (int32_t)(info & 0x7fffu) - 16384);
                            const int32_t o = out0 + u + (int32_t)(info >> 15);
                            if (to_i32) st_out((int32_t*)c.out + o, (int32_t)b);
                            else store(o, (uint64_t)b);
                        }
                    }
                } else if (U > 0) {
                    const uint64_t lm = __ballot(lv), below = (1ull << l) - 1ull;
                    const int32_t nl = __popcll(lm);
                    const int32_t dst = lv ? __popcll(lm & below) : nl + __popcll(~lm & below);
                    const int32_t ust = (int32_t)(linc - lc);
                    // rank and output offsets relative to u, 15 + 17 bits (rr <= 1024, ust and goff - out0 < 2^14)
                    const uint32_t pk = (uint32_t)(rr - ust + 16384) | ((uint32_t)(goff - out0 - ust) << 15);
                    const int32_t cust = __builtin_amdgcn_ds_permute(dst << 2, lv ? ust : 0x3fffffff);
                    const uint32_t cpk = (uint32_t)__builtin_amdgcn_ds_permute(dst << 2, (int32_t)pk);
                    for (int32_t u0 = 0; u0 < U; u0 += 64) {
                        const int32_t s = cust - u0;
                        const int32_t gb = __popcll(__ballot(cust <= u0)) - 1;  // group holding value u0
                        // marks and groups as in the one-byte path; a group starting at u0 itself is gb
                        const bool in = s > 0 && s < 64;
                        const int32_t mk = __builtin_amdgcn_ds_permute(in ? s << 2 : 0, in ? 1 : 0);
                        const int32_t gk = gb + bits_below(__ballot(mk != 0)) + mk;
                        const bool gfirst = mk != 0 || (l == 0 && __builtin_amdgcn_readlane(cust, gb) == u0);
                        const uint32_t info = (uint32_t)lane_get((int32_t)cpk, gk);
                        const int32_t u = u0 + l;
                        if (u < U) {
                            const int32_t rank = u + (int32_t)(info & 0x7fffu) - 16384;
                            const int32_t o = out0 + u + (int32_t)(info >> 15);
                            const int32_t ej = sm.u.v.list[rank];
                            const int32_t pv = rank > 0 ? (int32_t)sm.u.v.list[rank - 1] : -2;
                            // a group's first varint starts after its header (the byte after the previous
                            // group's last terminator; at the window's first group, after jlo)
                            const int32_t sj = gfirst ? max(pv + 2, jlo + 1) : pv + 1;
                            if (to_i32) st_out((int32_t*)c.out + o, (int32_t)win_vulong_lo32(sm, sj, ej));
                            else store(o, win_vulong(sm, sj, ej));
                        }
                    }
                }
                COVT_PHASE(c, 4);
            }
            if (G < 64 || out >= c.n) break;
        }
        done = out < c.n ? out : c.n;
        pos = woff + pj;
        wave_sync();
    }
    c.consumed = pos;
}

// bytes [a, b) of a 16-byte packet (per lane; a split chunk's edge packets)
__device__ __forceinline__ void store_packet_bytes(uint8_t* dst, const uint32_t (&pk)[4], int32_t a, int32_t b) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k >= a && k < b) st_out(dst + k, (uint8_t)(pk[k >> 2] >> (8 * (k & 3))));
}

// ORC RLE v1 byte reader (RunLengthByteReader); GeometryType.values()[b] range-checked for
// COVT_OP_BYTE_RLE_U8 (present / boolean bitsets: COVT_OP_BYTE_RLE_RAW, no check).
// Same window structure as run_rle_int; a byte-RLE group's length follows from its header byte.
// o0 as in run_rle_int; `exact`: bytes outside [o0, c.n) are never written (a split chunk shares its
// first and last 16-byte packets with its neighbours)
__device__ __forceinline__ void run_rle_byte(Ctx& c, int32_t o0 = 0, bool exact = false) {
    WaveSmem& sm = *c.sm;
    const int l = lane_id();
    Win w;
    w.valid = false;
    int32_t pos = 0, done = o0;
    bool bad = false;
    uint32_t cpk[4] = {0u, 0u, 0u, 0u};  // the carried partial packet (uniform) at output byte cpos
    int32_t cpos = -1;
    while (done < c.n && !c.err) {
        if (pos >= c.avail) { c.err = COVT_ERR_TRUNCATED; break; }
        COVT_PHASE(c, 7);
        win_load<MODE_RAW, VAL_NONE>(sm, c.sb, w, pos, c.avail);
        COVT_PHASE(c, 0);
        const int32_t woff = w.woff;
        const int32_t vend = (c.avail - woff) < kWin ? (c.avail - woff) : kWin;
        int32_t pj = pos - woff, out = done;
        bool lbad = false, first = true;
        // Jump tables: N1[j] = where the next group starts if a header sat at j (kWin: no group completes
        // there; a header's length follows from its byte alone), N8 = N1 applied eight times (three
        // in-place doublings; all reads of a round precede its writes within the wave).  Position kWin-1
        // never completes a group (groups take >= 2 bytes), so reads clamp the sentinel to it.
        lds_cu16* const N1 = (lds_cu16*)&sm.u.v.next[0];
        lds_cu16* const N8 = (lds_cu16*)&sm.u.v.list[0];
        {
            const uint32_t dw[4] = {w.d.x, w.d.y, w.d.z, w.d.w};
            uint32_t nx2[8];  // this lane's 16 entries, two per register
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int32_t j = 16 * l + k;
                const int32_t cbk = (int32_t)((dw[k >> 2] >> (8 * (k & 3))) & 0xffu);
                const int32_t e = cbk < 0x80 ? j + 2 : j + 0x101 - cbk;
                const uint32_t v = (j < vend && e <= vend) ? (uint32_t)e : (uint32_t)kWin;
                nx2[k >> 1] = (k & 1) ? (nx2[k >> 1] | (v << 16)) : v;
            }
            auto put = [&](uint16_t* t) {
                ((uint4*)t)[2 * l] = make_uint4(nx2[0], nx2[1], nx2[2], nx2[3]);
                ((uint4*)t)[2 * l + 1] = make_uint4(nx2[4], nx2[5], nx2[6], nx2[7]);
            };
            put(sm.u.v.next);
            wave_sync();
            lds_cu16* src = N1;
#pragma unroll 1
            for (int r = 0; r < 3; ++r) {  // N2 = N1 o N1, N4 = N2 o N2, N8 = N4 o N4
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t lo = src[min(nx2[k] & 0xffffu, (uint32_t)kWin - 1u)];
                    const uint32_t hi = src[min(nx2[k] >> 16, (uint32_t)kWin - 1u)];
                    nx2[k] = lo | (hi << 16);
                }
                put(sm.u.v.list);
                wave_sync();
                src = N8;
            }
        }
        COVT_PHASE(c, 1);
        while (true) {  // 64 groups at a time (lane g of `gs` = start of group g), each batch expanded
            int32_t G = 0;
            uint32_t gs = 0;
            const int32_t out0 = out;
            {  // lane g: g steps from pj = (g >> 3) N8 steps, then (g & 7) N1 steps (14 dependent reads)
                uint32_t cur = (uint32_t)pj;
                const int a = l >> 3, b = l & 7;
#pragma unroll
                for (int i = 0; i < 7; ++i) {
                    const uint32_t t = N8[min(cur, (uint32_t)kWin - 1u)];
                    cur = i < a ? t : cur;
                }
#pragma unroll
                for (int i = 0; i < 7; ++i) {
                    const uint32_t t = N1[min(cur, (uint32_t)kWin - 1u)];
                    cur = i < b ? t : cur;
                }
                const uint32_t succ = N1[min(cur, (uint32_t)kWin - 1u)];  // group g completes iff != kWin
                G = __popcll(__ballot(succ != (uint32_t)kWin));
                gs = l < G ? cur : ~0u;
                pj = (int32_t)(G < 64 ? lane_bcast(cur, G) : lane_bcast(succ, 63));
            }
            COVT_PHASE(c, 2);
            if (G == 0) {
                if (first) c.err = (woff + kWin >= c.avail) ? COVT_ERR_TRUNCATED : COVT_ERR_BAD_HEADER;
                break;
            }
            first = false;
            const bool gv = l < G;
            const int32_t pg = gv ? (int32_t)gs : 0;
            const uint32_t cb = gv ? win_byte(sm, pg) : 0u;
            const int32_t cnt = !gv ? 0 : (cb < 0x80u ? (int32_t)cb + 3 : 0x100 - (int32_t)cb);
            const uint32_t inc = incl_scan((uint32_t)cnt);
            const int32_t goff = out0 + (int32_t)(inc - (uint32_t)cnt);
            int32_t take = c.n - goff;
            take = take < 0 ? 0 : (take > cnt ? cnt : take);
            out = out0 + (int32_t)lane_bcast(inc, 63);
            if (out >= c.n) {  // stop after the group that reaches n
                const uint64_t fin = __ballot(gv && goff + cnt >= c.n);
                const int gl = __ffsll((long long)fin) - 1;
                const uint32_t nxt = lane_bcast(gs, gl + 1 < 64 ? gl + 1 : 63);
                pj = gl + 1 < G ? (int32_t)nxt : pj;
            }
            // (3) the batch's bytes [out0, outE) as aligned 16-byte packets, one per lane per step (full
            // nontemporal stores; a run-by-run expansion wrote partial lines, ~500 clocks per run).  A
            // packet's first group: binary search over the groups' output starts (ds_bpermute); then its
            // bytes group by group, a run's value or literal bytes straight from the window.  The packet
            // straddling the batch's end is carried into the next batch in registers.
            const bool isrun = cb < 0x80u;
            const uint32_t rv = win_byte(sm, pg + 1);  // a run's value
            lbad |= gv && isrun && take > 0 && rv > 5u;
            const int32_t outE = out < c.n ? out : c.n;
            const int32_t gst = gv ? goff : INT32_MAX, gen = gv ? goff + take : INT32_MAX;
            const int32_t gsrc = !gv ? 0 : (isrun ? (int32_t)(0x10000u | rv) : pg + 1);
            const int32_t P0 = out0 & ~15;
            for (int32_t s0 = P0; s0 < outE; s0 += 64 * 16) {
                const int32_t P = s0 + 16 * l, qe = min(P + 16, outE);
                int32_t q = max(P, out0);
                int32_t gi = 0;  // the last group starting at or before q
#pragma unroll
                for (int st = 32; st > 0; st >>= 1) {
                    const int32_t cand = gi + st;
                    const int32_t v = lane_get(gst, min(cand, 63));
                    gi = (cand < G && v <= q) ? cand : gi;
                }
                const bool hc = P == cpos;  // bytes before out0 come from the carried packet
                uint32_t pk[4] = {hc ? cpk[0] : 0u, hc ? cpk[1] : 0u, hc ? cpk[2] : 0u, hc ? cpk[3] : 0u};
                bool act = q < qe;
                while (__any(act)) {
                    const int32_t g = min(gi, 63);
                    const int32_t gs = lane_get(gst, g), ge = lane_get(gen, g), src = lane_get(gsrc, g);
                    const int32_t hi = min(ge, qe);
                    const int32_t a = q - P, b = hi - P;  // packet bytes [a, b) from group g
                    uint32_t x[4];
                    const bool lit = !(src & 0x10000);
                    if (lit) {
                        const int32_t A = src + (P - gs);  // window byte of packet byte 0 (may be < 0: masked)
                        const int32_t d = A >> 2;
                        const uint32_t sh = (uint32_t)(A & 3);
                        const uint32_t w0 = sm.u.v.win[d], w1 = sm.u.v.win[d + 1], w2 = sm.u.v.win[d + 2],
                                       w3 = sm.u.v.win[d + 3], w4 = sm.u.v.win[d + 4];
                        x[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
                        x[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
                        x[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
                        x[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
                    } else {
                        const uint32_t r4 = ((uint32_t)src & 0xffu) * 0x01010101u;
                        x[0] = x[1] = x[2] = x[3] = r4;
                    }
                    if (act) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t m = bytemask(b - 4 * k) & ~bytemask(a - 4 * k);
                            pk[k] = (pk[k] & ~m) | (x[k] & m);
                            const uint32_t v = x[k] & m;  // GeometryType.values()[b]: bytes > 5
                            lbad |= lit && (((v | ((v & 0x7f7f7f7fu) + 0x7a7a7a7au)) & 0x80808080u & m) != 0u);
                        }
                        q = hi;
                        ++gi;
                    }
                    act = q < qe;
                }
                if (P + 16 <= outE) {
                    if (P >= o0) st_out16((int32_t*)(c.out + P), make_int4((int)pk[0], (int)pk[1], (int)pk[2], (int)pk[3]));
                    else store_packet_bytes(c.out + P, pk, o0 - P, 16);  // a chunk's first packet
                }
                const uint64_t part = __ballot(P < outE && P + 16 > outE);
                if (part) {  // the batch's last packet, partial: carried
                    const int src = __ffsll((long long)part) - 1;
#pragma unroll
                    for (int k = 0; k < 4; ++k) cpk[k] = lane_bcast(pk[k], src);
                    cpos = (int32_t)lane_bcast((uint32_t)P, src);
                }
            }
            COVT_PHASE(c, 4);
            if (G < 64 || out >= c.n || pj >= vend) break;
        }
        bad |= __any(lbad);
        done = out < c.n ? out : c.n;
        pos = woff + pj;
        wave_sync();
    }
    // the last partial packet, stored whole (a stream's output slice is padded to 16 bytes) or, for a
    // chunk, byte by byte
    if (cpos >= 0 && (done & 15) && cpos == (done & ~15) && l == 0) {
        if (exact) store_packet_bytes(c.out + cpos, cpk, max(o0 - cpos, 0), done - cpos);
        else st_out16((int32_t*)(c.out + cpos), make_int4((int)cpk[0], (int)cpk[1], (int)cpk[2], (int)cpk[3]));
    }
    if (!c.err && bad && c.op == COVT_OP_BYTE_RLE_U8) c.err = COVT_ERR_BAD_HEADER;  // GeometryType.values()[b]
    c.consumed = pos;
}

// ---- FastPFOR ------------------------------------------------------------------------------
struct Words {
    const uint8_t* sb;
    int32_t nw;
    __device__ __forceinline__ uint32_t operator()(int64_t i) const { return ld_be32(sb + 4 * i); }
    // word i at a wave-uniform index, through the scalar cache (s_load; no vmcnt wait on the stores
    // in flight)
    __device__ __forceinline__ uint32_t uniform(int64_t i) const { return sld_be32(sb + 4 * i); }
};

// exception value X[k][i] (dataTobePacked[k]); words past the stream read as 0
__device__ __forceinline__ uint32_t xget(const Words& W, uint32_t xs, int k, uint32_t i) {
    const int64_t bit = (int64_t)(i & 31u) * k;
    const int64_t wi = (int64_t)xs + (int64_t)(i >> 5) * k + (bit >> 5);
    const int off = (int)(bit & 31);
    const uint64_t lo = wi < W.nw ? W(wi) : 0u;
    const uint64_t hi = (off + k > 32 && wi + 1 < W.nw) ? W(wi + 1) : 0u;
    const uint64_t m = k == 32 ? 0xffffffffull : ((1ull << k) - 1ull);
    return (uint32_t)(((lo | (hi << 32)) >> off) & m);
}
// One FastPFOR block header walked out of the byte container (FastPFOR.decodePage loop body).
struct FpfHdr {
    int32_t b, ce, idx;  // bit width, exception count, maxbits - b
    uint32_t xcur;       // cursor into dataTobePacked[idx] for this block
    int32_t bcoff;       // container offset of the exception positions
    int32_t next;        // container offset of the next block header
};
// Registers prefetched for one block.
struct FpfPre {
    uint4 raw;           // 16 raw bytes of the block's packed words (16-B aligned, lane-major)
    uint32_t pos;        // exception e = lane: its position in the block (e >= 64: LDS posx[])
    uint32_t x0, x1, x2; // exception e = lane: 12 bytes (4-B aligned) covering its packed word(s)
};

// 12 / 8 bytes from a 4-byte aligned global address
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef __attribute__((address_space(1))) const u32x3 g_v3;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x2 g_v2;

// FastPFOR (256-value blocks, 65536-value pages) + VariableByte, JavaFastPFOR 0.1.12 as called by
// DecodingUtils.java:316-444.  Per page the exception-array directory is read and the byte
// container is staged in LDS 1 KiB at a time; blocks then run software-pipelined: while block j
// is unpacked (4 consecutive values per lane), patched and scanned, block j+1's header is walked
// and its packed words, exception positions and exception values are already in flight.  The
// packed words are staged in LDS already aligned to the stream's word grid and byte-swapped, so a
// value costs one ds_read2_b32 and one v_alignbit_b32.
// Output values [v0, v1) only (a split chunk; the whole stream by default): pages before v0 are
// skipped after their directory, blocks before v0 in its page are walked (headers, exception cursors)
// but not decoded, the VariableByte tail and the zero fill belong to the range holding value n - 1.
// sum_only: no stores -- the transformed values (zigzag, or the raw Morton deltas) are summed into
// *sums (x,y ops: .x over even, .y over odd value indices).  `cr0`: the running sums before v0.
template <int OP, int K>
__device__ __forceinline__ void sum_values(const uint32_t (&v)[K], int64_t base, int32_t count, uint32_t& ax,
                                           uint32_t& ay) {
    const int l = lane_id();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool ok = l * K + k < count;
        const uint32_t z = ok ? (OP == COVT_OP_FPF_DELTA_MORTON ? v[k] : (uint32_t)zz32(v[k])) : 0u;
        const bool odd = OP == COVT_OP_FPF_ZZ_DELTA_XY && ((base + l * K + k) & 1);
        ax += odd ? 0u : z;
        ay += odd ? z : 0u;
    }
}
// The block loop's vmcnt waits.  Loads and stores retire in issue order through one counter (gfx950
// has no separate store counter), and the compiler sizes each wait at the loop header for the path
// with the fewest younger operations.  A page's first block is reached from the prefetch alone (no
// stores after it); every later block from the previous block's output stores.  Without help the wait
// for block j's prefetched words therefore also waited for block j-1's output stores on every other
// block (`s_waitcnt vmcnt(1)` instead of vmcnt(3) for Morton).  So the prefetch of the first block is
// followed by the same number of 16-byte stores as a block's sink issues: zeros, cached (they merge in
// L2 with the nontemporal stores of the real values that follow to the same addresses, from the same
// lane, in order).
template <int OP>
__device__ __forceinline__ void fpf_prime_stores(uint8_t* __restrict__ out, int64_t base) {
    const int64_t i0 = base + 4 * (int64_t)lane_id();
    const int4 z = make_int4(0, 0, 0, 0);
    if constexpr (OP == COVT_OP_FPF_DELTA_MORTON) {
        int4* o = (int4*)((int32_t*)out + 2 * i0);
        o[0] = z;
        o[1] = z;
    } else {
        *(int4*)((int32_t*)out + i0) = z;
    }
}
// (sum_only is a run-time flag: two template copies inlined into one chunk kernel made it 248 VGPRs)
// `skip`: a split chunk's state at its first block (header offset, packed-word offset, exception
// cursors), filled by the first pass and reused by the second.
struct FpfSkip {
    int32_t done = -1;  // page start (values) the state belongs to; -1: none
    int32_t cur0, pk;
    int xc;  // lane k: values of dataTobePacked[k] consumed before the chunk's first block
    // the page holding the chunk's first value: its start (values, -1: none) and word, and its parsed
    // directory (so the second pass neither re-walks earlier pages' directories nor this one's)
    int32_t pdone = -1, p_page, bytesize, ie_end;
    int xs, xz;
};
template <int OP>
__device__ __forceinline__ void run_fastpfor(Ctx& c, int32_t v0 = 0, int32_t v1 = INT32_MAX, Carry cr0 = Carry{0, 0},
                             bool sum_only = false, Carry* sums = nullptr, FpfSkip* skip = nullptr,
                             Carry* fin = nullptr) {
    WaveSmem& sm = *c.sm;
    const int l = lane_id();
    const Words W{c.sb, c.byte_length / 4};
    const int64_t nw = W.nw;
    const uint32_t sbmis = (uint32_t)((uintptr_t)c.sb & 15);  // stream base misalignment (uniform)
    const uint32_t bsel = be_sel(sbmis & 3u);  // a stream word from the 4-byte grid: one v_perm_b32
    Carry cr = cr0;
    uint32_t ax = 0, ay = 0;                  // sum_only: per-lane sums
    const bool has_end = v1 >= c.n;           // this range holds the stream's last value
    int32_t decoded = 0;
    int32_t L = 0;
    int64_t p = 1;
    int xs_v = 0, xz_v = -1, xc_v = 0;  // lane k: dataTobePacked[k] start word, size, values consumed
    FpfPre pre;                          // the first block's prefetch (its packed words: at the page start)
    int64_t mw0 = 0;                     // stream word of cbuf[0] (the meta window)
    bool xin = false;                    // the page's metadata fits the meta window
    if (c.byte_length > c.avail) { c.err = COVT_ERR_TRUNCATED; }
    if (!c.err && nw > 0) {
        // W[0] (L) and W[1] (the first page's whereMeta) share one scalar-cache line: one round trip
        const uint32_t head0 = W.uniform(0), head1 = W.uniform(1);  // (the input is padded past every stream)
        L = (int32_t)head0;
        if (L < 0) c.err = COVT_ERR_BAD_HEADER;
        L -= L % kFpfBlock;
        if (!c.err && L > c.n) c.err = COVT_ERR_COUNT_MISMATCH;
        int32_t done = 0;
        // 1 KiB of stream words from word w on the 16-byte grid, byte-swapped into dst[]:
        // dst[m] = W(base + m) for m < 255, base = w - (0..3) returned; words at or past the stream's end
        // (nw) read as 0, as JavaFastPFOR's reads past its int[] do.  One 16-byte load per lane, by the
        // lanes whose 16 bytes start before the stream's last word ends (like win_load: a short stream's
        // window would otherwise fetch up to 1 KiB past it).  Issued and finished separately, so other
        // loads can be in flight between.
        const uintptr_t s_end = (uintptr_t)(c.sb + 4 * nw);
        struct WordsRaw {
            uint4 r;
            int64_t base;
            uint32_t sh;
        };
        auto words_issue = [&](int64_t w) -> WordsRaw {
            const uintptr_t addr = (uintptr_t)(c.sb + 4 * w);
            const uintptr_t a16 = addr & ~(uintptr_t)15;
            const uint32_t o = (uint32_t)(addr & 15u);
            // lanes past the stream repeat the last granule (their words are zeroed by words_store): an
            // unmasked load, so the compiler's vmcnt waits stay partial (a masked one drains every load)
            const uint32_t lmax = s_end > a16 ? (uint32_t)((s_end - 1 - a16) >> 4) : 0u;
            WordsRaw q;
            q.r = ld128_off((const g_u8*)a16, 16u * min((uint32_t)l, lmax));
            q.base = uni64(w - (int64_t)(o >> 2));
            q.sh = o & 3u;
            return q;
        };
        auto words_store = [&](uint32_t* dst, const WordsRaw& q) -> int64_t {
            const uint32_t nx = lane_next(q.r.x);
            const uint32_t sel = be_sel(q.sh);
            const int64_t wl = q.base + 4 * l;  // stream word of dst[4 l]
            uint4 wv;
            wv.x = wl < nw ? be_word(q.r.y, q.r.x, sel) : 0u;
            wv.y = wl + 1 < nw ? be_word(q.r.z, q.r.y, sel) : 0u;
            wv.z = wl + 2 < nw ? be_word(q.r.w, q.r.z, sel) : 0u;
            wv.w = wl + 3 < nw ? be_word(nx, q.r.w, sel) : 0u;
            wave_sync();
            ((uint4*)dst)[l] = wv;
            wave_sync();
            return q.base;
        };
        auto load_words = [&](uint32_t* dst, int64_t w) -> int64_t { return words_store(dst, words_issue(w)); };
        while (!c.err && done < L) {
            done = uni(done);
            const bool cached = skip && skip->pdone >= 0;
            if (cached && done < skip->pdone) {  // second pass: pages before the chunk's, skipped outright
                done = skip->pdone;
                p = skip->p_page;
                continue;
            }
            const int32_t thissize = uni((L - done) < kFpfPage ? (L - done) : kFpfPage);
            const int64_t p0 = uni64(p);
            if (p0 >= nw) { c.err = COVT_ERR_TRUNCATED; break; }
            int64_t ie = p0 + (int32_t)(p0 == 1 ? head1 : W.uniform(p0));  // the page's bytesize word
            if (ie < 0 || ie >= nw) { c.err = COVT_ERR_TRUNCATED; break; }
            // One round trip for the page's metadata and its first block: the 1 KiB meta window from the
            // bytesize word (bytesize, the byte container, and for a small page the exception directory and
            // arrays too: 74 % of the bench batch's pages have <= 1 KiB of metadata) is staged in cbuf, and
            // a page decoded from its first block gets that block's packed words (word p0 + 1, bit width not
            // yet known: every lane up to the stream's end) in flight beside it.
            // (issued for every page, also one decoded from a later block (a split chunk's first page, which
            // requests its first block again): a load under a branch makes the compiler drain every load)
            const WordsRaw mq = words_issue(ie);
            const bool spec = v0 <= done && v1 > done;  // the range starts at this page's first block
            {
                const uintptr_t a16 = ((uintptr_t)c.sb + 4u * (uint32_t)(p0 + 1)) & ~(uintptr_t)15;
                const uint32_t lmax = s_end > a16 ? (uint32_t)((s_end - 1 - a16) >> 4) : 0u;
                pre.raw = ld128_off((const g_u8*)a16, 16u * min((uint32_t)l, lmax));
            }
            mw0 = words_store(sm.u.f.cbuf, mq);
            auto mword = [&](int64_t w) -> uint32_t { return uniu(sm.u.f.cbuf[w - mw0]); };
            const int32_t bytesize = (int32_t)mword(ie++);  // (ie - mw0 <= 3)
            if (bytesize < 0 || bytesize > kFpfBcCap) { c.err = COVT_ERR_BAD_HEADER; break; }
            xc_v = 0;
            const int64_t bcw = (bytesize + 3) / 4;
            const int64_t bc = ie;
            if (bc + bcw >= nw) { c.err = COVT_ERR_TRUNCATED; break; }
            ie += bcw;
            if (cached && done == skip->pdone) {
                ie = skip->ie_end;
                xs_v = skip->xs;
                xz_v = skip->xz;
            } else {
                // exception-array directory (bitmap, then size + packed words per set bit): from the meta
                // window, or -- past it -- from 1 KiB LDS windows of words in stage; the arrays'
                // start/size/cursor live in lanes 2..32 of VGPRs
                int64_t dbase = INT64_MIN / 2;
                auto dword = [&](int64_t w) -> uint32_t {
                    if (w >= mw0 && w < mw0 + 255) return mword(w);
                    if (w < dbase || w >= dbase + 255) dbase = load_words(sm.u.f.stage, w);
                    return uniu(sm.u.f.stage[w - dbase]);
                };
                uint32_t bm = dword(ie++) & ~1u;  // bit k-1 set: dataTobePacked[k] present (k >= 2)
                xs_v = 0;
                xz_v = -1;
                while (bm) {
                    const int32_t k = __builtin_ctz(bm) + 1;
                    bm &= bm - 1;
                    if (ie >= nw) { c.err = COVT_ERR_TRUNCATED; break; }
                    const int32_t size = (int32_t)dword(ie++);
                    if (size < 0) { c.err = COVT_ERR_BAD_HEADER; break; }
                    const int64_t groups = ((int64_t)size + 31) / 32;
                    xs_v = l == k ? (int)(uint32_t)ie : xs_v;
                    xz_v = l == k ? size : xz_v;
                    ie += groups * k;
                    ie -= ((groups * 32 - size) * k) / 32;
                }
                if (c.err) break;
                if (skip && v0 >= done && v0 < done + thissize) {  // the chunk's first page: kept for pass two
                    skip->pdone = done;
                    skip->p_page = (int32_t)p0;
                    skip->bytesize = bytesize;
                    skip->ie_end = (int32_t)ie;
                    skip->xs = xs_v;
                    skip->xz = xz_v;
                }
            }
            // the whole metadata section (container, directory, exception arrays) inside the meta window:
            // the container walk never reloads it and exception values are read from it (no global loads)
            xin = ie - mw0 <= 255;
            // lane 0 stands for "no exception array" in the header walk: an unbounded size (its cursor counts
            // the other blocks' exceptions, never read as one)
            xz_v = l == 0 ? INT32_MAX : xz_v;
            COVT_PHASE(c, 0);
            const int32_t nblocks_page = uni(thissize / kFpfBlock);
            // blocks of this page holding values of [v0, v1)
            const int32_t jb0 = v0 > done ? min((v0 - done) / kFpfBlock, nblocks_page) : 0;
            const int32_t nblocks = v1 <= done ? 0 : uni(min(nblocks_page, (int32_t)(((int64_t)v1 - done + kFpfBlock - 1) / kFpfBlock)));
            const int32_t nw32 = (int32_t)nw;
            const int32_t bclen = uni((int32_t)(bcw * 4));
            const uint8_t* cb8 = (const uint8_t*)sm.u.f.cbuf;
            int32_t cbase = (int32_t)(4 * (mw0 - bc));  // (the meta window holds the container's start)
            auto chunk_load = [&](int32_t at) {  // container bytes [cbase, cbase + 1020), cbase in (at - 16, at]
                cbase = (int32_t)(4 * (load_words(sm.u.f.cbuf, bc + (at >> 2)) - bc));
            };
            // One block header (FastPFOR.decodePage loop body): all checks merged into one uniform test.
            // The chunk is (re)loaded so that the header and up to 255 exception positions are inside.
            auto walk = [&](int32_t cur, FpfHdr& h) -> int32_t {
                cur = uni(cur);
                cbase = uni(cbase);
                if (!xin && (uint32_t)(cur - cbase) > (uint32_t)(1020 - 260)) chunk_load(cur);
                const int32_t j = cur - cbase;
                const uint32_t hw =
                    uniu(__builtin_amdgcn_alignbyte(sm.u.f.cbuf[(j >> 2) + 1], sm.u.f.cbuf[j >> 2], (uint32_t)j & 3u));
                const int32_t b = (int32_t)(int8_t)(hw & 0xffu);
                const int32_t ce = (int32_t)((hw >> 8) & 0xffu);
                const int32_t hasx = ce > 0 ? 1 : 0;
                // exceptions: index maxbits - b; 1 = the implicit 1 << b, 2..32 = dataTobePacked[idx] (a block
                // without exceptions gets 1, a valid index its exception code never reads)
                const int32_t idx = hasx ? (int32_t)(int8_t)((hw >> 16) & 0xffu) - b : 1;
                const int32_t k = (uint32_t)(idx - 2) <= 30u ? idx : 0;  // lane 0: no array
                const int32_t xsz = __builtin_amdgcn_readlane(xz_v, k);
                const int32_t xc = __builtin_amdgcn_readlane(xc_v, k);
                h.b = b;
                h.ce = ce;
                h.idx = idx;
                h.xcur = (uint32_t)xc;  // (read only for idx >= 2)
                h.bcoff = cur + 2 + hasx;
                h.next = h.bcoff + ce;
                xc_v += l == k ? ce : 0;
                // every check at once as the largest of differences that must not be positive (all operands
                // far below 2^30): the bit width in [0, 32], the header and its exception positions inside
                // the container, the index in [1, 32], the array holding ce more values
                const int32_t worst = max(max(max(b - 32, -b), h.next - bclen), max(max(idx - 32, 1 - idx), xc + ce - xsz));
                return worst > 0 ? COVT_ERR_BAD_HEADER : COVT_OK;
            };
            // (32-bit: a stream holds < 2^29 words)
            auto xword = [&](int32_t k, uint32_t xs, uint32_t i, uint32_t& xbit) -> int32_t {
                // 24-bit multiplies (full rate; v_mul_lo_u32 is quarter rate): k <= 32, i < 2^16
                const uint32_t bit = __umul24(i & 31u, (uint32_t)k);
                xbit = bit & 31u;
                return (int32_t)(xs + __umul24(i >> 5, (uint32_t)k) + (bit >> 5));
            };
            auto prefetch = [&](const FpfHdr& hv, int32_t pkv, FpfPre& pr, int slot, bool raw = true) {
                FpfHdr h;
                h.idx = uni(hv.idx);
                h.ce = uni(hv.ce);
                h.xcur = uniu(hv.xcur);
                h.bcoff = uni(hv.bcoff);
                const int32_t pk = uni(pkv);
                // loads consumed only in the next iteration (the vmcnt wait lands there).  The packed
                // words are requested only by the lanes whose 16 bytes the unpack reads (8b words from
                // word qoff <= 3, plus the next lane's first word): 2b + 2 lanes, not all 64.
                // Both loads are issued by every lane with no exec mask and from a uniform base plus a
                // 32-bit lane offset (the `saddr` form, no 64-bit address math per lane): lanes past the
                // 2b + 2 whose 16 bytes the unpack reads repeat the last one's address, lanes without an
                // exception read word 0.  A masked load or a select of its address under a branch made
                // the compiler drain every outstanding load (vmcnt(0)) right after issuing the prefetch.
                if (raw) {  // (a page's first block: its words were requested with the meta window)
                    const uintptr_t a16 = ((uintptr_t)c.sb + 4u * (uint32_t)pk) & ~(uintptr_t)15;
                    const uint32_t lraw = min((uint32_t)l, 2u * (uint32_t)uni(hv.b) + 1u);
                    pr.raw = ld128_off((const g_u8*)a16, 16u * lraw);
                }
                const int32_t k = h.idx;
                const uint32_t xs = k >= 2 ? (uint32_t)__builtin_amdgcn_readlane(xs_v, k) : 0u;
                uint32_t xb;
                const int32_t wx = xword(k >= 2 ? k : 2, xs, h.xcur + (uint32_t)l, xb);
                const uint32_t xon = (uint32_t)(k >= 2) & (uint32_t)(l < h.ce) & (uint32_t)(wx < nw32);
                // (a page whose metadata fits the meta window reads its exception words from LDS when the
                // block is patched: no load here.  Reading them here into pr.x* would make the compiler drain
                // every outstanding load first -- those registers are a global load's destination on the
                // other path)
                if (!xin) {
                    const uint32_t wi = (uint32_t)wx & (0u - xon);
                    const u32x3 xv = *(const g_v3*)((const g_u8*)(((uintptr_t)c.sb) & ~(uintptr_t)3) + 4u * wi);
                    pr.x0 = xv.x;
                    pr.x1 = xv.y;
                    pr.x2 = xv.z;
                }
                const int32_t pb = h.bcoff - cbase;  // positions of exception e at cbuf byte pb + e
                pr.pos = cb8[min(pb + l, 4 * 260 - 1)];
                if (h.ce > 64) {  // rare: keep positions 64.. in LDS (the chunk may move on)
#pragma unroll
                    for (int q = 1; q < 4; ++q)
                        sm.u.f.posx[slot][64 * (q - 1) + l] = cb8[min(pb + l + 64 * q, 4 * 260 - 1)];
                }
            };
            FpfHdr h;
            int32_t pk = (int32_t)p0 + 1;
            int32_t cur0 = 0;
            // headers of the page's blocks before the range: only their offsets, packed words and exception
            // cursors, one LDS read per header (each block is checked by the chunk that decodes it; the
            // container bound keeps this walk's reads in place), once per chunk
            if (jb0 > 0 && jb0 < nblocks && !c.err) {
                if (skip && skip->done == done) {  // (FpfSkip::done: set by the pre-walk below)
                    cur0 = skip->cur0;
                    pk = skip->pk;
                    xc_v = skip->xc;
                } else {
                    int32_t cur = 0, pkk = pk;
                    for (int32_t j = 0; j < jb0; ++j) {
                        if (!xin && (uint32_t)(cur - cbase) > (uint32_t)(1020 - 8)) chunk_load(cur);
                        const int32_t jj = cur - cbase;
                        const uint32_t hw = uniu(__builtin_amdgcn_alignbyte(sm.u.f.cbuf[(jj >> 2) + 1],
                                                                            sm.u.f.cbuf[jj >> 2], (uint32_t)jj & 3u));
                        const int32_t b = (int32_t)(int8_t)(hw & 0xffu);
                        const int32_t ce = (int32_t)((hw >> 8) & 0xffu);
                        const int32_t idx = (int32_t)(int8_t)((hw >> 16) & 0xffu) - b;
                        pkk += 8 * b;
                        xc_v += (ce > 0 && idx >= 2 && idx <= 32 && l == idx) ? ce : 0;
                        cur += ce > 0 ? 3 + ce : 2;
                        if (cur > bclen) { c.err = COVT_ERR_BAD_HEADER; break; }
                    }
                    cur0 = uni(cur);
                    pk = uni(pkk);
                    if (skip) {
                        skip->done = done;
                        skip->cur0 = cur0;
                        skip->pk = pk;
                        skip->xc = xc_v;
                    }
                }
                COVT_PHASE(c, 0);  // (the pre-walk counts with the directory)
            }
            // one block; the loop below alternates two register sets so that no in-flight prefetch
            // register is ever copied (a copy would force the vmcnt wait at the end of the iteration)
            auto block = [&](int32_t j, const FpfPre& pc, FpfPre& pn, int slot) {
                FpfHdr hc;
                hc.b = uni(h.b);
                hc.ce = uni(h.ce);
                hc.idx = uni(h.idx);
                hc.xcur = uniu(h.xcur);
                hc.bcoff = uni(h.bcoff);
                hc.next = uni(h.next);
                const int32_t pkc = uni(pk);
                const int32_t b = hc.b;
                // stage block j: LDS dword qoff + i = packed word i (aligned, byte-swapped)
                const uint32_t o = (sbmis + 4u * (uint32_t)pkc) & 15u;
                const int32_t qoff = (int32_t)(o >> 2);
                {
                    uint4 raw2 = make_uint4(0, 0, 0, 0);
                    if (b == 32) {  // rare: the 16 bytes past the first KiB (same for every lane; scalar load)
                        const uintptr_t a16 = ((uintptr_t)c.sb + 4u * (uint32_t)pkc) & ~(uintptr_t)15;
                        raw2 = sld128(a16 + 1024);
                    }
                    const uint32_t nxt = lane_next(pc.raw.x, raw2.x);
                    uint4 wv;
                    wv.x = be_word(pc.raw.y, pc.raw.x, bsel);
                    wv.y = be_word(pc.raw.z, pc.raw.y, bsel);
                    wv.z = be_word(pc.raw.w, pc.raw.z, bsel);
                    wv.w = be_word(nxt, pc.raw.w, bsel);
                    ((uint4*)sm.u.f.stage)[l] = wv;
                    if (b == 32 && l == 0) {
                        uint4 w2;
                        w2.x = be_word(raw2.y, raw2.x, bsel);
                        w2.y = be_word(raw2.z, raw2.y, bsel);
                        w2.z = be_word(raw2.w, raw2.z, bsel);
                        w2.w = be_word(0u, raw2.w, bsel);
                        ((uint4*)sm.u.f.stage)[64] = w2;
                    }
                }
                if (hc.ce > 0) ((uint4*)sm.u.f.patch)[l] = make_uint4(0, 0, 0, 0);
                wave_sync();
                COVT_PHASE(c, 1);
                // walk block j+1 and put its loads in flight.  The loads are issued unconditionally (the
                // last block re-reads its own words) so that every path has the same number of memory
                // ops in flight and the waits for this block's exception words stay partial.
                if (j + 1 < nblocks) {
                    c.err = walk(hc.next, h);
                    pk = pkc + 8 * b;
                    if (!c.err && pk + 8 * h.b > nw32) c.err = COVT_ERR_TRUNCATED;
                    if (c.err) return;
                }
                prefetch(h, pk, pn, slot ^ 1);
                COVT_PHASE(c, 2);
                // unpack: lane l -> values 4l..4l+3 of miniblock l/8
                uint32_t v[4];
                {
                    const uint32_t mask = b == 32 ? 0xffffffffu : ((1u << b) - 1u);
                    uint32_t bit = __umul24((uint32_t)(l & 7) * 4u, (uint32_t)b);
                    const int32_t wb = (int32_t)__umul24((uint32_t)(l >> 3), (uint32_t)b) + qoff;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int32_t wi = wb + (int32_t)(bit >> 5);
                        const uint32_t lo = sm.u.f.stage[wi], hi = sm.u.f.stage[wi + 1];
                        v[k] = __builtin_amdgcn_alignbit(hi, lo, bit & 31u) & mask;
                        bit += (uint32_t)b;
                    }
                }
                COVT_PHASE(c, 3);
#if defined(COVT_ABL_NOEXC)  // ablation build: exceptions not applied
                if (false) {
#else
                if (hc.ce > 0) {  // out[pos] |= (index == 1 ? 1 : exceptvalue) << b
#endif
                    const int32_t k = hc.idx;
                    const uint32_t xs = k >= 2 ? (uint32_t)__builtin_amdgcn_readlane(xs_v, k) : 0u;
                    const bool el = l < hc.ce;
                    uint32_t ex = 1u;
                    if (k != 1) {  // uniform
                        uint32_t xbit;
                        const int32_t wi = xword(k, xs, hc.xcur + (uint32_t)l, xbit);
                        uint32_t lo, hi;
                        if (xin) {  // meta window: words already swapped, 0 past the stream
                            const int32_t m = el ? wi - (int32_t)mw0 : 0;
                            lo = sm.u.f.cbuf[m];
                            hi = sm.u.f.cbuf[m + 1];
                        } else {
                            lo = wi < nw32 ? be_word(pc.x1, pc.x0, bsel) : 0u;  // words past the stream read as 0
                            hi = wi + 1 < nw32 ? be_word(pc.x2, pc.x1, bsel) : 0u;
                        }
                        // bits [xbit, xbit + k) of hi:lo (xbit < 32, k <= 32)
                        const uint32_t m = k == 32 ? 0xffffffffu : ((1u << k) - 1u);
                        ex = __builtin_amdgcn_alignbit(hi, lo, xbit) & m;
                    }
                    // lanes without an exception OR 0 into their own slot: no branch, no conflict
                    atomicOr(&sm.u.f.patch[el ? pc.pos : (uint32_t)(4 * l)], el ? ex << (b & 31) : 0u);
                    if (hc.ce > 64) {  // rare: more than 64 exceptions in the block
                        for (int q = 1; q < 4; ++q) {
                            const int32_t e = l + 64 * q;
                            if (e < hc.ce) {
                                const uint32_t ex = k == 1 ? 1u : xget(W, xs, k, hc.xcur + (uint32_t)e);
                                atomicOr(&sm.u.f.patch[sm.u.f.posx[slot][64 * (q - 1) + l]], ex << (b & 31));
                            }
                        }
                    }
                    wave_sync();
                    const uint4 pt = ((const uint4*)sm.u.f.patch)[l];
                    v[0] |= pt.x;
                    v[1] |= pt.y;
                    v[2] |= pt.z;
                    v[3] |= pt.w;
                }
                COVT_PHASE(c, 4);
#if defined(COVT_ABL_NOSTORE)  // ablation build: every block's output to the same 1 KiB (L2-resident)
                sink_values<OP, 4>(v, 0, 0, kFpfBlock, c.nb, c.out, cr);
#else
                if (sum_only)
                    sum_values<OP, 4>(v, (int64_t)done + (int64_t)j * kFpfBlock, kFpfBlock, ax, ay);
                else
                    sink_values<OP, 4>(v, (int64_t)done + (int64_t)j * kFpfBlock, 0, kFpfBlock, c.nb, c.out, cr);
#endif
                wave_sync();
                COVT_PHASE(c, 5);
            };
            FpfPre preB;
            if (jb0 < nblocks && !c.err) {
                c.err = walk(cur0, h);
                if (!c.err && pk + 8 * h.b > nw32) c.err = COVT_ERR_TRUNCATED;
                if (!c.err) {
                    prefetch(h, pk, pre, 0, !spec);
                    // (the loop is entered only from here, so its header sees these stores on every path)
                    if (!sum_only) fpf_prime_stores<OP>(c.out, (int64_t)done + (int64_t)jb0 * kFpfBlock);
                    int32_t j = jb0;
                    do {
                        block(j, pre, preB, 0);
                        if (j + 1 < nblocks && !c.err) block(j + 1, preB, pre, 1);
                        j += 2;
                    } while (j < nblocks && !c.err);
                }
            }
            done += thissize;
            p = ie;
            if (done >= v1) break;  // the range ends in this page
        }
        decoded = L;
        // VariableByte tail over words [p, nw): from the last page's meta window when the window holds it
        // (words (4 vpos & ~15) / 4 .. nw - 1 staged in cbuf; cbuf lies past the varint window and most of
        // its terminator list, so the window's first load reads it before anything is overwritten)
        if (!c.err && has_end && p < nw) {
            int32_t vpos = (int32_t)(4 * p);
            const int32_t base = L;
            Win w;
            w.valid = false;
            const bool tail_in = L > 0 && ((int64_t)(vpos & ~15) >> 2) >= mw0 && nw - mw0 <= 255;
            const int32_t got = varint_take<MODE_WORDREV, VAL_VB>(
                sm, c.sb, w, vpos, (int32_t)(4 * nw), c.n - L, true, c.err,
                [&](const uint32_t (&lo)[1], const uint32_t (&hi)[1], int32_t vb, int32_t, int32_t count) {
                    if (sum_only) sum_values<OP, 1>(lo, (int64_t)base + vb, count, ax, ay);
                    else sink_values<OP, 1>(lo, (int64_t)base + vb, 0, count, c.nb, c.out, cr);
                },
                0, nullptr, 0, tail_in ? sm.u.f.cbuf : nullptr, (int32_t)mw0);
            decoded = L + got;
        }
    }
    // values the codec did not produce stay 0 in Java's decompressedValues[]: transform them too
    if (!c.err && has_end) {
        for (int32_t b = decoded; !sum_only && b < c.n; b += 64) {
            uint32_t vv[1] = {0};
            sink_values<OP, 1>(vv, b, 0, c.n - b < 64 ? c.n - b : 64, c.nb, c.out, cr);
        }
        if (OP == COVT_OP_FPF_ZZ_DELTA_XY && (c.n & 1)) c.err = COVT_ERR_COUNT_MISMATCH;
    }
    COVT_PHASE(c, 7);
    c.consumed = c.byte_length;
    if (sum_only) {
        sums->x = lane_bcast(incl_scan(ax), 63);
        sums->y = lane_bcast(incl_scan(ay), 63);
    }
    if (fin) *fin = cr;  // the running sums after the range (from cr0)
}

// FastPFOR + VariableByte over a whole stream (the family kernels' path; split chunks keep run_fastpfor
// above).  Same page framing, directory and checks as run_fastpfor; what differs is how the blocks get
// their words and headers:
//  * packed words stream through LDS: a page's packed words are one contiguous run of stream words from
//    p0 + 1 (block j's 8 b words follow block j - 1's), so they are read in 1 KiB windows from the 128-byte
//    line holding word p0 + 1 -- one 16-byte load per lane, each window requested as soon as the previous
//    one is staged -- and staged byte-swapped into a 512-word ring (two windows).  A block waits only when
//    its words pass the staged end, on a load issued a window (about five blocks) earlier; no load address
//    depends on a block header.  Lane 63's last word needs the next window's first bytes: it is written
//    when that window is staged (the staged end lags by one word).
//  * block headers in batches of up to 64 (one serial walk of the header chain, one LDS read per header,
//    then lane-parallel: packed-word offsets and exception cursors by prefix sums, every check at once by
//    ballot); each block reads its state from those lanes.
// Blocks before a failing one are decoded and stored; the failing block's status is the stream's.
template <int OP>
__device__ __forceinline__ void run_fastpfor_stream(Ctx& c) {
    WaveSmem& sm = *c.sm;
    const int l = lane_id();
    const Words W{c.sb, c.byte_length / 4};
    const int32_t nw32 = W.nw;  // (32-bit word indices: a stream holds < 2^29 words)
    const uint32_t bsel = be_sel((uint32_t)((uintptr_t)c.sb & 3u));  // a stream word from the 4-byte grid
    Carry cr{0u, 0u};
    int32_t decoded = 0;
    int32_t L = 0;
    int32_t p = 1;
    int xs_v = 0, xz_v = -1, xc_v = 0;  // lane k: dataTobePacked[k] start word, size, values consumed
    int32_t mw0 = 0;                     // stream word of cbuf[0] (the meta window)
    if (c.byte_length > c.avail) { c.err = COVT_ERR_TRUNCATED; }
    if (!c.err && nw32 > 0) {
        const uint32_t head0 = W.uniform(0), head1 = W.uniform(1);
        L = (int32_t)head0;
        if (L < 0) c.err = COVT_ERR_BAD_HEADER;
        L -= L % kFpfBlock;
        if (!c.err && L > c.n) c.err = COVT_ERR_COUNT_MISMATCH;
        int32_t done = 0;
        const uintptr_t s_end = (uintptr_t)c.sb + 4u * (uint32_t)nw32;
        struct WordsRaw {
            uint4 r;
            int32_t base;
            uint32_t sh;
        };
        auto words_issue = [&](int32_t w) -> WordsRaw {
            const uintptr_t addr = (uintptr_t)c.sb + 4u * (uint32_t)w;
            const uintptr_t a16 = addr & ~(uintptr_t)15;
            const uint32_t o = (uint32_t)(addr & 15u);
            const uint32_t lmax = s_end > a16 ? (uint32_t)((s_end - 1 - a16) >> 4) : 0u;
            WordsRaw q;
            q.r = ld128_off((const g_u8*)a16, 16u * min((uint32_t)l, lmax));
            q.base = uni(w - (int32_t)(o >> 2));
            q.sh = o & 3u;
            return q;
        };
        auto words_store = [&](uint32_t* dst, const WordsRaw& q) -> int32_t {
            const uint32_t nx = lane_next(q.r.x);
            const uint32_t sel = be_sel(q.sh);
            const int32_t wl = q.base + 4 * l;
            uint4 wv;
            wv.x = wl < nw32 ? be_word(q.r.y, q.r.x, sel) : 0u;
            wv.y = wl + 1 < nw32 ? be_word(q.r.z, q.r.y, sel) : 0u;
            wv.z = wl + 2 < nw32 ? be_word(q.r.w, q.r.z, sel) : 0u;
            wv.w = wl + 3 < nw32 ? be_word(nx, q.r.w, sel) : 0u;
            wave_sync();
            ((uint4*)dst)[l] = wv;
            wave_sync();
            return q.base;
        };
        auto load_words = [&](uint32_t* dst, int32_t w) -> int32_t { return words_store(dst, words_issue(w)); };
        while (!c.err && done < L) {
            done = uni(done);
            const int32_t thissize = uni((L - done) < kFpfPage ? (L - done) : kFpfPage);
            const int32_t p0 = uni(p);
            if (p0 >= nw32) { c.err = COVT_ERR_TRUNCATED; break; }
            const int64_t ie0 = (int64_t)p0 + (int32_t)(p0 == 1 ? head1 : W.uniform(p0));  // the page's bytesize word
            if (ie0 < 0 || ie0 >= nw32) { c.err = COVT_ERR_TRUNCATED; break; }
            int32_t ie = (int32_t)ie0;
            // one round trip: the meta window (bytesize, byte container, small pages' directory and exception
            // arrays) and the first window of packed words, requested together (meta first: its wait does not
            // wait for the packed words)
            const WordsRaw mq = words_issue(ie);
            const uintptr_t pa = (uintptr_t)c.sb + 4u * (uint32_t)(p0 + 1);
            const uintptr_t A0 = pa & ~(uintptr_t)127;
            // last 16-byte granule of the stream relative to A0: lanes past it repeat it (unmasked loads)
            const uint32_t glast = s_end > A0 ? (uint32_t)((s_end - 1 - A0) & ~(uintptr_t)15) : 0u;
            // ring word m (window k, lane l, word i: m = 256 k + 4 l + i) holds stream word wbase + m
            const int32_t wbase = uni((int32_t)(p0 + 1) - (int32_t)((pa - A0) >> 2));
            uint4 R = ld128_off((const g_u8*)A0, min(16u * (uint32_t)l, glast));
            int32_t kst = 0;       // windows staged
            int32_t vend = wbase;  // stream words below vend are staged
            uint32_t prev63 = 0u;  // lane 63's last raw dword of the last staged window
            mw0 = words_store(sm.u.f.cbuf, mq);
            auto mword = [&](int32_t w) -> uint32_t { return uniu(sm.u.f.cbuf[w - mw0]); };
            const int32_t bytesize = (int32_t)mword(ie++);
            if (bytesize < 0 || bytesize > kFpfBcCap) { c.err = COVT_ERR_BAD_HEADER; break; }
            xc_v = 0;
            const int32_t bcw = (bytesize + 3) / 4;
            const int32_t bc = ie;
            if (bc + bcw >= nw32) { c.err = COVT_ERR_TRUNCATED; break; }
            ie += bcw;
            // the directory in 64-bit arithmetic (array sizes up to 2^31 - 1 move the cursor far past the
            // stream: caught by the next read's bound, or by the next page's), its end clamped to nw after
            int64_t ie64 = ie;
            {
                int32_t dbase = INT32_MIN / 2;
                auto dword = [&](int32_t w) -> uint32_t {
                    if (w >= mw0 && w < mw0 + 255) return mword(w);
                    // (the ring is free until the first window is staged)
                    if (w < dbase || w >= dbase + 255) dbase = load_words(sm.u.f.ring, w);
                    return uniu(sm.u.f.ring[w - dbase]);
                };
                uint32_t bm = dword((int32_t)ie64++) & ~1u;
                xs_v = 0;
                xz_v = -1;
                while (bm) {
                    const int32_t k = __builtin_ctz(bm) + 1;
                    bm &= bm - 1;
                    if (ie64 >= nw32) { c.err = COVT_ERR_TRUNCATED; break; }
                    const int32_t size = (int32_t)dword((int32_t)ie64++);
                    if (size < 0) { c.err = COVT_ERR_BAD_HEADER; break; }
                    const int64_t groups = ((int64_t)size + 31) / 32;
                    xs_v = l == k ? (int)(uint32_t)ie64 : xs_v;
                    xz_v = l == k ? size : xz_v;
                    ie64 += groups * k;
                    ie64 -= ((groups * 32 - size) * k) / 32;
                }
                if (c.err) break;
            }
            const bool xin = ie64 - mw0 <= 255;  // the page's whole metadata sits in the meta window
            ie = (int32_t)(ie64 < nw32 ? ie64 : (int64_t)nw32);  // (>= nw: the next page, or the tail, stops)
            COVT_PHASE(c, 0);
            const int32_t nblocks = uni(thissize / kFpfBlock);
            const int32_t bclen = uni((int32_t)(bcw * 4));
            const uint8_t* cb8 = (const uint8_t*)sm.u.f.cbuf;
            const g_u8* cbyte = (const g_u8*)(c.sb + 4u * (uint32_t)bc);  // container byte q: cbyte[q ^ 3]
            int32_t cbase = (int32_t)(4 * (mw0 - bc));
            auto chunk_load = [&](int32_t at) {  // container bytes [cbase, cbase + 1020), cbase in (at - 16, at]
                cbase = (int32_t)(4 * (load_words(sm.u.f.cbuf, bc + (at >> 2)) - bc));
            };
            // the next window of packed words: staged into the ring, the one after it requested
            bool fin = false;           // the current batch is the page's last (or fails)
            int32_t bneed = INT32_MAX;  // ... and its blocks need the words below this
            auto stage = [&]() {
                const int32_t k = uni(kst);
                const uint32_t nx = lane_next(R.x, 0u);
                const int32_t w0 = wbase + 256 * k + 4 * l;
                uint4 wv;
                wv.x = w0 < nw32 ? be_word(R.y, R.x, bsel) : 0u;
                wv.y = w0 + 1 < nw32 ? be_word(R.z, R.y, bsel) : 0u;
                wv.z = w0 + 2 < nw32 ? be_word(R.w, R.z, bsel) : 0u;
                wv.w = w0 + 3 < nw32 ? be_word(nx, R.w, bsel) : 0u;  // (lane 63: incomplete, not stored)
                const int32_t fw = wbase + 256 * k - 1;  // the previous window's last word
                const uint32_t fix = fw < nw32 ? be_word(lane_bcast(R.x, 0), prev63, bsel) : 0u;
                prev63 = lane_bcast(R.w, 63);
                const uint32_t ri = (uint32_t)(256 * k + 4 * l) & 511u;
                wave_sync();
                if (l < 63) {
                    *(uint4*)&sm.u.f.ring[ri] = wv;
                } else {
                    sm.u.f.ring[ri] = wv.x;
                    sm.u.f.ring[ri + 1] = wv.y;
                    sm.u.f.ring[ri + 2] = wv.z;
                }
                if (l == 0 && k > 0) sm.u.f.ring[(uint32_t)(256 * k - 1) & 511u] = fix;
                wave_sync();
                kst = k + 1;
                vend = wbase + 256 * (k + 1) - 1;
                // the next window, unless the page's last batch is staged far enough (a window requested past
                // a page's last needed word was up to 1 KiB of extra reads per page)
                if (!fin || vend < bneed)
                    R = ld128_off((const g_u8*)A0, min(1024u * (uint32_t)(k + 1) + 16u * (uint32_t)l, glast));
                wave_sync();  // (the request stays ahead of the stores that follow: see the block's wait)
            };
            int32_t cur = 0, pk = (int32_t)p0 + 1;
            for (int32_t jbat = 0, nbat = 0; jbat < nblocks && !c.err; jbat += nbat) {
                jbat = uni(jbat);
                nbat = uni(min(64, nblocks - jbat));
                // (1) the header chain: block jbat + g's header bytes and container offset to lane g.  A page
                // whose container is past the meta window reads it through 1 KiB chunks; a batch then holds
                // only blocks whose header and exception positions lie in the chunk loaded at its start, so the
                // chunk moves forward once per KiB of container and a block's positions never reload it (a
                // reload is a synchronous load: it waits for every request in flight)
                uint32_t hw_v = 0u;
                int32_t cur_v = bclen + 1;  // (past the container: no header)
                cur = uni(cur);
                cbase = uni(cbase);
                if (!xin && cur <= bclen && (uint32_t)(cur - cbase) > (uint32_t)(1020 - 258)) chunk_load(cur);
                for (int32_t g = 0; g < nbat; ++g) {
                    cur = uni(cur);
                    cbase = uni(cbase);
                    if (cur > bclen) break;  // the chain has left the container
                    if (!xin && cur - cbase > 1020 - 8) {  // the next header is past the chunk: a new batch
                        nbat = g;
                        break;
                    }
                    const int32_t q = cur - cbase;
                    const uint32_t hw =
                        uniu(__builtin_amdgcn_alignbyte(sm.u.f.cbuf[(q >> 2) + 1], sm.u.f.cbuf[q >> 2], (uint32_t)q & 3u));
                    const int32_t ce = (int32_t)((hw >> 8) & 0xffu);
                    const int32_t nx = cur + (ce > 0 ? 3 + ce : 2);
                    if (!xin && g > 0 && nx - cbase > 1020) {  // its positions are past the chunk: a new batch
                        nbat = g;
                        break;
                    }
                    hw_v = l == g ? hw : hw_v;
                    cur_v = l == g ? cur : cur_v;
                    cur = nx;
                }
                nbat = uni(nbat);
                if (nbat == 0) {  // (cannot happen: the chunk was loaded at the batch's first header)
                    c.err = COVT_ERR_BAD_HEADER;
                    break;
                }
                COVT_PHASE(c, 1);
                // (2) lane-parallel: fields, exception cursors (a prefix sum per exception width present),
                // packed-word offsets, checks
                const bool in = l < nbat;
                const int32_t b_v = (int32_t)(int8_t)(hw_v & 0xffu);
                const int32_t ce_v = (int32_t)((hw_v >> 8) & 0xffu);
                const bool hasx = ce_v > 0;
                const int32_t idx_v = hasx ? (int32_t)(int8_t)((hw_v >> 16) & 0xffu) - b_v : 1;
                const bool arr_k = hasx && idx_v >= 2 && idx_v <= 32;  // exceptions from dataTobePacked[idx]
                const bool arr = in && arr_k;
                int32_t xcur_v = 0;
                for (uint64_t todo = __ballot(arr); todo;) {
                    const int32_t kk = __builtin_amdgcn_readlane(idx_v, (int32_t)__builtin_ctzll(todo));
                    const bool mine = arr && idx_v == kk;
                    const uint32_t v = mine ? (uint32_t)ce_v : 0u;
                    const uint32_t s = incl_scan(v);
                    const int32_t base = __builtin_amdgcn_readlane(xc_v, kk);
                    xcur_v = mine ? base + (int32_t)(s - v) : xcur_v;
                    xc_v += l == kk ? (int32_t)lane_bcast(s, 63) : 0;
                    todo &= ~__ballot(mine);
                }
                const uint32_t w8 = in ? 8u * (uint32_t)(b_v & 63) : 0u;
                const uint32_t pinc = incl_scan(w8);
                const int32_t pk_v = pk + (int32_t)(pinc - w8);
                pk += (int32_t)lane_bcast(pinc, 63);
                int32_t nok = nbat;  // blocks of the batch before the first failing one
                int32_t ferr = 0;
                {
                    const int32_t xsz = lane_get(xz_v, arr_k ? idx_v : 0);
                    bool bad = (uint32_t)b_v > 32u || cur_v + 2 > bclen;
                    bad |= hasx && (cur_v + 3 + ce_v > bclen || (idx_v != 1 && !arr_k));
                    bad |= arr_k && (xsz < 0 || xcur_v + ce_v > xsz);
                    const bool trunc = pk_v + 8 * b_v > nw32;
                    const uint64_t fail = __ballot(in && (bad || trunc));
                    if (fail) {
                        nok = (int32_t)__builtin_ctzll(fail);
                        ferr = __builtin_amdgcn_readlane(bad ? COVT_ERR_BAD_HEADER : COVT_ERR_TRUNCATED, nok);
                    }
                }
                COVT_PHASE(c, 2);
                fin = jbat + nbat >= nblocks || ferr != 0;
                bneed = nok > 0 ? uni(__builtin_amdgcn_readlane(pk_v + 8 * b_v, nok - 1)) : 0;
                // the page's first window (requested with the meta window): vend >= p0 + 1 from here on.  (Before the
                // batch's first block on every path: the prime stores below then separate it from every wait.)
                if (jbat == 0) stage();
                // (3) the blocks.  Block g's fields, packed lane-side (b | ce << 8 | idx << 16 | xo << 24; the
                // positions' container offset), so that a block reads four lanes: xo = where its exception words sit
                // in xw (255: read from memory -- pages whose metadata the meta window holds read them from there)
                struct Hdr {
                    int32_t b, ce, idx, pk, bcoff, xo;
                    uint32_t xcur;
                };
                int32_t xo_v = 255;
                if (!xin) {
                    // The batch's exception words, gathered into xw by four requests at once: per block with an
                    // exception array, the words holding its values (one more for the straddling read).  One wait
                    // per batch instead of a dependent load per block: 97 % of the bench batch's blocks carry
                    // exceptions, and 79 % sit on pages whose metadata is past the meta window.  (Words past xw:
                    // those blocks read memory.)
                    const bool ab = arr && l < nok;
                    const int32_t k = ab ? idx_v : 2;
                    const uint32_t xs = (uint32_t)lane_get(xs_v, k);
                    const uint32_t b0 = __umul24((uint32_t)xcur_v, (uint32_t)k);
                    const uint32_t b1 = __umul24((uint32_t)(xcur_v + ce_v), (uint32_t)k);
                    const int32_t wlo = (int32_t)(xs + (b0 >> 5));
                    const int32_t wn = ab ? (int32_t)((b1 + 31u) >> 5) - (int32_t)(b0 >> 5) + 1 : 0;
                    const uint32_t winc = incl_scan((uint32_t)wn);
                    const int32_t wo = (int32_t)(winc - (uint32_t)wn);
                    const int32_t wend = (int32_t)winc;  // non-decreasing over the lanes
                    xo_v = ab && wend <= kFpfXw ? wo : 255;
                    const int32_t tot = uni(min((int32_t)lane_bcast(winc, 63), kFpfXw));
                    const g_u8* sb4 = (const g_u8*)(((uintptr_t)c.sb) & ~(uintptr_t)3);
                    u32x2 d[4];
                    bool okw[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {  // word t of xw: block g = the first whose words end past t
                        const int32_t t = 64 * r + l;
                        int32_t lo = 0, hi = 64;  // (65 outcomes: 7 halvings)
#pragma unroll
                        for (int s2 = 0; s2 < 7; ++s2) {
                            const int32_t mid = (lo + hi) >> 1;
                            const bool le = lane_get(wend, mid & 63) <= t;
                            const bool act = lo < hi;
                            lo = act && le ? mid + 1 : lo;
                            hi = act && !le ? mid : hi;
                        }
                        const int32_t g = min(lo, 63);
                        const int32_t w = lane_get(wlo, g) + (t - lane_get(wo, g));
                        okw[r] = t < tot && w < nw32;
                        d[r] = *(const g_v2*)(sb4 + 4u * (okw[r] ? (uint32_t)w : 0u));  // (unmasked: no drain)
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (64 * r + l < kFpfXw) sm.u.f.xw[64 * r + l] = okw[r] ? be_word(d[r].y, d[r].x, bsel) : 0u;
                    wave_sync();
                }
                const uint32_t f_v = (uint32_t)(b_v & 0xff) | ((uint32_t)ce_v << 8) | ((uint32_t)(idx_v & 0xff) << 16) |
                                     ((uint32_t)xo_v << 24);
                const int32_t bo_v = cur_v + (hasx ? 3 : 2);
                auto rec = [&](int32_t g, Hdr& h) {
                    const uint32_t f = uniu((uint32_t)__builtin_amdgcn_readlane((int32_t)f_v, g));
                    h.b = (int32_t)(f & 0xffu);
                    h.ce = (int32_t)((f >> 8) & 0xffu);
                    h.idx = (int32_t)(int8_t)((f >> 16) & 0xffu);
                    h.xo = (int32_t)(f >> 24);
                    h.xcur = uniu((uint32_t)__builtin_amdgcn_readlane(xcur_v, g));
                    h.bcoff = uni(__builtin_amdgcn_readlane(bo_v, g));
                    h.pk = uni(__builtin_amdgcn_readlane(pk_v, g));
                };
                // as many zero stores to the batch's first block as a block's sink issues (overwritten by its
                // values): every path from a window request to its wait then passes a store -- also when the
                // first block needs the next window at once -- so the compiler's vmcnt waits stay partial instead
                // of vmcnt(0) (which would also wait for the stores just issued)
                fpf_prime_stores<OP>(c.out, (int64_t)done + (int64_t)jbat * kFpfBlock);
                auto block = [&](int32_t g) {
                    Hdr hc;
                    rec(g, hc);
                    const int32_t b = hc.b;
                    // this block's words staged.  One window is always enough (vend >= pk: the previous block
                    // needed up to pk; a block needs <= 256 words), and never two stages back to back: every
                    // path from a window's request to its wait then passes a block's output stores, so the
                    // compiler's vmcnt wait there stays partial (a loop here, or a second stage, made it
                    // vmcnt(0) on every block: the stores just issued waited for too)
                    if (uni(vend) < hc.pk + 8 * b) stage();
                    if (hc.ce > 0) ((uint4*)sm.u.f.patch)[l] = make_uint4(0, 0, 0, 0);
                    COVT_PHASE(c, 3);
                    // unpack: lane l -> values 4l..4l+3 of miniblock l/8, words from the ring
                    uint32_t v[4];
                    {
                        const uint32_t mask = b == 32 ? 0xffffffffu : ((1u << b) - 1u);
                        uint32_t bit = __umul24((uint32_t)(l & 7) * 4u, (uint32_t)b);
                        const int32_t r0 = (hc.pk - wbase) & 511;
                        const int32_t wb = (int32_t)__umul24((uint32_t)(l >> 3), (uint32_t)b) + r0;
                        if (r0 + 8 * b <= 511) {
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                const int32_t wi = wb + (int32_t)(bit >> 5);
                                const uint32_t lo = sm.u.f.ring[wi], hi = sm.u.f.ring[wi + 1];
                                v[k] = __builtin_amdgcn_alignbit(hi, lo, bit & 31u) & mask;
                                bit += (uint32_t)b;
                            }
                        } else {  // the block wraps around the ring's end
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                const int32_t wi = wb + (int32_t)(bit >> 5);
                                const uint32_t lo = sm.u.f.ring[wi & 511], hi = sm.u.f.ring[(wi + 1) & 511];
                                v[k] = __builtin_amdgcn_alignbit(hi, lo, bit & 31u) & mask;
                                bit += (uint32_t)b;
                            }
                        }
                    }
                    COVT_PHASE(c, 4);
                    if (hc.ce > 0) {  // out[pos] |= (index == 1 ? 1 : exceptvalue) << b
                        const int32_t k = hc.idx;
                        const bool el = l < hc.ce;
                        // exception e = lane: its position (container byte bcoff + e, inside the chunk: batch rule)
                        const uint32_t pos = cb8[min(max(hc.bcoff - cbase + l, 0), 4 * 260 - 1)];
                        uint32_t ex = 1u;
                        if (k != 1) {  // uniform; k in [2, 32] (checked)
                            const uint32_t xs = (uint32_t)__builtin_amdgcn_readlane(xs_v, k);
                            // value i = xcur + e of dataTobePacked[k]: bits [i k, i k + k) of its words
                            const uint32_t bb = __umul24(hc.xcur + (uint32_t)l, (uint32_t)k);
                            const uint32_t xbit = bb & 31u;
                            uint32_t lo, hi;
                            if (xin) {  // meta window: words already swapped, 0 past the stream
                                const int32_t m = el ? (int32_t)(xs + (bb >> 5)) - mw0 : 0;
                                lo = sm.u.f.cbuf[m];
                                hi = sm.u.f.cbuf[m + 1];
                            } else if (hc.xo != 255) {  // the batch's gathered words
                                const int32_t m = el ? hc.xo + (int32_t)(bb >> 5) - (int32_t)(__umul24(hc.xcur, (uint32_t)k) >> 5) : 0;
                                lo = sm.u.f.xw[m];
                                hi = sm.u.f.xw[m + 1];
                            } else {  // (past xw: from memory)
                                const int32_t wi = (int32_t)(xs + (bb >> 5));
                                lo = el && wi < nw32 ? W(wi) : 0u;
                                hi = el && wi + 1 < nw32 ? W(wi + 1) : 0u;
                            }
                            const uint32_t m = k == 32 ? 0xffffffffu : ((1u << k) - 1u);
                            ex = __builtin_amdgcn_alignbit(hi, lo, xbit) & m;
                        }
                        atomicOr(&sm.u.f.patch[el ? pos : (uint32_t)(4 * l)], el ? ex << (b & 31) : 0u);
                        if (hc.ce > 64) {  // rare: more than 64 exceptions in the block (positions from memory)
                            const uint32_t xs = k >= 2 ? (uint32_t)__builtin_amdgcn_readlane(xs_v, k) : 0u;
                            for (int q = 1; q < 4; ++q) {
                                const int32_t e = l + 64 * q;
                                if (e < hc.ce) {
                                    const uint32_t ex2 = k == 1 ? 1u : xget(W, xs, k, hc.xcur + (uint32_t)e);
                                    const uint32_t ps = cbyte[(hc.bcoff + e) ^ 3];
                                    atomicOr(&sm.u.f.patch[ps], ex2 << (b & 31));
                                }
                            }
                        }
                        wave_sync();
                        const uint4 pt = ((const uint4*)sm.u.f.patch)[l];
                        v[0] |= pt.x;
                        v[1] |= pt.y;
                        v[2] |= pt.z;
                        v[3] |= pt.w;
                    }
                    COVT_PHASE(c, 5);
                    sink_values<OP, 4>(v, (int64_t)done + (int64_t)(jbat + g) * kFpfBlock, 0, kFpfBlock, c.nb, c.out, cr);
                    wave_sync();
                    COVT_PHASE(c, 6);
                };
                for (int32_t g = 0; g < nok; ++g) {
                    g = uni(g);
                    block(g);
                }
                if (ferr) c.err = ferr;
            }
            done += thissize;
            p = ie;
        }
        decoded = L;
        // VariableByte tail over words [p, nw): from the last page's meta window when it holds them
        if (!c.err && p < nw32) {
            int32_t vpos = (int32_t)(4 * p);
            const int32_t base = L;
            Win w;
            w.valid = false;
            const bool tail_in = L > 0 && ((vpos & ~15) >> 2) >= mw0 && nw32 - mw0 <= 255;
            const int32_t got = varint_take<MODE_WORDREV, VAL_VB>(
                sm, c.sb, w, vpos, 4 * nw32, c.n - L, true, c.err,
                [&](const uint32_t (&lo)[1], const uint32_t (&hi)[1], int32_t vb, int32_t, int32_t count) {
                    sink_values<OP, 1>(lo, (int64_t)base + vb, 0, count, c.nb, c.out, cr);
                },
                0, nullptr, 0, tail_in ? sm.u.f.cbuf : nullptr, (int32_t)mw0);
            decoded = L + got;
        }
    }
    // values the codec did not produce stay 0 in Java's decompressedValues[]: transform them too
    if (!c.err) {
        for (int32_t b = decoded; b < c.n; b += 64) {
            uint32_t vv[1] = {0};
            sink_values<OP, 1>(vv, b, 0, c.n - b < 64 ? c.n - b : 64, c.nb, c.out, cr);
        }
        if (OP == COVT_OP_FPF_ZZ_DELTA_XY && (c.n & 1)) c.err = COVT_ERR_COUNT_MISMATCH;
    }
    COVT_PHASE(c, 7);
    c.consumed = c.byte_length;
}

// A FastPFOR chunk's values were stored with the running sums from 0 at its first value: add the sums of
// the values before it (x / y alternate by value index for the coordinate op; v0 is a multiple of 256), in
// place, 16 bytes per lane.  (Morton codes are not linear in the sum: that op decodes twice instead.)
template <int OP>
__device__ __forceinline__ void fpf_add_carry(uint8_t* out, int32_t v0, int32_t v1, Carry cr) {
    const uint32_t cx = cr.x, cy = OP == COVT_OP_FPF_ZZ_DELTA_XY ? cr.y : cr.x;
    if ((cx | cy) == 0u) return;  // (uniform)
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): this wave's own stores of the range have completed
    int32_t* o = (int32_t*)out;
    typedef __attribute__((address_space(1))) i32x4 g_i4;
    // Eight 1 KiB loads in flight per round trip (a load -> add -> store loop waited out one HBM round trip
    // per KiB: the values were just written past L2; an 8192-value chunk spent most of its time here).  The
    // loads are unmasked (a lane past the range re-reads the range's last whole 16 bytes, not stored), the
    // stores masked; the range's last 0-3 values (a stream's end) element by element.
    const int32_t nq = (v1 - v0) >> 2;  // whole 16-byte quads
    const int32_t last = v0 + 4 * (nq > 0 ? nq - 1 : 0);
    constexpr int kDeep = 8;
    for (int32_t q0 = 0; q0 < nq; q0 += 64 * kDeep) {
        i32x4 v[kDeep];
#pragma unroll
        for (int k = 0; k < kDeep; ++k) v[k] = *(const g_i4*)(o + min(v0 + 4 * (q0 + 64 * k + lane_id()), last));
#pragma unroll
        for (int k = 0; k < kDeep; ++k) {
            const int32_t q = q0 + 64 * k + lane_id();
            if (q < nq)
                st_out16(o + v0 + 4 * q, make_int4((int32_t)((uint32_t)v[k].x + cx), (int32_t)((uint32_t)v[k].y + cy),
                                                   (int32_t)((uint32_t)v[k].z + cx), (int32_t)((uint32_t)v[k].w + cy)));
        }
    }
    const int32_t i = v0 + 4 * nq + lane_id();  // (v0 even: value i is an x value when i - v0 is even)
    if (i < v1) o[i] = (int32_t)((uint32_t)o[i] + (((i - v0) & 1) ? cy : cx));
}

// --------------------------------------------------------------------------------------------
// long streams split into chunks (COVT_FAMILY_SPLIT; plan rule and layout in include/covt.h)
// --------------------------------------------------------------------------------------------
// A long varint stream is a serial chain only through two things: where each value starts and the
// running sum of the delta ops.  Both are local once a chunk knows its first value and its
// predecessors' totals: every byte with bit 7 clear ends a Java-capped varint (a value's bytes are
// continuation bytes then one terminator, or four bytes), so the value after the last such byte
// before the chunk starts a value; values are owned by the chunk their last byte falls in.  Each
// chunk wave (1) finds its first owned value, (2) decodes its values once to count and sum them
// (no stores), (3) publishes that aggregate, (4) looks back over its predecessors' records (their
// inclusive prefix if published, else their aggregate and one step further back) for the values
// and sums before it, publishes its inclusive prefix, and (5) decodes again with that carry,
// storing its values at their global indices.  Chunks take tickets from a counter in launch order,
// so a chunk only ever waits on chunks whose waves were started before it.
constexpr int kSplitSlots = COVT_SPLIT_SLOTS;
struct Agg {
    int32_t cnt;
    uint32_t sx, sy;  // wrapping sums of the transformed values (x,y ops: of local-even / local-odd values)
};
// a's values followed by b's: b's parity flips when a holds an odd number of values.  A record
// with cnt < 0 is a chunk that found an error (its status in sx, the index of the failing value
// relative to the record's first value in sy): the earlier one wins.
__device__ __forceinline__ Agg agg_cat(const Agg& a, const Agg& b, bool xy) {
    if (a.cnt < 0) return a;
    if (b.cnt < 0) return Agg{b.cnt, b.sx, (uint32_t)a.cnt + b.sy};
    const bool sw = xy && (a.cnt & 1);
    return Agg{a.cnt + b.cnt, a.sx + (sw ? b.sy : b.sx), a.sy + (sw ? b.sx : b.sy)};
}
// A record is three 8-byte granules {tag, value} (cnt, sx, sy), each written by one relaxed
// agent-scope store (a write-through `sc1` store): the data is its own flag, so neither a release
// fence (an XCD L2 write-back) nor an acquire (an L1/L2 invalidation, which would cost every wave on
// the CU its cached windows) is needed -- a reader polls the granules with relaxed agent-scope
// (`sc1`) loads until all three carry the tag (cdna_hip_programming.md, publish/consume recipe R2).
// The launch zeroes every record beforehand (hipMemsetAsync in launch_grouped).
typedef __attribute__((address_space(1))) uint64_t g_u64;
__device__ __forceinline__ void rec_publish(covt_stream_result* rec, const Agg& a, uint32_t tag) {
    if (lane_id() == 0) {
        g_u64* g = (g_u64*)rec;
        const uint64_t t = (uint64_t)tag << 32;
        __hip_atomic_store(g, t | (uint32_t)a.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g + 1, t | a.sx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g + 2, t | a.sy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// the record if all three granules carry the tag
__device__ __forceinline__ bool rec_try(covt_stream_result* rec, uint32_t tag, Agg& a) {
    g_u64* g = (g_u64*)rec;
    const uint64_t x0 = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t x1 = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t x2 = __hip_atomic_load(g + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool ok = (uint32_t)(x0 >> 32) == tag && (uint32_t)(x1 >> 32) == tag && (uint32_t)(x2 >> 32) == tag;
    a = Agg{(int32_t)(uint32_t)x0, (uint32_t)x1, (uint32_t)x2};
    return uniu(ok ? 1u : 0u) != 0u;
}
// result entries of a chunk: 0 = the stream's result (chunk 0), 1-3 aggregate, 4-6 inclusive prefix,
// 7 = the family's ticket counter (first chunk of the launch)
constexpr int kRecAgg = 1, kRecIncl = 4, kRecTicket = 7;
static_assert(kSplitSlots == 8, "split record layout");
constexpr uint32_t kSpinLimit = 1u << 22;  // ~0.5 s of polling: a predecessor that never publishes
// values and sums before chunk `chunk` (ticket t) of a stream: its predecessors are tickets t-chunk..t-1
__device__ Agg lookback(covt_stream_result* res, int64_t t, int32_t chunk, bool xy, int32_t& err) {
    Agg acc{0, 0u, 0u};
    int64_t k = t - 1;
    uint32_t spins = 0;
    for (int32_t left = chunk; left > 0;) {
        covt_stream_result* r = res + kSplitSlots * k;
        Agg a;
        if (rec_try(r + kRecIncl, 2u, a)) {
            acc = agg_cat(a, acc, xy);
            break;
        }
        if (rec_try(r + kRecAgg, 1u, a)) {
            acc = agg_cat(a, acc, xy);
            --k;
            --left;
            continue;
        }
        if (++spins > kSpinLimit) { err = COVT_ERR_DEVICE; break; }
        __builtin_amdgcn_s_sleep(2);
    }
    return acc;
}

// One chunk [s, e) of a split varint stream (ops of split_op, include/covt_internal.h): Java's
// 4-byte-capped int varints, or 64-bit LEB128 (ids; INT_64 zigzag columns in format mode), where a value of
// more than 10 bytes is an error only if it is one of the first num_values (the one-wave decode reads
// no further): a chunk that meets one counts the values before it and publishes an error record
// carrying its index, and whichever chunk finds that index below num_values reports the status.
template <int OP>
__device__ __forceinline__ void run_varint_chunk(Ctx& c, int32_t s, int32_t e, int32_t chunk, covt_stream_result* res, int64_t t) {
    // (COVT_OP_VARINT_ZZ_DELTA_S64 is not split: its 64-bit running sums took this kernel from 65 to 113
    // VGPRs with a scratch spill)
    constexpr bool kU64 = OP == COVT_OP_VARINT_U64 || OP == COVT_OP_VARINT_ZZ_S64;
    constexpr int kVal = kU64 ? VAL_U64_STRICT : VAL_J4;
    constexpr bool kXY = OP == COVT_OP_VARINT_ZZ_DELTA_XY;
    constexpr bool kZZ = OP == COVT_OP_VARINT_ZZ_I32 || OP == COVT_OP_VARINT_ZZ_DELTA_I32 || kXY ||
                         OP == COVT_OP_VARINT_ZZ_I32_AS_I64 || OP == COVT_OP_VARINT_ZZ_DELTA_I64;
    constexpr bool kSum = OP == COVT_OP_VARINT_ZZ_DELTA_I32 || kXY || OP == COVT_OP_VARINT_DELTA_MORTON ||
                          OP == COVT_OP_VARINT_ZZ_DELTA_I64;
    const int l = lane_id();
    // (1) the last byte before s with bit 7 clear ends a value; search back 1 KiB at a time
    int32_t p = 0;
    if (chunk > 0) {
        const uintptr_t lo = (uintptr_t)c.sb & ~(uintptr_t)15;
        int32_t hi = s, last = -1;
        while (hi > 0) {
            uintptr_t w0 = ((uintptr_t)(c.sb + hi) & ~(uintptr_t)15);
            w0 = w0 >= lo + 1008 ? w0 - 1008 : lo;
            const uint4 d = ld128(w0 + 16 * (uintptr_t)l);
            const int32_t q0 = (int32_t)((intptr_t)(w0 + 16 * (uintptr_t)l) - (intptr_t)c.sb);
            const uint32_t T = ~hibits16(d) & 0xffffu & range16(-q0, hi - q0);
            const uint32_t best = T ? (uint32_t)(q0 + 31 - __builtin_clz(T)) + 1u : 0u;
            const uint32_t m = wave_max(best);
            if (m) { last = (int32_t)m - 1; break; }
            hi = (int32_t)((intptr_t)w0 - (intptr_t)c.sb);
        }
        p = last + 1;
        // Java-capped: values of 4 continuation bytes may still end before s: skip them
        while (!kU64 && p < s) {
            const uint32_t x = uniu(ld_le32(c.sb + p));
            const uint32_t u = ~x & 0x80808080u;
            const int32_t len = u ? (__builtin_ctz(u) >> 3) + 1 : 4;
            if (p + len - 1 >= s) break;
            p += len;
        }
    }
    // (2) count and sum the values ending in [s, e); (3) + (4) publish, look back, publish the
    // inclusive prefix; (5) decode again with the carry, values past num_values not stored.  One
    // varint_take call site for both passes (two inlined copies doubled the kernel's registers).
    Win w;
    int32_t err = 0, ferr = 0, cnt = 0, take = 0, pos = p, bad = -1;
    Agg excl{0, 0u, 0u};
#pragma nounroll
    for (int pass = 0; pass < 2; ++pass) {
        uint32_t ax = 0, ay = 0;
        Carry cr{excl.sx, excl.sy};
        uint64_t acc = 0;  // (the split 64-bit ops carry no running sum)
        const int32_t g0 = excl.cnt;
        w.valid = false;
        pos = p;
        const int32_t got = varint_take<MODE_RAW, kVal, 4>(
            *c.sm, c.sb, w, pos, e, pass == 0 ? INT32_MAX : take, pass == 0, err,
            [&](const uint32_t (&lo)[4], const uint32_t (&hi)[4], int32_t base, int32_t first, int32_t count) {
                if (pass == 1) {
                    if constexpr (kU64) sink_u64<OP>(lo, hi, (int64_t)g0 + base, first, count, (int64_t*)c.out, acc);
                    else sink_values<OP, 4>(lo, (int64_t)g0 + base, first, count, c.nb, c.out, cr);
                } else if (kSum) {
                    const int32_t s0 = 4 * l - first;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const bool ok = s0 + k >= 0 && s0 + k < count;
                        const uint32_t z = ok ? (kZZ ? (uint32_t)zz32(lo[k]) : lo[k]) : 0u;
                        const bool odd = kXY && (((uint32_t)(base + 4 * l + k)) & 1u);
                        ax += odd ? 0u : z;
                        ay += odd ? z : 0u;
                    }
                }
            },
            pass == 0 ? 0 : g0, &bad);
        if (pass == 1) break;
        cnt = got;
        if (kU64 && err) {
            cnt = bad;  // the values before the over-long one
        } else if (kU64 && pos < e) {
            // the chunk's tail without a terminator: fine if the window reached the chunk end (the value
            // ends in a later chunk), over-long otherwise (the one-wave decode's BAD_HEADER)
            const int32_t aligned = (int32_t)(((uintptr_t)(c.sb + pos) & ~(uintptr_t)15) - (uintptr_t)c.sb);
            if (aligned + kWin < e) {
                err = COVT_ERR_BAD_HEADER;
                bad = cnt;
            }
        }
        Agg mine{cnt, 0u, 0u};
        if (err) {
            mine = Agg{INT32_MIN, (uint32_t)err, (uint32_t)cnt};
        } else if (kSum) {
            mine.sx = lane_bcast(incl_scan(ax), 63);
            mine.sy = kXY ? lane_bcast(incl_scan(ay), 63) : 0u;
        }
        covt_stream_result* rec = res + kSplitSlots * t;
        int32_t lerr = 0;
        if (chunk == 0) {
            rec_publish(rec + kRecIncl, mine, 2u);
        } else {
            rec_publish(rec + kRecAgg, mine, 1u);
            excl = lookback(res, t, chunk, kXY, lerr);
            rec_publish(rec + kRecIncl, lerr ? Agg{INT32_MIN, (uint32_t)lerr, 0u} : agg_cat(excl, mine, kXY), 2u);
        }
        if (lerr) {  // a predecessor never published
            err = lerr;
            bad = 0;
            excl = Agg{0, 0u, 0u};
            break;
        }
        if (excl.cnt < 0) return;  // an earlier chunk failed: it reports the stream if it must
        if (err && excl.cnt + bad < c.n) ferr = err;  // else past num_values: never read
        err = 0;
        take = min(cnt, c.n - excl.cnt);
        pos = p;
        if (take <= 0) break;
    }
    if (ferr) err = ferr;
    // the stream's result, from the chunk holding its last value (or the last chunk if it is short, or
    // the chunk that failed within the first num_values)
    covt_stream_result* r0 = res + kSplitSlots * (t - chunk);
    const bool has_last = !err && excl.cnt < c.n && excl.cnt + cnt >= c.n;
    const bool short_end = !err && e >= c.byte_length && excl.cnt + cnt < c.n;
    if (l == 0 && (has_last || short_end || err)) {
        covt_stream_result r;
        r.status = err ? err : (has_last ? COVT_OK : COVT_ERR_TRUNCATED);
        r.consumed = pos;
        *r0 = r;
    }
}

// One chunk [v0, v1) (values, whole 256-value blocks; the last chunk ends at num_values) of a split
// FastPFOR stream: the same two passes as run_varint_chunk over run_fastpfor's value range (pass one
// sums without storing, pass two stores with the carry).  Each chunk walks the page directories and
// the block headers before its range itself, so chunks depend on each other only through the sums.
template <int OP>
__device__ __forceinline__ void run_fastpfor_chunk(Ctx& c, int32_t v0, int32_t v1, int32_t chunk, covt_stream_result* res,
                                   int64_t t, const covt_stream_desc* __restrict__ cd) {
    constexpr bool kXY = OP == COVT_OP_FPF_ZZ_DELTA_XY;
    Carry carry{0u, 0u};
    int32_t err = 0;
    FpfSkip skip;
    {  // the plan's walk of the headers before the chunk (pads [2..7], covt_host.cpp fpf_chunk_states)
        auto slot = [&](int i) -> const int32_t* {
            return (const int32_t*)((const uint8_t*)(cd + 2 + i / 7) + covt_fpf_state_byte(i % 7));
        };
        if (uni(*slot(0)) == 1) {
            const int l = lane_id();
            skip.done = uni(*slot(1));
            skip.cur0 = uni(*slot(2));
            skip.pk = uni(*slot(3));
            skip.xc = l <= 32 ? *slot(4 + l) : 0;
        }
    }
    // The delta ops are linear in the carry: one decode stores the chunk's values with its own running
    // sums (from 0), publishes them, and after the look-back adds the predecessors' sums in place (an
    // 8 KiB read-modify-write for a 2048-value chunk instead of a second decode).  Morton decodes twice:
    // a pass of sums only, then the decode with the carry.
    constexpr bool kOnce = OP != COVT_OP_FPF_DELTA_MORTON;
    // fpf_add_carry adds the carry in place: right only for int32 outputs indexed by value whose values are
    // linear in the running sum (x / y by value parity for XY, whose chunks start at even values -- v0 is a
    // multiple of 256).  Any other op listed in split_fpf_op (covt_internal.h) must decode twice.
    static_assert(OP == COVT_OP_FPF_ZZ_DELTA_I32 || OP == COVT_OP_FPF_ZZ_DELTA_XY || OP == COVT_OP_FPF_DELTA_MORTON,
                  "split FastPFOR op without a carry rule");
    static_assert(!kOnce || OP == COVT_OP_FPF_ZZ_DELTA_I32 || OP == COVT_OP_FPF_ZZ_DELTA_XY,
                  "in-place carry only for the linear int32 ops");
#pragma nounroll
    for (int pass = 0; pass < 2; ++pass) {  // one inlined copy of the decoder for both passes
        Carry sums{0u, 0u};
        c.err = 0;
        run_fastpfor<OP>(c, v0, v1, carry, pass == 0 && !kOnce, &sums, &skip, kOnce ? &sums : nullptr);
        if (pass == 1) {
            err = c.err;
            break;
        }
        const int32_t own_err = c.err;
        const Agg mine = own_err ? Agg{INT32_MIN, (uint32_t)own_err, 0u} : Agg{v1 - v0, sums.x, sums.y};
        covt_stream_result* rec = res + kSplitSlots * t;
        Agg excl{0, 0u, 0u};
        if (chunk == 0) {
            rec_publish(rec + kRecIncl, mine, 2u);
        } else {
            rec_publish(rec + kRecAgg, mine, 1u);
            excl = lookback(res, t, chunk, kXY, err);
            rec_publish(rec + kRecIncl, err ? Agg{INT32_MIN, (uint32_t)err, 0u} : agg_cat(excl, mine, kXY), 2u);
        }
        if (!err && excl.cnt < 0) err = (int32_t)excl.sx;  // an earlier chunk's error
        if (!err) err = own_err;
        if (err) break;
        carry = Carry{excl.sx, excl.sy};
        if (kOnce) {  // the values are stored: add the carry (chunk 0: none)
            fpf_add_carry<OP>(c.out, v0, v1 < c.n ? v1 : c.n, carry);
            break;
        }
    }
    if (lane_id() == 0 && (v1 >= c.n || err)) {  // the last chunk (or an error) sets the stream's result
        covt_stream_result r;
        r.status = err;
        r.consumed = c.byte_length;
        res[kSplitSlots * (t - chunk)] = r;
    }
}

// One chunk of a split ORC RLE stream: whole groups, located by the plan's host walk (pads: [1] the
// chunk's bytes [s, e), [2] its values [v0, v0 + nv), [3] the stream's consumed bytes).  Groups carry
// no state across, so a chunk needs no look-back: it decodes like a stream of its own into its slice
// of the stream's output.  The stream's result entry (zeroed before the launch) takes the first chunk's
// consumed count and the lowest failing status (the plan splits only streams whose group structure it
// walked: what remains is the GeometryType range check, BAD_HEADER from any chunk).
__device__ __forceinline__ void run_rle_chunk(Ctx& c, const covt_stream_desc* __restrict__ cd, int32_t chunk, covt_stream_result* res,
                              int64_t t) {
    const int32_t s = (int32_t)cd[1].in_off, e = (int32_t)cd[1].out_off;
    const int32_t v0 = (int32_t)cd[2].in_off, nv = (int32_t)cd[2].out_off;
    c.sb += s;
    c.avail = c.byte_length = e - s;
    c.n = v0 + nv;
    if (c.op == COVT_OP_BYTE_RLE_U8 || c.op == COVT_OP_BYTE_RLE_RAW) run_rle_byte(c, v0, true);
    else run_rle_int(c, v0);
    if (lane_id() == 0) {
        covt_stream_result* r0 = res + kSplitSlots * (t - chunk);
        if (c.err) atomicMin(&r0->status, c.err);
        if (chunk == 0) r0->consumed = (int32_t)cd[3].in_off;
    }
}

// One split chunk per wave, chunks in ticket order (tickets from a counter in the split region's
// result entries).  K: kSplitVarint, kSplitFpf, kSplitRle (COVT_FAMILY_SPLIT, _SPLIT_FPF, _SPLIT_RLE).
constexpr int kSplitVarint = 0, kSplitFpf = 1, kSplitRle = 2;
template <int K>
__device__ __forceinline__ int64_t decode_split_chunk(WaveSmem* sm, const uint8_t* __restrict__ in, const covt_stream_desc* __restrict__ descs,
                                      int64_t n_chunks, uint8_t* __restrict__ out, covt_stream_result* __restrict__ res) {
    constexpr bool FPF = K == kSplitFpf;
    uint32_t* ctr = (uint32_t*)(res + kRecTicket);  // the first chunk's ticket entry
    uint32_t tk = 0;
    if (lane_id() == 0) tk = atomicAdd(ctr, 1u);
    const int64_t t = (int64_t)lane_bcast(tk, 0);
    if (t >= n_chunks) return -1;
    // chunks are pieces of the launch's longest streams: the same raised priority as a long stream's wave
    __builtin_amdgcn_s_setprio(COVT_CHUNK_PRIO);
    const covt_stream_desc d = descs[kSplitSlots * t];
    const covt_stream_desc rg = descs[kSplitSlots * t + 1];  // the chunk's byte range
    Ctx c;
    c.sm = sm;
    c.sb = in + d.in_off;
    c.out = out + d.out_off;
    c.avail = d.byte_length;
    c.n = d.num_values;
    c.nb = d.num_bits;
    c.op = d.op;
    c.byte_length = d.byte_length;
    c.err = 0;
    c.consumed = 0;
#ifdef COVT_TIMING  // phase clocks -> entries 2..7 of the chunk descriptor's phase row (0, 1: duration, start)
    c.ph_last = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < kPhases; ++k) c.ph[k] = 0;
    struct PhaseOut {
        Ctx& c;
        const covt_stream_desc* row;
        __device__ ~PhaseOut() {
            if (covt_phase_buf && lane_id() == 0) {
                uint32_t* r = covt_phase_buf + (row - covt_phase_desc0) * kPhases;
                for (int k = 0; k < kPhases - 2; ++k) r[2 + k] = c.ph[k];
            }
        }
    } phase_out{c, descs + kSplitSlots * t};
#endif
    const int32_t chunk = d.avail, s = (int32_t)rg.in_off, e = (int32_t)rg.out_off;
    if constexpr (K == kSplitRle) {
        run_rle_chunk(c, descs + kSplitSlots * t, chunk, res, t);
        return t;
    }
    if constexpr (FPF) {
        switch (d.op) {
        case COVT_OP_FPF_ZZ_DELTA_I32: run_fastpfor_chunk<COVT_OP_FPF_ZZ_DELTA_I32>(c, s, e, chunk, res, t, descs + kSplitSlots * t); break;
        case COVT_OP_FPF_ZZ_DELTA_XY: run_fastpfor_chunk<COVT_OP_FPF_ZZ_DELTA_XY>(c, s, e, chunk, res, t, descs + kSplitSlots * t); break;
        default: run_fastpfor_chunk<COVT_OP_FPF_DELTA_MORTON>(c, s, e, chunk, res, t, descs + kSplitSlots * t); break;
        }
        return t;
    }
    switch (d.op) {
    case COVT_OP_VARINT_I32: run_varint_chunk<COVT_OP_VARINT_I32>(c, s, e, chunk, res, t); break;
    case COVT_OP_VARINT_ZZ_I32: run_varint_chunk<COVT_OP_VARINT_ZZ_I32>(c, s, e, chunk, res, t); break;
    case COVT_OP_VARINT_ZZ_DELTA_I32: run_varint_chunk<COVT_OP_VARINT_ZZ_DELTA_I32>(c, s, e, chunk, res, t); break;
    case COVT_OP_VARINT_ZZ_DELTA_XY: run_varint_chunk<COVT_OP_VARINT_ZZ_DELTA_XY>(c, s, e, chunk, res, t); break;
    case COVT_OP_VARINT_DELTA_MORTON: run_varint_chunk<COVT_OP_VARINT_DELTA_MORTON>(c, s, e, chunk, res, t); break;
    case COVT_OP_VARINT_I32_AS_I64: run_varint_chunk<COVT_OP_VARINT_I32_AS_I64>(c, s, e, chunk, res, t); break;
    case COVT_OP_VARINT_ZZ_I32_AS_I64: run_varint_chunk<COVT_OP_VARINT_ZZ_I32_AS_I64>(c, s, e, chunk, res, t); break;
    case COVT_OP_VARINT_ZZ_DELTA_I64: run_varint_chunk<COVT_OP_VARINT_ZZ_DELTA_I64>(c, s, e, chunk, res, t); break;
    case COVT_OP_VARINT_U64: run_varint_chunk<COVT_OP_VARINT_U64>(c, s, e, chunk, res, t); break;
    default: run_varint_chunk<COVT_OP_VARINT_ZZ_S64>(c, s, e, chunk, res, t); break;
    }
    return t;
}

__host__ __device__ constexpr int op_family(int op) { return covt_op_family(op); }

// One wave per descriptor; waves whose descriptor belongs to another family return at once (used
// when the caller's descriptors are not grouped by family).
// Split chunks (COVT_FAMILY_SPLIT) have a kernel of their own: inside the varint family kernel their
// code raised it from 31 to 72 VGPRs with a scratch spill (varint family alone 0.63 -> 0.88 ms).
// (FPF: the FastPFOR chunks, COVT_FAMILY_SPLIT_FPF, their own kernel and ticket sequence for the same reason)
template <int K>
__global__ __launch_bounds__(64 * kWavesPerBlock) void decode_split_kernel(const uint8_t* __restrict__ in,
                                                                           const covt_stream_desc* __restrict__ descs,
                                                                           int64_t n_chunks, uint8_t* __restrict__ out,
                                                                           covt_stream_result* __restrict__ res) {
    constexpr int kStride = K == kSplitFpf ? kFamSmemFpf : K == kSplitRle ? kFamSmemRle : kFamSmemVarint;
    __shared__ __attribute__((aligned(16))) uint8_t smem[kWavesPerBlock * kStride];
    const int wv = uni((int)(threadIdx.x >> 6));
#ifdef COVT_TIMING  // profiling build: a chunk's (duration, start) in 100 MHz ticks -> phase row of its descriptor
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const int64_t t = decode_split_chunk<K>((WaveSmem*)(smem + wv * kStride), in, descs, n_chunks, out, res);
#ifdef COVT_TIMING
    if (t >= 0 && covt_phase_buf && lane_id() == 0) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        uint32_t* row = covt_phase_buf + (descs + kSplitSlots * t - covt_phase_desc0) * kPhases;
        row[0] = (uint32_t)(t_end - t_start);
        row[1] = (uint32_t)t_start;
    }
#else
    (void)t;
#endif
}

// One stream of family FAM on this wave (descriptor sid; `smem`: the wave's scratch).
// FS (FastPFOR only): whole streams through run_fastpfor_stream (the ring / batched-header path) instead of
// run_fastpfor; the launch picks it for batches of many FastPFOR streams (covt_launch_family_split)
template <int FAM, bool FS = false>
__device__ __forceinline__ void decode_family_wave(uint8_t* smem, const uint8_t* __restrict__ in,
                                                   const covt_stream_desc* __restrict__ descs, int64_t sid,
                                                   uint8_t* __restrict__ out, covt_stream_result* __restrict__ res) {
    const covt_stream_desc d = descs[sid];
    if ((d.flags & (COVT_DESC_LANE | COVT_DESC_SPLIT | COVT_DESC_SPLIT_PAD)) || op_family(d.op) != FAM) return;
    // long streams are the kernel's critical path: let their waves win instruction arbitration
    if (d.byte_length > kLongStream || d.num_values > kLongStream) __builtin_amdgcn_s_setprio(COVT_LONG_PRIO);
#ifdef COVT_TIMING  // profiling build (libcovt_timing.so): result = (duration, start) in 100 MHz ticks
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    Ctx c;
    c.sm = (WaveSmem*)smem;
    c.sb = in + d.in_off;
    c.out = out + d.out_off;
    c.avail = d.avail;
    c.n = d.num_values;
    c.nb = d.num_bits;
    c.op = d.op;
    c.byte_length = d.byte_length;
    c.err = 0;
    c.consumed = 0;
#ifdef COVT_TIMING
    c.ph_last = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < kPhases; ++k) c.ph[k] = 0;
#endif
    if (c.n < 0 || c.avail < 0 || c.byte_length < 0) {
        c.err = COVT_ERR_INVALID_ARG;
    } else if (FAM == COVT_FAMILY_RLE) {
        if (c.op == COVT_OP_BYTE_RLE_U8 || c.op == COVT_OP_BYTE_RLE_RAW) { if (c.n > 0) run_rle_byte(c); }
        else if (c.op == COVT_OP_RLE_U64 || c.op == COVT_OP_RLE_I32 || c.op == COVT_OP_RLE_S64) { if (c.n > 0) run_rle_int(c); }
        else c.err = COVT_ERR_UNSUPPORTED_ENCODING;
#if defined(COVT_ABL_ONEOP)  // ablation build (instruction-cache footprint): one code path per family
    } else if (FAM == COVT_FAMILY_VARINT) {
        if (c.op == COVT_OP_VARINT_U64) run_varint_stream<COVT_OP_VARINT_U64>(c);
        else run_varint_stream<COVT_OP_VARINT_ZZ_DELTA_I32>(c);
    } else if (true) {
        run_fastpfor<COVT_OP_FPF_ZZ_DELTA_I32>(c);
#endif
    } else if (FAM == COVT_FAMILY_VARINT) {
        switch (c.op) {  // one uniform switch per stream; the loops are specialised per op
        case COVT_OP_VARINT_I32: run_varint_stream<COVT_OP_VARINT_I32>(c); break;
        case COVT_OP_VARINT_ZZ_I32: run_varint_stream<COVT_OP_VARINT_ZZ_I32>(c); break;
        case COVT_OP_VARINT_ZZ_DELTA_I32: run_varint_stream<COVT_OP_VARINT_ZZ_DELTA_I32>(c); break;
        case COVT_OP_VARINT_ZZ_DELTA_XY: run_varint_stream<COVT_OP_VARINT_ZZ_DELTA_XY>(c); break;
        case COVT_OP_VARINT_DELTA_MORTON: run_varint_stream<COVT_OP_VARINT_DELTA_MORTON>(c); break;
        case COVT_OP_VARINT_U64: run_varint_stream<COVT_OP_VARINT_U64>(c); break;
        case COVT_OP_VARINT_I32_AS_I64: run_varint_stream<COVT_OP_VARINT_I32_AS_I64>(c); break;
        case COVT_OP_VARINT_ZZ_I32_AS_I64: run_varint_stream<COVT_OP_VARINT_ZZ_I32_AS_I64>(c); break;
        case COVT_OP_VARINT_ZZ_S64: run_varint_stream<COVT_OP_VARINT_ZZ_S64>(c); break;
        case COVT_OP_VARINT_ZZ_DELTA_S64: run_varint_stream<COVT_OP_VARINT_ZZ_DELTA_S64>(c); break;
        default: run_varint_stream<COVT_OP_VARINT_ZZ_DELTA_I64>(c); break;
        }
    } else {
        if constexpr (FS) {
            switch (c.op) {
            case COVT_OP_FPF_ZZ_DELTA_I32: run_fastpfor_stream<COVT_OP_FPF_ZZ_DELTA_I32>(c); break;
            case COVT_OP_FPF_ZZ_DELTA_XY: run_fastpfor_stream<COVT_OP_FPF_ZZ_DELTA_XY>(c); break;
            default: run_fastpfor_stream<COVT_OP_FPF_DELTA_MORTON>(c); break;
            }
        } else {
            switch (c.op) {
            case COVT_OP_FPF_ZZ_DELTA_I32: run_fastpfor<COVT_OP_FPF_ZZ_DELTA_I32>(c); break;
            case COVT_OP_FPF_ZZ_DELTA_XY: run_fastpfor<COVT_OP_FPF_ZZ_DELTA_XY>(c); break;
            default: run_fastpfor<COVT_OP_FPF_DELTA_MORTON>(c); break;
            }
        }
    }
    if (lane_id() == 0) {
        covt_stream_result r;
        r.status = c.err;
        r.consumed = c.consumed;
#ifdef COVT_TIMING
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        r.status = c.err ? -1 : (int32_t)(t_end - t_start);
        r.consumed = (int32_t)(uint32_t)t_start;
        if (covt_phase_buf)
            for (int k = 0; k < kPhases; ++k) covt_phase_buf[(descs + sid - covt_phase_desc0) * kPhases + k] = c.ph[k];
#endif
        res[sid] = r;
    }
}

#ifndef COVT_FPF_WAVES
#define COVT_FPF_WAVES 7  // A/B: waves per SIMD the FastPFOR family kernel (run_fastpfor) is register-budgeted for
#endif
#ifndef COVT_FPF_STREAM_WAVES
#define COVT_FPF_STREAM_WAVES 8  // ... and its run_fastpfor_stream variant (7 -> 8: launch 1.504 -> 1.495 ms)
#endif
template <int FAM, bool FS = false>
__global__ __launch_bounds__(64 * kWavesPerBlock) __attribute__((amdgpu_waves_per_eu(FAM == COVT_FAMILY_FASTPFOR ? (FS ? COVT_FPF_STREAM_WAVES : COVT_FPF_WAVES) : 7))) void decode_family_kernel(const uint8_t* __restrict__ in,
                                                            const covt_stream_desc* __restrict__ descs,
                                                            int64_t n_streams, uint8_t* __restrict__ out,
                                                            covt_stream_result* __restrict__ res) {
    constexpr int kStride = FAM == COVT_FAMILY_RLE ? kFamSmemRle
                            : FAM == COVT_FAMILY_VARINT ? kFamSmemVarint : kFamSmemFpf;
    __shared__ __attribute__((aligned(16))) uint8_t smem[kWavesPerBlock * kStride];
    const int wv = uni((int)(threadIdx.x >> 6));
    const int64_t sid = (int64_t)blockIdx.x * kWavesPerBlock + wv;
    if (sid >= n_streams) return;
    decode_family_wave<FAM, FS>(smem + wv * kStride, in, descs, sid, out, res);
}

// --------------------------------------------------------------------------------------------
// lane-per-stream path: small RLE streams (the plan's lane limits, flagged by the plan), one
// stream per lane, decoded serially the way RunLengthIntegerReader / RunLengthByteReader read them.
// A wave-per-stream decode spends its fixed window/index setup on a handful of values; here 64
// such streams share one wave's instructions.
// --------------------------------------------------------------------------------------------
#ifndef COVT_LANE_SLOT
#define COVT_LANE_SLOT 17
#endif
constexpr int kLaneSlot = COVT_LANE_SLOT;  // LDS dwords per lane: a sliding window of 4 * kLaneSlot bytes (68)
static_assert(kLaneSlot % 4 == 1, "16-byte granules plus one dword");
struct LaneBytes {  // the lane's stream through a window in its LDS slot; one-dword read cache
    const uint8_t* sb;
    uint32_t* slot;
    int32_t avail;
    int32_t w0;  // stream offset of slot byte 0 (4-byte aligned in memory)
    int32_t cq;
    uint32_t cw;
    // window = stream bytes [w0, w0 + 68) from p's 4-byte aligned address; up to 4 x 16 B + 4 B loads at
    // once, only those holding stream bytes (a 10-byte stream loads 16 bytes, not 68)
    __device__ __forceinline__ void load(int32_t p) {
        const uintptr_t a = (uintptr_t)(sb + p), a4 = a & ~(uintptr_t)3;
        w0 = p - (int32_t)(a & 3u);
        const int32_t need = avail - w0;  // window bytes that are stream bytes
        uint32_t st[kLaneSlot];
#pragma unroll
        for (int k = 0; k < kLaneSlot / 4; ++k) {
            u32x4 v = {0u, 0u, 0u, 0u};
            if (16 * k < need) v = *(const __attribute__((address_space(1))) u32x4*)(a4 + 16 * k);
            st[4 * k] = v.x;
            st[4 * k + 1] = v.y;
            st[4 * k + 2] = v.z;
            st[4 * k + 3] = v.w;
        }
        st[kLaneSlot - 1] = 4 * (kLaneSlot - 1) < need ? *g32(a4 + 4 * (kLaneSlot - 1)) : 0u;
#pragma unroll
        for (int k = 0; k < kLaneSlot; ++k) slot[k * 256] = st[k];
        cq = -1;
    }
    // bytes [p, p + 4) little-endian (two slot dwords and a byte align)
    __device__ __forceinline__ uint32_t at4(int32_t p) {
        if (p + 4 - w0 > 4 * kLaneSlot) load(p);
        const int32_t a = p - w0, q = a >> 2;
        const uint32_t d0 = slot[q * 256], d1 = (a & 3) ? slot[(q + 1) * 256] : 0u;
        cq = -1;
        return __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)(a & 3));
    }
    __device__ __forceinline__ uint32_t at(int32_t p) {
        if (p - w0 >= 4 * kLaneSlot) load(p);  // slides forward (reads are sequential)
        const int32_t a = p - w0, q = a >> 2;
        if (q != cq) {
            cq = q;
            cw = slot[q * 256];
        }
        return (cw >> (8u * (uint32_t)(a & 3))) & 0xffu;
    }
};
// orc SerializationUtils.readVulong (shift masked to 6 bits)
__device__ __forceinline__ int32_t lane_vulong(LaneBytes& in, int32_t& p, uint64_t& v) {
    uint64_t r = 0;
    uint32_t sh = 0, b;
    do {
        if (p >= in.avail) return COVT_ERR_TRUNCATED;
        b = in.at(p++);
        r |= (uint64_t)(b & 0x7fu) << (sh & 63u);
        sh += 7;
    } while (b & 0x80u);
    v = r;
    return COVT_OK;
}
// A lane's output gathered into 16-byte packets: one store per 16 bytes instead of one per value
// (each lane writes a different stream, so every store instruction touches 64 separate lines).
// The last packet is written whole: stream outputs start 16-byte aligned and are padded to 16.
struct Pack16 {
    uint32_t w0, w1, w2, w3;
    uint32_t nb;   // bytes in the packet
    uint8_t* dst;  // the packet's address
    __device__ __forceinline__ void flush() {
        *(uint4*)dst = make_uint4(w0, w1, w2, w3);
        dst += 16;
    }
    __device__ __forceinline__ void put32(uint32_t v) {
        const uint32_t k = (nb >> 2) & 3u;
        w0 = k == 0 ? v : w0;
        w1 = k == 1 ? v : w1;
        w2 = k == 2 ? v : w2;
        w3 = k == 3 ? v : w3;
        nb += 4;
        if ((nb & 15u) == 0) flush();
    }
    __device__ __forceinline__ void put8(uint32_t b) {
        const uint32_t k = (nb >> 2) & 3u, sh = 8u * (nb & 3u);
        const uint32_t m = ~(0xffu << sh), x = b << sh;
        w0 = k == 0 ? (w0 & m) | x : w0;
        w1 = k == 1 ? (w1 & m) | x : w1;
        w2 = k == 2 ? (w2 & m) | x : w2;
        w3 = k == 3 ? (w3 & m) | x : w3;
        nb += 1;
        if ((nb & 15u) == 0) flush();
    }
    // a run of k elements base + i * delta (E = 4: int32, E = 8: int64), whole packet slots per step:
    // a run costs k / (16 / E) steps instead of k (the other lanes of the wave wait on the longest)
    template <int E>
    __device__ __forceinline__ void put_run(int64_t base, int32_t delta, int32_t k) {
        constexpr int PER = 16 / E;  // elements per packet
        while (k > 0) {
            const int32_t slot = (int32_t)((nb / E) & (PER - 1));
            const int32_t m = min(PER - slot, k);
            uint32_t w[4] = {w0, w1, w2, w3};
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                const int32_t i = j - slot;
                if (i >= 0 && i < m) {
                    const uint64_t v = (uint64_t)base + (uint64_t)(int64_t)(int32_t)(i * delta);
                    if (E == 4) {
                        w[j] = (uint32_t)v;
                    } else {
                        w[2 * j] = (uint32_t)v;
                        w[2 * j + 1] = (uint32_t)(v >> 32);
                    }
                }
            }
            w0 = w[0];
            w1 = w[1];
            w2 = w[2];
            w3 = w[3];
            base = (int64_t)((uint64_t)base + (uint64_t)(int64_t)(int32_t)(m * delta));
            k -= m;
            nb += (uint32_t)(m * E);
            if ((nb & 15u) == 0) flush();
        }
    }
    // k copies of byte b, up to 16 per step
    __device__ __forceinline__ void put_bytes(uint32_t b, int32_t k) {
        const uint32_t rep = (b & 0xffu) * 0x01010101u;
        while (k > 0) {
            const int32_t slot = (int32_t)(nb & 15u);
            const int32_t m = min(16 - slot, k);
            uint32_t w[4] = {w0, w1, w2, w3};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t lo = max(slot - 4 * j, 0), hi = min(slot + m - 4 * j, 4);  // bytes [lo, hi) of dword j
                if (hi > lo) {
                    const uint32_t mask = (hi >= 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u)) & ~((1u << (8 * lo)) - 1u);
                    w[j] = (w[j] & ~mask) | (rep & mask);
                }
            }
            w0 = w[0];
            w1 = w[1];
            w2 = w[2];
            w3 = w[3];
            k -= m;
            nb += (uint32_t)m;
            if ((nb & 15u) == 0) flush();
        }
    }
    // four bytes (little-endian in v) at any byte position of the packet
    __device__ __forceinline__ void put4(uint32_t v) {
        const uint32_t sh = 8u * (nb & 3u), k = (nb >> 2) & 3u;
        const uint32_t lo = v << sh, hi = sh ? v >> (32u - sh) : 0u;
        const uint32_t mlo = 0xffffffffu << sh;
        uint32_t w[4] = {w0, w1, w2, w3};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((uint32_t)j == k) w[j] = (w[j] & ~mlo) | lo;
        w0 = w[0];
        w1 = w[1];
        w2 = w[2];
        w3 = w[3];
        nb += 4;
        if ((nb & 15u) < 4u) {  // crossed into the next packet: flush, carry the high bytes
            flush();
            w0 = hi;
        } else if (sh) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((uint32_t)j == k + 1u) w[j] = hi;
            w0 = w[0];
            w1 = w[1];
            w2 = w[2];
            w3 = w[3];
        }
    }
    __device__ __forceinline__ void finish() {
        if (nb & 15u) flush();
    }
};
__device__ void lane_rle_int(LaneBytes& in, int op, int32_t n, uint8_t* out, int32_t& err, int32_t& consumed) {
    const bool is_signed = op == COVT_OP_RLE_S64, to_i32 = op == COVT_OP_RLE_I32;
    int32_t o = 0, done = 0;
    Pack16 pk{0, 0, 0, 0, 0, out};
    auto put = [&](int64_t v) {
        pk.put32((uint32_t)v);
        if (!to_i32) pk.put32((uint32_t)((uint64_t)v >> 32));
        ++done;
    };
    while (done < n) {
        if (o >= in.avail) { err = COVT_ERR_TRUNCATED; return; }
        const uint32_t control = in.at(o++);
        if (control < 0x80u) {  // run: control + 3 values base + i * delta
            const int32_t cnt = (int32_t)control + 3;
            if (o >= in.avail) { err = COVT_ERR_TRUNCATED; return; }
            const int32_t delta = (int32_t)(int8_t)in.at(o++);
            uint64_t raw;
            if ((err = lane_vulong(in, o, raw))) return;
            const int64_t b = is_signed ? zz64(raw) : (int64_t)raw;
            const int32_t k = cnt < n - done ? cnt : n - done;
            if (to_i32) pk.put_run<4>(b, delta, k);
            else pk.put_run<8>(b, delta, k);
            done += k;
        } else {  // literals: 256 - control varints, all read even past n
            const int32_t cnt = 0x100 - (int32_t)control;
            for (int32_t i = 0; i < cnt; ++i) {
                uint64_t raw;
                if ((err = lane_vulong(in, o, raw))) return;
                if (done < n) put(is_signed ? zz64(raw) : (int64_t)raw);
            }
        }
    }
    pk.finish();
    consumed = o;
}
__device__ void lane_rle_byte(LaneBytes& in, int32_t n, uint8_t* out, bool check, int32_t& err, int32_t& consumed) {
    int32_t o = 0, done = 0;
    bool bad = false;
    Pack16 pk{0, 0, 0, 0, 0, out};
    while (done < n) {
        if (o >= in.avail) { err = COVT_ERR_TRUNCATED; return; }
        const uint32_t control = in.at(o++);
        if (control < 0x80u) {
            const int32_t cnt = (int32_t)control + 3;
            if (o >= in.avail) { err = COVT_ERR_TRUNCATED; return; }
            const uint32_t b = in.at(o++);
            bad |= b > 5u;
            const int32_t k = cnt < n - done ? cnt : n - done;
            pk.put_bytes(b, k);
            done += k;
        } else {
            const int32_t cnt = 0x100 - (int32_t)control;
            if (o + cnt > in.avail) { err = COVT_ERR_TRUNCATED; return; }
            const int32_t take = cnt < n - done ? cnt : n - done;  // literals past n are skipped
            int32_t i = 0;
            if (!check) {  // (no value check) four bytes per step
                for (; i + 4 <= take; i += 4, o += 4) pk.put4(in.at4(o));
            }
            for (; i < take; ++i) {
                const uint32_t b = in.at(o++);
                bad |= b > 5u;
                pk.put8(b);
            }
            done += take;
            o += cnt - take;
        }
    }
    pk.finish();
    if (bad && check) err = COVT_ERR_BAD_HEADER;  // GeometryType.values()[b]
    consumed = o;
}

// One lane-family stream on this lane (`slot`: the lane's column of a [kLaneSlot][256] dword array)
__device__ __forceinline__ void decode_lane_one(uint32_t* slot, const uint8_t* __restrict__ in,
                                                const covt_stream_desc* __restrict__ descs, int64_t sid,
                                                uint8_t* __restrict__ out, covt_stream_result* __restrict__ res) {
    const covt_stream_desc d = descs[sid];
    if (!(d.flags & COVT_DESC_LANE)) return;
#ifdef COVT_TIMING
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    int32_t err = 0, consumed = 0;
    // the stream's first 68 bytes into the lane's slot (dword k of lane t at slots[k * 256 + t])
    LaneBytes lb{in + d.in_off, slot, d.avail, 0, -1, 0u};
    lb.load(0);
    if (d.num_values < 0 || d.avail < 0) err = COVT_ERR_INVALID_ARG;
    else if (d.op == COVT_OP_BYTE_RLE_U8 || d.op == COVT_OP_BYTE_RLE_RAW)
        lane_rle_byte(lb, d.num_values, out + d.out_off, d.op == COVT_OP_BYTE_RLE_U8, err, consumed);
    else if (d.op == COVT_OP_RLE_U64 || d.op == COVT_OP_RLE_S64 || d.op == COVT_OP_RLE_I32)
        lane_rle_int(lb, d.op, d.num_values, out + d.out_off, err, consumed);
    else err = COVT_ERR_UNSUPPORTED_ENCODING;
    covt_stream_result r;
    r.status = err;
    r.consumed = err ? 0 : consumed;
#ifdef COVT_TIMING
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    r.status = err ? -1 : (int32_t)(t_end - t_start);
    r.consumed = (int32_t)(uint32_t)t_start;
#endif
    res[sid] = r;
}

__global__ __launch_bounds__(256) void decode_lane_kernel(const uint8_t* __restrict__ in,
                                                          const covt_stream_desc* __restrict__ descs,
                                                          int64_t n_streams, uint8_t* __restrict__ out,
                                                          covt_stream_result* __restrict__ res) {
    __shared__ uint32_t slots[256 * kLaneSlot];
    const int64_t sid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (sid >= n_streams) return;
    decode_lane_one(slots + threadIdx.x, in, descs, sid, out, res);
}

// ---- small batches: every family and split region in ONE launch ----------------------------------------
// The grouped launch forks up to four HIP streams so the families run concurrently; for a batch far
// smaller than the GPU (BASELINE configs 2-4: one tile to 61 tiles) the fork / event / join overhead and
// the hardware-queue start-up (a queue's first kernel started up to 26 us late behind another queue's,
// profiles/r02/config_timeline_fpf_state.txt) exceed the decode itself.  This kernel holds every family
// as a segment of one grid, longest work first (workgroups dispatch in blockIdx order): FastPFOR chunks,
// varint chunks, RLE chunks, FastPFOR, RLE, varint streams, then the lane family (128 streams per
// workgroup).  Each segment runs the same device code as its own kernel.
struct FusedSegs {
    const covt_stream_desc* desc[COVT_NUM_FAMILIES];
    covt_stream_result* res[COVT_NUM_FAMILIES];
    int64_t n[COVT_NUM_FAMILIES];  // descriptors (split regions: chunks x kSplitSlots)
    uint32_t wg_end[COVT_NUM_FAMILIES];  // cumulative workgroups, segment order kFusedOrder
};
constexpr int kFusedOrder[COVT_NUM_FAMILIES] = {COVT_FAMILY_SPLIT_FPF, COVT_FAMILY_SPLIT, COVT_FAMILY_SPLIT_RLE,
                                                COVT_FAMILY_FASTPFOR, COVT_FAMILY_RLE, COVT_FAMILY_VARINT,
                                                COVT_FAMILY_LANE};
constexpr int kFusedLds = (kWavesPerBlock * kFamSmemRle > 256 * kLaneSlot * 4) ? kWavesPerBlock * kFamSmemRle
                                                                              : 256 * kLaneSlot * 4;
static_assert(kFamSmemRle >= kFamSmemFpf && kFamSmemRle >= kFamSmemVarint, "RLE scratch is the largest");
// the lane segment: one stream per thread, each in its column of the [kLaneSlot][256] slot array
static_assert(64 * kWavesPerBlock <= 256, "a fused workgroup's threads must fit the 256 lane-slot columns");
static_assert(kFusedLaneStreams == 64 * kWavesPerBlock, "host wave estimate: lane streams per fused workgroup");

__global__ __launch_bounds__(64 * kWavesPerBlock) __attribute__((amdgpu_waves_per_eu(4))) void decode_fused_kernel(const uint8_t* __restrict__ in,
                                                                           uint8_t* __restrict__ out, FusedSegs sg) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kFusedLds];
    const uint32_t b = blockIdx.x;
    // the segment of this workgroup (constant indices only: a dynamically indexed kernel argument would be
    // copied to scratch)
    int fam = COVT_FAMILY_LANE;
    uint32_t local = 0, prev = 0;
    const covt_stream_desc* d = nullptr;
    covt_stream_result* r = nullptr;
    int64_t n = 0;
    bool found = false;
#pragma unroll
    for (int k = 0; k < COVT_NUM_FAMILIES; ++k) {
        const int f = kFusedOrder[k];
        if (!found && b < sg.wg_end[k]) {
            found = true;
            fam = f;
            local = b - prev;
            d = sg.desc[f];
            r = sg.res[f];
            n = sg.n[f];
        }
        prev = sg.wg_end[k];
    }
    if (!found) return;
    const int wv = uni((int)(threadIdx.x >> 6));
    uint8_t* wsm = smem + wv * kFamSmemRle;
    switch (fam) {
    case COVT_FAMILY_SPLIT_FPF:
        decode_split_chunk<kSplitFpf>((WaveSmem*)wsm, in, d, n / kSplitSlots, out, r);
        break;
    case COVT_FAMILY_SPLIT:
        decode_split_chunk<kSplitVarint>((WaveSmem*)wsm, in, d, n / kSplitSlots, out, r);
        break;
    case COVT_FAMILY_SPLIT_RLE:
        decode_split_chunk<kSplitRle>((WaveSmem*)wsm, in, d, n / kSplitSlots, out, r);
        break;
    case COVT_FAMILY_LANE: {
        const int64_t sid = (int64_t)local * (64 * kWavesPerBlock) + threadIdx.x;
        if (sid < n) decode_lane_one((uint32_t*)smem + threadIdx.x, in, d, sid, out, r);
        break;
    }
    default: {
        const int64_t sid = (int64_t)local * kWavesPerBlock + wv;
        if (sid >= n) break;
        if (fam == COVT_FAMILY_FASTPFOR) decode_family_wave<COVT_FAMILY_FASTPFOR>(wsm, in, d, sid, out, r);
        else if (fam == COVT_FAMILY_RLE) decode_family_wave<COVT_FAMILY_RLE>(wsm, in, d, sid, out, r);
        else decode_family_wave<COVT_FAMILY_VARINT>(wsm, in, d, sid, out, r);
    }
    }
}

}  // namespace covt

// The fused small-batch launch (covt::decode_fused_kernel): family f's descriptors at d_desc + off[f],
// its results at d_res + off[f].  Split regions' records must be zeroed before (launch_grouped does).
extern "C" int covt_launch_fused(const uint8_t* d_in, const covt_stream_desc* d_desc, const int64_t counts[COVT_NUM_FAMILIES],
                                 uint8_t* d_out, covt_stream_result* d_res, hipStream_t stream) {
    covt::FusedSegs sg{};
    int64_t off = 0;
    for (int f = 0; f < COVT_NUM_FAMILIES; ++f) {
        if (counts[f] < 0) return COVT_ERR_INVALID_ARG;
        sg.desc[f] = d_desc + off;
        sg.res[f] = d_res + off;
        sg.n[f] = counts[f];
        off += counts[f];
    }
    uint64_t wg = 0;
    for (int k = 0; k < COVT_NUM_FAMILIES; ++k) {
        const int f = covt::kFusedOrder[k];
        const int64_t n = f == COVT_FAMILY_SPLIT || f == COVT_FAMILY_SPLIT_FPF || f == COVT_FAMILY_SPLIT_RLE
                              ? counts[f] / covt::kSplitSlots : counts[f];
        const int64_t per = f == COVT_FAMILY_LANE ? 64 * kWavesPerBlock : kWavesPerBlock;
        wg += (uint64_t)((n + per - 1) / per);
        if (wg > 0x7fffffffull) return COVT_ERR_INVALID_ARG;
        sg.wg_end[k] = (uint32_t)wg;
    }
    if (wg == 0) return COVT_OK;
    hipLaunchKernelGGL(covt::decode_fused_kernel, dim3((unsigned)wg), dim3(64 * kWavesPerBlock), 0, stream,
                       d_in, d_out, sg);
    return hipGetLastError() == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
}

extern "C" int covt_launch_family_split_mode(int fam, const uint8_t* d_in, const covt_stream_desc* d_desc,
                                             int64_t n_streams, uint8_t* d_out, covt_stream_result* d_res,
                                             const covt_stream_desc* d_split, int64_t n_split,
                                             covt_stream_result* d_split_res, hipStream_t stream, int fpf_mode) {
    if (fpf_mode != 0 && fpf_mode != COVT_LAUNCH_FPF_STREAM && fpf_mode != COVT_LAUNCH_FPF_CLASSIC)
        return COVT_ERR_INVALID_ARG;
    if (n_split < 0 || n_split % covt::kSplitSlots) return COVT_ERR_INVALID_ARG;
    if (n_split && fam != COVT_FAMILY_VARINT && fam != COVT_FAMILY_FASTPFOR && fam != COVT_FAMILY_RLE)
        return COVT_ERR_INVALID_ARG;
    if (n_streams <= 0 && n_split == 0) return COVT_OK;
    if (n_streams < 0) n_streams = 0;
    if (fam == COVT_FAMILY_LANE) {
        const int64_t lblocks = (n_streams + 255) / 256;
        if (lblocks > 0x7fffffff) return COVT_ERR_INVALID_ARG;
        hipLaunchKernelGGL(covt::decode_lane_kernel, dim3((unsigned)lblocks), dim3(256), 0, stream, d_in, d_desc,
                           n_streams, d_out, d_res);
        return hipGetLastError() == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
    }
    const int64_t n_chunks = n_split / covt::kSplitSlots;
    const dim3 block(64 * kWavesPerBlock);
    if (n_chunks > 0) {  // the chunks first, on the same stream (the same hardware queue) as the family
        const int64_t sblocks = (n_chunks + kWavesPerBlock - 1) / kWavesPerBlock;
        if (sblocks > 0x7fffffff) return COVT_ERR_INVALID_ARG;
        if (fam == COVT_FAMILY_FASTPFOR)
            hipLaunchKernelGGL(covt::decode_split_kernel<covt::kSplitFpf>, dim3((unsigned)sblocks), block, 0, stream,
                               d_in, d_split, n_chunks, d_out, d_split_res);
        else if (fam == COVT_FAMILY_RLE)
            hipLaunchKernelGGL(covt::decode_split_kernel<covt::kSplitRle>, dim3((unsigned)sblocks), block, 0, stream,
                               d_in, d_split, n_chunks, d_out, d_split_res);
        else
            hipLaunchKernelGGL(covt::decode_split_kernel<covt::kSplitVarint>, dim3((unsigned)sblocks), block, 0,
                               stream, d_in, d_split, n_chunks, d_out, d_split_res);
        if (hipGetLastError() != hipSuccess) return COVT_ERR_DEVICE;
    }
    if (n_streams <= 0) return COVT_OK;
    const int64_t blocks = (n_streams + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0x7fffffff) return COVT_ERR_INVALID_ARG;
    const dim3 grid((unsigned)blocks);
    switch (fam) {
    case COVT_FAMILY_RLE:
        hipLaunchKernelGGL(covt::decode_family_kernel<COVT_FAMILY_RLE>, grid, block, 0, stream, d_in, d_desc,
                           n_streams, d_out, d_res);
        break;
    case COVT_FAMILY_VARINT:
        hipLaunchKernelGGL(covt::decode_family_kernel<COVT_FAMILY_VARINT>, grid, block, 0, stream, d_in, d_desc,
                           n_streams, d_out, d_res);
        break;
    case COVT_FAMILY_FASTPFOR:
        // the ring / batched-header variant for batches of many FastPFOR streams: there it takes the launch 1.525 ->
        // 1.474 ms, while in smaller batches -- a strong-scaling shard -- the per-block pipeline of run_fastpfor
        // keeps the family shorter (N = 2 shard 0.962 -> 0.883 ms)
        if (fpf_mode == COVT_LAUNCH_FPF_STREAM || (fpf_mode == 0 && n_streams >= kFpfStreamMinStreams))
            hipLaunchKernelGGL((covt::decode_family_kernel<COVT_FAMILY_FASTPFOR, true>), grid, block, 0, stream, d_in,
                               d_desc, n_streams, d_out, d_res);
        else
            hipLaunchKernelGGL((covt::decode_family_kernel<COVT_FAMILY_FASTPFOR, false>), grid, block, 0, stream, d_in,
                               d_desc, n_streams, d_out, d_res);
        break;
    default: return COVT_ERR_INVALID_ARG;
    }
    return hipGetLastError() == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
}

extern "C" int covt_launch_family_split(int fam, const uint8_t* d_in, const covt_stream_desc* d_desc,
                                        int64_t n_streams, uint8_t* d_out, covt_stream_result* d_res,
                                        const covt_stream_desc* d_split, int64_t n_split, covt_stream_result* d_split_res,
                                        hipStream_t stream) {
    return covt_launch_family_split_mode(fam, d_in, d_desc, n_streams, d_out, d_res, d_split, n_split, d_split_res,
                                         stream, 0);
}

extern "C" int covt_launch_family(int fam, const uint8_t* d_in, const covt_stream_desc* d_desc, int64_t n_streams,
                                  uint8_t* d_out, covt_stream_result* d_res, hipStream_t stream) {
    return covt_launch_family_split(fam, d_in, d_desc, n_streams, d_out, d_res, nullptr, 0, nullptr, stream);
}

extern "C" int covt_op_family_of(int op) { return covt::op_family(op); }

#ifdef COVT_TIMING
// profiling build only: per-stream phase clocks go to d_buf[n_streams][8] (launch order)
extern "C" int covt_debug_set_phase_buffer(void* d_buf, const void* d_desc0) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(covt::covt_phase_desc0), &d_desc0, sizeof(d_desc0)) != hipSuccess) return -5;
    return hipMemcpyToSymbol(HIP_SYMBOL(covt::covt_phase_buf), &d_buf, sizeof(d_buf)) == hipSuccess ? 0 : -5;
}
#endif
