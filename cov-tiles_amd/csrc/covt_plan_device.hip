// covt_plan_device.hip -- the Id / Geometry plan built on the GPU from tiles already resident in HBM
// (include/covt.h "Device-side plan").
//
// The host plan (covt_plan_create, covt_host.cpp) walks each tile's container metadata on host
// threads -- the host half of CovtParser.decodeCovt (CovtParser.java:53-133) and decodeLayerMetadata
// (:574-652) -- and turns every Id / Geometry stream into a descriptor.  This file does the same walk
// with one wave per tile, so a caller whose tiles are already in HBM gets a decodable descriptor table
// without a round trip through the host:
//   1. walk_count   one wave per tile: the container walk, counting the tile's streams and output bytes
//                   and leaving up to 128 stream records per tile in slots
//   2. prefix sums  (hipcub) of the per-tile counts and output bytes -> each tile's first stream and
//                   output offset; one 32-byte D2H of the totals to size the stream arrays
//   3. emit_slots   each stream's covt_stream_info from the slots (output slices 128-byte aligned, in tile
//                   order: the host plan's layout, byte for byte) and its 16-bit launch key (launch_key,
//                   covt_internal.h); walk_emit walks the tiles with more streams again
//   4. radix sort   two 8-bit stable passes of the launch keys (ties in tile order) -> launch order; the
//                   high-byte pass counts the families
//   5. fill_descs   descriptor k from the k-th stream in launch order (writing it in the sort's last
//                   scatter instead measured slower: the scatter's rounds expose the gather's latency)
// The split rule is the host plan's (split plans: split_mark .. fpf_states_walk below); property columns
// (COVT_PLAN_PROPERTIES) add a property walk per tile and their stream entries after the tile's own.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>

#include "covt.h"
#include "covt_internal.h"
#include "covt_walk.h"
#include "covt_props_plan.h"

struct covt_device_plan {
    int dev = 0;
    int32_t n_tiles = 0, format = 0, id_mode = 0;
    int64_t n_streams = 0, n_descs = 0, out_bytes = 0, in_bytes = 0, out_payload = 0, vertices = 0;
    int32_t spec_redo = 0;  // the stream part ran again with counted sizes (a bound-sized plan that missed)
    int64_t fam_counts[COVT_NUM_FAMILIES] = {};
    void* tile_arena = nullptr;    // status, per-tile counts and prefix sums, totals, scan scratch
    void* stream_arena = nullptr;  // infos, values, keys, launch order, descriptors, sort scratch
    void* desc_arena = nullptr;    // split plans: the descriptors and their streams (n_descs each)
    void* geo_arena = nullptr;     // geometry columns (covt_device_plan_geometry): records, descriptors
    bool geo_built = false;
    int64_t n_geo = 0, asm_bytes = 0;
    covt_geom_info* d_ginfo = nullptr;
    covt_geom_desc* d_gdesc = nullptr;
    void* prop_arena = nullptr;    // property columns (COVT_PLAN_PROPERTIES): records, infos, descriptors
    void* scratch = nullptr;       // creation-time scratch (the property walk's record slots), freed on the way
    int64_t n_props = 0, prop_bytes = 0;
    covt_prop_info* d_pinfo = nullptr;
    covt_prop_desc* d_pdesc = nullptr;
    int32_t* d_status = nullptr;
    covt_stream_info* d_info = nullptr;
    covt_stream_desc* d_desc = nullptr;
    uint32_t* d_order = nullptr;  // descriptor k decodes (a chunk of) stream d_order[k]
};

namespace {

// The plan's arenas come from a per-device stream-ordered pool that keeps freed memory (up to
// kPoolKeep bytes) for the next plan: a plain hipMalloc of the ~100 MB stream arena between the plan's
// two host syncs cost ~0.15 ms of the 10k-tile plan (profiles/r04, kernel trace gap).  The retained memory
// is invisible to other allocators (PyTorch's cache): 1 GiB covers a 10k-tile property plan's arenas, and
// covt_device_plan_pool_trim hands it back on request.
constexpr uint64_t kPoolKeep = 1ull << 30;
hipMemPool_t plan_pool(int dev) {
    static std::mutex mu;
    static hipMemPool_t pools[64] = {};
    if (dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    if (!pools[dev]) {
        hipMemPoolProps pp{};
        pp.allocType = hipMemAllocationTypePinned;
        pp.location.type = hipMemLocationTypeDevice;
        pp.location.id = dev;
        hipMemPool_t mp = nullptr;
        if (hipMemPoolCreate(&mp, &pp) != hipSuccess) return nullptr;
        uint64_t keep = kPoolKeep;
        (void)hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &keep);
        pools[dev] = mp;
    }
    return pools[dev];
}
hipError_t plan_malloc(void** q, size_t n, int dev, hipStream_t s) {
    hipMemPool_t mp = plan_pool(dev);
    if (!mp) return hipErrorOutOfMemory;
    return hipMallocFromPoolAsync(q, n, mp, s);
}

// device totals (int64 slots)
enum { T_STREAMS = 0, T_OUT = 1, T_IN = 2, T_PAYLOAD = 3, T_VERTS = 4, T_LANE = 5, T_FAM = 8,
       T_RCH = 8 + COVT_NUM_FAMILIES, T_N = T_RCH + 1 };

// One tile's bytes, read through a 64-byte window held in registers: four 16-byte loads issued
// together (one memory latency per 64 bytes of the front-to-back metadata walk instead of four).
// Only granules overlapping the tile are loaded (each lies inside the allocation holding the tile);
// every byte the walk uses is inside [0, len).
// compile-time packing of a name literal (bytes [from, from + 8) of its first len bytes)
__host__ __device__ constexpr uint64_t cstrlen(const char* s) { return *s ? 1 + cstrlen(s + 1) : 0; }
__host__ __device__ constexpr uint64_t pk(const char* s, uint64_t from, uint64_t len) {
    uint64_t v = 0;
    for (uint64_t i = from; i < from + 8 && i < len; ++i) v |= (uint64_t)(uint8_t)s[i] << (8 * (i - from));
    return v;
}

// the walking lanes' 64-byte windows (dynamic LDS: 64 bytes per lane of the workgroup)
extern __shared__ uint4 covt_walk_win[];

// Window refill (Rd::peek8): loads the window for byte address a into LDS and returns its base.  Out
// of line and with value arguments only, so the walk has one copy of it (inlined at every read site, the
// walk kernels were ~12k instructions) and the reader's state stays in registers.
__device__ __forceinline__ uint4 window_ld(const uint8_t* t, int64_t len, uintptr_t b) {
    const uintptr_t lo = (uintptr_t)t, hi = lo + (uintptr_t)len;
    return (b + 16 > lo && b < hi) ? *reinterpret_cast<const uint4*>(b) : make_uint4(0, 0, 0, 0);
}
template <bool kWave>
__device__ __noinline__ uintptr_t window_refill(const uint8_t* t, int64_t len, uintptr_t a) {
    if (kWave) {
        const uintptr_t lo = (uintptr_t)t;
        const uintptr_t b = (a - lo > 128 ? a - 128 : lo) & ~(uintptr_t)15;
        if (threadIdx.x < 32) covt_walk_win[threadIdx.x] = window_ld(t, len, b + 16 * threadIdx.x);
        return b;
    }
    const uintptr_t b = a & ~(uintptr_t)15;
    uint4* w = covt_walk_win + threadIdx.x * 4;
    const uint4 v0 = window_ld(t, len, b), v1 = window_ld(t, len, b + 16), v2 = window_ld(t, len, b + 32),
                v3 = window_ld(t, len, b + 48);
    w[0] = v0;
    w[1] = v1;
    w[2] = v2;
    w[3] = v3;
    return b;
}

// bytes [off, off + 8) of an LDS window: three dword reads issued together (one LDS latency; the window
// is readable 4 bytes past off + 8) and two byte-aligns, no branch on the alignment
__device__ __forceinline__ uint64_t win_bytes8(const uint32_t* w, uint32_t off) {
    const uint32_t k = off >> 2, s = off & 3u;
    const uint32_t d0 = w[k], d1 = w[k + 1], d2 = w[k + 2];
    return ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32) | __builtin_amdgcn_alignbyte(d1, d0, s);
}

template <bool kWave>
struct Rd {
    const uint8_t* t;
    int64_t len;   // < 2^31 (walk_tile), so tile offsets compare as 32-bit values below
    int64_t wo;    // the window's start as a tile offset (its address is 16-byte aligned)
    // 8 bytes at tile offset i from a window of the tile kept in LDS (only its base is carried through
    // the walk's loops: a register window of 16 dwords cost ~1,400 64-bit moves per kernel at loop edges).
    // Lane layout: 64 bytes per lane, refilled by that lane.  Wave layout: 512 bytes per wave, refilled by
    // 32 lanes at once (one 16-byte load each) starting 128 bytes before the byte wanted, so the walk's
    // look-backs (a column's name, the geometry column's type-ordered rescans) stay inside the window.
    // Bytes past the tile are unspecified: callers mask by len.
    static constexpr uint32_t kWin = kWave ? 512 : 64;
    __device__ __forceinline__ uint64_t peek8(int32_t i) {
        const uint4* w = covt_walk_win + (kWave ? 0 : threadIdx.x * 4);
        uint32_t off = (uint32_t)i - (uint32_t)wo;  // wraps when i < wo
        if (off > kWin - 8) {
            const uintptr_t b = window_refill<kWave>(t, len, (uintptr_t)(t + i));  // out of line: one copy
            wo = (int64_t)(b - (uintptr_t)t);
            if (kWave) wo = (int64_t)(int32_t)__builtin_amdgcn_readfirstlane((int)(int32_t)wo);
            off = (uint32_t)i - (uint32_t)wo;
        }
        return win_bytes8(reinterpret_cast<const uint32_t*>(w), off);  // (off <= kWin - 8)
    }
    __device__ __forceinline__ int at(int32_t i) { return (int)(peek8(i) & 0xff); }
    // (wave layout) the window holds bytes [i, i + n) (n <= 384); returns i's offset in it
    __device__ __forceinline__ uint32_t ensure(int32_t i, uint32_t n) {
        uint32_t off = (uint32_t)i - (uint32_t)wo;
        if (off > kWin - n) {
            const uintptr_t b = window_refill<kWave>(t, len, (uintptr_t)(t + i));
            wo = (int64_t)(int32_t)__builtin_amdgcn_readfirstlane((int)(int32_t)(int64_t)(b - (uintptr_t)t));
            off = (uint32_t)i - (uint32_t)wo;
        }
        return off;
    }
    // low n bytes (n <= 8) of x's 7-bit groups packed (LEB128 payload)
    __device__ __forceinline__ static uint64_t leb_pack(uint64_t x, int n) {
        x = (n >= 8 ? x : x & ((1ull << (8 * n)) - 1)) & 0x7f7f7f7f7f7f7f7full;
        x = (x & 0x007f007f007f007full) | ((x & 0x7f007f007f007f00ull) >> 1);
        x = (x & 0x00003fff00003fffull) | ((x & 0x3fff00003fff0000ull) >> 2);
        return (x & 0x000000000fffffffull) | ((x & 0x0fffffff00000000ull) >> 4);
    }
    // rd_uv (covt_host.cpp): 64-bit LEB128, at most 10 bytes; up to 8 bytes decoded from one word
    __device__ __forceinline__ bool uv(int32_t& o, uint64_t& v) {
        const int32_t avail = (int32_t)len - (int32_t)o;
        if (avail <= 0) return false;
        const uint64_t w = peek8(o);
        {  // values of up to 4 bytes (nearly all metadata) in 32-bit arithmetic
            const uint32_t w4 = (uint32_t)w;
            uint32_t stop4 = ~w4 & 0x80808080u;
            if (avail < 4) stop4 &= (1u << (8 * avail)) - 1;
            if (stop4) {
                const int n = (__builtin_ctz(stop4) >> 3) + 1;
                uint32_t x = (n >= 4 ? w4 : w4 & ((1u << (8 * n)) - 1)) & 0x7f7f7f7fu;
                x = (x & 0x007f007fu) | ((x & 0x7f007f00u) >> 1);
                v = (x & 0x3fffu) | ((x & 0x3fff0000u) >> 2);
                o += n;
                return true;
            }
        }
        uint64_t stop = ~w & 0x8080808080808080ull;
        if (avail < 8) stop &= (1ull << (8 * avail)) - 1;  // only the tile's bytes
        if (stop) {
            const int n = (__builtin_ctzll(stop) >> 3) + 1;
            v = leb_pack(w, n);
            o += n;
            return true;
        }
        if (avail < 8) return false;  // no terminator before the tile's end
        v = leb_pack(w, 8);           // 9- or 10-byte value
        int32_t q = o + 8;
#pragma unroll 1
        for (int i = 8; i < 10; ++i) {
            if (q >= len) return false;
            const int b = at(q++);
            v |= (uint64_t)(b & 0x7f) << (7 * i);
            if (!(b & 0x80)) {
                o = q;
                return true;
            }
        }
        return false;
    }
    // LEB128 payload of the low n (<= 4) bytes of x
    __device__ __forceinline__ static uint32_t leb_pack4(uint32_t x, int n) {
        x = (n >= 4 ? x : x & ((1u << (8 * n)) - 1)) & 0x7f7f7f7fu;
        x = (x & 0x007f007fu) | ((x & 0x7f007f00u) >> 1);
        return (x & 0x3fffu) | ((x & 0x3fff0000u) >> 2);
    }
    // Gen C stream record tail (numValues, byteLength varints and the encoding byte) from one 64-bit word
    // when both varints have at most 4 bytes and all of it lies in the tile; false (nothing consumed)
    // otherwise, and the caller reads the fields one by one (same values and statuses)
    __device__ __forceinline__ bool rec3(int32_t& o, uint64_t& nv, uint64_t& bl, int& enc) {
        const int32_t avail = (int32_t)len - o;
        if (avail < 3) return false;
        const uint64_t w = peek8(o);
        uint64_t stop = ~w & 0x8080808080808080ull;
        if (avail < 8) stop &= (1ull << (8 * avail)) - 1;
        if (!stop) return false;
        const int e1 = __builtin_ctzll(stop) >> 3;  // numValues' last byte
        if (e1 > 3) return false;
        const uint64_t stop2 = stop & (~0ull << (8 * (e1 + 1)));
        if (!stop2) return false;
        const int e2 = __builtin_ctzll(stop2) >> 3;  // byteLength's last byte
        if (e2 - e1 > 4 || e2 + 1 >= avail || e2 + 1 >= 8) return false;
        nv = leb_pack4((uint32_t)w, e1 + 1);
        bl = leb_pack4((uint32_t)(w >> (8 * (e1 + 1))), e2 - e1);
        enc = (int)((w >> (8 * (e2 + 1))) & 0xff);
        o += e2 + 2;
        return true;
    }
    // rd_j4: DecodingUtils.decodeVarint with its 4-byte cap (DecodingUtils.java:157-186): a byte
    // without bit 7 among the first three ends the value, else the fourth byte does
    __device__ __forceinline__ bool j4(int32_t& o, int32_t& v) {
        const int32_t avail = (int32_t)len - (int32_t)o;
        if (avail <= 0) return false;
        const uint32_t w4 = (uint32_t)peek8(o);
        const uint32_t stop = ~w4 & 0x808080u;
        const int n = stop ? (__builtin_ctz(stop) >> 3) + 1 : 4;
        if (n > avail) return false;
        uint32_t x = (n >= 4 ? w4 : w4 & ((1u << (8 * n)) - 1)) & 0x7f7f7f7fu;
        x = (x & 0x007f007fu) | ((x & 0x7f007f00u) >> 1);
        v = (int32_t)((x & 0x3fffu) | ((x & 0x3fff0000u) >> 2));
        o += n;
        return true;
    }
    // the first 16 bytes of a name at o (n <= 16) packed little-endian (register compares below)
    __device__ __forceinline__ void pack16(int32_t o, uint64_t n, uint64_t& lo, uint64_t& hi) {
        lo = peek8(o);
        if (n < 8) lo &= (1ull << (8 * n)) - 1;
        hi = 0;
        if (n > 8) {
            hi = peek8(o + 8);
            if (n < 16) hi &= (1ull << (8 * (n - 8))) - 1;
        }
    }
    // name at o (n bytes) == the literal (constants evaluated at compile time: a runtime walk of the
    // literal's bytes would be a memory load per character)
#define COVT_IS(o, n, str)                                                                             \
    ([&]() {                                                                                           \
        constexpr uint64_t n_ = cstrlen(str), l_ = pk(str, 0, n_), h_ = pk(str, 8, n_);                \
        static_assert(n_ <= 16, "names up to 16 bytes");                                               \
        if ((uint64_t)(n) != n_) return false;                                                         \
        uint64_t lo_, hi_;                                                                             \
        r.pack16((o), n_, lo_, hi_);                                                                   \
        return lo_ == l_ && hi_ == h_;                                                                 \
    }())
    // genc_stream_type: Gen C stream name -> StreamType (-1: other)
    __device__ __forceinline__ int stream_type(int32_t o, uint64_t n) {
        if (n < 4 || n > 16) return -1;
        uint64_t lo, hi;
        pack16(o, n, lo, hi);
#define COVT_NAME(str, v)                                                              \
    {                                                                                  \
        constexpr uint64_t n_ = cstrlen(str), l_ = pk(str, 0, n_), h_ = pk(str, 8, n_); \
        if (n == n_ && lo == l_ && hi == h_) return v;                                 \
    }
        COVT_NAME("data", ST_DATA)
        COVT_NAME("length", ST_LENGTH)
        COVT_NAME("present", ST_PRESENT)
        COVT_NAME("dictionary", ST_DICTIONARY)
        COVT_NAME("geometry_types", ST_GEOMETRY_TYPES)
        COVT_NAME("geometry_offsets", ST_GEOMETRY_OFFSETS)
        COVT_NAME("part_offsets", ST_PART_OFFSETS)
        COVT_NAME("ring_offsets", ST_RING_OFFSETS)
        COVT_NAME("vertex_offsets", ST_VERTEX_OFFSETS)
        COVT_NAME("vertex_buffer", ST_VERTEX_BUFFER)
#undef COVT_NAME
        return -1;
    }
    // byte_rle_length: bytes of an ORC byte-RLE stream of n values at o (-1: runs past the tile)
    __device__ __forceinline__ int32_t byte_rle_length(int32_t o, int32_t n) {
        int32_t q = o;
        int64_t done = 0;
        while (done < n) {
            if (q >= len) return -1;
            const int c = at(q++);
            if (c < 0x80) done += c + 3, q += 1;
            else done += 0x100 - c, q += 0x100 - c;
            if (q > len) return -1;
        }
        return (int32_t)(q - o);
    }
};

// Gen C container (walk_genc, covt_host.cpp) in one pass over each layer's
// column metadata: the host walk's metadata checks in the same order (same first failing status), data
// offsets relative to the layer's data start (known once its metadata is read: the emitter rebases the
// layer's streams then), and the host's per-column data bound checked once at the end of the layer (the
// data cursor only grows, so the last column's check fires iff any column's does).  Geometry streams
// are laid out in StreamType order (a rescan of that column's few streams).
template <bool kWave, class E>
__device__ __forceinline__ int walk_genc_dev(Rd<kWave>& r, E& emit) {
    const int32_t len = (int32_t)r.len;  // 32-bit cursors (walk_tile: tiles under 2 GiB)
    int32_t o = 0;
    uint64_t version, nlayers;
    if (!r.uv(o, version) || !r.uv(o, nlayers)) return COVT_ERR_TRUNCATED;
    if (version != 1) return COVT_ERR_BAD_HEADER;
    for (uint64_t L = 0; L < nlayers; ++L) {
        uint64_t nlen, extent, nfeat, ncols;
        if (!r.uv(o, nlen) || nlen > (uint64_t)(len - o)) return COVT_ERR_TRUNCATED;
        o += (int32_t)nlen;
        if (!r.uv(o, extent) || !r.uv(o, nfeat) || !r.uv(o, ncols)) return COVT_ERR_TRUNCATED;
        if (ncols > 4096) return COVT_ERR_BAD_HEADER;
        const int nb = nbits_of_extent(extent);
        int64_t d = 0;  // data bytes of the layer's columns so far
        emit.layer_begin();
        for (uint32_t c = 0; c < (uint32_t)ncols; ++c) {
            uint64_t cn, ns, sn, nv, bl;
            if (!r.uv(o, cn) || cn > (uint64_t)(len - o) || (uint64_t)(len - o) - cn < 2) return COVT_ERR_TRUNCATED;
            const int32_t name = o;
            o += (int32_t)cn;
            const int dtype = r.at(o), ctype = r.at(o + 1);
            o += 2;
            if (!r.uv(o, ns)) return COVT_ERR_TRUNCATED;
            if (ns > 256) return COVT_ERR_BAD_HEADER;
            const int kind = COVT_IS(name, cn, "id") ? 0 : (COVT_IS(name, cn, "geometry") || dtype == 6) ? 1 : 2;
            const int32_t s0 = o;
            // wave layout: the geometry column's streams (type, encoding, sizes) go to an LDS table as
            // they are read, and the type-ordered layout below reads the table; the lane layout
            // re-reads the column's metadata once per type instead (each re-read parses the names)
            uint4* geo = covt_walk_win + Rd<kWave>::kWin / 16;
            constexpr bool kTable = kWave;
            uint32_t present = 0;  // geometry stream types seen
            for (uint32_t s = 0; s < (uint32_t)ns; ++s) {
                if (!r.uv(o, sn) || sn > (uint64_t)(len - o)) return COVT_ERR_TRUNCATED;
                const int type = kind == 0 || (kTable && kind == 1) ? r.stream_type(o, sn) : -1;
                o += (int32_t)sn;
                int enc;
                if (!r.rec3(o, nv, bl, enc)) {
                    if (!r.uv(o, nv) || !r.uv(o, bl) || o >= len) return COVT_ERR_TRUNCATED;
                    enc = r.at(o++);
                }
                if (nv > 0x7fffffff || bl > 0x7fffffff) return COVT_ERR_BAD_HEADER;
                if (kind == 0 && type == ST_DATA)
                    emit(RawStream{(int32_t)L, 0, ST_DATA, enc, ctype, (int32_t)nv, (int32_t)bl, nb, d});
                if (kind != 1) d += (int64_t)bl;
                if (kTable && kind == 1) {
                    geo[s] = make_uint4((uint32_t)(type & 0xff) | ((uint32_t)enc << 8), (uint32_t)nv, (uint32_t)bl, 0);
                    if (type >= ST_GEOMETRY_TYPES && type <= ST_VERTEX_BUFFER) present |= 1u << type;
                }
            }
            if (kind == 1 && kTable) {  // types 4..9 in type order (metadata order within a type), then the rest
                for (int want = ST_GEOMETRY_TYPES; want <= ST_VERTEX_BUFFER; ++want) {
                    if (!(present >> want & 1)) continue;
                    for (uint32_t s = 0; s < (uint32_t)ns; ++s) {
                        const uint4 g = geo[s];
                        if ((int)(g.x & 0xff) != want) continue;
                        emit(RawStream{(int32_t)L, 1, want, (int)(g.x >> 8), ctype, (int32_t)g.y, (int32_t)g.z, nb, d});
                        d += (int64_t)g.z;
                    }
                }
                for (uint32_t s = 0; s < (uint32_t)ns; ++s) {
                    const uint4 g = geo[s];
                    const int type = (int)(int8_t)(g.x & 0xff);
                    if (type < ST_GEOMETRY_TYPES || type > ST_VERTEX_BUFFER) d += (int64_t)g.z;
                }
            } else if (kind == 1) {  // streams of types 4..9 in type order, then the rest (all checked above)
                for (int want = ST_GEOMETRY_TYPES; want <= ST_VERTEX_BUFFER + 1; ++want) {
                    int32_t q = s0;
                    for (uint32_t s = 0; s < (uint32_t)ns; ++s) {
                        r.uv(q, sn);
                        const int type = r.stream_type(q, sn);
                        q += (int32_t)sn;
                        r.uv(q, nv);
                        r.uv(q, bl);
                        const int enc = r.at(q++);
                        const bool isgeo = type >= ST_GEOMETRY_TYPES && type <= ST_VERTEX_BUFFER;
                        if (want <= ST_VERTEX_BUFFER ? type != want : isgeo) continue;
                        if (isgeo) emit(RawStream{(int32_t)L, 1, type, enc, ctype, (int32_t)nv, (int32_t)bl, nb, d});
                        d += (int64_t)bl;
                    }
                }
            }
        }
        if (d > (int64_t)(len - o)) return COVT_ERR_TRUNCATED;
        emit.layer_end(o);  // the layer's data starts where its metadata ends
        o += (int32_t)d;
    }
    return o == len ? COVT_OK : COVT_ERR_BAD_HEADER;
}

// Gen D container (walk_gend, covt_host.cpp; CovtParser.decodeLayerMetadata, CovtParser.java:574-652).
// A column's streams follow TreeMap<StreamType> order, the last metadata entry of a type winning.
template <bool kWave, class E>
__device__ __forceinline__ int walk_gend_dev(Rd<kWave>& r, E& emit) {
    const int32_t len = (int32_t)r.len;  // 32-bit cursors (walk_tile: tiles under 2 GiB)
    int32_t o = 0;
    int32_t layer = 0;
    while (o < len) {
        const bool optimized = r.at(o++) & 1;
        int32_t v, extent, nfeat, ncols;
        if (!r.j4(o, v)) return COVT_ERR_TRUNCATED;
        if (!optimized) {
            if (v < 0 || v > len - o) return COVT_ERR_TRUNCATED;
            o += v;
        }
        if (!r.j4(o, extent) || !r.j4(o, nfeat) || !r.j4(o, ncols)) return COVT_ERR_TRUNCATED;
        if (ncols < 0 || ncols > 4096) return COVT_ERR_BAD_HEADER;
        const int32_t meta = o;
        for (int32_t ci = 0; ci < ncols; ++ci) {  // metadata checks
            int32_t x;
            if (optimized || ci == 0) {
                if (!r.j4(o, x)) return COVT_ERR_TRUNCATED;
            } else {
                if (!r.j4(o, x) || x < 0 || x > len - o) return COVT_ERR_TRUNCATED;
                o += x;
            }
            if (o >= len) return COVT_ERR_TRUNCATED;
            const int desc = r.at(o++), dtype = (desc >> 3) & 0xF, ctype = desc & 0x7;
            if (ctype > 4) return COVT_ERR_BAD_HEADER;
            for (;;) {
                if (o >= len) return COVT_ERR_TRUNCATED;
                const int sd = r.at(o++), type = sd >> 4, enc = sd & 0xF;
                if (type > ST_M || enc > 9) return COVT_ERR_BAD_HEADER;
                int32_t nv, bl;
                if (!r.j4(o, nv) || !r.j4(o, bl)) return COVT_ERR_TRUNCATED;
                if ((dtype == 8 && type == ST_VERTEX_BUFFER) || (type == ST_DATA && ctype == CT_PLAIN) ||
                    type == ST_DICTIONARY)
                    break;
            }
        }
        const int nb = nbits_of_extent((uint32_t)extent);
        int32_t m = meta;
        int64_t d = o;  // data cursor (64-bit: a column's streams may sum past 2^31 before its bound check)
        emit.layer_begin();
        for (int32_t ci = 0; ci < ncols; ++ci) {
            int32_t x, kind;
            if (optimized || ci == 0) {
                r.j4(m, x);
                kind = x == 0 ? 0 : (x == 1 ? 1 : 2);
            } else {
                r.j4(m, x);
                kind = COVT_IS(m, x, "id") ? 0 : COVT_IS(m, x, "geometry") ? 1 : 2;
                m += x;
            }
            const int desc = r.at(m++), dtype = (desc >> 3) & 0xF, ctype = desc & 0x7;
            const int32_t s0 = m;
            uint32_t have = 0;  // stream types present
            for (;;) {
                const int sd = r.at(m++), type = sd >> 4;
                int32_t nv, bl;
                r.j4(m, nv);
                r.j4(m, bl);
                have |= 1u << type;
                if ((dtype == 8 && type == ST_VERTEX_BUFFER) || (type == ST_DATA && ctype == CT_PLAIN) ||
                    type == ST_DICTIONARY)
                    break;
            }
            if (kind == 2 && dtype != 0) {  // implicit present stream (walk_gend)
                const int32_t pl = r.byte_rle_length((int32_t)d, nfeat < 0 ? 0 : (int32_t)(((int64_t)nfeat + 7) / 8));
                if (pl < 0) return COVT_ERR_TRUNCATED;
                d += pl;
            }
            for (int type = 0; type < 12; ++type) {
                if (!(have >> type & 1) || (kind == 2 && type == ST_PRESENT)) continue;
                int enc = 0;
                int32_t nv = 0, bl = 0;
                for (int32_t q = s0; q < m;) {  // the last entry of this type
                    const int sd = r.at(q++);
                    int32_t a, b;
                    r.j4(q, a);
                    r.j4(q, b);
                    if ((sd >> 4) == type) enc = sd & 0xF, nv = a, bl = b;
                }
                const bool hot = (kind == 0 && type == ST_DATA) ||
                                 (kind == 1 && type >= ST_GEOMETRY_TYPES && type <= ST_VERTEX_BUFFER);
                if (hot) emit(RawStream{layer, kind, type, enc, ctype, nv, bl, nb, d});
                if (bl < 0) return COVT_ERR_BAD_HEADER;
                d += bl;
            }
            if (d > len) return COVT_ERR_TRUNCATED;
        }
        emit.layer_end(0);
        o = (int32_t)d;
        ++layer;
    }
    return COVT_OK;
}

__device__ inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

// a stream's launch key (launch_key, covt_internal.h) as its entry is written; lm: the batch's lane limits
// (lane_limits, or -1 when the batch has fewer lane streams than lane_min: totals[T_LANE] is known before
// the entries are written -- walk_count counts them)
__device__ __forceinline__ uint32_t entry_key(int32_t op, int32_t nv, int32_t bl, int64_t out_elems, int32_t elem,
                                              int32_t lm) {
    const bool lane = lane_stream(op, nv, bl, lm);
    const uint32_t fam = lane ? (uint32_t)COVT_FAMILY_LANE : (uint32_t)covt_op_family(op);
    return launch_key(fam, lane, op, (int64_t)bl + out_elems * elem / 4);
}

// ---- speculative Gen C walk (one wave per tile) -------------------------------------------------------
// The serial walk spends ~90 scalar instructions per metadata varint (~75k per tile: 2.2 ms for the 10k-
// tile bench batch, profiles/r02).  Most of a Gen C tile's metadata is a chain of records of two shapes:
// column headers (name, dataType, columnType, numStreams) and stream records (name, numValues, byteLength,
// encoding).  So the wave stages kFwSpan bytes of metadata (+ 256 bytes of look-ahead) in LDS and every lane
// parses, at each position (256 at a time, as the walk reaches them), the record that WOULD start there -- a stream record's length and
// byteLength, a column header's length, stream count, kind (id / geometry / other) and columnType -- into
// two tables; the walk then follows the chain one LDS read per record and parses fields only for the
// Id / Geometry streams it emits.  Anything outside the fast grammar (a name or varint longer than the
// tables hold, a record past the tile, a check the serial walk would fail) makes the tile fall back to the
// serial walk (walk_genc_dev), which then gives the exact statuses; a successful fast walk emits the same
// records in the same order.
#ifndef COVT_FW_SPAN
#define COVT_FW_SPAN 512
#endif
constexpr int kFwSpan = COVT_FW_SPAN;  // table positions per window (a multiple of 256)
constexpr int kFwBytes = kFwSpan + 256;  // window bytes: the positions + 256 bytes of look-ahead
constexpr int kFwGeo = 32;  // geometry streams per column the fast walk holds (more: the serial walk)
constexpr int kFastFallback = 1;
struct FastSmem {
    uint32_t win[kFwBytes / 4 + 4];
    uint32_t stab[kFwSpan];  // stream record at j: length | byteLength << 8 (0: not fast)
    uint32_t ctab[kFwSpan];  // column header at j: length | numStreams << 8 | kind << 17 | columnType << 19 |
                             // min(dataType, 31) << 27 (0: not fast)
};
// the property walk's extra tables (after FastSmem; the Id walk neither builds nor allocates them)
struct FastSmemRec {
    uint32_t rtab[kFwSpan];  // stream record at j: numValues | (StreamType of its name + 1) << 28
    uint8_t etab[kFwSpan];   // its encoding
};
// LDS: Rd<true>'s 512-byte window, then the geometry table (kFwGeo entries for the fast walk, 256 for the
// serial one, which overlaps the fast walk's tables: it only runs once they are abandoned).  Small
// enough for ~6 waves per SIMD: the walk is a latency-bound chain, so resident tiles set its rate.
constexpr size_t kFastSmemOffset = 512 + kFwGeo * 16;
constexpr size_t kWalkLds = kFastSmemOffset + sizeof(FastSmem) > 512 + 256 * 16 ? kFastSmemOffset + sizeof(FastSmem)
                                                                                  : 512 + 256 * 16;

// StreamType of a stream name of n bytes (lo: bytes 0-7, hi: 8-15, masked to n; -1: none)
__device__ __forceinline__ int fast_name_type(uint32_t n, uint64_t lo, uint64_t hi) {
    int type = -1;
    if (n >= 4 && n <= 16) {
#define COVT_FNAME(str, v)                                                              \
    {                                                                                   \
        constexpr uint64_t n_ = cstrlen(str), l_ = pk(str, 0, n_), h_ = pk(str, 8, n_); \
        if (n == n_ && lo == l_ && hi == h_) type = v;                                  \
    }
        COVT_FNAME("data", ST_DATA)
        COVT_FNAME("length", ST_LENGTH)
        COVT_FNAME("present", ST_PRESENT)
        COVT_FNAME("dictionary", ST_DICTIONARY)
        COVT_FNAME("geometry_types", ST_GEOMETRY_TYPES)
        COVT_FNAME("geometry_offsets", ST_GEOMETRY_OFFSETS)
        COVT_FNAME("part_offsets", ST_PART_OFFSETS)
        COVT_FNAME("ring_offsets", ST_RING_OFFSETS)
        COVT_FNAME("vertex_offsets", ST_VERTEX_OFFSETS)
        COVT_FNAME("vertex_buffer", ST_VERTEX_BUFFER)
#undef COVT_FNAME
    }
    return type;
}

// The same for a uniform name (the walk's scalar path): the candidate picked by length (and by the first
// byte where two names share one), then one compare.  The ten compare chains above cost the scalar unit
// ~60 instructions per Id / Geometry record, and the walk is bound by scalar issue.
__device__ __forceinline__ int fast_name_type_u(uint32_t n, uint64_t lo, uint64_t hi) {
    const uint32_t c0 = (uint32_t)lo & 0xffu;
    int t = -1;
    uint64_t el = 0, eh = 0;
#define COVT_FNAME_U(str, v)                                                      \
    {                                                                             \
        constexpr uint64_t n_ = cstrlen(str), l_ = pk(str, 0, n_), h_ = pk(str, 8, n_); \
        t = v;                                                                    \
        el = l_;                                                                  \
        eh = h_;                                                                  \
    }
    switch (n) {
    case 4: COVT_FNAME_U("data", ST_DATA) break;
    case 6: COVT_FNAME_U("length", ST_LENGTH) break;
    case 7: COVT_FNAME_U("present", ST_PRESENT) break;
    case 10: COVT_FNAME_U("dictionary", ST_DICTIONARY) break;
    case 12:
        if (c0 == 'p') COVT_FNAME_U("part_offsets", ST_PART_OFFSETS)
        else COVT_FNAME_U("ring_offsets", ST_RING_OFFSETS)
        break;
    case 13: COVT_FNAME_U("vertex_buffer", ST_VERTEX_BUFFER) break;
    case 14:
        if (c0 == 'g') COVT_FNAME_U("geometry_types", ST_GEOMETRY_TYPES)
        else COVT_FNAME_U("vertex_offsets", ST_VERTEX_OFFSETS)
        break;
    case 16: COVT_FNAME_U("geometry_offsets", ST_GEOMETRY_OFFSETS) break;
    default: return -1;
    }
#undef COVT_FNAME_U
    return lo == el && hi == eh ? t : -1;
}

struct FastGenc {
    const uint8_t* t;
    int32_t len;
    int32_t wb;  // tile offset of window byte 0 (16-byte aligned address; may be < 0 at the tile start)
    uint32_t segs;  // window positions [256 k, 256 k + 256) whose record tables are built: bit k
    uint32_t lim;   // window positions [0, lim) all have their tables built
    FastSmem* fs;
    FastSmemRec* fr = nullptr;  // the property walk's tables (null: not built)
    // bytes [q, q + 8) of the window, q per lane (q <= kFwBytes - 8)
    __device__ __forceinline__ uint64_t peek8(int32_t q) const {
        const uint32_t* w = fs->win;
        const int32_t k = q >> 2;
        const uint32_t s = (uint32_t)q & 3u;
        const uint32_t d0 = w[k], d1 = w[k + 1], d2 = w[k + 2];
        return ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32) | __builtin_amdgcn_alignbyte(d1, d0, s);
    }
    __device__ __forceinline__ uint64_t upeek8(int32_t q) const {  // uniform q
        const uint64_t v = peek8(q);
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
               (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    }
    // the window holding tile offset `at` (its record tables are built on demand, 256 positions at a time:
    // a layer's metadata is often a few hundred bytes)
    __device__ void load(int32_t at) {
        const int l = threadIdx.x;
        const uintptr_t lo = (uintptr_t)t;
        const uintptr_t b = (lo + (uintptr_t)(int64_t)at) & ~(uintptr_t)15;
        wb = (int32_t)(int64_t)(b - lo);
        wb = __builtin_amdgcn_readfirstlane(wb);
        segs = 0;
        lim = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
        for (int i = 0; i < kFwBytes / 16; i += 64)
            if (i + 64 <= kFwBytes / 16 || i + l < kFwBytes / 16)
                ((uint4*)fs->win)[i + l] = window_ld(t, len, b + 16 * (uintptr_t)(i + l));
        if (l == 0) ((uint4*)fs->win)[kFwBytes / 16] = make_uint4(0, 0, 0, 0);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    // the record tables of window positions [256 sg, 256 sg + 256)
    __device__ void build(int sg) {
        const int l = threadIdx.x;
        constexpr uint64_t kId = pk("id", 0, 2), kGeo = pk("geometry", 0, 8);
#pragma unroll 1
        for (int i = 0; i < 4; ++i) {
            const int32_t q = 256 * sg + l + 64 * i, j = wb + q;
            uint32_t se = 0, ce = 0, re = 0;
            uint8_t ee = 0;
            const uint64_t nm = peek8(q + 1);              // name bytes (a stream / column name)
            const uint32_t n = fs->win[q >> 2] >> (8 * (q & 3)) & 0xffu;  // its length (one LEB128 byte)
            if (j >= 0 && n < 0x80u) {
                const int32_t p = q + 1 + (int32_t)n;
                const uint64_t w = peek8(p);
                // stream record: numValues (<= 4 bytes), byteLength (<= 4 bytes, < 2^24), encoding
                const uint64_t stop = ~w & 0x8080808080808080ull;
                const int e1 = stop ? __builtin_ctzll(stop) >> 3 : 8;
                const uint64_t stop2 = e1 < 7 ? stop & (~0ull << (8 * (e1 + 1))) : 0ull;
                const int e2 = stop2 ? __builtin_ctzll(stop2) >> 3 : 8;
                if (e1 <= 3 && e2 - e1 <= 4 && e2 <= 6) {
                    uint32_t x = (uint32_t)(w >> (8 * (e1 + 1)));
                    const int nb = e2 - e1;
                    x = (nb >= 4 ? x : x & ((1u << (8 * nb)) - 1u)) & 0x7f7f7f7fu;
                    x = (x & 0x007f007fu) | ((x & 0x7f007f00u) >> 1);
                    const uint32_t bl = (x & 0x3fffu) | ((x & 0x3fff0000u) >> 2);
                    const int32_t slen = 1 + (int32_t)n + e2 + 2;
                    if (bl < (1u << 24) && j + slen <= len) se = (uint32_t)slen | (bl << 8);
                    if (fr && se) {  // the property walk's fields: name's StreamType, numValues, encoding
                        uint32_t v = (uint32_t)w;
                        v = (e1 >= 3 ? v : v & ((1u << (8 * (e1 + 1))) - 1u)) & 0x7f7f7f7fu;
                        v = (v & 0x007f007fu) | ((v & 0x7f007f00u) >> 1);
                        const uint32_t nv = (v & 0x3fffu) | ((v & 0x3fff0000u) >> 2);
                        const uint64_t lo = n >= 8 ? nm : nm & ((1ull << (8 * n)) - 1);
                        uint64_t hi = 0;
                        if (n > 8) {
                            hi = peek8(q + 9);
                            if (n < 16) hi &= (1ull << (8 * (n - 8))) - 1;
                        }
                        re = nv | ((uint32_t)(fast_name_type(n, lo, hi) + 1) << 28);
                        ee = (uint8_t)(w >> (8 * (e2 + 1)));
                    }
                }
                // column header: dataType, columnType, numStreams (1-2 byte LEB128, <= 256)
                const uint32_t b2 = (uint32_t)(w >> 16) & 0xffu, b3 = (uint32_t)(w >> 24) & 0xffu;
                const uint32_t ns = b2 < 0x80u ? b2 : ((b2 & 0x7fu) | (b3 << 7));
                const int32_t nsb = b2 < 0x80u ? 1 : (b3 < 0x80u ? 2 : 0);
                const int32_t clen = 1 + (int32_t)n + 2 + nsb;
                if (nsb && ns <= 256u && j + clen <= len) {
                    const uint32_t dtype = (uint32_t)w & 0xffu, ctype = (uint32_t)(w >> 8) & 0xffu;
                    const bool id = n == 2 && (nm & 0xffffull) == kId;
                    const bool geo = (n == 8 && nm == kGeo) || dtype == 6;
                    const uint32_t kind = id ? 0u : geo ? 1u : 2u;
                    ce = (uint32_t)clen | (ns << 8) | (kind << 17) | (ctype << 19) | ((dtype < 31u ? dtype : 31u) << 27);
                }
            }
            fs->stab[q] = se;
            fs->ctab[q] = ce;
            if (fr) {
                fr->rtab[q] = re;
                fr->etab[q] = ee;
            }
        }
        segs |= 1u << sg;
        lim = (segs & 1u) ? ((kFwSpan > 256 && (segs & 2u)) ? 512u : 256u) : 0u;
        static_assert(kFwSpan == 512 || kFwSpan == 256, "lim: one or two table segments");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    __device__ __forceinline__ int32_t at(int32_t o) {  // the window offset of tile offset o (loads, builds)
        if ((uint32_t)(o - wb) >= (uint32_t)kFwSpan) load(o);
        const int32_t q = o - wb;
        if (!((segs >> (q >> 8)) & 1u)) build(q >> 8);
        return q;
    }
    // the same with one compare when the tables already cover o (the Id walk's property-record loop, whose
    // scalar instructions bound the walk)
    __device__ __forceinline__ int32_t at_run(int32_t o) {
        const int32_t q = o - wb;
        if ((uint32_t)q < lim) return q;
        return at(o);
    }
    // window offset of tile offset o for plain byte reads (no tables needed)
    __device__ __forceinline__ int32_t at_bytes(int32_t o) {
        if ((uint32_t)(o - wb) >= (uint32_t)kFwSpan) load(o);
        return o - wb;
    }
    // a uniform LEB128 value of at most 4 bytes at o (false: longer, or past the tile)
    __device__ __forceinline__ bool uv4(int32_t& o, uint32_t& v) {
        if (o >= len) return false;
        const int32_t q = at_bytes(o);
        const uint32_t w = (uint32_t)upeek8(q);
        const uint32_t stop = ~w & 0x80808080u;
        if (!stop) return false;
        const int nb = (__builtin_ctz(stop) >> 3) + 1;
        if (o + nb > len) return false;
        uint32_t x = (nb >= 4 ? w : w & ((1u << (8 * nb)) - 1u)) & 0x7f7f7f7fu;
        x = (x & 0x007f007fu) | ((x & 0x7f007f00u) >> 1);
        v = (x & 0x3fffu) | ((x & 0x3fff0000u) >> 2);
        o += nb;
        return true;
    }
    // a fast stream record at o (its table entry se != 0): StreamType of its name, numValues, encoding
    __device__ __forceinline__ void rec(int32_t q, uint32_t se, int& type, int32_t& nv, int& enc) {
        const uint64_t w0 = upeek8(q);
        const uint32_t n = (uint32_t)w0 & 0xffu;
        uint64_t lo = upeek8(q + 1), hi = 0;
        if (n < 8) lo &= (1ull << (8 * n)) - 1;
        if (n > 8) {
            hi = upeek8(q + 9);
            if (n < 16) hi &= (1ull << (8 * (n - 8))) - 1;
        }
        type = fast_name_type_u(n, lo, hi);
        const uint64_t w = upeek8(q + 1 + (int32_t)n);
        const uint64_t stop = ~w & 0x8080808080808080ull;  // (the table checked: numValues <= 4 bytes)
        const int e1 = __builtin_ctzll(stop) >> 3;
        uint32_t x = (uint32_t)w;
        x = (e1 >= 3 ? x : x & ((1u << (8 * (e1 + 1))) - 1u)) & 0x7f7f7f7fu;
        x = (x & 0x007f007fu) | ((x & 0x7f007f00u) >> 1);
        nv = (int32_t)((x & 0x3fffu) | ((x & 0x3fff0000u) >> 2));
        enc = (int)((w >> (8 * ((se & 0xffu) - 2 - n))) & 0xffu);  // the record's last byte
    }
};

// The fast walk of one Gen C tile (walk_genc_dev's grammar and emission order); kFastFallback when the
// tile leaves the fast grammar (the caller then runs walk_genc_dev from scratch with a fresh emitter).
template <class E>
__device__ int walk_genc_fast(FastGenc& f, E& emit) {
    const int32_t len = f.len;
    int32_t o = 0;
    uint32_t version, nlayers;
    if (!f.uv4(o, version) || !f.uv4(o, nlayers) || version != 1) return kFastFallback;
    uint4* geo = covt_walk_win + Rd<true>::kWin / 16;  // the geometry column's streams (as walk_genc_dev)
    for (uint32_t L = 0; L < nlayers; ++L) {
        uint32_t nlen, extent, nfeat, ncols;
        if (!f.uv4(o, nlen) || nlen > (uint32_t)(len - o)) return kFastFallback;
        o += (int32_t)nlen;
        if (!f.uv4(o, extent) || !f.uv4(o, nfeat) || !f.uv4(o, ncols) || ncols > 4096) return kFastFallback;
        const int nb = nbits_of_extent(extent);
        int64_t d = 0;
        emit.layer_begin();
        for (uint32_t c = 0; c < ncols; ++c) {
            const uint32_t ce = (uint32_t)__builtin_amdgcn_readfirstlane((int)f.fs->ctab[f.at_run(o)]);
            if (!ce) return kFastFallback;
            const uint32_t ns = (ce >> 8) & 0x1ffu, kind = (ce >> 17) & 3u;
            const int ctype = (int)(ce >> 19) & 0xff;
            if (kind == 1 && ns > (uint32_t)kFwGeo) return kFastFallback;
            o += (int32_t)(ce & 0xffu);
            if (kind == 2) {  // a property column (most records): only its data bytes, in a loop of its own
                // (a position with no fast record there (entry 0) is remembered in `miss` -- one scalar OR
                // per record -- and the walk falls back after the column; meanwhile it steps 255 bytes and
                // counts 2^24 - 1 data bytes, and emits nothing.  32-bit sums: < 2^9 * 2^24 per column)
                // (the window offset carried instead of the tile offset, a count-down loop: fewer scalar
                // instructions per record, the walk's bound)
                uint32_t dd = 0, miss = 0;
                int32_t q = o - f.wb;
                for (uint32_t left = ns; left != 0; --left) {
                    if ((uint32_t)q >= f.lim) q = f.at(q + f.wb);  // (a window reload moves wb)
                    uint32_t se = (uint32_t)__builtin_amdgcn_readfirstlane((int)f.fs->stab[q]);
                    miss |= se == 0u;
                    se = se ? se : 0xffffffffu;
                    dd += se >> 8;
                    q += (int32_t)(se & 0xffu);
                }
                if (miss) return kFastFallback;  // (a tile over 16 MiB could otherwise pass the overrun check)
                o = q + f.wb;
                d += dd;
                continue;
            }
            uint32_t present = 0;
            for (uint32_t s = 0; s < ns; ++s) {
                const int32_t q = f.at(o);
                const uint32_t se = (uint32_t)__builtin_amdgcn_readfirstlane((int)f.fs->stab[q]);
                if (!se) return kFastFallback;
                const int32_t bl = (int32_t)(se >> 8);
                if (kind != 2) {
                    int type, enc;
                    int32_t nv;
                    f.rec(q, se, type, nv, enc);
                    if (kind == 0) {
                        if (type == ST_DATA) emit(RawStream{(int32_t)L, 0, ST_DATA, enc, ctype, nv, bl, nb, d});
                    } else {
                        if (threadIdx.x == 0) geo[s] = make_uint4((uint32_t)(type & 0xff) | ((uint32_t)enc << 8), (uint32_t)nv, (uint32_t)bl, 0);
                        if (type >= ST_GEOMETRY_TYPES && type <= ST_VERTEX_BUFFER) present |= 1u << type;
                    }
                }
                if (kind != 1) d += bl;
                o += (int32_t)(se & 0xffu);
            }
            if (kind == 1) {  // types 4..9 in type order (metadata order within a type), then the rest
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                // stream s in lane s (ns <= kFwGeo <= 64); each type's streams by one ballot, emitted in
                // lane order (a scan of the table per type cost six dependent LDS reads per stream)
                const uint32_t ls = threadIdx.x;
                const uint4 g = ls < ns ? geo[ls] : make_uint4(0xffu, 0u, 0u, 0u);
                const uint32_t gt = g.x & 0xffu;
                for (int want = ST_GEOMETRY_TYPES; want <= ST_VERTEX_BUFFER; ++want) {
                    if (!(present >> want & 1)) continue;
                    uint64_t m = __ballot(ls < ns && gt == (uint32_t)want);
                    while (m) {
                        const int sl = __builtin_ctzll(m);
                        m &= m - 1;
                        const uint32_t gx = (uint32_t)__builtin_amdgcn_readlane((int)g.x, sl);
                        const int32_t gy = __builtin_amdgcn_readlane((int)g.y, sl);
                        const int32_t gz = __builtin_amdgcn_readlane((int)g.z, sl);
                        emit(RawStream{(int32_t)L, 1, want, (int)(gx >> 8), ctype, gy, gz, nb, d});
                        d += (int64_t)gz;
                    }
                }
                uint64_t mo = __ballot(ls < ns && (gt < (uint32_t)ST_GEOMETRY_TYPES || gt > (uint32_t)ST_VERTEX_BUFFER));
                while (mo) {  // the rest: only their data bytes
                    const int sl = __builtin_ctzll(mo);
                    mo &= mo - 1;
                    d += (int64_t)__builtin_amdgcn_readlane((int)g.z, sl);
                }
            }
        }
        if (d > (int64_t)(len - o)) return kFastFallback;
        emit.layer_end(o);
        o += (int32_t)d;
    }
    return o == len ? COVT_OK : kFastFallback;
}

template <bool kWave, class E>
__device__ __forceinline__ int walk_tile(const uint8_t* bytes, uint64_t n_bytes, uint64_t off, uint64_t size, int32_t format, E& emit) {
    if (off > n_bytes || size > n_bytes - off) return COVT_ERR_INVALID_ARG;
    if (size > 0x7ff00000ull) return COVT_ERR_INVALID_ARG;  // device plan limit: tiles under 2 GiB
    Rd<kWave> r;
    r.t = bytes + off;
    r.len = (int64_t)size;
    r.wo = -(int64_t)0x40000000;  // no window yet (every offset misses it)
    if (kWave && format == COVT_FORMAT_GENC) {  // the speculative walk first; the serial one on a fallback
        FastGenc f;
        f.t = r.t;
        f.len = (int32_t)size;
        f.wb = -(int32_t)0x40000000;
        f.segs = 0;
        f.lim = 0;
        f.fs = (FastSmem*)((uint8_t*)covt_walk_win + kFastSmemOffset);
        const E fresh = emit;
        const int st = walk_genc_fast(f, emit);
        if (st != kFastFallback) return st;
        emit = fresh;
    }
    return format == COVT_FORMAT_GENC ? walk_genc_dev(r, emit) : walk_gend_dev(r, emit);
}

// the walks' tile order in a property plan: largest first (the batch's few 442 KB tiles were the property
// walk's tail when they started late: 10k-tile plan 3.16-3.21 -> 2.95-2.99 ms; an Id / Geometry plan
// gains nothing from it and would pay the sort, ~0.04 ms)
__global__ void tile_iota(uint32_t* __restrict__ v, int32_t n) {
    const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) v[i] = (uint32_t)i;
}

// Records a tile's walk leaves for emit_slots: up to kSlots per tile (the fixture library's busiest
// tile has 67 Id / Geometry streams); a tile with more is walked again by walk_emit
constexpr int kSlots = 128;
#ifndef COVT_DEFER_SUMS
#define COVT_DEFER_SUMS 1
#endif
#ifndef COVT_PLAN_SPEC
#define COVT_PLAN_SPEC 1
#endif
// a plan is built without the mid-plan synchronisation when its tiles at this many streams each would exceed
// the split bound (split_max_streams): such a plan splits nothing, so the guess is rarely wrong
constexpr int64_t kSpecStreamsPerTile = 32;
// ... and its stream arena is sized to this many streams per tile (the bench batch averages 43, the fixture
// library's busiest tile has 67): a batch averaging more is redone with its counted size (a third sync)
constexpr int64_t kSpecCapPerTile = 64;

struct CountEmit {
    int32_t id_mode;
    RawStream* slots = nullptr;  // this tile's kSlots record slots, or null
    bool writer = true, wave = false;
    int64_t n = 0, out = 0, k0 = 0;
    int64_t fpf_w = 1, cost = 0, cmax = 0;  // the split rule's cost: sum, and the largest split cost
    // a wave walk with slots: a slotted record is only written here, its op, output bytes and costs are
    // summed by the whole wave after the walk (slot_sums): 17.0k -> 15.3k scalar instructions per tile of the
    // bench batch (the walk is bound by scalar issue; plan 0.64 -> 0.63 ms, paired)
    bool defer = false;

    __device__ void operator()(const RawStream& s) {
        if (defer && n < kSlots) {
            if (writer) slots[n] = s;
            ++n;
            return;
        }
        int op, elem;
        int64_t nvals, oe;
        choose_op(s, id_mode, op, nvals, elem, oe);
        if (slots && writer && n < kSlots) slots[n] = s;
        ++n;
        const int64_t ob = (op == COVT_OP_NONE ? 0 : oe) * elem;
        out = align_out(out + ob);
        const int64_t c = (int64_t)s.bl + ob / 4;  // covt_plan_create's stream_cost
        cost += c;
        const int64_t sc = split_fpf_op(op) ? c + (fpf_w - 1) * (ob / 4) : c;
        cmax = sc > cmax ? sc : cmax;
    }
    // the slotted records' sums (defer), one lane per record: output bytes (each stream's slice aligned, so
    // the walk's running align_out sum is the sum of the aligned sizes), split cost sum and maximum
    __device__ void slot_sums() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        const int64_t m = n < kSlots ? n : kSlots;
        int64_t so = 0, sc = 0, sm = 0;
        for (int64_t j = threadIdx.x; j < m; j += 64) {
            int op, elem;
            int64_t nvals, oe;
            const RawStream r = slots[j];
            choose_op(r, id_mode, op, nvals, elem, oe);
            const int64_t ob = (op == COVT_OP_NONE ? 0 : oe) * elem;
            so += align_out(ob);
            const int64_t c = (int64_t)r.bl + ob / 4;
            sc += c;
            const int64_t x = split_fpf_op(op) ? c + (fpf_w - 1) * (ob / 4) : c;
            sm = x > sm ? x : sm;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            so += __shfl_xor(so, d, 64);
            sc += __shfl_xor(sc, d, 64);
            const int64_t x = __shfl_xor(sm, d, 64);
            sm = x > sm ? x : sm;
        }
        out += so;
        cost += sc;
        cmax = sm > cmax ? sm : cmax;
    }
    __device__ void layer_begin() { k0 = n; }
    __device__ void layer_end(int64_t data_start) {  // rebase the layer's recorded data offsets
        if (!data_start || !slots) return;
        const int64_t e = n < kSlots ? n : kSlots;
        if (wave) {  // one lane per record (lane 0 wrote them)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            for (int64_t j = k0 + threadIdx.x; j < e; j += 64) slots[j].off += data_start;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        } else {
            for (int64_t j = k0; j < e; ++j) slots[j].off += data_start;
        }
    }
};

// Walk kernels in two layouts (covt_plan_options.device_walk):
//  * 0 (default): a wave per tile, its lanes in lockstep on values the compiler proves uniform (the
//    walk compiles to scalar code, 32-54 VGPRs), a 512-byte LDS window refilled by 32 lanes at once,
//    lane 0 writing the records and all lanes rebasing a layer's offsets;
//  * k >= 2: k lanes per workgroup, a lane per tile with a 64-byte window (lanes diverge, so k = 1 is
//    best: 1 / 2 / 4 / 16 lanes measured 7.9 / 8.6 / 8.1 / 11.9 ms for the whole plan).
// Both take ~0.7 ms for one tile alone and ~3.6 ms per walk kernel for the 10k-tile batch
// (profiles/r02/device_plan_ab.txt); the walk is a serial chain per tile whose step time neither the
// scalar nor the lane layout changes.
#ifdef COVT_PLAN_TIMING  // profiling build (tools/walk_timeline.py): each tile's walk (start, end), 100 MHz ticks
__device__ uint64_t* covt_walk_clock;
#endif
template <bool kWave>
__global__ void walk_count(const uint8_t* __restrict__ bytes, uint64_t n_bytes, const uint64_t* __restrict__ offs,
                           const uint64_t* __restrict__ sizes, int32_t n_tiles, int32_t format, int32_t id_mode,
                           int32_t* __restrict__ status, int64_t* __restrict__ cnt, int64_t* __restrict__ ob,
                           RawStream* __restrict__ slots, int64_t fpf_w, int64_t* __restrict__ tcost,
                           const uint32_t* __restrict__ order) {
    int32_t t = kWave ? (int32_t)blockIdx.x : (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t > n_tiles) return;
    if (order && t < n_tiles) t = (int32_t)order[t];  // (largest tiles first)
    if (t == n_tiles) {  // the prefix sums' total slot
        if (!kWave || threadIdx.x == 0) cnt[t] = 0, ob[t] = 0;
        return;
    }
    CountEmit e{id_mode};
    e.slots = slots ? slots + (size_t)t * kSlots : nullptr;
    e.writer = !kWave || threadIdx.x == 0;
    e.wave = kWave;
    e.fpf_w = fpf_w;
    e.defer = kWave && COVT_DEFER_SUMS && e.slots;
#ifdef COVT_PLAN_TIMING
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const int st = walk_tile<kWave>(bytes, n_bytes, offs[t], sizes[t], format, e);
    if (kWave && e.defer && st == COVT_OK) e.slot_sums();
#ifdef COVT_PLAN_TIMING
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    if (kWave && threadIdx.x == 0 && covt_walk_clock) {
        covt_walk_clock[2 * (size_t)t] = t_start;
        covt_walk_clock[2 * (size_t)t + 1] = t_end;
    }
#endif
    if (!kWave || threadIdx.x == 0) {
        status[t] = st;
        cnt[t] = st ? 0 : e.n;  // a failed tile contributes nothing
        ob[t] = st ? 0 : e.out;
        tcost[2 * (size_t)t] = st ? 0 : e.cost;
        tcost[2 * (size_t)t + 1] = st ? 0 : e.cmax;
    }
}

// The first plan totals in one 32-byte block (one D2H): streams, output bytes, the batch's split cost and
// its largest stream split cost (covt_plan_create_ex step 3: nothing splits unless that passes the threshold)
__global__ void __launch_bounds__(1024) plan_head(const int64_t* __restrict__ cb, const int64_t* __restrict__ obb,
                                                  const int64_t* __restrict__ tcost, int32_t n_tiles,
                                                  int64_t* __restrict__ head, const unsigned long long* __restrict__ pacc) {
    __shared__ int64_t part[16][2];
    int64_t sum = 0, mx = 0;
    for (int32_t t = threadIdx.x; t < n_tiles; t += 1024) {
        sum += tcost[2 * (size_t)t];
        const int64_t m = tcost[2 * (size_t)t + 1];
        mx = m > mx ? m : mx;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        sum += __shfl_xor(sum, d, 64);
        const int64_t m = __shfl_xor(mx, d, 64);
        mx = m > mx ? m : mx;
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6][0] = sum, part[threadIdx.x >> 6][1] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t a = 0, b = 0;
        for (int i = 0; i < 16; ++i) a += part[i][0], b = part[i][1] > b ? part[i][1] : b;
        if (pacc) {  // the property streams' split costs (prop_sizes)
            a += (int64_t)pacc[2 + 1];
            b = (int64_t)pacc[2 + 2] > b ? (int64_t)pacc[2 + 2] : b;
        }
        head[0] = cb[n_tiles];
        head[1] = obb[n_tiles];
        head[2] = a;
        head[3] = b;
    }
}

struct InfoEmit {
    int32_t tile, id_mode;
    int64_t tile_off;
    covt_stream_info* info;
    int32_t* nvals;
    int64_t k, out, in_bytes = 0, payload = 0, verts = 0, lane = 0, k0 = 0;
    int32_t lane_max, lm = -1;
    uint32_t* keys = nullptr;
    int64_t cap = INT64_MAX;  // entries the arena holds (a plan sized to a bound)
    bool writer, wave;
    __device__ void layer_begin() { k0 = k; }
    __device__ void layer_end(int64_t data_start) {  // rebase the layer's data offsets (this lane's own stores)
        if (!data_start) return;
        if (wave) {  // the layer's records, one lane each (lane 0 wrote them: a barrier-free wave is in order)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            for (int64_t j = k0 + threadIdx.x; j < k && j < cap; j += 64) info[j].in_off += data_start;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        } else {
            for (int64_t j = k0; j < k && j < cap; ++j) info[j].in_off += data_start;
        }
    }
    __device__ void operator()(const RawStream& s) {
        int op, elem;
        int64_t nv, oe;
        choose_op(s, id_mode, op, nv, elem, oe);
        covt_stream_info si;
        si.tile = tile;
        si.layer = s.layer;
        si.column_kind = s.kind;
        si.stream_type = s.type;
        si.encoding = s.enc;
        si.column_type = s.ctype;
        si.num_values = s.nv;
        si.byte_length = s.bl;
        si.num_bits = s.nb;
        si.op = op;
        si.elem_bytes = elem;
        si.desc_index = -1;
        si.in_off = tile_off + s.off;
        si.out_elems = op == COVT_OP_NONE ? 0 : oe;
        si.out_off = out;
        out = align_out(out + si.out_elems * elem);
        in_bytes += s.bl;
        payload += si.out_elems * elem;
        if (s.kind == 1 && s.type == ST_VERTEX_BUFFER) verts += (s.ctype == CT_ICE || s.ctype == CT_ICE_MORTON) ? s.nv : s.nv / 2;
        lane += lane_stream(op, (int32_t)nv, s.bl, lane_max);
        if (writer && k < cap) {
            info[k] = si;
            nvals[k] = (int32_t)nv;
            if (keys) keys[k] = entry_key(op, (int32_t)nv, s.bl, si.out_elems, elem, lm);
        }
        ++k;
    }
};

template <bool kWave>
__global__ void walk_emit(const uint8_t* __restrict__ bytes, uint64_t n_bytes, const uint64_t* __restrict__ offs,
                          const uint64_t* __restrict__ sizes, int32_t n_tiles, int32_t format, int32_t id_mode,
                          const int32_t* __restrict__ status, const int64_t* __restrict__ cnt_base,
                          const int64_t* __restrict__ ob_base, int32_t lane_max, covt_stream_info* __restrict__ info,
                          int32_t* __restrict__ nvals, long long* __restrict__ tsum,
                          const int64_t* __restrict__ cnt, uint32_t* __restrict__ keys, int32_t lm, int64_t cap) {
    const int32_t t = kWave ? (int32_t)blockIdx.x : (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= n_tiles || status[t]) return;
    if (cnt && cnt[t] <= kSlots) return;  // emit_slots has this tile's records
    InfoEmit e{t, id_mode, (int64_t)offs[t], info, nvals, cnt_base[t], ob_base[t]};
    e.lane_max = lane_max;
    e.lm = lm;
    e.keys = keys;
    e.cap = cap;
    e.writer = !kWave || threadIdx.x == 0;
    e.wave = kWave;
    walk_tile<kWave>(bytes, n_bytes, offs[t], sizes[t], format, e);
    if (e.writer) *(longlong4*)(tsum + 4 * (size_t)t) = make_longlong4(e.in_bytes, e.payload, e.verts, e.lane);
}

// The records walk_count left in a tile's slots -> covt_stream_info, one lane per record: output slices
// by a wave prefix sum of their aligned sizes (the walk's running align_out sum), totals by a wave
// reduction.  Tiles with more than kSlots streams are left to walk_emit.
__global__ void emit_slots(const uint64_t* __restrict__ offs, int32_t n_tiles, int32_t id_mode,
                           const int32_t* __restrict__ status, const int64_t* __restrict__ cnt,
                           const int64_t* __restrict__ cnt_base, const int64_t* __restrict__ ob_base,
                           const RawStream* __restrict__ slots, int32_t lane_max, covt_stream_info* __restrict__ info,
                           int32_t* __restrict__ nvals, long long* __restrict__ tsum, uint32_t* __restrict__ keys,
                           int32_t lm, int64_t cap) {
    const int32_t t = blockIdx.x;
    if (t >= n_tiles || status[t]) return;
    const int64_t n = cnt[t];
    if (n > kSlots) return;
    const int lane = threadIdx.x;
    const int64_t base = cnt_base[t], tile_off = (int64_t)offs[t];
    int64_t out = ob_base[t];
    long long in_bytes = 0, payload = 0, verts = 0, nlane = 0;
    for (int64_t j0 = 0; j0 < n; j0 += 64) {
        const int64_t j = j0 + lane;
        const bool valid = j < n;
        RawStream s{};
        int op = COVT_OP_NONE, elem = 4;
        int64_t nv = 0, oe = 0;
        if (valid) {
            s = slots[(size_t)t * kSlots + j];
            choose_op(s, id_mode, op, nv, elem, oe);
        }
        const int64_t out_elems = op == COVT_OP_NONE ? 0 : oe;
        const long long size = valid ? align_out(out_elems * elem) : 0;
        long long incl = size;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const long long u = __shfl_up(incl, d, 64);
            if (lane >= d) incl += u;
        }
        if (valid && base + j < cap) {  // (cap: a plan sized to a bound; the overflow is caught on the host)
            covt_stream_info si;
            si.tile = t;
            si.layer = s.layer;
            si.column_kind = s.kind;
            si.stream_type = s.type;
            si.encoding = s.enc;
            si.column_type = s.ctype;
            si.num_values = s.nv;
            si.byte_length = s.bl;
            si.num_bits = s.nb;
            si.op = op;
            si.elem_bytes = elem;
            si.desc_index = -1;
            si.in_off = tile_off + s.off;
            si.out_elems = out_elems;
            si.out_off = out + (incl - size);
            info[base + j] = si;
            nvals[base + j] = (int32_t)nv;
            if (keys) keys[base + j] = entry_key(op, (int32_t)nv, s.bl, out_elems, elem, lm);
            in_bytes += s.bl;
            payload += out_elems * elem;
            if (s.kind == 1 && s.type == ST_VERTEX_BUFFER)
                verts += (s.ctype == CT_ICE || s.ctype == CT_ICE_MORTON) ? s.nv : s.nv / 2;
            nlane += lane_stream(op, (int32_t)nv, s.bl, lane_max);
        }
        out += __shfl(incl, 63, 64);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        in_bytes += __shfl_xor(in_bytes, d, 64);
        payload += __shfl_xor(payload, d, 64);
        verts += __shfl_xor(verts, d, 64);
        nlane += __shfl_xor(nlane, d, 64);
    }
    if (lane == 0) *(longlong4*)(tsum + 4 * (size_t)t) = make_longlong4(in_bytes, payload, verts, nlane);
}

// The per-tile sums (input bytes, payload, vertices, lane streams; zero for failed tiles) -> totals: one
// workgroup (same-address atomics from every tile serialise in L2: ~0.5 ms for 10k tiles)
__global__ void __launch_bounds__(1024) reduce_tiles(const long long* __restrict__ tsum, int32_t n_tiles,
                                                     unsigned long long* __restrict__ totals,
                                                     const unsigned long long* __restrict__ pacc) {
    __shared__ long long part[16][4];
    long long a[4] = {0, 0, 0, 0};
    for (int32_t t = threadIdx.x; t < n_tiles; t += 1024) {
        const longlong4 v = *(const longlong4*)(tsum + 4 * (size_t)t);
        a[0] += v.x, a[1] += v.y, a[2] += v.z, a[3] += v.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) a[k] += __shfl_xor(a[k], d, 64);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 4; ++k) part[w][k] = a[k];
    __syncthreads();
    if (threadIdx.x < 4) {
        long long x = 0;
        for (int i = 0; i < 16; ++i) x += part[i][threadIdx.x];
        if (pacc) {  // + the property streams' (prop_sizes: bytes, payload, lane streams; no vertices)
            const int k = threadIdx.x;
            x += (long long)(k == 0 ? pacc[0] : k == 1 ? pacc[1] : k == 3 ? pacc[2] : 0ull);
        }
        totals[T_IN + threadIdx.x] = (unsigned long long)x;  // T_IN, T_PAYLOAD, T_VERTS, T_LANE
    }
}

// Launch keys of a split plan (covt_plan_create_ex step 3): the family and descriptor count of each stream
// from split_mark / rle_chunks_walk.  (Unsplit plans write the keys with the stream entries and count the
// families in the sort.)
static_assert(COVT_NUM_FAMILIES <= 8 && kLaunchFamShift == 13, "launch keys: 16 bits, two radix passes");
__global__ void stream_keys(const covt_stream_info* info, const int32_t* nvals, int64_t n, int32_t lane_max,
                            int64_t lane_min, unsigned long long* totals, uint32_t* keys, const uint8_t* sfam,
                            const int64_t* sndesc) {
    __shared__ unsigned long long fam_n[COVT_NUM_FAMILIES];
    if (threadIdx.x < COVT_NUM_FAMILIES) fam_n[threadIdx.x] = 0;
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t fam = 0xffu;
    if (i < n) {
        const covt_stream_info& s = info[i];
        const int32_t lm = (int64_t)totals[T_LANE] < lane_min ? -1 : lane_max;
        const bool lane = lane_stream(s.op, nvals[i], s.byte_length, lm);
        fam = sfam ? (uint32_t)sfam[i] : lane ? (uint32_t)COVT_FAMILY_LANE : (uint32_t)covt_op_family(s.op);
        const int64_t c = (int64_t)s.byte_length + s.out_elems * s.elem_bytes / 4;
        keys[i] = launch_key(fam, fam == COVT_FAMILY_LANE, s.op, c);
        if (sndesc) atomicAdd(&fam_n[fam], (unsigned long long)sndesc[i]);
    }
    if (!sndesc) {  // one descriptor per stream: a ballot per family (same-address LDS atomics serialized)
#pragma unroll
        for (int f = 0; f < COVT_NUM_FAMILIES; ++f) {
            const uint64_t b = __ballot(fam == (uint32_t)f);
            if (b && (threadIdx.x & 63) == 0) atomicAdd(&fam_n[f], (unsigned long long)__popcll(b));
        }
    }
    __syncthreads();
    if (threadIdx.x < COVT_NUM_FAMILIES && fam_n[threadIdx.x])
        atomicAdd(&totals[T_FAM + threadIdx.x], fam_n[threadIdx.x]);
}

// ---- launch order: a stable LSD radix sort of the streams' 16-bit launch keys, two 8-bit passes of
// three launches each: per-chunk digit counts, one workgroup's scan of them (digit-major, so chunk order
// inside a digit), and the scatter, each wave ranking its 64 keys among equal digits with eight ballots
constexpr int kSortBuckets = 256;
constexpr int kSortChunk = 4096;  // keys per workgroup (4 rounds of 1024)

// info non-null (the first pass of an unsplit plan): a batch with fewer lane streams than lane_min gets
// its keys again without the lane family first (the entries were keyed with it)
__global__ void __launch_bounds__(256) order_hist(uint32_t* __restrict__ keys, int64_t n, int32_t nb, int shift,
                                                  uint32_t* __restrict__ ghist, const covt_stream_info* __restrict__ info,
                                                  const int32_t* __restrict__ nvals, int64_t lane_min,
                                                  const unsigned long long* __restrict__ totals,
                                                  const int64_t* __restrict__ dn) {
    if (dn) n = min(n, *dn);  // (a plan sized to a bound: the counted streams, from the device)
    if (dn && (int64_t)blockIdx.x * kSortChunk >= n && blockIdx.x > 0) return;  // (chunks past them: never read)
    __shared__ uint32_t h[kSortBuckets];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kSortChunk;
    const bool rekey = info && (int64_t)totals[T_LANE] < lane_min;
    for (int j = threadIdx.x; j < kSortChunk; j += 256) {
        const int64_t i = base + j;
        if (i >= n) continue;
        uint32_t key = keys[i];
        if (rekey) {
            const covt_stream_info& si = info[i];
            key = entry_key(si.op, nvals[i], si.byte_length, si.out_elems, si.elem_bytes, -1);
            keys[i] = key;
        }
        atomicAdd(&h[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    ghist[(size_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// vals null: the identity (the first pass).  scanned: gpos holds the scanned offsets; else gpos holds
// order_hist's counts and each workgroup sums the ones before it (nb <= kSortFuseChunks: one launch less)
constexpr int kSortFuseChunks = 512;
__global__ void __launch_bounds__(1024) order_scatter(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                      int64_t n, int32_t nb, int shift, const uint32_t* __restrict__ gpos,
                                                      int scanned, uint32_t* __restrict__ okeys, uint32_t* __restrict__ ovals,
                                                      unsigned long long* __restrict__ ftot, const int64_t* __restrict__ dn) {
    const int32_t stride = nb;  // (ghist rows: one count per launched chunk)
    if (dn) {  // a plan sized to a bound: the counted streams and their chunks only
        n = min(n, *dn);
        nb = max(1, (int32_t)((n + kSortChunk - 1) / kSortChunk));
        if ((int32_t)blockIdx.x >= nb) return;
    }
    __shared__ uint32_t run[kSortBuckets];
    __shared__ uint32_t wc[16][kSortBuckets];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    // ftot (the high-byte pass of the launch keys): workgroup 0 writes the streams per family (a family is
    // 2^(kLaunchFamShift - 8) consecutive digits)
    constexpr int kFamDigits = 1 << (kLaunchFamShift - 8);
    if (scanned) {
        if (threadIdx.x < kSortBuckets) run[threadIdx.x] = gpos[(size_t)threadIdx.x * stride + blockIdx.x];
        if (ftot && blockIdx.x == 0 && threadIdx.x < COVT_NUM_FAMILIES) {
            const int d0 = threadIdx.x * kFamDigits, d1 = d0 + kFamDigits;
            const uint32_t end = d1 < kSortBuckets ? gpos[(size_t)d1 * stride] : (uint32_t)n;
            ftot[threadIdx.x] = end - gpos[(size_t)d0 * stride];
        }
    } else {
        // digit totals and the counts of the chunks before this one (4 threads per digit)
        const int dg = threadIdx.x >> 2, part = threadIdx.x & 3;
        const uint32_t* row = gpos + (size_t)dg * stride;
        uint32_t tot = 0, pre = 0;
#pragma unroll 8
        for (int c = part; c < nb; c += 4) {
            const uint32_t v = row[c];
            tot += v;
            pre += c < (int)blockIdx.x ? v : 0u;
        }
        tot += __shfl_xor(tot, 1, 64);
        tot += __shfl_xor(tot, 2, 64);
        pre += __shfl_xor(pre, 1, 64);
        pre += __shfl_xor(pre, 2, 64);
        uint32_t* ts = &wc[0][0];  // (scratch before the rounds)
        if (part == 0) ts[dg] = tot;
        __syncthreads();
        if (threadIdx.x < 64) {  // exclusive scan of the 256 digit totals: 4 per lane, then the lanes
            const uint32_t a0 = ts[4 * l], a1 = ts[4 * l + 1], a2 = ts[4 * l + 2], a3 = ts[4 * l + 3];
            const uint32_t sl = a0 + a1 + a2 + a3;
            uint32_t x = sl;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                if (l >= d) x += y;
            }
            x -= sl;
            ts[kSortBuckets + 4 * l] = x;
            ts[kSortBuckets + 4 * l + 1] = x + a0;
            ts[kSortBuckets + 4 * l + 2] = x + a0 + a1;
            ts[kSortBuckets + 4 * l + 3] = x + a0 + a1 + a2;
        }
        __syncthreads();
        if (part == 0) run[dg] = ts[kSortBuckets + dg] + pre;
        if (ftot && blockIdx.x == 0 && threadIdx.x < COVT_NUM_FAMILIES) {
            unsigned long long f = 0;
            for (int q = 0; q < kFamDigits; ++q) f += ts[threadIdx.x * kFamDigits + q];
            ftot[threadIdx.x] = f;
        }
        __syncthreads();
    }
    const int64_t base = (int64_t)blockIdx.x * kSortChunk;
    for (int r = 0; r < kSortChunk / 1024; ++r) {
        for (int k = threadIdx.x; k < 16 * kSortBuckets; k += 1024) (&wc[0][0])[k] = 0;
        __syncthreads();
        const int64_t e = base + r * 1024 + threadIdx.x;
        const bool valid = e < n;
        const uint32_t key = valid ? keys[e] : 0u, dg = (key >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const bool b = (dg >> bit) & 1u;
            const uint64_t bb = __ballot(b);
            peers &= b ? bb : ~bb;
        }
        const uint64_t below = peers & ((1ull << l) - 1ull);
        const uint32_t rank = (uint32_t)__popcll(below);
        if (valid && below == 0) wc[w][dg] = (uint32_t)__popcll(peers);  // the lowest lane of each digit
        __syncthreads();
        if (threadIdx.x < kSortBuckets) {  // waves in order, after the chunk's earlier keys
            uint32_t x = run[threadIdx.x];
            for (int q = 0; q < 16; ++q) {
                const uint32_t c = wc[q][threadIdx.x];
                wc[q][threadIdx.x] = x;
                x += c;
            }
            run[threadIdx.x] = x;
        }
        __syncthreads();
        if (valid) {
            const uint32_t pos = wc[w][dg] + rank;
            okeys[pos] = key;
            ovals[pos] = vals ? vals[e] : (uint32_t)e;
        }
        __syncthreads();
    }
}

__device__ __forceinline__ void fill_desc(covt_stream_info* info, const int32_t* nvals, const uint32_t* keys,
                                          const uint32_t* order, int64_t k, covt_stream_desc* desc) {
    const uint32_t i = order[k];
    covt_stream_info& si = info[i];
    covt_stream_desc d;
    d.in_off = (uint64_t)si.in_off;
    d.out_off = (uint64_t)si.out_off;
    d.avail = si.byte_length;
    d.num_values = nvals[i];
    d.op = (uint8_t)si.op;
    d.num_bits = (uint8_t)si.num_bits;
    d.flags = (keys[k] >> kLaunchFamShift) == COVT_FAMILY_LANE ? COVT_DESC_LANE : 0;
    d.byte_length = si.byte_length;
    desc[k] = d;
    si.desc_index = (int32_t)k;
}
// dn: a plan sized to a bound (the counted streams from the device, a grid-stride loop over them)
__global__ void fill_descs(covt_stream_info* info, const int32_t* nvals, const uint32_t* keys, const uint32_t* order,
                           int64_t n, covt_stream_desc* desc, const int64_t* __restrict__ dn) {
    if (dn) n = min(n, *dn);
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        fill_desc(info, nvals, keys, order, k, desc);
}

// ---- Split plans (covt_plan_create_ex step 3 on the device; only when some stream's split cost passes
// the batch's threshold, i.e. small batches: their long poles are cut into chunks decoded by separate
// waves).  The same rule, chunk layout and descriptor order as the host plan:
//   split_mark       one thread per stream: family, descriptor count (varint: byte chunks, FastPFOR: value
//                    chunks of whole blocks), and the lists of RLE candidates and split FastPFOR streams
//   rle_chunks_walk  one wave per RLE candidate: its group framing (rle_chunks in covt_host.cpp) and chunk
//                    records; a stream it frames in two chunks or more becomes COVT_FAMILY_SPLIT_RLE
//   stream_keys / sort, then the descriptor offsets (a scan of the counts in launch order; one D2H)
//   fill_split_descs one thread per descriptor (RLE chunks from the walk's records); then fpf_states_walk
//                    writes the FastPFOR chunks' start states (fpf_chunk_states in covt_host.cpp)
enum { T_NRLE = 6, T_NFPF = 7 };  // list lengths (totals slots)

__global__ void split_mark(const covt_stream_info* __restrict__ info, const int32_t* __restrict__ nvals, int64_t n,
                           int32_t lane_max, int64_t lane_min, int64_t smin, int64_t split_chunk, int64_t split_values,
                           int64_t fpf_w, unsigned long long* __restrict__ totals, uint8_t* __restrict__ sfam,
                           int64_t* __restrict__ sndesc, uint32_t* __restrict__ rle_list, uint32_t* __restrict__ fpf_list) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const covt_stream_info& s = info[i];
    const int32_t nv = nvals[i];
    const int32_t lm = (int64_t)totals[T_LANE] < lane_min ? -1 : lane_max;
    const bool lane = lane_stream(s.op, nv, s.byte_length, lm);
    const int64_t ob4 = s.out_elems * s.elem_bytes / 4, cost = (int64_t)s.byte_length + ob4;
    const bool fpf = split_fpf_op(s.op);
    const int64_t scost = fpf ? cost + (fpf_w - 1) * ob4 : cost;
    const bool split = split_stream(s.op, nv, scost, smin, split_values);
    int fam = split ? (fpf ? COVT_FAMILY_SPLIT_FPF : COVT_FAMILY_SPLIT) : lane ? COVT_FAMILY_LANE : covt_op_family(s.op);
    int64_t nd = 1;
    if (split) {
        const int64_t unit = fpf ? split_values : split_chunk, tot = fpf ? nv : s.byte_length;
        nd = (tot + unit - 1) / unit * COVT_SPLIT_SLOTS;
        if (fpf) fpf_list[atomicAdd(&totals[T_NFPF], 1ull)] = (uint32_t)i;
    } else if (split_rle_op(s.op) && cost > smin && nv > 0) {
        rle_list[atomicAdd(&totals[T_NRLE], 1ull)] = (uint32_t)i;
    }
    sfam[i] = (uint8_t)fam;
    sndesc[i] = nd;
}

// One stream's bytes for the split walkers (a wave each, lanes in lockstep): a 4 KiB LDS window refilled
// by all 64 lanes at once (four 16-byte loads each, one memory latency per 4 KiB of a long stream)
struct StreamRd {
    static constexpr uint32_t kWin = 4096;
    const uint8_t* t;
    int64_t len;
    int32_t wo;  // the window's start as a stream offset (16-byte aligned address)
    __device__ void refill(int32_t i) {
        const uintptr_t lo = (uintptr_t)t;
        const uintptr_t b = (lo + (uintptr_t)(int64_t)i) & ~(uintptr_t)15;
        wo = __builtin_amdgcn_readfirstlane((int32_t)(int64_t)(b - lo));
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = window_ld(t, len, b + 16 * (uintptr_t)(threadIdx.x + 64 * k));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
        for (int k = 0; k < 4; ++k) covt_walk_win[threadIdx.x + 64 * k] = v[k];
        if (threadIdx.x == 0) covt_walk_win[kWin / 16] = make_uint4(0, 0, 0, 0);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    // the window holds bytes [i, i + n) (n <= 512); returns i's offset in it
    __device__ __forceinline__ uint32_t ensure(int32_t i, uint32_t n) {
        if ((uint32_t)(i - wo) > kWin - n) refill(i);
        return (uint32_t)(i - wo);
    }
    // bytes [i, i + 8) (past the stream: unspecified, callers mask by len)
    __device__ __forceinline__ uint64_t peek8(int32_t i) {
        return win_bytes8(reinterpret_cast<const uint32_t*>(covt_walk_win), ensure(i, 8));
    }
    __device__ __forceinline__ int at(int32_t i) { return (int)(peek8(i) & 0xff); }
};
constexpr size_t kStreamRdLds = StreamRd::kWin + 16;

// skips cnt LEB128 values from pos (false: the stream ends first): 64 bytes per step, a lane per byte
__device__ __forceinline__ bool skip_varints(StreamRd& r, int32_t& pos, int32_t len, int32_t cnt) {
    const int lane = threadIdx.x;
    while (cnt > 0) {
        if (pos >= len) return false;
        const uint32_t off = r.ensure(pos, 64);
        const uint8_t* w = (const uint8_t*)covt_walk_win + off;
        const bool term = pos + lane < len && !(w[lane] & 0x80);
        const uint64_t m = __ballot(term);
        const int pc = __builtin_popcountll(m);
        if (pc < cnt) {
            if (len - pos <= 64) return false;
            pos += 64;
            cnt -= pc;
            continue;
        }
        const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint64_t sel = __ballot(term && below == cnt - 1);
        pos += __builtin_ctzll(sel) + 1;
        return true;
    }
    return true;
}

// rle_chunks (covt_host.cpp) for one stream: its chunks {first byte, end byte, first value, values} into
// rec[0, cap) (cap: the bound (cost / unit + 2)), the chunk count (0: not framed), the consumed bytes
__device__ int32_t rle_walk(StreamRd& r, int32_t len, int op, int32_t n, int32_t elem, int64_t unit, int32_t& consumed,
                            int4* rec, int64_t cap) {
    const bool byte_rle = op == COVT_OP_BYTE_RLE_U8 || op == COVT_OP_BYTE_RLE_RAW;
    int32_t pos = 0, v = 0, cs = 0, cv = 0, nch = 0;
    auto chunk = [&](int32_t e, int32_t nvc) {
        if (threadIdx.x == 0 && nch < cap) rec[nch] = make_int4(cs, e, cv, nvc);
        ++nch;
    };
    while (v < n) {
        if (pos >= len) return 0;
        if ((int64_t)(pos - cs) + (int64_t)(v - cv) * elem / 4 >= unit) {  // cut before this group
            chunk(pos, v - cv);
            cs = pos;
            cv = v;
        }
        const uint64_t w = r.peek8(pos);
        const int32_t h = (int32_t)(w & 0xff);
        if (h < 0x80) {
            if (byte_rle) {
                if (pos + 2 > len) return 0;
                pos += 2;
            } else {  // header, delta byte, base varint (ends within the word: one step)
                const int32_t avail = len - pos;
                uint64_t x = w | (avail < 8 ? 0x8080808080808080ull & (~0ull << (8 * (avail > 0 ? avail : 0))) : 0ull);
                const uint64_t term = ~x & 0x8080808080808080ull & ~0xffffull;
                if (pos + 2 > len) return 0;
                if (term) {
                    pos += (__builtin_ctzll(term) >> 3) + 1;
                } else {
                    pos += 2;
                    if (!skip_varints(r, pos, len, 1)) return 0;
                }
            }
            v += h + 3;
        } else {
            const int32_t cnt = 256 - h;
            ++pos;
            if (byte_rle) {
                if (pos + cnt > len) return 0;
                pos += cnt;
            } else if (!skip_varints(r, pos, len, cnt)) {
                return 0;
            }
            v += cnt;
        }
    }
    chunk(pos, n - cv);
    consumed = pos;
    return nch;
}

// one wave per RLE candidate: a stream framed in >= 2 chunks becomes a split RLE stream, its chunk records
// at rle_base[i] of the chunk scratch (cap records reserved per candidate) and its consumed bytes
__global__ void rle_chunks_walk(const uint8_t* __restrict__ bytes, const covt_stream_info* __restrict__ info,
                                const int32_t* __restrict__ nvals, unsigned long long* __restrict__ totals,
                                const uint32_t* __restrict__ rle_list, int64_t unit, uint8_t* __restrict__ sfam,
                                int64_t* __restrict__ sndesc, int4* __restrict__ chunks, int64_t chunk_cap,
                                int64_t* __restrict__ rle_base, int32_t* __restrict__ rle_cons) {
    const int64_t nl = (int64_t)totals[T_NRLE];
    for (int64_t c = blockIdx.x; c < nl; c += gridDim.x) {
        const uint32_t i = rle_list[c];
        const covt_stream_info& si = info[i];
        const int32_t nv = nvals[i];
        const int64_t cap = ((int64_t)si.byte_length + (int64_t)nv * si.elem_bytes / 4) / unit + 2;
        unsigned long long base = 0;
        if (threadIdx.x == 0) base = atomicAdd(&totals[T_RCH], (unsigned long long)cap);
        base = __shfl(base, 0, 64);
        if ((int64_t)base + cap > chunk_cap) continue;  // (cannot happen: the host sized the scratch for every bound)
        StreamRd r;
        r.t = bytes + si.in_off;
        r.len = si.byte_length;
        r.wo = -0x40000000;
        int32_t consumed = 0;
        const int32_t nch = rle_walk(r, si.byte_length, si.op, nv, si.elem_bytes, unit, consumed, chunks + base, cap);
        if (nch >= 2 && threadIdx.x == 0) {
            sfam[i] = COVT_FAMILY_SPLIT_RLE;
            sndesc[i] = (int64_t)nch * COVT_SPLIT_SLOTS;
            rle_base[i] = (int64_t)base;
            rle_cons[i] = consumed;
        }
    }
}

// descriptor counts in launch order (for their exclusive scan)
__global__ void gather_ndesc(const uint32_t* __restrict__ order, const int64_t* __restrict__ sndesc, int64_t n,
                             int64_t* __restrict__ dn) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) dn[k] = sndesc[order[k]];
    if (k == n) dn[k] = 0;
}

// descriptor j: its stream (binary search of the launch-order offsets), then the stream's descriptor or the
// chunk / pad j - dpos of a split varint or FastPFOR stream (FastPFOR states: fpf_states_walk; split RLE
// streams: rle_chunks_walk<true>).  The first descriptor of a stream sets its desc_index.
__global__ void fill_split_descs(covt_stream_info* __restrict__ info, const int32_t* __restrict__ nvals,
                                 const uint32_t* __restrict__ order, const int64_t* __restrict__ dpos, int64_t ns,
                                 int64_t n_desc, const uint8_t* __restrict__ sfam, int64_t split_chunk,
                                 int64_t split_values, const int4* __restrict__ chunks, const int64_t* __restrict__ rle_base,
                                 const int32_t* __restrict__ rle_cons, covt_stream_desc* __restrict__ desc,
                                 uint32_t* __restrict__ dorder) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_desc) return;
    int64_t lo = 0, hi = ns;  // the last k with dpos[k] <= j
    while (hi - lo > 1) {
        const int64_t m = (lo + hi) >> 1;
        if (dpos[m] <= j) lo = m;
        else hi = m;
    }
    const int64_t k = lo, q = j - dpos[k];
    const uint32_t i = order[k];
    dorder[j] = i;
    covt_stream_info& si = info[i];
    const int fam = sfam[i];
    if (q == 0) si.desc_index = (int32_t)j;
    covt_stream_desc d;
    d.in_off = (uint64_t)si.in_off;
    d.out_off = (uint64_t)si.out_off;
    d.avail = si.byte_length;
    d.num_values = nvals[i];
    d.op = (uint8_t)si.op;
    d.num_bits = (uint8_t)si.num_bits;
    d.flags = fam == COVT_FAMILY_LANE ? COVT_DESC_LANE : 0;
    d.byte_length = si.byte_length;
    if (fam != COVT_FAMILY_SPLIT && fam != COVT_FAMILY_SPLIT_FPF && fam != COVT_FAMILY_SPLIT_RLE) {
        desc[j] = d;
        return;
    }
    const int64_t c = q / COVT_SPLIT_SLOTS, slot = q % COVT_SPLIT_SLOTS;
    if (fam == COVT_FAMILY_SPLIT_RLE) {  // the chunk records of rle_chunks_walk
        covt_stream_desc x{};
        if (slot == 0) {
            x = d;
            x.flags = COVT_DESC_SPLIT | COVT_DESC_SPLIT_RLE;
            x.avail = (int32_t)c;
        } else {
            x.flags = COVT_DESC_SPLIT_PAD | COVT_DESC_SPLIT_RLE;
            const int4 r = chunks[rle_base[i] + c];
            if (slot == 1) x.in_off = (uint64_t)r.x, x.out_off = (uint64_t)r.y;
            if (slot == 2) x.in_off = (uint64_t)r.z, x.out_off = (uint64_t)r.w;
            if (slot == 3) x.in_off = (uint64_t)rle_cons[i];
        }
        desc[j] = x;
        return;
    }
    const bool fpf = fam == COVT_FAMILY_SPLIT_FPF;
    const uint16_t fflag = fpf ? COVT_DESC_SPLIT_FPF : 0;
    if (slot == 0) {
        d.flags = COVT_DESC_SPLIT | fflag;
        d.avail = (int32_t)c;
        desc[j] = d;
        return;
    }
    covt_stream_desc pd{};
    pd.flags = COVT_DESC_SPLIT_PAD | fflag;
    if (slot == 1) {
        const int64_t unit = fpf ? split_values : split_chunk, total = fpf ? (int64_t)d.num_values : (int64_t)d.byte_length;
        pd.in_off = (uint64_t)(c * unit);
        pd.out_off = (uint64_t)((c + 1) * unit < total ? (c + 1) * unit : total);
    }
    desc[j] = pd;
}

// fpf_chunk_states (covt_host.cpp) for each split FastPFOR stream, one wave each (lanes in lockstep; lane
// k <= 32 holds the exception cursor of array k): the start state of every chunk the page / block header
// walk reaches, in the chunk's pads [2..7] (state slot m: pad 2 + m / 7, field m % 7)
__global__ void fpf_states_walk(const uint8_t* __restrict__ bytes, const covt_stream_info* __restrict__ info,
                                const int32_t* __restrict__ nvals, const unsigned long long* __restrict__ totals,
                                const uint32_t* __restrict__ fpf_list, int64_t unit, covt_stream_desc* __restrict__ desc) {
    const int64_t nl = (int64_t)totals[T_NFPF];
    const int lane = threadIdx.x;
    for (int64_t li = blockIdx.x; li < nl; li += gridDim.x) {
        const uint32_t i = fpf_list[li];
        const covt_stream_info& si = info[i];
        const int32_t n = nvals[i], byte_length = si.byte_length;
        const int64_t nch = ((int64_t)n + unit - 1) / unit;
        covt_stream_desc* out = desc + si.desc_index;
        StreamRd r;
        r.t = bytes + si.in_off;
        r.len = byte_length;
        r.wo = -0x40000000;
        auto W = [&](int64_t w) -> uint32_t { return __builtin_bswap32((uint32_t)r.peek8((int32_t)(4 * w))); };
        const int64_t nw = byte_length / 4;
        if (nw <= 0 || unit % 256) continue;
        int32_t L = (int32_t)W(0);
        if (L < 0) continue;
        L -= L % 256;
        if (L > n) continue;
        int64_t p = 1;
        int32_t done = 0;
        bool stop = false;
        while (done < L && !stop) {
            const int32_t thissize = L - done < 65536 ? L - done : 65536;
            const int64_t p0 = p;
            if (p0 >= nw) break;
            int64_t ie = p0 + (int32_t)W(p0);
            if (ie < 0 || ie >= nw) break;
            const int32_t bytesize = (int32_t)W(ie++);
            if (bytesize < 0 || bytesize > 3 * 65536 / 256 + 65536) break;
            const int64_t bcw = (bytesize + 3) / 4, bc = ie;
            if (bc + bcw >= nw) break;
            ie += bcw;
            uint32_t bm = W(ie++) & ~1u;
            while (bm) {
                const int32_t k = __builtin_ctz(bm) + 1;
                bm &= bm - 1;
                if (ie >= nw) {
                    stop = true;
                    break;
                }
                const int32_t size = (int32_t)W(ie++);
                if (size < 0) {
                    stop = true;
                    break;
                }
                const int64_t groups = ((int64_t)size + 31) / 32;
                ie += groups * k - ((groups * 32 - size) * k) / 32;
            }
            if (stop) break;
            const int32_t bclen = (int32_t)(bcw * 4), nblk = thissize / 256;
            // container bytes cur, cur + 1, cur + 2 (byte q at stream byte 4 bc + (q ^ 3)): one 8-byte read
            // of the two words holding them
            const int32_t cbase = (int32_t)(4 * bc);
            int32_t cur = 0, xc = 0;  // xc: this lane's array cursor (lane k <= 32)
            int64_t pk = p0 + 1;
            // the next chunk start past the page's first block (a multiple of unit; no 64-bit division per block)
            int64_t ci = ((int64_t)done + 256 + unit - 1) / unit, cut = ci * unit;
            for (int32_t j = 0; j < nblk; ++j) {
                const int64_t v = (int64_t)done + (int64_t)j * 256;
                if (v == cut) {  // chunk ci starts at block j (> 0) of this page
                    const bool own = ci < nch;
                    covt_stream_desc* o = out + (size_t)ci * COVT_SPLIT_SLOTS;
                    ++ci;
                    cut += unit;
                    const int32_t xv = __shfl(xc, lane >= 4 ? lane - 4 : 0, 64);
                    const int32_t val = lane == 0 ? 1 : lane == 1 ? done : lane == 2 ? cur : lane == 3 ? (int32_t)pk : xv;
                    if (own && lane < 37) *(int32_t*)((uint8_t*)(o + 2 + lane / 7) + covt_fpf_state_byte(lane % 7)) = val;
                }
                if (cur + 3 > bclen + 1) {
                    stop = true;
                    break;
                }
                const uint64_t x = r.peek8(cbase + 4 * (cur >> 2));
                auto cb = [&](int32_t q) -> uint32_t {
                    return (uint32_t)(x >> (8 * (4 * ((q >> 2) - (cur >> 2)) + ((q & 3) ^ 3)))) & 0xffu;
                };
                const int32_t hb = (int32_t)(int8_t)cb(cur), ce = (int32_t)cb(cur + 1);
                const int32_t idx = ce > 0 && cur + 2 < bclen ? (int32_t)(int8_t)cb(cur + 2) - hb : 0;
                pk += 8 * hb;
                if (ce > 0 && idx >= 2 && idx <= 32 && lane == idx) xc += ce;
                cur += ce > 0 ? 3 + ce : 2;
                if (cur > bclen) {
                    stop = true;
                    break;
                }
            }
            done += thissize;
            p = ie;
        }
    }
}

// ---- Property columns (COVT_PLAN_PROPERTIES; covt_host.cpp walk_genc / walk_gend's property records,
// plan_property and plan_property_layout).  The host plan puts a tile's property streams after its Id /
// Geometry streams and gives them output slices in that order; here:
//   prop_walk<false>  one wave per tile (largest tiles first): the container walk again, counting property
//                     (sub)columns and keeping each tile's first kPropSlots records in its slots
//   scan              -> each tile's first record; one D2H (the record count sizes the arrays)
//   prop_compact      the slots -> the records' places (PropRaw, tile-relative offsets); prop_walk<true>
//                     walks again only the tiles with more records than slots
//   prop_sizes        a thread per record: its decode streams (prop_streams, the host's rule), their count
//                     and aligned output bytes; the records' byte / payload / lane / cost totals
//   scans + tile_totals  each tile's streams and output bytes = Id / Geometry + property
// and once the stream arrays exist, prop_fill writes the records' stream entries and covt_prop_info,
// prop_layout / prop_layout_fill the property output slices, a stable radix sort the largest-first
// materialization order and prop_desc_fill the covt_prop_desc table.
struct PropSm {  // a property column's stream, as the Gen C walk reads it
    uint32_t h0, h8;  // localized string columns: hashes of the name and of its bytes from 8 on (names_hash)
    int32_t noff, nlen, nv, bl;
    int32_t off;      // layer-data-relative
    uint16_t enc, role;  // role: PR_* bits of the name, classified while the window holds it
};
enum { PR_PRESENT = 1, PR_DATA = 2, PR_LENGTH = 4, PR_DICTIONARY = 8, PR_PRESENT_LANG = 16 };
constexpr int kPropMaxStreams = 256;  // numStreams bound of the walk (walk_genc: > 256 is BAD_HEADER)
// LDS: Rd<true>'s window, the fast walk's window and tables (walk_count's layout)
constexpr size_t kPropRecOffset = (kFastSmemOffset + sizeof(FastSmem) + 15) & ~(size_t)15;
constexpr size_t kPropWalkLds = kPropRecOffset + sizeof(FastSmemRec) > kWalkLds ? kPropRecOffset + sizeof(FastSmemRec) : kWalkLds;

// A property column's stream table in registers: entry s in lane s % 64, slot s / 64 (32 VGPRs).  It
// was 7 KB of LDS per wave, which halved the walk's resident waves against the Id walk's -- and the walk
// is a latency-bound chain, so resident tiles set its rate.
struct PropTab {
    uint32_t h0[4], h8[4];
    int32_t noff[4], nlen[4], nv[4], bl[4], off[4];
    uint32_t er[4];  // enc | role << 16
    template <class T>
    static __device__ __forceinline__ T pick(const T (&a)[4], uint32_t j) {  // a[j], j uniform
        return j == 0 ? a[0] : j == 1 ? a[1] : j == 2 ? a[2] : a[3];
    }
    __device__ __forceinline__ void set(uint32_t s, const PropSm& v) {  // (s, v uniform)
        // selects, not conditional stores: those were merged into one store at a computed index (scratch)
        const bool me = threadIdx.x == (s & 63u);
        const uint32_t j = s >> 6, e = (uint32_t)v.enc | ((uint32_t)v.role << 16);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const bool w = me && k == j;
            h0[k] = w ? v.h0 : h0[k];
            h8[k] = w ? v.h8 : h8[k];
            noff[k] = w ? v.noff : noff[k];
            nlen[k] = w ? v.nlen : nlen[k];
            nv[k] = w ? v.nv : nv[k];
            bl[k] = w ? v.bl : bl[k];
            off[k] = w ? v.off : off[k];
            er[k] = w ? e : er[k];
        }
    }
    static __device__ __forceinline__ int32_t rl(int32_t x, uint32_t ln) { return __builtin_amdgcn_readlane(x, (int)ln); }
    __device__ __forceinline__ PropSm get(uint32_t s) const {  // entry s (uniform), on every lane
        const uint32_t j = s >> 6, ln = s & 63u;
        PropSm v;
        v.h0 = (uint32_t)rl((int32_t)pick(h0, j), ln);
        v.h8 = (uint32_t)rl((int32_t)pick(h8, j), ln);
        v.noff = rl(pick(noff, j), ln);
        v.nlen = rl(pick(nlen, j), ln);
        v.nv = rl(pick(nv, j), ln);
        v.bl = rl(pick(bl, j), ln);
        v.off = rl(pick(off, j), ln);
        const uint32_t e = (uint32_t)rl((int32_t)pick(er, j), ln);
        v.enc = (uint16_t)(e & 0xffffu);
        v.role = (uint16_t)(e >> 16);
        return v;
    }
    // the highest entry below ns whose role has any of `bits` (-1: none)
    __device__ __forceinline__ int32_t last_role(uint32_t ns, uint32_t bits, uint32_t notbits) const {
        for (int32_t j = 3; j >= 0; --j) {
            const uint32_t k = 64u * (uint32_t)j + threadIdx.x;
            const uint32_t role = pick(er, (uint32_t)j) >> 16;
            const uint64_t b = __ballot(k < ns && (role & bits) && !(role & notbits));
            if (b) return 64 * j + 63 - __builtin_clzll(b);
        }
        return -1;
    }
};

// bytes [a, a + n) == bytes [b, b + n) of the tile (names; uniform)
__device__ __forceinline__ bool names_equal(Rd<true>& r, int32_t a, int32_t b, int32_t n) {
    for (int32_t i = 0; i < n; i += 8) {
        const int32_t k = n - i < 8 ? n - i : 8;
        const uint64_t m = k >= 8 ? ~0ull : ((1ull << (8 * k)) - 1);
        if ((r.peek8(a + i) & m) != (r.peek8(b + i) & m)) return false;
    }
    return true;
}
// a hash of bytes [a, a + n) (equal bytes, equal hashes): read while the walk's window holds the name, so
// the localized columns' name matching below compares hashes and confirms a match with names_equal --
// one window refill per match instead of a refill per byte compared (two names of a long column lie
// further apart than the window, and the all-pairs compare ping-ponged between them: ~9 ms per walk)
__device__ __forceinline__ uint32_t names_hash(Rd<true>& r, int32_t a, int32_t n) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)(uint32_t)n;
    for (int32_t i = 0; i < n; i += 8) {
        const int32_t k = n - i < 8 ? n - i : 8;
        const uint64_t m = k >= 8 ? ~0ull : ((1ull << (8 * k)) - 1);
        h = (h ^ (r.peek8(a + i) & m)) * 0xff51afd7ed558ccdull;
        h ^= h >> 29;
    }
    return (uint32_t)(h ^ (h >> 32));
}

// Gen C property records (walk_genc's props branch): a column's streams in metadata order, roles by
// name; LOCALIZED_DICTIONARY strings as one sub-column per present_<lang> stream
template <class PE>
__device__ int prop_walk_genc(Rd<true>& r, PE& pe, PropTab& tab) {
    const int32_t len = (int32_t)r.len;
    int32_t o = 0;
    uint64_t version, nlayers;
    if (!r.uv(o, version) || !r.uv(o, nlayers)) return COVT_ERR_TRUNCATED;
    if (version != 1) return COVT_ERR_BAD_HEADER;
    for (uint64_t L = 0; L < nlayers; ++L) {
        uint64_t nlen, extent, nfeat, ncols;
        if (!r.uv(o, nlen) || nlen > (uint64_t)(len - o)) return COVT_ERR_TRUNCATED;
        o += (int32_t)nlen;
        if (!r.uv(o, extent) || !r.uv(o, nfeat) || !r.uv(o, ncols)) return COVT_ERR_TRUNCATED;
        if (ncols > 4096) return COVT_ERR_BAD_HEADER;
        int64_t d = 0;
        pe.layer_begin();
        for (uint32_t c = 0; c < (uint32_t)ncols; ++c) {
            uint64_t cn, ns, sn, nv, bl;
            if (!r.uv(o, cn) || cn > (uint64_t)(len - o) || (uint64_t)(len - o) - cn < 2) return COVT_ERR_TRUNCATED;
            const int32_t name = o;
            o += (int32_t)cn;
            const int dtype = r.at(o), ctype = r.at(o + 1);
            o += 2;
            if (!r.uv(o, ns)) return COVT_ERR_TRUNCATED;
            if (ns > 256) return COVT_ERR_BAD_HEADER;
            const int kind = COVT_IS(name, cn, "id") ? 0 : (COVT_IS(name, cn, "geometry") || dtype == 6) ? 1 : 2;
            const bool localized = kind == 2 && genc_prop_type(dtype) == COVT_PROP_STRING && ctype == 2;
            for (uint32_t q = 0; q < (uint32_t)ns; ++q) {
                if (!r.uv(o, sn) || sn > (uint64_t)(len - o)) return COVT_ERR_TRUNCATED;
                const int32_t sname = o;
                o += (int32_t)sn;
                int enc;
                if (!r.rec3(o, nv, bl, enc)) {
                    if (!r.uv(o, nv) || !r.uv(o, bl) || o >= len) return COVT_ERR_TRUNCATED;
                    enc = r.at(o++);
                }
                if (nv > 0x7fffffff || bl > 0x7fffffff) return COVT_ERR_BAD_HEADER;
                if (kind == 2) {  // the name's role (and, localized, its hashes) while the window holds it
                    uint32_t role = 0;
                    if (COVT_IS(sname, sn, "present")) role |= PR_PRESENT;
                    if (COVT_IS(sname, sn, "data")) role |= PR_DATA;
                    if (COVT_IS(sname, sn, "length")) role |= PR_LENGTH;
                    if (COVT_IS(sname, sn, "dictionary")) role |= PR_DICTIONARY;
                    uint32_t h0 = 0, h8 = 0;
                    if (localized) {
                        if (sn > 8 && r.peek8(sname) == pk("present_", 0, 8)) {
                            role |= PR_PRESENT_LANG;
                            h8 = names_hash(r, sname + 8, (int32_t)sn - 8);
                        }
                        h0 = names_hash(r, sname, (int32_t)sn);
                    }
                    tab.set(q, PropSm{h0, h8, sname, (int32_t)sn, (int32_t)nv, (int32_t)bl, (int32_t)d, (uint16_t)enc,
                                      (uint16_t)role});
                }
                d += (int64_t)bl;
            }
            if (kind != 2) continue;
            PropRaw p = prop_init((int32_t)L, (int32_t)c, (int32_t)nfeat);
            p.name_off = name;
            p.name_len = (int32_t)cn;
            p.type = genc_prop_type(dtype);
            p.ctype = ctype;
            if (localized) {
                prop_localized(r, pe, tab, ns, p);
            } else {
                for (uint32_t q = 0; q < (uint32_t)ns; ++q) {
                    const PropSm sm = tab.get(q);
                    if (sm.role & PR_PRESENT) prop_stream(p, 0, sm.off, sm.nv, sm.bl, sm.enc);
                    if (sm.role & PR_DATA) prop_stream(p, 1, sm.off, sm.nv, sm.bl, sm.enc);
                    if (sm.role & PR_LENGTH) prop_stream(p, 2, sm.off, sm.nv, sm.bl, sm.enc);
                    if (sm.role & PR_DICTIONARY) prop_stream(p, 3, sm.off, sm.nv, sm.bl, sm.enc);
                }
                pe(p);
            }
        }
        if (d > (int64_t)(len - o)) return COVT_ERR_TRUNCATED;
        pe.layer_end(o);  // the layer's data starts where its metadata ends
        o += (int32_t)d;
    }
    return o == len ? COVT_OK : COVT_ERR_BAD_HEADER;
}

// names_hash of every stream name of a localized column at once, a lane per stream (name bytes read from
// the tile): on the scalar unit, the walk's bound, two hashes cost ~60 instructions per stream.  h8 (the
// bytes after "present_") for the present_<lang> streams.
__device__ __forceinline__ uint64_t tile_bytes8(const uint8_t* t, int32_t len, int32_t off) {
    const uintptr_t lo = (uintptr_t)t, hi = lo + (uintptr_t)(uint32_t)len, a = lo + (uintptr_t)(uint32_t)off;
    const uintptr_t a4 = a & ~(uintptr_t)3;
    auto ld4 = [&](uintptr_t x) -> uint32_t {  // dwords overlapping the tile lie inside its allocation
        return (x + 4 > lo && x < hi) ? *(const __attribute__((address_space(1))) uint32_t*)x : 0u;
    };
    const uint32_t d0 = ld4(a4), d1 = ld4(a4 + 4), d2 = ld4(a4 + 8), sh = (uint32_t)(a & 3u);
    return ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32) | __builtin_amdgcn_alignbyte(d1, d0, sh);
}
__device__ __forceinline__ uint32_t names_hash_lane(const uint8_t* t, int32_t len, int32_t a, int32_t n, int32_t nmax) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)(uint32_t)n;
    for (int32_t i = 0; i < nmax; i += 8) {  // (the wave's longest name sets the trip count)
        const int32_t k = n - i < 8 ? n - i : 8;
        const uint64_t m = k >= 8 ? ~0ull : ((1ull << (8 * (k > 0 ? k : 0))) - 1);
        uint64_t hn = (h ^ (tile_bytes8(t, len, a + i) & m)) * 0xff51afd7ed558ccdull;
        hn ^= hn >> 29;
        h = i < n ? hn : h;
    }
    return (uint32_t)(h ^ (h >> 32));
}
__device__ __forceinline__ void names_hash_lanes(const uint8_t* t, int32_t len, PropTab& tab, uint32_t ns) {
    for (uint32_t j = 0; 64 * j < ns; ++j) {
        const bool v = 64 * j + threadIdx.x < ns;
        const int32_t noff = PropTab::pick(tab.noff, j), nlen = v ? PropTab::pick(tab.nlen, j) : 0;
        const bool lang = v && ((PropTab::pick(tab.er, j) >> 16) & PR_PRESENT_LANG);
        int32_t nmax = nlen;
#pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) nmax = max(nmax, __shfl_xor(nmax, sh));
        nmax = __builtin_amdgcn_readfirstlane(nmax);
        const uint32_t h0 = v ? names_hash_lane(t, len, noff, nlen, nmax) : 0u;
        const uint32_t h8 = lang ? names_hash_lane(t, len, noff + 8, nlen - 8, nmax) : 0u;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            tab.h0[k] = k == j ? h0 : tab.h0[k];
            tab.h8[k] = k == j ? h8 : tab.h8[k];
        }
    }
}

// The localized sub-columns of a Gen C string column from its stream table (prop_walk_genc's rule): one
// per present_<lang> stream, with the last stream named <lang> as data and the last length / dictionary
template <class PE>
__device__ __forceinline__ void prop_localized(Rd<true>& r, PE& pe, const PropTab& tab, uint32_t ns, const PropRaw& p) {
    const int32_t ls = tab.last_role(ns, PR_LENGTH, 0), ds = tab.last_role(ns, PR_DICTIONARY, PR_LENGTH);
    const PropSm lsm = tab.get(ls >= 0 ? (uint32_t)ls : 0u), dsm = tab.get(ds >= 0 ? (uint32_t)ds : 0u);
    int32_t lang = 0;
    for (uint32_t j = 0; 64 * j < ns; ++j) {  // the present_<lang> streams in order
        uint64_t pm = __ballot(64 * j + threadIdx.x < ns && ((PropTab::pick(tab.er, j) >> 16) & PR_PRESENT_LANG));
        while (pm) {
            const uint32_t q = 64 * j + (uint32_t)__builtin_ctzll(pm);
            pm &= pm - 1;
            const PropSm sm = tab.get(q);
            const int32_t ll = sm.nlen - 8;
            // the last stream named <lang>: 64 candidates per step, hash matches confirmed from the highest
            // down (a serial all-pairs scan was ~ns^2 dependent LDS reads: ms per tile)
            int dd = -1;
            for (int32_t k0 = ((int32_t)ns - 1) & ~63; k0 >= 0 && dd < 0; k0 -= 64) {
                const uint32_t jj = (uint32_t)k0 >> 6;
                const int32_t k = k0 + (int32_t)threadIdx.x;
                const bool m = k < (int32_t)ns && PropTab::pick(tab.nlen, jj) == ll && PropTab::pick(tab.h0, jj) == sm.h8;
                uint64_t bal = __ballot(m);
                while (bal && dd < 0) {
                    const int hi = 63 - __builtin_clzll(bal);
                    if (names_equal(r, PropTab::rl(PropTab::pick(tab.noff, jj), (uint32_t)hi), sm.noff + 8, ll)) dd = k0 + hi;
                    bal &= ~(1ull << hi);
                }
            }
            PropRaw x = p;
            x.lang = lang++;
            x.lang_off = sm.noff + 8;
            x.lang_len = ll;
            prop_stream(x, 0, sm.off, sm.nv, sm.bl, sm.enc);
            if (dd >= 0) {
                const PropSm dm = tab.get((uint32_t)dd);
                prop_stream(x, 1, dm.off, dm.nv, dm.bl, dm.enc);
            }
            if (ls >= 0) prop_stream(x, 2, lsm.off, lsm.nv, lsm.bl, lsm.enc);
            if (ds >= 0) prop_stream(x, 3, dsm.off, dsm.nv, dsm.bl, dsm.enc);
            pe(x);
        }
    }
}

// prop_walk_genc on walk_count's speculative tables (FastGenc): a column header and a stream record are
// one LDS read each, and a stream's name, numValues and encoding are parsed only in property columns.
// kFastFallback when the tile leaves the fast grammar (the caller walks it with prop_walk_genc); a
// successful fast walk emits the same records.
template <class PE>
__device__ int prop_walk_genc_fast(FastGenc& f, Rd<true>& r, PE& pe, PropTab& tab) {
    const int32_t len = f.len;
    int32_t o = 0;
    uint32_t version, nlayers;
    if (!f.uv4(o, version) || !f.uv4(o, nlayers) || version != 1) return kFastFallback;
    for (uint32_t L = 0; L < nlayers; ++L) {
        uint32_t nlen, extent, nfeat, ncols;
        if (!f.uv4(o, nlen) || nlen > (uint32_t)(len - o)) return kFastFallback;
        o += (int32_t)nlen;
        if (!f.uv4(o, extent) || !f.uv4(o, nfeat) || !f.uv4(o, ncols) || ncols > 4096) return kFastFallback;
        int64_t d = 0;
        pe.layer_begin();
        for (uint32_t c = 0; c < ncols; ++c) {
            const int32_t qc = f.at_run(o);
            const uint32_t ce = (uint32_t)__builtin_amdgcn_readfirstlane((int)f.fs->ctab[qc]);
            if (!ce) return kFastFallback;
            const uint32_t ns = (ce >> 8) & 0x1ffu, kind = (ce >> 17) & 3u;
            if (kind != 2) {  // Id / Geometry: only their data bytes
                o += (int32_t)(ce & 0xffu);
                for (uint32_t s = 0; s < ns; ++s) {
                    const uint32_t se = (uint32_t)__builtin_amdgcn_readfirstlane((int)f.fs->stab[f.at_run(o)]);
                    if (!se) return kFastFallback;
                    d += (int32_t)(se >> 8);
                    o += (int32_t)(se & 0xffu);
                }
                continue;
            }
            const int32_t n = (int32_t)((__builtin_amdgcn_readfirstlane((int)f.fs->win[qc >> 2]) >> (8 * (qc & 3))) &
                                        0xff);  // the name's length (one LEB128 byte)
            const int dtype = (int)(ce >> 27);  // (min(dataType, 31): the same property type)
            const int ctype = (int)(ce >> 19) & 0xff;
            PropRaw p = prop_init((int32_t)L, (int32_t)c, (int32_t)nfeat);
            p.name_off = o + 1;
            p.name_len = n;
            p.type = genc_prop_type(dtype);
            p.ctype = ctype;
            const bool localized = p.type == COVT_PROP_STRING && ctype == 2;
            if (localized && ns > (uint32_t)kPropMaxStreams) return kFastFallback;  // (the table's bound)
            o += (int32_t)(ce & 0xffu);
            // the column's role streams in lanes 0..3 (lane = StreamType, the last stream of a role wins): a
            // select per field, where prop_stream on the record in scalar registers cost ~24 scalar
            // instructions per stream (the walk is bound by scalar issue)
            int64_t v_off = -1;
            int32_t v_nv = 0, v_bl = 0, v_enc = 0;
            for (uint32_t s = 0; s < ns; ++s) {
                const int32_t q = f.at_run(o);
                const uint32_t se = (uint32_t)__builtin_amdgcn_readfirstlane((int)f.fs->stab[q]);
                const uint32_t re = (uint32_t)__builtin_amdgcn_readfirstlane((int)f.fr->rtab[q]);
                const int enc = __builtin_amdgcn_readfirstlane((int)f.fr->etab[q]);
                if (!se) return kFastFallback;
                const int type = (int)(re >> 28) - 1;
                const int32_t nv = (int32_t)(re & 0x0fffffffu);
                const int32_t bl = (int32_t)(se >> 8);
                const uint32_t role = type >= ST_PRESENT && type <= ST_DICTIONARY ? 1u << type : 0u;
                if (localized) {  // (the names' hashes: after the column, a lane per stream)
                    const int32_t sn = (int32_t)(f.upeek8(q) & 0xffu);
                    uint32_t rl = role;
                    if (sn > 8 && f.upeek8(q + 1) == pk("present_", 0, 8)) rl |= PR_PRESENT_LANG;
                    tab.set(s, PropSm{0u, 0u, o + 1, sn, nv, bl, (int32_t)d, (uint16_t)enc, (uint16_t)rl});
                } else if (role) {  // the roles applied in metadata order (the last stream of a role wins)
                    const bool me = threadIdx.x == (uint32_t)type;
                    v_off = me ? d : v_off;
                    v_nv = me ? nv : v_nv;
                    v_bl = me ? bl : v_bl;
                    v_enc = me ? enc : v_enc;
                }
                d += bl;
                o += (int32_t)(se & 0xffu);
            }
            if (localized) {
                names_hash_lanes(f.t, f.len, tab, ns);
                prop_localized(r, pe, tab, ns, p);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    p.s_off[q] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v_off >> 32), q) << 32) |
                                           (uint32_t)__builtin_amdgcn_readlane((int)v_off, q));
                    p.s_nv[q] = __builtin_amdgcn_readlane(v_nv, q);
                    p.s_bl[q] = __builtin_amdgcn_readlane(v_bl, q);
                    p.s_enc[q] = __builtin_amdgcn_readlane(v_enc, q);
                }
                pe(p);
            }
        }
        if (d > (int64_t)(len - o)) return kFastFallback;
        pe.layer_end(o);
        o += (int32_t)d;
    }
    return o == len ? COVT_OK : kFastFallback;
}

// Gen D property records (walk_gend's props branch): the implicit present stream, then data / length /
// dictionary in TreeMap<StreamType> order (the last metadata entry of a type)
template <class PE>
__device__ int prop_walk_gend(Rd<true>& r, PE& pe) {
    const int32_t len = (int32_t)r.len;
    int32_t o = 0;
    int32_t layer = 0;
    while (o < len) {
        const bool optimized = r.at(o++) & 1;
        int32_t v, extent, nfeat, ncols;
        if (!r.j4(o, v)) return COVT_ERR_TRUNCATED;
        if (!optimized) {
            if (v < 0 || v > len - o) return COVT_ERR_TRUNCATED;
            o += v;
        }
        if (!r.j4(o, extent) || !r.j4(o, nfeat) || !r.j4(o, ncols)) return COVT_ERR_TRUNCATED;
        if (ncols < 0 || ncols > 4096) return COVT_ERR_BAD_HEADER;
        const int32_t meta = o;
        for (int32_t ci = 0; ci < ncols; ++ci) {  // skip the metadata (checked by the Id / Geometry walk)
            int32_t x;
            if (optimized || ci == 0) {
                if (!r.j4(o, x)) return COVT_ERR_TRUNCATED;
            } else {
                if (!r.j4(o, x) || x < 0 || x > len - o) return COVT_ERR_TRUNCATED;
                o += x;
            }
            if (o >= len) return COVT_ERR_TRUNCATED;
            const int desc = r.at(o++), dtype = (desc >> 3) & 0xF, ctype = desc & 0x7;
            if (ctype > 4) return COVT_ERR_BAD_HEADER;
            for (;;) {
                if (o >= len) return COVT_ERR_TRUNCATED;
                const int sd = r.at(o++), type = sd >> 4, enc = sd & 0xF;
                if (type > ST_M || enc > 9) return COVT_ERR_BAD_HEADER;
                int32_t nv, bl;
                if (!r.j4(o, nv) || !r.j4(o, bl)) return COVT_ERR_TRUNCATED;
                if ((dtype == 8 && type == ST_VERTEX_BUFFER) || (type == ST_DATA && ctype == CT_PLAIN) ||
                    type == ST_DICTIONARY)
                    break;
            }
        }
        int32_t m = meta;
        int64_t d = o;
        pe.layer_begin();
        for (int32_t ci = 0; ci < ncols; ++ci) {
            int32_t x, kind;
            int32_t name_off = -1, name_len = 0;
            if (optimized || ci == 0) {
                r.j4(m, x);
                kind = x == 0 ? 0 : (x == 1 ? 1 : 2);
            } else {
                r.j4(m, x);
                kind = COVT_IS(m, x, "id") ? 0 : COVT_IS(m, x, "geometry") ? 1 : 2;
                name_off = m;
                name_len = x;
                m += x;
            }
            const int desc = r.at(m++), dtype = (desc >> 3) & 0xF, ctype = desc & 0x7;
            const int32_t s0 = m;
            uint32_t have = 0;
            for (;;) {
                const int sd = r.at(m++), type = sd >> 4;
                int32_t nv, bl;
                r.j4(m, nv);
                r.j4(m, bl);
                have |= 1u << type;
                if ((dtype == 8 && type == ST_VERTEX_BUFFER) || (type == ST_DATA && ctype == CT_PLAIN) ||
                    type == ST_DICTIONARY)
                    break;
            }
            PropRaw p = prop_init(layer, ci, nfeat);
            if (kind == 2 && dtype != 0) {  // the implicit present stream
                const int32_t pl = r.byte_rle_length((int32_t)d, nfeat < 0 ? 0 : (int32_t)(((int64_t)nfeat + 7) / 8));
                if (pl < 0) return COVT_ERR_TRUNCATED;
                prop_stream(p, 0, d, nfeat, pl, 7);
                d += pl;
            }
            for (int type = 0; type < 12; ++type) {
                if (!(have >> type & 1) || (kind == 2 && type == ST_PRESENT)) continue;
                int enc = 0;
                int32_t nv = 0, bl = 0;
                for (int32_t q = s0; q < m;) {  // the last entry of this type
                    const int sd = r.at(q++);
                    int32_t a, b;
                    r.j4(q, a);
                    r.j4(q, b);
                    if ((sd >> 4) == type) enc = sd & 0xF, nv = a, bl = b;
                }
                if (bl < 0) return COVT_ERR_BAD_HEADER;
                if (type > ST_PRESENT && type <= ST_DICTIONARY) prop_stream(p, type, d, nv, bl, enc);
                d += bl;
            }
            if (d > len) return COVT_ERR_TRUNCATED;
            if (kind == 2) {
                p.name_off = name_off;
                p.name_len = name_len;
                p.type = gend_prop_type(dtype);
                p.ctype = ctype;
                pe(p);
            }
        }
        pe.layer_end(0);
        o = (int32_t)d;
        ++layer;
    }
    return COVT_OK;
}

struct PropCountEmit {
    int64_t n = 0;
    __device__ void operator()(const PropRaw&) { ++n; }
    __device__ void layer_begin() {}
    __device__ void layer_end(int64_t) {}
};
struct PropRecEmit {
    PropRaw* recs;    // this tile's first record
    int32_t* rtile;   // (null: the tile's slots, no tile column)
    int32_t t;
    int64_t n = 0, k0 = 0;
    int64_t cap = INT64_MAX;  // records kept (slots: kPropSlots; the rest are only counted)
    __device__ void operator()(const PropRaw& q) {
        if (threadIdx.x == 0 && n < cap) {
            recs[n] = q;
            if (rtile) rtile[n] = t;
        }
        ++n;
    }
    __device__ void layer_begin() { k0 = n; }
    __device__ void layer_end(int64_t data_start) {  // Gen C: data offsets relative to the layer's data start
        if (!data_start) return;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        const int64_t e = n < cap ? n : cap;
        for (int64_t j = k0 + threadIdx.x; j < e; j += 64)
            for (int q = 0; q < 4; ++q)
                if (recs[j].s_off[q] >= 0) recs[j].s_off[q] += data_start;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
};

// a tile's property records: Gen C through the fast walk first (the serial walk on a fallback)
template <class PE>
__device__ __forceinline__ int prop_walk_tile(Rd<true>& r, PE& e, PropTab& tab, int32_t format) {
    if (format != COVT_FORMAT_GENC) return prop_walk_gend(r, e);
    FastGenc f;
    f.t = r.t;
    f.len = (int32_t)r.len;
    f.wb = -(int32_t)0x40000000;
    f.segs = 0;
    f.lim = 0;
    f.fs = (FastSmem*)((uint8_t*)covt_walk_win + kFastSmemOffset);
    f.fr = (FastSmemRec*)((uint8_t*)covt_walk_win + kPropRecOffset);
    const PE fresh = e;
    const int st = prop_walk_genc_fast(f, r, e, tab);
    if (st != kFastFallback) return st;
    e = fresh;
    return prop_walk_genc(r, e, tab);
}

// one wave per tile (tiles the Id / Geometry walk failed contribute nothing).  EMIT false: count the
// records, keeping the first kPropSlots of each tile in its slots (`recs` = the slot array, null: count
// only); EMIT true: write them at pcb[t] -- only for the tiles with more records than slots when `pcnt` is
// given (the others are copied from their slots by prop_compact)
constexpr int kPropSlots = 256;
constexpr size_t kPropSlotBytes = (size_t)2 << 30;  // slot memory a plan may take (10k tiles: 328 MB)
// The two walks read the same metadata as the Id / Geometry walk, which accepted the tile, so they cannot
// fail on it; if one does anyway (a divergence between the walkers) the count walk raises `diverged` and
// the plan fails with COVT_ERR_BAD_HEADER instead of dropping the tile's property columns, and the emit
// walk never writes past the records its count walk found (pcb[t + 1] - pcb[t]).
template <bool EMIT>
__global__ void prop_walk(const uint8_t* __restrict__ bytes, uint64_t n_bytes, const uint64_t* __restrict__ offs,
                          const uint64_t* __restrict__ sizes, int32_t n_tiles, int32_t format,
                          const int32_t* __restrict__ status, int64_t* __restrict__ pcnt,
                          const int64_t* __restrict__ pcb, PropRaw* __restrict__ recs, int32_t* __restrict__ rtile,
                          const uint32_t* __restrict__ order, unsigned long long* __restrict__ diverged,
                          bool slotted) {
    int32_t t = (int32_t)blockIdx.x;
    if (t > n_tiles) return;
    if (order && t < n_tiles) t = (int32_t)order[t];  // (largest tiles first)
    if (t == n_tiles || status[t]) {  // (t == n_tiles: the prefix sum's total slot)
        if (!EMIT && threadIdx.x == 0) pcnt[t] = 0;
        return;
    }
    if (EMIT && pcnt[t] <= kPropSlots && slotted) return;  // (in its slots)
    Rd<true> r;
    r.t = bytes + offs[t];
    r.len = (int64_t)sizes[t];
    r.wo = -(int64_t)0x40000000;
    PropTab tab;
    if (EMIT) {
        PropRecEmit e{recs + pcb[t], rtile + pcb[t], t};
        e.cap = pcb[t + 1] - pcb[t];
        (void)prop_walk_tile(r, e, tab, format);
    } else if (recs) {
        PropRecEmit e{recs + (size_t)t * kPropSlots, nullptr, t};
        e.cap = kPropSlots;
        const int st = prop_walk_tile(r, e, tab, format);
        if (threadIdx.x == 0) {
            pcnt[t] = st ? 0 : e.n;
            if (st) atomicOr(diverged, 1ull);
        }
    } else {
        PropCountEmit e;
        const int st = prop_walk_tile(r, e, tab, format);
        if (threadIdx.x == 0) {
            pcnt[t] = st ? 0 : e.n;
            if (st) atomicOr(diverged, 1ull);
        }
    }
}

// the records of the tiles whose records fit their slots -> their place at pcb[t] (a wave per tile)
__global__ void __launch_bounds__(64) prop_compact(const PropRaw* __restrict__ slots, const int64_t* __restrict__ pcnt,
                                                   const int64_t* __restrict__ pcb, int32_t n_tiles,
                                                   PropRaw* __restrict__ recs, int32_t* __restrict__ rtile) {
    const int32_t t = (int32_t)blockIdx.x;
    if (t >= n_tiles) return;
    const int64_t n = pcnt[t];
    if (n <= 0 || n > kPropSlots) return;
    static_assert(sizeof(PropRaw) % 16 == 0, "records copy as 16-byte words");
    constexpr int kW = (int)(sizeof(PropRaw) / 16);
    const uint4* src = (const uint4*)(slots + (size_t)t * kPropSlots);
    uint4* dst = (uint4*)(recs + pcb[t]);
    for (int64_t i = threadIdx.x; i < n * kW; i += 64) dst[i] = src[i];
    for (int64_t i = threadIdx.x; i < n; i += 64) rtile[pcb[t] + i] = t;
}

enum { PA_IN = 0, PA_PAYLOAD = 1, PA_LANE = 2, PA_COST = 3, PA_CMAX = 4, PA_DIVERGED = 7, PA_N = 8 };
// a thread per record: its decode streams (prop_streams), their count and aligned output bytes, and the
// records' totals (stream / in-place bytes, payload, lane-family streams, split cost and its maximum)
__global__ void __launch_bounds__(256) prop_sizes(const PropRaw* __restrict__ recs, int64_t n_rec, int32_t id_mode,
                                                  int32_t lane_max, int64_t* __restrict__ rs_cnt,
                                                  int64_t* __restrict__ rs_ob, unsigned long long* __restrict__ acc) {
    __shared__ unsigned long long part[4][5];
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long a[5] = {0, 0, 0, 0, 0};
    if (r < n_rec) {
        const PropRaw q = recs[r];
        PropStreams ps;
        prop_streams(q, id_mode, ps);
        int64_t ob = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {  // (k: the role)
            if (!(ps.has >> k & 1u)) continue;
            const int64_t bytes = ps.count[k] * ps.elem[k];
            const int32_t bl = q.s_bl[k];
            ob = align_out(ob + bytes);
            a[PA_PAYLOAD] += (unsigned long long)bytes;
            a[PA_LANE] += lane_stream(ps.op[k], (int32_t)ps.count[k], bl, lane_max) ? 1ull : 0ull;
            const unsigned long long c = (unsigned long long)((int64_t)bl + bytes / 4);
            a[PA_COST] += c;
            a[PA_CMAX] = c > a[PA_CMAX] ? c : a[PA_CMAX];
        }
        a[PA_IN] = (unsigned long long)ps.in_bytes;
        rs_cnt[r] = ps.n;
        rs_ob[r] = ob;
    } else if (r == n_rec) {
        rs_cnt[r] = 0;
        rs_ob[r] = 0;
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const unsigned long long x = __shfl_xor(a[k], d, 64);
            a[k] = k == PA_CMAX ? (x > a[k] ? x : a[k]) : a[k] + x;
        }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 5; ++k) part[threadIdx.x >> 6][k] = a[k];
    __syncthreads();
    if (threadIdx.x < 5) {
        unsigned long long x = 0;
        for (int w = 0; w < 4; ++w) {
            const unsigned long long y = part[w][threadIdx.x];
            x = threadIdx.x == PA_CMAX ? (y > x ? y : x) : x + y;
        }
        if (threadIdx.x == PA_CMAX) atomicMax(&acc[PA_CMAX], x);
        else if (x) atomicAdd(&acc[threadIdx.x], x);
    }
}

// each tile's streams and output bytes: its Id / Geometry ones + its records' (slot n_tiles: 0)
__global__ void tile_totals(const int64_t* __restrict__ cnt, const int64_t* __restrict__ ob, const int64_t* __restrict__ pcb,
                            const int64_t* __restrict__ rsb, const int64_t* __restrict__ rob, int32_t n_tiles,
                            int64_t* __restrict__ tc, int64_t* __restrict__ to) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > n_tiles) return;
    if (t == n_tiles) {
        tc[t] = to[t] = 0;
        return;
    }
    const int64_t r0 = pcb[t], r1 = pcb[t + 1];
    tc[t] = cnt[t] + (rsb[r1] - rsb[r0]);
    to[t] = ob[t] + (rob[r1] - rob[r0]);
}

// a thread per record: its stream entries (after the tile's Id / Geometry streams, output slices after
// theirs, as plan_property appends them) and its covt_prop_info / flags
__global__ void prop_fill(const PropRaw* __restrict__ recs, const int32_t* __restrict__ rtile, int64_t n_rec,
                          int32_t id_mode, const uint64_t* __restrict__ offs, const int64_t* __restrict__ cnt,
                          const int64_t* __restrict__ ob, const int64_t* __restrict__ cb, const int64_t* __restrict__ obb,
                          const int64_t* __restrict__ pcb, const int64_t* __restrict__ rsb, const int64_t* __restrict__ rob,
                          covt_stream_info* __restrict__ info, int32_t* __restrict__ nvals, covt_prop_info* __restrict__ pinfo,
                          uint16_t* __restrict__ pflags, int64_t* __restrict__ pin, uint32_t* __restrict__ keys,
                          int32_t lm) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rec) return;
    const int32_t t = rtile[r];
    const PropRaw q = recs[r];
    PropStreams ps;
    prop_streams(q, id_mode, ps);
    const int64_t r0 = pcb[t];
    int64_t si_k = cb[t] + cnt[t] + (rsb[r] - rsb[r0]);
    int64_t out = obb[t] + ob[t] + (rob[r] - rob[r0]);
    const int64_t tile_off = (int64_t)offs[t];
    covt_prop_info pi = prop_info_of(q, t, tile_off);
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // (k: the role)
        if (!(ps.has >> k & 1u)) continue;
        const int role = k;
        const int32_t cnt_k = (int32_t)ps.count[k];
        covt_stream_info si;
        si.tile = t;
        si.layer = q.layer;
        si.column_kind = 2;
        si.stream_type = role;
        si.encoding = q.s_enc[k];
        si.column_type = q.ctype;
        si.num_values = q.s_nv[k];
        si.byte_length = q.s_bl[k];
        si.num_bits = 0;
        si.op = ps.op[k];
        si.elem_bytes = ps.elem[k];
        si.desc_index = -1;
        si.in_off = tile_off + q.s_off[k];
        si.out_elems = ps.count[k];
        si.out_off = out;
        out = align_out(out + ps.count[k] * ps.elem[k]);
        info[si_k] = si;
        nvals[si_k] = cnt_k;
        if (keys) keys[si_k] = entry_key(si.op, cnt_k, si.byte_length, si.out_elems, si.elem_bytes, lm);
        pi.stream[k] = (int32_t)si_k;
        ++si_k;
    }
    pin[2 * r] = pi.out_off[1];  // the FLOAT data / STRING dictionary input offsets (plan_property_layout's
    pin[2 * r + 1] = pi.out_off[3];  // in_float / in_dict)
    pinfo[r] = pi;
    pflags[r] = ps.flags;
}

// property output layout (plan_property_layout): bytes per record, then their offsets
__global__ void prop_layout(const covt_prop_info* __restrict__ pinfo, const uint16_t* __restrict__ pflags, int64_t n_rec,
                            int64_t* __restrict__ psz) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > n_rec) return;
    if (r == n_rec) {
        psz[r] = 0;
        return;
    }
    const covt_prop_info pi = pinfo[r];
    const bool own = (pflags[r] & COVT_PROP_DICT_OWNER) != 0;
    int64_t sz[4];
    prop_layout_sizes(pi, own, sz);
    psz[r] = sz[0] + sz[1] + (pi.type == COVT_PROP_STRING && own ? sz[2] + sz[3] : 0);
}
__global__ void prop_layout_fill(covt_prop_info* __restrict__ pinfo, const uint16_t* __restrict__ pflags, int64_t n_rec,
                                 const int64_t* __restrict__ poff) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rec) return;
    covt_prop_info& pi = pinfo[r];
    const bool own = (pflags[r] & COVT_PROP_DICT_OWNER) != 0;
    int64_t sz[4];
    prop_layout_sizes(pi, own, sz);
    const int64_t off = poff[r];
    pi.out_off[0] = off;
    pi.out_off[1] = off + sz[0];
    if (pi.type == COVT_PROP_STRING && own) {
        pi.out_off[2] = off + sz[0] + sz[1];
        pi.out_off[3] = off + sz[0] + sz[1] + sz[2];
        return;
    }
    pi.out_off[2] = pi.out_off[3] = -1;
    if (pi.type != COVT_PROP_STRING || pi.lang <= 0 || r - pi.lang < 0) return;
    // a localized sub-column shares its column's dictionary: the owner is language 0, lang rows back
    const int64_t w = r - pi.lang;
    const covt_prop_info& po = pinfo[w];
    if (!(pflags[w] & COVT_PROP_DICT_OWNER) || po.tile != pi.tile || po.layer != pi.layer || po.column != pi.column)
        return;
    int64_t so[4];
    prop_layout_sizes(po, true, so);
    pi.out_off[2] = poff[w] + so[0] + so[1];
    pi.out_off[3] = poff[w] + so[0] + so[1] + so[2];
}
__global__ void prop_order_keys(const covt_prop_info* __restrict__ pinfo, int64_t n_rec, uint64_t* __restrict__ keys,
                                uint32_t* __restrict__ vals) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rec) return;
    keys[r] = prop_order_key(pinfo[r]);
    vals[r] = (uint32_t)r;
}
// the sort's order -> each record's row (so prop_desc_fill reads the records in order and scatters only
// its descriptor writes: gathering a record, its streams and flags per row was 182 us on the 10k batch)
__global__ void prop_rank(const uint32_t* __restrict__ order, int64_t n_rec, uint32_t* __restrict__ rank) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n_rec) rank[order[k]] = (uint32_t)k;
}
__global__ void prop_desc_fill(covt_prop_info* __restrict__ pinfo, const uint16_t* __restrict__ pflags,
                               const int64_t* __restrict__ pin, const uint32_t* __restrict__ rank, int64_t n_rec,
                               const covt_stream_info* __restrict__ info, covt_prop_desc* __restrict__ pdesc) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rec) return;
    const uint32_t k = rank[r];
    covt_prop_info& pi = pinfo[r];
    auto s_out = [&](int role) -> int64_t { return pi.stream[role] >= 0 ? info[pi.stream[role]].out_off : -1; };
    covt_prop_desc d;
    d.present_off = s_out(0);
    d.data_off = pi.type == COVT_PROP_FLOAT ? pin[2 * r] : s_out(1);
    d.length_off = s_out(2);
    d.dict_in_off = pi.type == COVT_PROP_STRING ? pin[2 * r + 1] : -1;
    for (int m = 0; m < 4; ++m) d.out_off[m] = pi.out_off[m];
    for (int m = 0; m < 3; ++m) d.res[m] = pi.stream[m] >= 0 ? info[pi.stream[m]].desc_index : -1;
    d.n_features = pi.n_features;
    d.n_data = pi.n_data;
    d.n_dict = pi.n_dict;
    d.dict_bytes = pi.dict_bytes;
    d.type = (int16_t)pi.type;
    d.flags = (int16_t)pflags[r];
    pi.desc_index = (int32_t)k;
    pdesc[k] = d;
}

// ---- Geometry columns (covt_device_plan_geometry; covt_host.cpp plan_geometry): a column is a run of
// adjacent geometry streams of one (tile, layer); its record holds the source streams, the assembly
// capacities and its six 16-byte aligned output slices; descriptors go largest (coordinates +
// features) first, ties in tile order.
__device__ __forceinline__ bool geo_same(const covt_stream_info& a, const covt_stream_info& b) {
    return a.column_kind == 1 && b.column_kind == 1 && a.tile == b.tile && a.layer == b.layer;
}
__global__ void geom_mark(const covt_stream_info* __restrict__ info, int64_t ns, int64_t* __restrict__ gst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > ns) return;
    gst[i] = i < ns && info[i].column_kind == 1 && !(i > 0 && geo_same(info[i - 1], info[i])) ? 1 : 0;
}
__global__ void geom_columns(const covt_stream_info* __restrict__ info, int64_t ns, int32_t format,
                             const int64_t* __restrict__ gst, const int64_t* __restrict__ gpos,
                             covt_geom_info* __restrict__ ginfo, int64_t* __restrict__ colbytes) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ns || !gst[i]) return;
    const covt_stream_info& s0 = info[i];
    covt_geom_info g{};
    g.tile = s0.tile;
    g.layer = s0.layer;
    g.column_type = s0.column_type;
    for (int k = 0; k < 6; ++k) g.stream[k] = -1;
    int64_t len[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t j = i; j < ns && geo_same(s0, info[j]); ++j) {
        const covt_stream_info& s = info[j];
        const int k = s.stream_type - ST_GEOMETRY_TYPES;
        if (k < 0 || k > 5) continue;
#pragma unroll
        for (int m = 0; m < 6; ++m) {  // (constant indices: g and len stay in registers, not scratch)
            if (m != k) continue;
            g.stream[m] = (int32_t)j;
            len[m] = m == 5 ? s.out_elems / 2 : s.out_elems;  // vertexBuffer: x,y pairs
        }
        if (k == 5) g.column_type = s.column_type;
    }
    g.n_features = (int32_t)len[0];
    const int64_t vs = g.stream[4] >= 0 ? len[4] : len[5];
    const int64_t pcap = vs + len[2], rcap = vs + len[2] + len[3];
    g.flags = (format == COVT_FORMAT_GENC && (g.column_type == CT_ICE || g.column_type == CT_ICE_MORTON))
                  ? (int32_t)COVT_GEOM_CLOSED_IN_STREAM : 0;
    const int64_t ccap = vs + ((g.flags & COVT_GEOM_CLOSED_IN_STREAM) ? 0 : len[3]);
    const bool fits = rcap <= COVT_GEOM_MAX_CAP && ccap <= COVT_GEOM_MAX_CAP && len[0] <= COVT_GEOM_MAX_CAP;
    g.part_cap = fits ? (int32_t)pcap : 0;
    g.ring_cap = fits ? (int32_t)rcap : 0;
    g.coord_cap = fits ? (int32_t)ccap : 0;
    if (!fits) g.flags = (int32_t)((uint32_t)g.flags | COVT_GEOM_TOO_LARGE);
    const int64_t nf = fits ? len[0] : 0;
    const int64_t bytes[6] = {4 * (nf + 1), 4 * ((int64_t)g.part_cap + 1), 4 * ((int64_t)g.ring_cap + 1),
                              8 * (int64_t)g.coord_cap, 4 * (int64_t)g.part_cap, 4 * (int64_t)g.ring_cap};
    int64_t off = 0;
    for (int k = 0; k < 6; ++k) {  // local to the column; geom_keys adds its base
        g.out_off[k] = off;
        off = align16(off + bytes[k]);
    }
    const int64_t c = gpos[i];
    ginfo[c] = g;
    colbytes[c] = off;
}
__global__ void geom_keys(covt_geom_info* __restrict__ ginfo, int64_t nc, const int64_t* __restrict__ coloff,
                          uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    covt_geom_info& g = ginfo[c];
    for (int k = 0; k < 6; ++k) g.out_off[k] += coloff[c];
    keys[c] = (1ull << 40) - (uint64_t)((int64_t)g.coord_cap + g.n_features);
    vals[c] = (uint32_t)c;
}
__global__ void geom_descs(const covt_stream_info* __restrict__ info, covt_geom_info* __restrict__ ginfo,
                           const uint32_t* __restrict__ order, int64_t nc, covt_geom_desc* __restrict__ gdesc) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nc) return;
    covt_geom_info& g = ginfo[order[k]];
    covt_geom_desc d{};
    for (int m = 0; m < 6; ++m) {
        const int32_t si = g.stream[m];
        d.in_off[m] = si >= 0 ? info[si].out_off : -1;
        d.in_len[m] = si >= 0 ? (int32_t)(m == 5 ? info[si].out_elems / 2 : info[si].out_elems) : 0;
        d.in_res[m] = si >= 0 ? info[si].desc_index : -1;  // its decode status gates the column
        d.out_off[m] = g.out_off[m];
    }
    d.part_cap = g.part_cap;
    d.ring_cap = g.ring_cap;
    d.coord_cap = g.coord_cap;
    d.flags = g.flags;
    g.desc_index = (int32_t)k;
    gdesc[k] = d;
}

size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }


}  // namespace

#ifdef COVT_PLAN_TIMING
extern "C" int covt_debug_walk_clock(void* p) {  // 2 x n_tiles uint64 on the device (null: off)
    return hipMemcpyToSymbol(HIP_SYMBOL(covt_walk_clock), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif
extern "C" {

int covt_device_plan_create(const uint8_t* d_bytes, uint64_t n_bytes, const uint64_t* d_tile_offsets,
                            const uint64_t* d_tile_sizes, int32_t n_tiles, int32_t format, int32_t id_mode,
                            void* hip_stream, covt_device_plan** out) {
    return covt_device_plan_create_opts(d_bytes, n_bytes, d_tile_offsets, d_tile_sizes, n_tiles, format, id_mode,
                                        nullptr, hip_stream, out);
}

int covt_device_plan_create_opts(const uint8_t* d_bytes, uint64_t n_bytes, const uint64_t* d_tile_offsets,
                                 const uint64_t* d_tile_sizes, int32_t n_tiles, int32_t format, int32_t id_mode,
                                 const covt_plan_options* opts, void* hip_stream, covt_device_plan** out) {
    covt_plan_options o;
    if (!covt_resolve_options(opts, o) || (o.flags & ~COVT_PLAN_PROPERTIES)) return COVT_ERR_INVALID_ARG;
    const bool props = (o.flags & COVT_PLAN_PROPERTIES) != 0;
    if (!out || n_tiles < 0 || (n_tiles && (!d_bytes || !d_tile_offsets || !d_tile_sizes))) return COVT_ERR_INVALID_ARG;
    if (format != COVT_FORMAT_GENC && format != COVT_FORMAT_GEND) return COVT_ERR_INVALID_ARG;
    if (id_mode != COVT_ID_FORMAT && id_mode != COVT_ID_JAVA) return COVT_ERR_INVALID_ARG;
    *out = nullptr;
    auto* p = new covt_device_plan();
    p->n_tiles = n_tiles;
    p->format = format;
    p->id_mode = id_mode;
    hipStream_t s = (hipStream_t)hip_stream;
    auto fail = [&](int st) {
        covt_device_plan_destroy(p);
        return st;
    };
#define DCHK(x)                                   \
    do {                                          \
        if ((x) != hipSuccess) return fail(COVT_ERR_DEVICE); \
    } while (0)
    DCHK(hipGetDevice(&p->dev));
    const size_t nt1 = (size_t)n_tiles + 1;
    // tile arena: status | cnt | ob | cnt_base | ob_base | totals | head | per-tile sums | per-tile costs |
    // scan scratch | slots
    size_t scan_tmp = 0;
    DCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (int64_t*)nullptr, (int64_t*)nullptr, (int)nt1, s));
    // [+ properties: per-tile record counts | their prefix | streams and output bytes per tile | totals]
    const size_t o_cnt = up256(nt1 * 4), o_ob = o_cnt + up256(nt1 * 8), o_cb = o_ob + up256(nt1 * 8),
                 o_obb = o_cb + up256(nt1 * 8), o_tot = o_obb + up256(nt1 * 8), o_head = o_tot + up256(T_N * 8),
                 o_ts = o_head + 256, o_tc = o_ts + up256(nt1 * 32), o_tmp = o_tc + up256(nt1 * 16),
                 o_pc = o_tmp + up256(scan_tmp), o_pcb = o_pc + (props ? up256(nt1 * 8) : 0),
                 o_ttc = o_pcb + (props ? up256(nt1 * 8) : 0), o_tto = o_ttc + (props ? up256(nt1 * 8) : 0),
                 o_pacc = o_tto + (props ? up256(nt1 * 8) : 0), o_slots = o_pacc + (props ? 256 : 0);
    // device_walk 0: a wave per tile with per-tile slots; 1: the same walk twice; k >= 2: k lanes per workgroup
    const int wl = o.device_walk >= 2 ? o.device_walk : 0;
    const bool use_slots = o.device_walk == 0;
    const size_t tile_bytes = o_slots + (use_slots ? up256((size_t)n_tiles * kSlots * sizeof(RawStream)) : 0);
    DCHK(plan_malloc(&p->tile_arena, tile_bytes, p->dev, s));
    uint8_t* ta = (uint8_t*)p->tile_arena;
    p->d_status = (int32_t*)ta;
    int64_t *cnt = (int64_t*)(ta + o_cnt), *ob = (int64_t*)(ta + o_ob), *cb = (int64_t*)(ta + o_cb),
            *obb = (int64_t*)(ta + o_obb), *head = (int64_t*)(ta + o_head), *tcost = (int64_t*)(ta + o_tc);
    auto* totals = (unsigned long long*)(ta + o_tot);
    auto* tsum = (long long*)(ta + o_ts);
    DCHK(hipMemsetAsync(totals, 0, T_N * 8, s));
    DCHK(hipMemsetAsync(tsum, 0, nt1 * 32, s));  // failed tiles leave zeros
    const int64_t fpf_w = o.fpf_split_weight;
    const int32_t lane_max = lane_limits(o.lane_max_bytes, o.lane_max_values);
    const int64_t lane_min = o.lane_min_streams;
    // 0: a wave per tile, its lanes in lockstep; k > 0: k lanes per workgroup, a lane per tile
    RawStream* slots = use_slots ? (RawStream*)(ta + o_slots) : nullptr;
    // property plans of more than 256 tiles: both walks largest tiles first (a stable descending sort of
    // the sizes)
    uint32_t* order = nullptr;
    void* order_mem = nullptr;
    if (props && n_tiles > 256) {
        size_t otmp = 0;
        DCHK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, otmp, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                          (const uint32_t*)nullptr, (uint32_t*)nullptr, n_tiles, 0, 40, s));
        const size_t nt = (size_t)n_tiles;
        DCHK(plan_malloc(&order_mem, up256(nt * 8) + 2 * up256(nt * 4) + up256(otmp), p->dev, s));
        uint8_t* om = (uint8_t*)order_mem;
        uint32_t* iota = (uint32_t*)(om + up256(nt * 8));
        order = (uint32_t*)(om + up256(nt * 8) + up256(nt * 4));
        tile_iota<<<(n_tiles + 255) / 256, 256, 0, s>>>(iota, n_tiles);
        const hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(
            om + up256(nt * 8) + 2 * up256(nt * 4), otmp, d_tile_sizes, (uint64_t*)om, iota, order, n_tiles, 0, 40, s);
        if (e != hipSuccess) {
            (void)hipFreeAsync(order_mem, s);
            return fail(COVT_ERR_DEVICE);
        }
    }
    struct OrderFree {  // (stream-ordered: after the walks that read it)
        void* m;
        hipStream_t q;
        ~OrderFree() { if (m) (void)hipFreeAsync(m, q); }
    } order_free{order_mem, s};
    const uint32_t* id_order = order;
    const uint32_t* prop_order = order;
    if (wl == 0)
        walk_count<true><<<(int)nt1, 64, kWalkLds, s>>>(d_bytes, n_bytes, d_tile_offsets, d_tile_sizes, n_tiles, format,
                                                        id_mode, p->d_status, cnt, ob, slots, fpf_w, tcost, id_order);
    else
        walk_count<false><<<(int)((nt1 + wl - 1) / wl), wl, (size_t)wl * 64 + 16, s>>>(
            d_bytes, n_bytes, d_tile_offsets, d_tile_sizes, n_tiles, format, id_mode, p->d_status, cnt, ob, nullptr,
            fpf_w, tcost, id_order);
    DCHK(hipGetLastError());
    // property columns: their records (a count walk, one D2H for the record count, the emitting walk), each
    // record's streams and output bytes, and each tile's totals = Id / Geometry + property
    int64_t *pcnt = nullptr, *pcb = nullptr, *rs_cnt = nullptr, *rs_ob = nullptr, *rsb = nullptr, *rob = nullptr;
    unsigned long long* pacc = nullptr;
    PropRaw* recs = nullptr;
    PropRaw* prop_slots = nullptr;  // the property walk's per-tile record slots (freed once copied)
    int32_t* rtile = nullptr;
    int64_t n_rec = 0;
    size_t pscan_tmp = 0, psort_tmp = 0;
    size_t po_rt = 0, po_rc = 0, po_ro = 0, po_rsb = 0, po_rob = 0, po_pi = 0, po_pf = 0, po_pin = 0, po_psz = 0,
           po_poff = 0, po_k0 = 0, po_k1 = 0, po_v0 = 0, po_v1 = 0, po_pd = 0, po_st = 0, po_sc = 0, prop_total = 0;
    const int64_t* scan_cnt = cnt;
    const int64_t* scan_ob = ob;
    if (props) {
        pcnt = (int64_t*)(ta + o_pc);
        pcb = (int64_t*)(ta + o_pcb);
        pacc = (unsigned long long*)(ta + o_pacc);
        DCHK(hipMemsetAsync(pacc, 0, 256, s));
        // one walk counting the records and keeping up to kPropSlots per tile (batches whose slots would
        // take more than kPropSlotBytes walk twice: count, then emit)
        void* pslots = nullptr;
        const size_t slot_bytes = (size_t)n_tiles * kPropSlots * sizeof(PropRaw);
        if (slot_bytes <= kPropSlotBytes && n_tiles > 0) DCHK(plan_malloc(&pslots, slot_bytes, p->dev, s));
        prop_slots = (PropRaw*)pslots;
        p->scratch = pslots;  // (a failure on the way frees it with the plan)
        prop_walk<false><<<(int)nt1, 64, kPropWalkLds, s>>>(d_bytes, n_bytes, d_tile_offsets, d_tile_sizes, n_tiles, format,
                                                           p->d_status, pcnt, nullptr, prop_slots, nullptr, prop_order,
                                                           pacc + PA_DIVERGED, prop_slots != nullptr);
        DCHK(hipGetLastError());
        DCHK(hipcub::DeviceScan::ExclusiveSum(ta + o_tmp, scan_tmp, pcnt, pcb, (int)nt1, s));
        unsigned long long head[2] = {0, 0};  // record count, walk divergence
        DCHK(hipMemcpyAsync(&head[0], pcb + n_tiles, 8, hipMemcpyDeviceToHost, s));
        DCHK(hipMemcpyAsync(&head[1], pacc + PA_DIVERGED, 8, hipMemcpyDeviceToHost, s));
        DCHK(hipStreamSynchronize(s));
        n_rec = (int64_t)head[0];
        if (head[1]) return fail(COVT_ERR_BAD_HEADER);  // the property walk failed a tile the Id walk accepted
        if (n_rec > 0x7fffffff) return fail(COVT_ERR_INVALID_ARG);
        const size_t nr = (size_t)(n_rec > 0 ? n_rec : 1), nr1 = nr + 1;
        DCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, pscan_tmp, (int64_t*)nullptr, (int64_t*)nullptr, (int)nr1, s));
        DCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, psort_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                (uint32_t*)nullptr, (uint32_t*)nullptr, (int)nr, 0, 41, s));
        // property arena: records | their tiles | stream counts | output bytes | both prefixes | infos | flags |
        // in-place input offsets | layout sizes | layout offsets | order keys / values in, out | descriptors |
        // sort scratch | scan scratch
        po_rt = up256(nr * sizeof(PropRaw));
        po_rc = po_rt + up256(nr * 4);
        po_ro = po_rc + up256(nr1 * 8);
        po_rsb = po_ro + up256(nr1 * 8);
        po_rob = po_rsb + up256(nr1 * 8);
        po_pi = po_rob + up256(nr1 * 8);
        po_pf = po_pi + up256(nr * sizeof(covt_prop_info));
        po_pin = po_pf + up256(nr * 2);
        po_psz = po_pin + up256(nr * 16);
        po_poff = po_psz + up256(nr1 * 8);
        po_k0 = po_poff + up256(nr1 * 8);
        po_k1 = po_k0 + up256(nr * 8);
        po_v0 = po_k1 + up256(nr * 8);
        po_v1 = po_v0 + up256(nr * 4);
        po_pd = po_v1 + up256(nr * 4);
        po_st = po_pd + up256(nr * sizeof(covt_prop_desc));
        po_sc = po_st + up256(psort_tmp);
        prop_total = po_sc + up256(pscan_tmp);
        DCHK(plan_malloc(&p->prop_arena, prop_total, p->dev, s));
        uint8_t* pa = (uint8_t*)p->prop_arena;
        recs = (PropRaw*)pa;
        rtile = (int32_t*)(pa + po_rt);
        rs_cnt = (int64_t*)(pa + po_rc);
        rs_ob = (int64_t*)(pa + po_ro);
        rsb = (int64_t*)(pa + po_rsb);
        rob = (int64_t*)(pa + po_rob);
        p->n_props = n_rec;
        p->d_pinfo = (covt_prop_info*)(pa + po_pi);
        p->d_pdesc = (covt_prop_desc*)(pa + po_pd);
        if (n_rec > 0) {
            if (prop_slots) {  // from the slots; the tiles with more records walk again
                prop_compact<<<n_tiles, 64, 0, s>>>(prop_slots, pcnt, pcb, n_tiles, recs, rtile);
                DCHK(hipGetLastError());
            }
            prop_walk<true><<<n_tiles, 64, kPropWalkLds, s>>>(d_bytes, n_bytes, d_tile_offsets, d_tile_sizes, n_tiles,
                                                             format, p->d_status, pcnt, pcb, recs, rtile, nullptr,
                                                             pacc + PA_DIVERGED, prop_slots != nullptr);
            DCHK(hipGetLastError());
        }
        if (prop_slots) {
            p->scratch = nullptr;
            DCHK(hipFreeAsync(prop_slots, s));  // (stream-ordered: after the copy)
            prop_slots = nullptr;
        }
        const int32_t lane_max0 = lane_limits(o.lane_max_bytes, o.lane_max_values);
        prop_sizes<<<(int)((nr1 + 255) / 256), 256, 0, s>>>(recs, n_rec, id_mode, lane_max0, rs_cnt, rs_ob, pacc);
        DCHK(hipGetLastError());
        DCHK(hipcub::DeviceScan::ExclusiveSum(pa + po_sc, pscan_tmp, rs_cnt, rsb, (int)(n_rec + 1), s));
        DCHK(hipcub::DeviceScan::ExclusiveSum(pa + po_sc, pscan_tmp, rs_ob, rob, (int)(n_rec + 1), s));
        int64_t *tcn = (int64_t*)(ta + o_ttc), *ton = (int64_t*)(ta + o_tto);
        tile_totals<<<(int)((nt1 + 255) / 256), 256, 0, s>>>(cnt, ob, pcb, rsb, rob, n_tiles, tcn, ton);
        DCHK(hipGetLastError());
        scan_cnt = tcn;
        scan_ob = ton;
    }
    DCHK(hipcub::DeviceScan::ExclusiveSum(ta + o_tmp, scan_tmp, scan_cnt, cb, (int)nt1, s));
    DCHK(hipcub::DeviceScan::ExclusiveSum(ta + o_tmp, scan_tmp, scan_ob, obb, (int)nt1, s));
    plan_head<<<1, 1024, 0, s>>>(cb, obb, tcost, n_tiles, head, pacc);
    DCHK(hipGetLastError());
    // Id / Geometry plans of many tiles skip the host synchronisation between the walk and the stream entries
    // (~57 us of the 10k-tile plan's 0.62 ms, profiles/r05): the stream arena is sized to a bound, the kernels
    // take the stream count from the device (head[0]), and the count and the split decision are checked at the
    // plan's final synchronisation -- a plan past the bound, or one that splits, runs this part again with the
    // counted sizes.  (Property plans synchronise for their record count anyway.)
    int64_t hd[4] = {0, 0, 0, 0};
    const int64_t spec_cap = std::min<int64_t>((int64_t)kSortFuseChunks * kSortChunk, (int64_t)n_tiles * kSpecCapPerTile);
    const bool spec = COVT_PLAN_SPEC && !props && wl == 0 && slots && o.split_max_streams > 0 &&
                      (int64_t)n_tiles * kSpecStreamsPerTile > o.split_max_streams;
    if (!spec) {
        DCHK(hipMemcpyAsync(hd, head, sizeof(hd), hipMemcpyDeviceToHost, s));
        DCHK(hipStreamSynchronize(s));
    }
    auto splits = [&](int64_t ns, int64_t& smin) {  // the split threshold (covt_plan_create_ex step 3)
        smin = o.split_min;
        if (smin >= 0 && o.split_ratio > 0) smin = std::max<int64_t>(smin, hd[2] / o.split_ratio);
        return smin >= 0 && ns > 0 && hd[3] > smin && (o.split_max_streams <= 0 || ns <= o.split_max_streams);
    };
    // the stream entries, their launch order and descriptors; sp: sized to spec_cap, nothing split
    auto stream_part = [&](bool sp) -> int {
    const int64_t ns = sp ? spec_cap : hd[0];
    const int64_t* dns = sp ? head : nullptr;
    const int64_t ecap = sp ? spec_cap : INT64_MAX;
    if (!sp) {
        p->n_streams = ns;
        p->n_descs = ns;
        p->out_bytes = hd[1];
    }
    if (ns > 0x7fffffff) return fail(COVT_ERR_INVALID_ARG);
    // nothing splits unless the largest cost passes the threshold
    int64_t smin = 0;
    const bool splitting = !sp && splits(ns, smin);
    const int64_t grow = split_grow_factor(hd[2], o.split_grow);
    const int64_t schunk = o.split_chunk * grow, svalues = o.split_values * grow;
    // stream arena: info | nvals | launch buckets | sorted buckets | launch order | bucket counts | descs [|
    // split: family | desc counts | offsets | RLE list | FastPFOR list | scan scratch]
    size_t dscan_tmp = 0;
    if (splitting)
        DCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, dscan_tmp, (int64_t*)nullptr, (int64_t*)nullptr, (int)(ns + 1), s));
    const size_t n = (size_t)(ns > 0 ? ns : 1);
    const int32_t nb = (int32_t)((n + kSortChunk - 1) / kSortChunk);  // counting-sort chunks
    // more chunks than one scatter workgroup sums itself: their counts scanned by hipcub into bscan
    const bool scanned = nb > kSortFuseChunks;
    const size_t mh = (size_t)kSortBuckets * nb;
    size_t hscan_tmp = 0;
    if (scanned)
        DCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, hscan_tmp, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)mh, s));
    // RLE chunk records: every candidate reserves (its cost / split_chunk + 2) <= the batch's
    const int64_t chunk_cap = splitting ? hd[2] / o.split_chunk + 2 * ns + 2 : 0;
    const size_t o_nv = up256(n * sizeof(covt_stream_info)), o_k0 = o_nv + up256(n * 4), o_k1 = o_k0 + up256(n * 4),
                 o_v0 = o_k1 + up256(n * 4), o_v1 = o_v0 + up256(n * 4), o_h = o_v1 + up256(n * 4),
                 o_hs = o_h + up256(mh * 4), o_ht = o_hs + (scanned ? up256(mh * 4) : 0),
                 o_d = o_ht + (scanned ? up256(hscan_tmp) : 0),
                 o_sf = o_d + up256(n * sizeof(covt_stream_desc)),
                 o_sn = o_sf + up256(n), o_dn = o_sn + up256(n * 8), o_dp = o_dn + up256((n + 1) * 8),
                 o_rl = o_dp + up256((n + 1) * 8), o_fl = o_rl + up256(n * 4), o_rb = o_fl + up256(n * 4),
                 o_rc = o_rb + up256(n * 8), o_ch = o_rc + up256(n * 4), o_ds = o_ch + up256((size_t)chunk_cap * 16),
                 stream_bytes = splitting ? o_ds + up256(dscan_tmp) : o_sf;
    DCHK(plan_malloc(&p->stream_arena, stream_bytes, p->dev, s));
    uint8_t* sa = (uint8_t*)p->stream_arena;
    p->d_info = (covt_stream_info*)sa;
    int32_t* nvals = (int32_t*)(sa + o_nv);
    uint32_t *q0 = (uint32_t*)(sa + o_k0), *q1 = (uint32_t*)(sa + o_k1), *v0 = (uint32_t*)(sa + o_v0),
             *v1 = (uint32_t*)(sa + o_v1);
    uint32_t* bhist = (uint32_t*)(sa + o_h);
    uint32_t* bscan = scanned ? (uint32_t*)(sa + o_hs) : bhist;
    p->d_order = v1;
    p->d_desc = (covt_stream_desc*)(sa + o_d);
    // launch order: the stable radix sort of the launch keys q0 (low byte: -> q1, v0; high byte: -> q0, v1)
    unsigned long long* fam_tot = splitting ? nullptr : totals + T_FAM;  // (split plans: stream_keys counts)
    auto launch_order = [&]() {
        for (int pass = 0; pass < 2; ++pass) {
            order_hist<<<nb, 256, 0, s>>>(pass ? q1 : q0, ns, nb, 8 * pass, bhist,
                                          pass == 0 && !splitting ? p->d_info : nullptr, nvals, lane_min, totals, dns);
            if (scanned) {
                const hipError_t e = hipcub::DeviceScan::ExclusiveSum(sa + o_ht, hscan_tmp, bhist, bscan, (int)mh, s);
                if (e != hipSuccess) return e;
            }
            if (pass == 0) order_scatter<<<nb, 1024, 0, s>>>(q0, nullptr, ns, nb, 0, bscan, scanned, q1, v0, nullptr, dns);
            else order_scatter<<<nb, 1024, 0, s>>>(q1, v0, ns, nb, 8, bscan, scanned, q0, v1, fam_tot, dns);
        }
        return hipGetLastError();
    };
    // unsplit plans: the launch keys written with the stream entries, taking every small RLE stream to the
    // lane family (the sort's first pass redoes them when the batch has fewer such streams than lane_min:
    // the count is known once the entries are written); split plans: stream_keys after split_mark
    uint32_t* ekeys = splitting ? nullptr : q0;
    const int32_t lm = lane_max;
    if (n_tiles) {
        if (slots) {
            emit_slots<<<n_tiles, 64, 0, s>>>(d_tile_offsets, n_tiles, id_mode, p->d_status, cnt, cb, obb, slots,
                                              lane_max, p->d_info, nvals, tsum, ekeys, lm, ecap);
            DCHK(hipGetLastError());
        }
        if (wl == 0)  // (with slots: only tiles with more than kSlots streams walk again)
            walk_emit<true><<<n_tiles, 64, kWalkLds, s>>>(d_bytes, n_bytes, d_tile_offsets, d_tile_sizes, n_tiles, format,
                                                          id_mode, p->d_status, cb, obb, lane_max, p->d_info, nvals, tsum,
                                                          slots ? cnt : nullptr, ekeys, lm, ecap);
        else
            walk_emit<false><<<(n_tiles + wl - 1) / wl, wl, (size_t)wl * 64 + 16, s>>>(
                d_bytes, n_bytes, d_tile_offsets, d_tile_sizes, n_tiles, format, id_mode, p->d_status, cb, obb,
                lane_max, p->d_info, nvals, tsum, nullptr, ekeys, lm, ecap);
        DCHK(hipGetLastError());
        reduce_tiles<<<1, 1024, 0, s>>>(tsum, n_tiles, totals, pacc);
        DCHK(hipGetLastError());
        if (props && n_rec > 0) {  // the property streams after each tile's Id / Geometry ones
            uint8_t* pa = (uint8_t*)p->prop_arena;
            prop_fill<<<(int)((n_rec + 255) / 256), 256, 0, s>>>(recs, rtile, n_rec, id_mode, d_tile_offsets, cnt, ob, cb,
                                                                 obb, pcb, rsb, rob, p->d_info, nvals, p->d_pinfo,
                                                                 (uint16_t*)(pa + po_pf), (int64_t*)(pa + po_pin), ekeys,
                                                                 lm);
            DCHK(hipGetLastError());
        }
    }
    const int blocks_s = (int)((ns + 255) / 256);
    if (ns > 0 && !splitting) {
        DCHK(launch_order());
        fill_descs<<<sp ? std::min(blocks_s, 2048) : blocks_s, 256, 0, s>>>(p->d_info, nvals, q0, v1, ns, p->d_desc, dns);
        DCHK(hipGetLastError());
    } else if (splitting) {
        auto* sfam = (uint8_t*)(sa + o_sf);
        auto *sndesc = (int64_t*)(sa + o_sn), *dn = (int64_t*)(sa + o_dn), *dpos = (int64_t*)(sa + o_dp);
        auto *rle_list = (uint32_t*)(sa + o_rl), *fpf_list = (uint32_t*)(sa + o_fl);
        const int walkers = (int)std::min<int64_t>(ns, 1024);
        split_mark<<<blocks_s, 256, 0, s>>>(p->d_info, nvals, ns, lane_max, lane_min, smin, schunk,
                                            svalues, fpf_w, totals, sfam, sndesc, rle_list, fpf_list);
        DCHK(hipGetLastError());
        auto* chunks = (int4*)(sa + o_ch);
        auto* rle_base = (int64_t*)(sa + o_rb);
        auto* rle_cons = (int32_t*)(sa + o_rc);
        rle_chunks_walk<<<walkers, 64, kStreamRdLds, s>>>(d_bytes, p->d_info, nvals, totals, rle_list, schunk, sfam,
                                                 sndesc, chunks, chunk_cap, rle_base, rle_cons);
        DCHK(hipGetLastError());
        stream_keys<<<blocks_s, 256, 0, s>>>(p->d_info, nvals, ns, lane_max, lane_min, totals, q0, sfam, sndesc);
        DCHK(hipGetLastError());
        DCHK(launch_order());
        gather_ndesc<<<(int)((ns + 256) / 256), 256, 0, s>>>(v1, sndesc, ns, dn);
        DCHK(hipGetLastError());
        DCHK(hipcub::DeviceScan::ExclusiveSum(sa + o_ds, dscan_tmp, dn, dpos, (int)(ns + 1), s));
        int64_t nd = 0;
        DCHK(hipMemcpyAsync(&nd, dpos + ns, 8, hipMemcpyDeviceToHost, s));
        DCHK(hipStreamSynchronize(s));
        // descriptor arena: descriptors | the stream of each
        DCHK(plan_malloc(&p->desc_arena, up256((size_t)nd * sizeof(covt_stream_desc)) + up256((size_t)nd * 4), p->dev, s));
        p->n_descs = nd;
        p->d_desc = (covt_stream_desc*)p->desc_arena;
        p->d_order = (uint32_t*)((uint8_t*)p->desc_arena + up256((size_t)nd * sizeof(covt_stream_desc)));
        fill_split_descs<<<(int)((nd + 255) / 256), 256, 0, s>>>(p->d_info, nvals, v1, dpos, ns, nd, sfam, schunk,
                                                                 svalues, chunks, rle_base, rle_cons, p->d_desc,
                                                                 p->d_order);
        DCHK(hipGetLastError());
        fpf_states_walk<<<walkers, 64, kStreamRdLds, s>>>(d_bytes, p->d_info, nvals, totals, fpf_list, svalues, p->d_desc);
        DCHK(hipGetLastError());
    }
    return COVT_OK;
    };
    {
        const int st = stream_part(spec);
        if (st) return st;  // (fail() has destroyed the plan)
    }

    if (props) {  // property output layout and the largest-first descriptor order (after the stream descriptors)
        uint8_t* pa = (uint8_t*)p->prop_arena;
        auto* pflags = (uint16_t*)(pa + po_pf);
        auto *psz = (int64_t*)(pa + po_psz), *poff = (int64_t*)(pa + po_poff);
        const int pb = (int)((n_rec + 256) / 256);
        prop_layout<<<pb, 256, 0, s>>>(p->d_pinfo, pflags, n_rec, psz);
        DCHK(hipGetLastError());
        DCHK(hipcub::DeviceScan::ExclusiveSum(pa + po_sc, pscan_tmp, psz, poff, (int)(n_rec + 1), s));
        DCHK(hipMemcpyAsync(&p->prop_bytes, poff + n_rec, 8, hipMemcpyDeviceToHost, s));
        if (n_rec > 0) {
            prop_layout_fill<<<pb, 256, 0, s>>>(p->d_pinfo, pflags, n_rec, poff);
            auto *pk0 = (uint64_t*)(pa + po_k0), *pk1 = (uint64_t*)(pa + po_k1);
            auto *pv0 = (uint32_t*)(pa + po_v0), *pv1 = (uint32_t*)(pa + po_v1);
            prop_order_keys<<<pb, 256, 0, s>>>(p->d_pinfo, n_rec, pk0, pv0);
            DCHK(hipGetLastError());
            DCHK(hipcub::DeviceRadixSort::SortPairs(pa + po_st, psort_tmp, pk0, pk1, pv0, pv1, (int)n_rec, 0, 41, s));
            prop_rank<<<pb, 256, 0, s>>>(pv1, n_rec, pv0);  // (pv0, the sort's input values, is free)
            prop_desc_fill<<<pb, 256, 0, s>>>(p->d_pinfo, pflags, (const int64_t*)(pa + po_pin), pv0, n_rec, p->d_info,
                                              p->d_pdesc);
            DCHK(hipGetLastError());
        }
    }
    unsigned long long tot[T_N];
    DCHK(hipMemcpyAsync(tot, totals, sizeof(tot), hipMemcpyDeviceToHost, s));
    if (spec) DCHK(hipMemcpyAsync(hd, head, sizeof(hd), hipMemcpyDeviceToHost, s));
    DCHK(hipStreamSynchronize(s));
    if (spec) {
        int64_t smin = 0;
        if (hd[0] > spec_cap || splits(hd[0], smin)) {  // past the bound, or a split plan: with the counted sizes
            ++p->spec_redo;
            DCHK(hipFreeAsync(p->stream_arena, s));
            p->stream_arena = nullptr;
            DCHK(hipMemsetAsync(totals + T_FAM, 0, COVT_NUM_FAMILIES * 8, s));
            const int st = stream_part(false);
            if (st) return st;
            DCHK(hipMemcpyAsync(tot, totals, sizeof(tot), hipMemcpyDeviceToHost, s));
            DCHK(hipStreamSynchronize(s));
        } else {
            p->n_streams = hd[0];
            p->n_descs = hd[0];
            p->out_bytes = hd[1];
        }
    }
#undef DCHK
    p->in_bytes = (int64_t)tot[T_IN];
    p->out_payload = (int64_t)tot[T_PAYLOAD];
    p->vertices = (int64_t)tot[T_VERTS];
    for (int f = 0; f < COVT_NUM_FAMILIES; ++f) p->fam_counts[f] = (int64_t)tot[T_FAM + f];
    *out = p;
    return COVT_OK;
}

int covt_device_plan_pool_trim(int device, uint64_t keep_bytes) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return COVT_ERR_INVALID_ARG;
    hipMemPool_t mp = plan_pool(device);
    if (!mp) return COVT_ERR_DEVICE;
    int cur = 0;
    const bool sw = hipGetDevice(&cur) == hipSuccess && cur != device && hipSetDevice(device) == hipSuccess;
    (void)hipDeviceSynchronize();  // (freed arenas return to the pool in stream order)
    const hipError_t e = hipMemPoolTrimTo(mp, (size_t)keep_bytes);
    if (sw) (void)hipSetDevice(cur);
    return e == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
}

void covt_device_plan_destroy(covt_device_plan* p) {
    if (!p) return;
    int cur = 0;
    const bool sw = hipGetDevice(&cur) == hipSuccess && cur != p->dev && hipSetDevice(p->dev) == hipSuccess;
    // (hipFree's implicit device synchronization, then the arenas back to the pool)
    (void)hipDeviceSynchronize();
    for (void* q : {p->tile_arena, p->stream_arena, p->desc_arena, p->geo_arena, p->prop_arena, p->scratch})
        if (q) (void)hipFreeAsync(q, nullptr);
    (void)hipStreamSynchronize(nullptr);
    if (sw) (void)hipSetDevice(cur);
    delete p;
}

int64_t covt_device_plan_num_streams(const covt_device_plan* p) { return p ? p->n_streams : 0; }
int64_t covt_device_plan_num_descs(const covt_device_plan* p) { return p ? p->n_descs : 0; }
int64_t covt_device_plan_output_bytes(const covt_device_plan* p) { return p ? p->out_bytes : 0; }

int covt_device_plan_totals(const covt_device_plan* p, int64_t* in_bytes, int64_t* out_bytes, int64_t* vertices) {
    if (!p) return COVT_ERR_INVALID_ARG;
    if (in_bytes) *in_bytes = p->in_bytes;
    if (out_bytes) *out_bytes = p->out_payload;
    if (vertices) *vertices = p->vertices;
    return COVT_OK;
}

int covt_device_plan_family_counts(const covt_device_plan* p, int64_t counts[COVT_NUM_FAMILIES]) {
    if (!p || !counts) return COVT_ERR_INVALID_ARG;
    for (int f = 0; f < COVT_NUM_FAMILIES; ++f) counts[f] = p->fam_counts[f];
    return COVT_OK;
}

const covt_stream_desc* covt_device_plan_descs_device(const covt_device_plan* p) { return p ? p->d_desc : nullptr; }
const covt_stream_info* covt_device_plan_streams_device(const covt_device_plan* p) { return p ? p->d_info : nullptr; }
const int32_t* covt_device_plan_tile_status_device(const covt_device_plan* p) { return p ? p->d_status : nullptr; }
const uint32_t* covt_device_plan_order_device(const covt_device_plan* p) { return p ? p->d_order : nullptr; }

int covt_device_plan_copy(const covt_device_plan* p, covt_stream_info* streams, covt_stream_desc* descs,
                          int32_t* tile_status) {
    if (!p) return COVT_ERR_INVALID_ARG;
    const size_t ns = (size_t)p->n_streams, nd = (size_t)p->n_descs;
    if (streams && ns && hipMemcpy(streams, p->d_info, ns * sizeof(covt_stream_info), hipMemcpyDeviceToHost) != hipSuccess)
        return COVT_ERR_DEVICE;
    if (descs && nd && hipMemcpy(descs, p->d_desc, nd * sizeof(covt_stream_desc), hipMemcpyDeviceToHost) != hipSuccess)
        return COVT_ERR_DEVICE;
    if (tile_status && p->n_tiles &&
        hipMemcpy(tile_status, p->d_status, (size_t)p->n_tiles * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return COVT_ERR_DEVICE;
    return COVT_OK;
}

int covt_device_plan_geometry(covt_device_plan* p, void* hip_stream) {
    if (!p) return COVT_ERR_INVALID_ARG;
    if (p->geo_built) return COVT_OK;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || (cur != p->dev && hipSetDevice(p->dev) != hipSuccess)) return COVT_ERR_DEVICE;
    struct Restore {
        int cur, dev;
        ~Restore() { if (cur != dev) (void)hipSetDevice(cur); }
    } restore{cur, p->dev};
    hipStream_t s = (hipStream_t)hip_stream;
    const int64_t ns = p->n_streams;
    const size_t n1 = (size_t)ns + 1;
    size_t scan_tmp = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (int64_t*)nullptr, (int64_t*)nullptr, (int)n1, s) != hipSuccess)
        return COVT_ERR_DEVICE;
    // stage 1 arena: column starts | their indices | scan scratch
    void* tmp = nullptr;
    const size_t o_gp = up256(n1 * 8), o_t = o_gp + up256(n1 * 8);
    if (plan_malloc(&tmp, o_t + up256(scan_tmp), p->dev, s) != hipSuccess) return COVT_ERR_DEVICE;
    struct Free {  // stream-ordered: after the work on s that uses it
        void* q;
        hipStream_t s;
        ~Free() { if (q) (void)hipFreeAsync(q, s); }
    } free_tmp{tmp, s};
    int64_t *gst = (int64_t*)tmp, *gpos = (int64_t*)((uint8_t*)tmp + o_gp);
    const int blocks = (int)((n1 + 255) / 256);
    geom_mark<<<blocks, 256, 0, s>>>(p->d_info, ns, gst);
    if (hipGetLastError() != hipSuccess) return COVT_ERR_DEVICE;
    if (hipcub::DeviceScan::ExclusiveSum((uint8_t*)tmp + o_t, scan_tmp, gst, gpos, (int)n1, s) != hipSuccess)
        return COVT_ERR_DEVICE;
    int64_t nc = 0;
    if (hipMemcpyAsync(&nc, gpos + ns, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return COVT_ERR_DEVICE;
    // geometry arena: records | descriptors | column bytes | column offsets | keys in/out | vals in/out | scratch
    const size_t m = (size_t)(nc > 0 ? nc : 1);
    size_t sort_tmp = 0, cscan_tmp = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)nc, 0, 41, s) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, cscan_tmp, (int64_t*)nullptr, (int64_t*)nullptr, (int)(nc + 1), s) != hipSuccess)
        return COVT_ERR_DEVICE;
    const size_t o_gd = up256(m * sizeof(covt_geom_info)), o_cb = o_gd + up256(m * sizeof(covt_geom_desc)),
                 o_co = o_cb + up256((m + 1) * 8), o_k0 = o_co + up256((m + 1) * 8), o_k1 = o_k0 + up256(m * 8),
                 o_v0 = o_k1 + up256(m * 8), o_v1 = o_v0 + up256(m * 4), o_st = o_v1 + up256(m * 4),
                 o_cs = o_st + up256(sort_tmp), total = o_cs + up256(cscan_tmp);
    // the arena is the plan's only on success: a failed build frees it (a retry allocates afresh)
    void* arena = nullptr;
    if (plan_malloc(&arena, total, p->dev, s) != hipSuccess) return COVT_ERR_DEVICE;
    Free free_arena{arena, s};
    uint8_t* g = (uint8_t*)arena;
    p->d_ginfo = (covt_geom_info*)g;
    p->d_gdesc = (covt_geom_desc*)(g + o_gd);
    int64_t *colbytes = (int64_t*)(g + o_cb), *coloff = (int64_t*)(g + o_co);
    uint64_t *k0 = (uint64_t*)(g + o_k0), *k1 = (uint64_t*)(g + o_k1);
    uint32_t *v0 = (uint32_t*)(g + o_v0), *v1 = (uint32_t*)(g + o_v1);
    if (hipMemsetAsync(colbytes, 0, (m + 1) * 8, s) != hipSuccess) return COVT_ERR_DEVICE;
    int64_t asm_bytes = 0;
    if (nc > 0) {
        geom_columns<<<(int)((ns + 255) / 256), 256, 0, s>>>(p->d_info, ns, p->format, gst, gpos, p->d_ginfo, colbytes);
        if (hipGetLastError() != hipSuccess) return COVT_ERR_DEVICE;
        if (hipcub::DeviceScan::ExclusiveSum(g + o_cs, cscan_tmp, colbytes, coloff, (int)(nc + 1), s) != hipSuccess)
            return COVT_ERR_DEVICE;
        const int cb = (int)((nc + 255) / 256);
        geom_keys<<<cb, 256, 0, s>>>(p->d_ginfo, nc, coloff, k0, v0);
        if (hipGetLastError() != hipSuccess) return COVT_ERR_DEVICE;
        if (hipcub::DeviceRadixSort::SortPairs(g + o_st, sort_tmp, k0, k1, v0, v1, (int)nc, 0, 41, s) != hipSuccess)
            return COVT_ERR_DEVICE;
        geom_descs<<<cb, 256, 0, s>>>(p->d_info, p->d_ginfo, v1, nc, p->d_gdesc);
        if (hipGetLastError() != hipSuccess) return COVT_ERR_DEVICE;
        if (hipMemcpyAsync(&asm_bytes, coloff + nc, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return COVT_ERR_DEVICE;
    }
    if (p->geo_arena) (void)hipFreeAsync(p->geo_arena, s);
    p->geo_arena = arena;
    free_arena.q = nullptr;
    p->n_geo = nc;
    p->asm_bytes = asm_bytes;
    p->geo_built = true;
    return COVT_OK;
}

int64_t covt_device_plan_num_property_columns(const covt_device_plan* p) { return p ? p->n_props : 0; }
int64_t covt_device_plan_property_bytes(const covt_device_plan* p) { return p ? p->prop_bytes : 0; }
const covt_prop_desc* covt_device_plan_property_descs_device(const covt_device_plan* p) { return p ? p->d_pdesc : nullptr; }
int covt_device_plan_property_copy(const covt_device_plan* p, covt_prop_info* infos, covt_prop_desc* descs) {
    if (!p) return COVT_ERR_INVALID_ARG;
    if (p->n_props == 0) return COVT_OK;
    if (infos && hipMemcpy(infos, p->d_pinfo, (size_t)p->n_props * sizeof(covt_prop_info), hipMemcpyDeviceToHost) != hipSuccess)
        return COVT_ERR_DEVICE;
    if (descs && hipMemcpy(descs, p->d_pdesc, (size_t)p->n_props * sizeof(covt_prop_desc), hipMemcpyDeviceToHost) != hipSuccess)
        return COVT_ERR_DEVICE;
    return COVT_OK;
}
int covt_device_plan_materialize(const covt_device_plan* p, const uint8_t* d_in, const uint8_t* d_decoded,
                                 const covt_stream_result* d_res, uint8_t* d_props, covt_prop_result* d_pres,
                                 void* hip_stream) {
    if (!p) return COVT_ERR_INVALID_ARG;
    return covt_materialize_properties_device(d_in, d_decoded, d_res, p->d_pdesc, p->n_props, d_props, d_pres, hip_stream);
}

int64_t covt_device_plan_num_geometry_columns(const covt_device_plan* p) { return p && p->geo_built ? p->n_geo : 0; }
int64_t covt_device_plan_assembly_bytes(const covt_device_plan* p) { return p && p->geo_built ? p->asm_bytes : 0; }
const covt_geom_desc* covt_device_plan_geometry_descs_device(const covt_device_plan* p) {
    return p && p->geo_built ? p->d_gdesc : nullptr;
}

int covt_device_plan_geometry_copy(const covt_device_plan* p, covt_geom_info* infos, covt_geom_desc* descs) {
    if (!p || !p->geo_built) return COVT_ERR_INVALID_ARG;
    const size_t nc = (size_t)p->n_geo;
    if (infos && nc && hipMemcpy(infos, p->d_ginfo, nc * sizeof(covt_geom_info), hipMemcpyDeviceToHost) != hipSuccess)
        return COVT_ERR_DEVICE;
    if (descs && nc && hipMemcpy(descs, p->d_gdesc, nc * sizeof(covt_geom_desc), hipMemcpyDeviceToHost) != hipSuccess)
        return COVT_ERR_DEVICE;
    return COVT_OK;
}

int covt_device_plan_assemble(covt_device_plan* p, const uint8_t* d_decoded, const covt_stream_result* d_res,
                              uint8_t* d_asm, covt_geom_result* d_gres, void* hip_stream) {
    if (!p) return COVT_ERR_INVALID_ARG;
    const int st = covt_device_plan_geometry(p, hip_stream);
    if (st) return st;
    return covt_assemble_geometry_device(d_decoded, d_res, p->d_gdesc, p->n_geo, d_asm, d_gres, hip_stream);
}

int covt_device_plan_decode(const covt_device_plan* p, const uint8_t* d_in, uint8_t* d_out, covt_stream_result* d_res,
                            void* hip_stream) {
    if (!p || (p->n_descs && (!d_in || !d_res || (p->out_bytes && !d_out)))) return COVT_ERR_INVALID_ARG;
    return covt_decode_streams_device_grouped(d_in, p->d_desc, p->fam_counts, d_out, d_res, hip_stream);
}

}  // extern "C"
