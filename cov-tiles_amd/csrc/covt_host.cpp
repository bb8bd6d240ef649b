// covt_host.cpp -- host side of libcovt: container walkers (plan), the C-ABI of include/covt.h,
// device contexts and the multi-GPU shard driver.
//
// The container walk is the host half of CovtParser.decodeCovt (CovtParser.java:53-133): it reads
// only metadata (tens of bytes per layer) and turns every Id / Geometry stream into a 32-byte
// covt_stream_desc.  Output sizes are known from numValues before anything is decoded, so one pass
// assigns every stream its output slice; the GPU then decodes all streams of all tiles in one launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <memory>
#include <mutex>
#include <numeric>
#include <thread>
#include <unordered_map>
#include <vector>

#include "covt.h"
#include "covt_internal.h"
#include "covt_walk.h"
#include "covt_props_plan.h"

namespace {

bool name_is(const uint8_t* t, int64_t off, int64_t len, const char* s) {
    return (size_t)len == std::strlen(s) && std::memcmp(t + off, s, (size_t)len) == 0;
}
// PropRaw, the property walkers' record, and the planning rule: covt_props_plan.h (shared with the device plan)

// LEB128 (metadata of Gen C is written with EncodingUtils.encodeVarints, i.e. 64-bit varints)
bool rd_uv(const uint8_t* t, size_t len, size_t& o, uint64_t& v) {
    v = 0;
    for (int i = 0; i < 10; ++i) {
        if (o >= len) return false;
        const uint8_t b = t[o++];
        v |= (uint64_t)(b & 0x7f) << (7 * i);
        if (!(b & 0x80)) return true;
    }
    return false;
}
// DecodingUtils.decodeVarint (4-byte cap) as used by the Gen D metadata reader
bool rd_j4(const uint8_t* t, size_t len, size_t& o, int32_t& v) {
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        if (o >= len) return false;
        const uint8_t b = t[o++];
        r |= (uint32_t)(b & 0x7f) << (7 * i);
        if (i < 3 && !(b & 0x80)) break;
    }
    v = (int32_t)r;
    return true;
}
int genc_stream_type(const uint8_t* s, uint64_t n) {
    static const char* kNames[] = {"present", "data", "length", "dictionary", "geometry_types",
                                   "geometry_offsets", "part_offsets", "ring_offsets", "vertex_offsets",
                                   "vertex_buffer"};
    for (int i = 0; i < 10; ++i)
        if (std::strlen(kNames[i]) == n && std::memcmp(kNames[i], s, n) == 0) return i;
    return -1;
}

// Gen C container (all committed fixtures), SURVEY.md Appendix A.1.  Geometry streams are laid
// out in StreamType order whatever their metadata order; other columns in metadata order.
int walk_genc(const uint8_t* t, size_t len, std::vector<RawStream>& out, std::vector<PropRaw>* props) {
    size_t o = 0;
    uint64_t version, nlayers;
    if (!rd_uv(t, len, o, version) || !rd_uv(t, len, o, nlayers)) return COVT_ERR_TRUNCATED;
    if (version != 1) return COVT_ERR_BAD_HEADER;
    struct SM { int type, enc; int64_t nv, bl, name_off, name_len, off; };
    struct CM { int kind, dtype, ctype; int64_t name_off, name_len; std::vector<SM> s; };
    static thread_local std::vector<CM> cols;  // reused across tiles: no allocation per column
    for (uint64_t L = 0; L < nlayers; ++L) {
        uint64_t nlen, extent, nfeat, ncols;
        if (!rd_uv(t, len, o, nlen) || nlen > len - o) return COVT_ERR_TRUNCATED;  // (no wrap)
        o += nlen;
        if (!rd_uv(t, len, o, extent) || !rd_uv(t, len, o, nfeat) || !rd_uv(t, len, o, ncols))
            return COVT_ERR_TRUNCATED;
        if (ncols > 4096) return COVT_ERR_BAD_HEADER;
        cols.assign(ncols, CM{});
        for (auto& c : cols) {
            uint64_t cn, ns;
            if (!rd_uv(t, len, o, cn) || cn > len - o || len - o - cn < 2) return COVT_ERR_TRUNCATED;
            const uint8_t* name = t + o;
            c.name_off = (int64_t)o;
            c.name_len = (int64_t)cn;
            o += cn;
            c.dtype = t[o++];
            c.ctype = t[o++];
            c.kind = (cn == 2 && !std::memcmp(name, "id", 2)) ? 0
                     : ((cn == 8 && !std::memcmp(name, "geometry", 8)) || c.dtype == 6) ? 1 : 2;
            if (!rd_uv(t, len, o, ns)) return COVT_ERR_TRUNCATED;
            if (ns > 256) return COVT_ERR_BAD_HEADER;
            c.s.resize(ns);
            for (auto& s : c.s) {
                uint64_t sn, nv, bl;
                if (!rd_uv(t, len, o, sn) || sn > len - o) return COVT_ERR_TRUNCATED;
                // stream names matter for Id / Geometry columns; property streams only when planned
                s.type = (c.kind != 2 || props) ? genc_stream_type(t + o, sn) : -1;
                s.name_off = (int64_t)o;
                s.name_len = (int64_t)sn;
                o += sn;
                if (!rd_uv(t, len, o, nv) || !rd_uv(t, len, o, bl) || o >= len) return COVT_ERR_TRUNCATED;
                s.enc = t[o++];
                if (nv > 0x7fffffff || bl > 0x7fffffff) return COVT_ERR_BAD_HEADER;
                s.nv = (int64_t)nv;
                s.bl = (int64_t)bl;
            }
        }
        const int nb = nbits_of_extent(extent);
        for (auto& c : cols) {
            if (c.kind == 1) {
                for (int type = ST_GEOMETRY_TYPES; type <= ST_VERTEX_BUFFER; ++type)
                    for (auto& s : c.s)
                        if (s.type == type) {
                            out.push_back({(int32_t)L, 1, type, s.enc, c.ctype, (int32_t)s.nv, (int32_t)s.bl, nb,
                                           (int64_t)o});
                            o += s.bl;
                        }
                for (auto& s : c.s)
                    if (s.type < ST_GEOMETRY_TYPES || s.type > ST_VERTEX_BUFFER) o += s.bl;
            } else {
                for (auto& s : c.s) {
                    if (c.kind == 0 && s.type == ST_DATA)
                        out.push_back({(int32_t)L, 0, ST_DATA, s.enc, c.ctype, (int32_t)s.nv, (int32_t)s.bl, nb,
                                       (int64_t)o});
                    s.off = (int64_t)o;
                    o += s.bl;
                }
            }
            if (o > len) return COVT_ERR_TRUNCATED;
            if (props && c.kind == 2) {  // streams of a property column in metadata order
                PropRaw p = prop_init((int32_t)L, (int32_t)(&c - cols.data()), (int32_t)nfeat);
                p.name_off = c.name_off;
                p.name_len = (int32_t)c.name_len;
                p.type = genc_prop_type(c.dtype);
                p.ctype = c.ctype;
                if (p.type == COVT_PROP_STRING && c.ctype == 2) {
                    // LOCALIZED_DICTIONARY: (present_<lang>, <lang>)*, then the shared length + dictionary
                    const SM *ls = nullptr, *ds = nullptr;
                    for (const SM& s : c.s) {
                        if (name_is(t, s.name_off, s.name_len, "length")) ls = &s;
                        else if (name_is(t, s.name_off, s.name_len, "dictionary")) ds = &s;
                    }
                    int32_t lang = 0;
                    for (const SM& s : c.s) {
                        if (s.name_len <= 8 || std::memcmp(t + s.name_off, "present_", 8)) continue;
                        const int64_t ll = s.name_len - 8;
                        const SM* d = nullptr;
                        for (const SM& k : c.s)
                            if (k.name_len == ll && !std::memcmp(t + k.name_off, t + s.name_off + 8, (size_t)ll)) d = &k;
                        PropRaw q = p;
                        q.lang = lang++;
                        q.lang_off = s.name_off + 8;
                        q.lang_len = (int32_t)ll;
                        prop_stream(q, 0, s.off, (int32_t)s.nv, (int32_t)s.bl, s.enc);
                        if (d) prop_stream(q, 1, d->off, (int32_t)d->nv, (int32_t)d->bl, d->enc);
                        if (ls) prop_stream(q, 2, ls->off, (int32_t)ls->nv, (int32_t)ls->bl, ls->enc);
                        if (ds) prop_stream(q, 3, ds->off, (int32_t)ds->nv, (int32_t)ds->bl, ds->enc);
                        props->push_back(q);
                    }
                } else {
                    static const char* kRoles[4] = {"present", "data", "length", "dictionary"};
                    for (const SM& s : c.s)
                        for (int r = 0; r < 4; ++r)
                            if (name_is(t, s.name_off, s.name_len, kRoles[r]))
                                prop_stream(p, r, s.off, (int32_t)s.nv, (int32_t)s.bl, s.enc);
                    props->push_back(p);
                }
            }
        }
    }
    return o == len ? COVT_OK : COVT_ERR_BAD_HEADER;
}

// Bytes an ORC byte-RLE stream of n values starting at tile offset o occupies (control bytes walked,
// values skipped); -1 if it runs past the tile.
int32_t byte_rle_length(const uint8_t* t, size_t len, size_t o, int32_t n) {
    size_t q = o;
    int64_t done = 0;
    while (done < n) {
        if (q >= len) return -1;
        const uint32_t c = t[q++];
        if (c < 0x80u) { done += c + 3; q += 1; }
        else { done += 0x100 - c; q += 0x100 - c; }
        if (q > len) return -1;
    }
    return (int32_t)(q - o);
}

// Gen D container: CovtParser.decodeLayerMetadata (CovtParser.java:574-652) + the column loop
// of decodeCovt (:56-85).  Streams of a column follow TreeMap<StreamType> order.
int walk_gend(const uint8_t* t, size_t len, std::vector<RawStream>& out, std::vector<PropRaw>* props) {
    size_t o = 0;
    int32_t layer = 0;
    struct SM { int enc; int32_t nv, bl; bool have; };
    struct CM { int kind, dtype, ctype; int64_t name_off; int32_t name_len; SM s[12]; };
    std::vector<CM> cols;
    while (o < len) {
        const int hdr = t[o++];
        const bool optimized = hdr & 1;
        int32_t v, extent, nfeat, ncols;
        if (!rd_j4(t, len, o, v)) return COVT_ERR_TRUNCATED;
        if (!optimized) {  // decodeString: varint length + UTF-8 bytes
            if (v < 0 || o + (size_t)v > len) return COVT_ERR_TRUNCATED;
            o += (size_t)v;
        }
        if (!rd_j4(t, len, o, extent) || !rd_j4(t, len, o, nfeat) || !rd_j4(t, len, o, ncols))
            return COVT_ERR_TRUNCATED;
        if (ncols < 0 || ncols > 4096) return COVT_ERR_BAD_HEADER;
        cols.assign((size_t)ncols, CM{});
        for (int32_t ci = 0; ci < ncols; ++ci) {
            CM& c = cols[(size_t)ci];
            c.name_off = -1;
            c.name_len = 0;
            if (optimized || ci == 0) {
                int32_t cid;
                if (!rd_j4(t, len, o, cid)) return COVT_ERR_TRUNCATED;
                c.kind = cid == 0 ? 0 : (cid == 1 ? 1 : 2);
            } else {
                int32_t sl;
                if (!rd_j4(t, len, o, sl) || sl < 0 || o + (size_t)sl > len) return COVT_ERR_TRUNCATED;
                c.kind = (sl == 2 && !std::memcmp(t + o, "id", 2)) ? 0
                         : (sl == 8 && !std::memcmp(t + o, "geometry", 8)) ? 1 : 2;
                c.name_off = (int64_t)o;
                c.name_len = sl;
                o += (size_t)sl;
            }
            if (o >= len) return COVT_ERR_TRUNCATED;
            const int desc = t[o++];
            c.dtype = (desc >> 3) & 0xF;
            c.ctype = desc & 0x7;
            if (c.ctype > 4) return COVT_ERR_BAD_HEADER;
            for (;;) {
                if (o >= len) return COVT_ERR_TRUNCATED;
                const int sd = t[o++];
                const int type = sd >> 4, enc = sd & 0xF;
                if (type > ST_M || enc > 9) return COVT_ERR_BAD_HEADER;
                int32_t nv, bl;
                if (!rd_j4(t, len, o, nv) || !rd_j4(t, len, o, bl)) return COVT_ERR_TRUNCATED;
                c.s[type] = SM{enc, nv, bl, true};
                if (c.dtype == 8 && type == ST_VERTEX_BUFFER) break;
                if (type == ST_DATA && c.ctype == CT_PLAIN) break;
                if (type == ST_DICTIONARY) break;
            }
        }
        const int nb = nbits_of_extent((uint32_t)extent);
        for (auto& c : cols) {
            PropRaw p = prop_init(layer, (int32_t)(&c - cols.data()), nfeat);
            if (c.kind == 2 && c.dtype != 0) {
                // implicit present stream: its bytes lead the column without metadata
                // (CovtConverter.addNamedColumnMetadata skips PRESENT, :452-458; CovtParser.java:296 reads
                // ceil(numFeatures/8) bytes with the 3-argument decodeByteRle); BOOLEAN (0) has none
                const int32_t pl = byte_rle_length(t, len, o, nfeat < 0 ? 0 : (int32_t)(((int64_t)nfeat + 7) / 8));
                if (pl < 0) return COVT_ERR_TRUNCATED;
                prop_stream(p, 0, (int64_t)o, nfeat, pl, 7);
                o += (size_t)pl;
            }
            for (int type = 0; type < 12; ++type) {
                const SM& s = c.s[type];
                if (!s.have || (c.kind == 2 && type == ST_PRESENT)) continue;
                const bool hot = (c.kind == 0 && type == ST_DATA) ||
                                 (c.kind == 1 && type >= ST_GEOMETRY_TYPES && type <= ST_VERTEX_BUFFER);
                if (hot) out.push_back({layer, c.kind, type, s.enc, c.ctype, s.nv, s.bl, nb, (int64_t)o});
                if (s.bl < 0) return COVT_ERR_BAD_HEADER;
                if (type > ST_PRESENT && type <= ST_DICTIONARY) prop_stream(p, type, (int64_t)o, s.nv, s.bl, s.enc);
                o += (size_t)s.bl;
            }
            if (o > len) return COVT_ERR_TRUNCATED;
            if (props && c.kind == 2) {  // TreeMap<StreamType> order: present, data, length, dictionary
                p.name_off = c.name_off;
                p.name_len = c.name_len;
                p.type = gend_prop_type(c.dtype);
                p.ctype = c.ctype;
                props->push_back(p);
            }
        }
        ++layer;
    }
    return COVT_OK;
}

inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

// f(begin, end) over [0, n) split into nthr contiguous ranges, one host thread each (the caller's thread
// takes the first); small inputs run on the caller's thread alone
template <class F>
void par_for(int32_t nthr, int64_t n, F&& f) {
    if (nthr <= 1 || n < 2) {
        f((int64_t)0, n);
        return;
    }
    const int64_t nt = std::min<int64_t>(nthr, n);
    std::vector<std::thread> th;
    for (int64_t k = 1; k < nt; ++k) th.emplace_back([&f, k, n, nt] { f(n * k / nt, n * (k + 1) / nt); });
    f((int64_t)0, n / nt);
    for (auto& x : th) x.join();
}

// Launch-order keys: a stable LSD radix sort (11-bit digits, passes whose digit is the same for every
// key skipped), so equal keys keep plan (tile) order.  std::sort of the 432k keys of a 10k-tile plan
// took ~50 ms of the plan; this takes a few.
struct SortKey {
    uint64_t k;
    uint32_t i;
};
inline int key_family(uint64_t k) {
#ifdef COVT_EXACT_ORDER
    return (int)(k >> 60);
#else
    return (int)(k >> kLaunchFamShift);
#endif
}
void radix_sort(std::vector<SortKey>& a) {
    const size_t n = a.size();
    if (n < 2) return;
    std::vector<SortKey> tmp(n);
    uint64_t all_or = 0, all_and = ~0ull;
    for (const SortKey& x : a) all_or |= x.k, all_and &= x.k;
    const uint64_t varying = all_or ^ all_and;
    for (int sh = 0; sh < 64; sh += 11) {
        if (!((varying >> sh) & 0x7ffull)) continue;
        size_t cnt[2048] = {};
        for (const SortKey& x : a) ++cnt[(x.k >> sh) & 0x7ff];
        size_t s = 0;
        for (size_t& c : cnt) { const size_t v = c; c = s; s += v; }
        for (const SortKey& x : a) tmp[cnt[(x.k >> sh) & 0x7ff]++] = x;
        a.swap(tmp);
    }
}

// ---- per-thread device context for the stream-level API -----------------------------------------
struct DevCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    uint8_t* d_out = nullptr;
    size_t out_cap = 0;
    covt_stream_desc* d_desc = nullptr;
    covt_stream_result* d_res = nullptr;
    ~DevCtx() {
        if (device < 0) return;
        (void)hipSetDevice(device);
        if (d_in) (void)hipFree(d_in);
        if (d_out) (void)hipFree(d_out);
        if (d_desc) (void)hipFree(d_desc);
        if (d_res) (void)hipFree(d_res);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

bool grow(uint8_t*& p, size_t& cap, size_t need) {
    if (need <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t c = std::max<size_t>(need, 1 << 16);
    c = (c + 4095) & ~(size_t)4095;
    if (hipMalloc(&p, c) != hipSuccess) return false;
    cap = c;
    return true;
}

DevCtx* ctx() {
    thread_local DevCtx c;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    if (c.device != dev) {
        c.~DevCtx();
        new (&c) DevCtx();
        c.device = dev;
        if (hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
        if (hipMalloc(&c.d_desc, sizeof(covt_stream_desc)) != hipSuccess) return nullptr;
        if (hipMalloc(&c.d_res, sizeof(covt_stream_result)) != hipSuccess) return nullptr;
    }
    return &c;
}

// Decode one stream held in host memory: `region` bytes become the device stream payload.
int run_one(const uint8_t* region, size_t region_len, size_t pad_to, int op, int32_t n, int32_t byte_length, int nb,
            void* out, size_t out_bytes, covt_stream_result* res) {
    DevCtx* c = ctx();
    if (!c) return COVT_ERR_DEVICE;
    const size_t payload = std::max(region_len, pad_to);
    if (!grow(c->d_in, c->in_cap, payload + COVT_INPUT_PADDING)) return COVT_ERR_DEVICE;
    if (!grow(c->d_out, c->out_cap, out_bytes + 16)) return COVT_ERR_DEVICE;
    if (region_len && hipMemcpyAsync(c->d_in, region, region_len, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return COVT_ERR_DEVICE;
    if (payload > region_len &&  // Arrays.copyOfRange zero-pads past the source (DecodingUtils.java:317)
        hipMemsetAsync(c->d_in + region_len, 0, payload - region_len, c->stream) != hipSuccess)
        return COVT_ERR_DEVICE;
    covt_stream_desc d{};
    d.in_off = 0;
    d.out_off = 0;
    d.avail = (int32_t)std::min<size_t>(payload, 0x7fffffff);
    d.num_values = n;
    d.op = (uint8_t)op;
    d.num_bits = (uint8_t)nb;
    d.byte_length = byte_length;
    if (hipMemcpyAsync(c->d_desc, &d, sizeof d, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return COVT_ERR_DEVICE;
    int st = covt_launch_family(covt_op_family_of(op), c->d_in, c->d_desc, 1, c->d_out, c->d_res, c->stream);
    if (st) return st;
    if (out_bytes && hipMemcpyAsync(out, c->d_out, out_bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        return COVT_ERR_DEVICE;
    if (hipMemcpyAsync(res, c->d_res, sizeof *res, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        return COVT_ERR_DEVICE;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return COVT_ERR_DEVICE;
    return COVT_OK;
}

// stream-level wrappers: varint / RLE ops read [pos, buf_len) (Java reads up to the array end)
// Most bytes decoding n values of `op` can read from *pos on: Java's capped varints take <= 4 bytes
// each (DecodingUtils.java:157-186); an ORC RLE reader reads whole groups, so past n values it may
// still read the rest of the last group (<= 128 literal varints of <= 10 bytes, RunLengthIntegerReader;
// <= 128 literal bytes, RunLengthByteReader).  The stream-level calls copy only that much of the
// caller's array to the device instead of everything up to its end.
size_t max_stream_bytes(int op, int32_t n) {
    const size_t v = (size_t)std::max(n, 0);
    switch (op) {
        case COVT_OP_RLE_U64: case COVT_OP_RLE_S64: case COVT_OP_RLE_I32: return 11 * v + 2 + 128 * 10;
        case COVT_OP_BYTE_RLE_RAW: case COVT_OP_BYTE_RLE_U8: return 2 * v + 1 + 128;
        case COVT_OP_VARINT_U64: return 10 * v;
        default: return 4 * v;  // 4-byte-capped int32 varints (x,y coordinates: num_values varints)
    }
}

// Length of ORC RunLengthByteWriter's encoding of v[0..n) (orc-core 1.8.1; EncodingUtils.encodeByteRle,
// EncodingUtils.java:123-135): runs of 3..130 equal bytes -> 2 bytes, literal groups of <= 128 -> 1 + k.
int64_t orc_byte_rle_length(const uint8_t* v, int32_t n) {
    constexpr int kMinRepeat = 3, kMaxLiteral = 128, kMaxRepeat = 127 + kMinRepeat;
    int64_t len = 0;
    int num = 0, tail = 0;
    bool repeat = false;
    uint8_t first = 0, last = 0;
    auto flush = [&] {
        if (num) len += repeat ? 2 : 1 + num;
        repeat = false;
        tail = num = 0;
    };
    for (int32_t i = 0; i < n; ++i) {
        const uint8_t x = v[i];
        if (num == 0) {
            first = last = x;
            num = tail = 1;
        } else if (repeat) {
            if (x == first) {
                if (++num == kMaxRepeat) flush();
            } else {
                flush();
                first = last = x;
                num = tail = 1;
            }
        } else {
            tail = x == last ? tail + 1 : 1;
            if (tail == kMinRepeat) {
                if (num + 1 == kMinRepeat) {
                    repeat = true;
                    ++num;
                } else {
                    num -= kMinRepeat - 1;  // the literal prefix before the run is written first
                    flush();
                    first = x;
                    repeat = true;
                    num = kMinRepeat;
                }
            } else {
                last = x;
                if (++num == kMaxLiteral) flush();
            }
        }
    }
    flush();
    return len;
}

int stream_call(const uint8_t* buf, size_t buf_len, int32_t* pos, int op, int32_t n, int nb, void* out,
                size_t elem_bytes, size_t out_elems) {
    if (!pos || n < 0 || (!buf && buf_len) || (!out && out_elems)) return COVT_ERR_INVALID_ARG;
    if (*pos < 0 || (size_t)*pos > buf_len) return COVT_ERR_TRUNCATED;
    covt_stream_result r{};
    const size_t rl = std::min(buf_len - (size_t)*pos, max_stream_bytes(op, n));
    int st = run_one(buf + *pos, rl, 0, op, n, 0, nb, out, elem_bytes * out_elems, &r);
    if (st) return st;
    if (r.status) return r.status;
    *pos += r.consumed;
    return COVT_OK;
}
int fpf_call(const uint8_t* buf, size_t buf_len, int32_t* pos, int op, int32_t n, int32_t byte_length, int nb,
             void* out, size_t out_elems) {
    if (!pos || n < 0 || byte_length < 0 || (!buf && buf_len) || (!out && out_elems)) return COVT_ERR_INVALID_ARG;
    if (*pos < 0) return COVT_ERR_INVALID_ARG;
    const size_t start = std::min<size_t>((size_t)*pos, buf_len);
    const size_t rl = std::min<size_t>(buf_len - start, (size_t)byte_length);
    covt_stream_result r{};
    int st = run_one(buf + start, rl, (size_t)byte_length, op, n, byte_length, nb, out, 4 * out_elems, &r);
    if (st) return st;
    if (r.status) return r.status;
    *pos += byte_length;
    return COVT_OK;
}

// Fork/join of the family kernels: the first on the caller's stream, the others on auxiliary
// streams ordered by events (capturable into a hipGraph).  The auxiliary streams and events come
// from a process-wide per-device pool: a launch takes a set, enqueues, and hands it back, so
// concurrent callers (one host thread per device, JNI threads) never share one and nothing leaks
// when threads come and go; the pool holds as many sets as launches ever overlapped.
constexpr int kForkAux = 3;
struct ForkCtx {
    int device = -1;
    hipStream_t aux[kForkAux] = {nullptr, nullptr, nullptr};
    hipEvent_t fork = nullptr, join[kForkAux] = {nullptr, nullptr, nullptr};
};
std::mutex g_fork_mu;
std::vector<ForkCtx*> g_fork_free;

void fork_destroy(ForkCtx* f) {
    for (int i = 0; i < kForkAux; ++i) {
        if (f->aux[i]) (void)hipStreamDestroy(f->aux[i]);
        if (f->join[i]) (void)hipEventDestroy(f->join[i]);
    }
    if (f->fork) (void)hipEventDestroy(f->fork);
    delete f;
}
ForkCtx* fork_acquire(int dev) {
    {
        std::lock_guard<std::mutex> g(g_fork_mu);
        for (size_t i = 0; i < g_fork_free.size(); ++i)
            if (g_fork_free[i]->device == dev) {
                ForkCtx* f = g_fork_free[i];
                g_fork_free.erase(g_fork_free.begin() + (std::ptrdiff_t)i);
                return f;
            }
    }
    auto* f = new ForkCtx();
    f->device = dev;
    bool ok = true;
    for (int i = 0; i < kForkAux && ok; ++i)
        ok = hipStreamCreateWithFlags(&f->aux[i], hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&f->join[i], hipEventDisableTiming) == hipSuccess;
    if (ok) ok = hipEventCreateWithFlags(&f->fork, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        fork_destroy(f);
        return nullptr;
    }
    return f;
}
void fork_release(ForkCtx* f) {
    std::lock_guard<std::mutex> g(g_fork_mu);
    g_fork_free.push_back(f);
}

int launch_grouped(const uint8_t* d_in, const covt_stream_desc* d_desc, const int64_t counts[COVT_NUM_FAMILIES],
                   uint8_t* d_out, covt_stream_result* d_res, hipStream_t s, int mode = COVT_LAUNCH_AUTO) {
    const int fpf_mode = mode & (COVT_LAUNCH_FPF_STREAM | COVT_LAUNCH_FPF_CLASSIC);
    mode &= ~(COVT_LAUNCH_FPF_STREAM | COVT_LAUNCH_FPF_CLASSIC);
    if (fpf_mode == (COVT_LAUNCH_FPF_STREAM | COVT_LAUNCH_FPF_CLASSIC)) return COVT_ERR_INVALID_ARG;
    if (mode != COVT_LAUNCH_AUTO && mode != COVT_LAUNCH_FUSED && mode != COVT_LAUNCH_FORKED) return COVT_ERR_INVALID_ARG;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return COVT_ERR_DEVICE;
    if (s) {  // the auxiliary streams must belong to the device of the caller's stream
        int sdev = -1;
        if (hipStreamGetDevice(s, &sdev) != hipSuccess || sdev != dev) return COVT_ERR_DEVICE;
    }
    ForkCtx* fp = fork_acquire(dev);
    if (!fp) return COVT_ERR_DEVICE;
    struct Back { ForkCtx* f; ~Back() { fork_release(f); } } back{fp};
    ForkCtx& f = *fp;
    int64_t off[COVT_NUM_FAMILIES];
    off[0] = 0;
    for (int k = 1; k < COVT_NUM_FAMILIES; ++k) off[k] = off[k - 1] + counts[k - 1];
    // Up to four queues: the first with work runs on the caller's stream, the others on up to three
    // auxiliary streams forked from and joined back into it -- four hardware queues with the caller's,
    // HIP's default per process (a fifth stream would share a queue and serialise behind another).  A
    // launch that needs one queue forks nothing.  Without split streams: FastPFOR, varint, RLE, lane.
    // With them: varint chunks ahead of the varint family and the RLE chunks behind it (no extra fork
    // for a varint-only launch such as BASELINE config 2; with the RLE chunks ahead of the RLE family
    // instead, that family's longest stream started only after them: config 3 0.150 -> 0.132 ms), the
    // RLE family (and lane, which the plan makes only for large batches that split nothing), and the
    // FastPFOR chunks on a queue of their own.  The split regions' look-back records and
    // ticket counters (their result entries) are zeroed on the caller's stream before the fork.
    constexpr int kSplitV = COVT_FAMILY_SPLIT, kSplitF = COVT_FAMILY_SPLIT_FPF, kSplitR = COVT_FAMILY_SPLIT_RLE;
    const int64_t n_split = counts[kSplitV] + counts[kSplitF] + counts[kSplitR];  // contiguous regions
    const bool splits = n_split > 0;
    auto n_of = [&](int fam) { return fam < 0 ? 0 : counts[fam]; };
    struct Q {
        int fam[3];
    };
    Q qs[4];
    int nq = 0;
    auto add = [&](int a, int b2, int c3) {
        Q q{{-1, -1, -1}};
        int k = 0;
        for (int f : {a, b2, c3})
            if (n_of(f) > 0) q.fam[k++] = f;
        if (k) qs[nq++] = q;
    };
    if (splits && hipMemsetAsync(d_res + off[kSplitV], 0, (size_t)n_split * sizeof(covt_stream_result), s) != hipSuccess)
        return COVT_ERR_DEVICE;
    {  // a small batch: one fused launch on the caller's stream (no fork / join)
        const int64_t waves = n_split / COVT_SPLIT_SLOTS + counts[COVT_FAMILY_FASTPFOR] + counts[COVT_FAMILY_RLE] +
                              counts[COVT_FAMILY_VARINT] +
                              (counts[COVT_FAMILY_LANE] + kFusedLaneStreams - 1) / kFusedLaneStreams;
        if (mode == COVT_LAUNCH_FUSED || (mode == COVT_LAUNCH_AUTO && waves <= kFusedMaxWaves))
            return covt_launch_fused(d_in, d_desc, counts, d_out, d_res, s);
    }
    if (splits) {
        // RLE chunks behind the varint queue (round 2 A/B: with the RLE family, config 3 0.132 -> 0.150 ms)
        add(kSplitV, COVT_FAMILY_VARINT, kSplitR);
        add(COVT_FAMILY_FASTPFOR, -1, -1);
        add(COVT_FAMILY_RLE, COVT_FAMILY_LANE, -1);
        add(kSplitF, -1, -1);
    } else {
        // queue order FastPFOR, varint, RLE, lane (round 2 A/B of all orders: within noise)
        for (int f : {COVT_FAMILY_FASTPFOR, COVT_FAMILY_VARINT, COVT_FAMILY_RLE, COVT_FAMILY_LANE}) add(f, -1, -1);
    }
    if (nq > 1 && hipEventRecord(f.fork, s) != hipSuccess) return COVT_ERR_DEVICE;
    int st = COVT_OK;
    int nforked = 0;
    for (int i = 0; i < nq && !st; ++i) {
        hipStream_t q = s;
        if (i > 0) {
            q = f.aux[i - 1];
            if (hipStreamWaitEvent(q, f.fork, 0) != hipSuccess) return COVT_ERR_DEVICE;
            nforked = i;
        }
        for (int k = 0; k < 3 && !st; ++k) {
            const int fam = qs[i].fam[k];
            if (fam < 0) continue;
            if (fam != kSplitV && fam != kSplitF && fam != kSplitR) {
                st = covt_launch_family_split_mode(fam, d_in, d_desc + off[fam], counts[fam], d_out, d_res + off[fam],
                                                   nullptr, 0, nullptr, q, fpf_mode);
                continue;
            }
            const int kind = fam == kSplitV ? COVT_FAMILY_VARINT : fam == kSplitR ? COVT_FAMILY_RLE : COVT_FAMILY_FASTPFOR;
            st = covt_launch_family_split(kind, d_in, nullptr, 0, d_out, nullptr, d_desc + off[fam], counts[fam],
                                          d_res + off[fam], q);
        }
    }
    for (int i = 0; i < nforked; ++i) {
        if (hipEventRecord(f.join[i], f.aux[i]) != hipSuccess) return COVT_ERR_DEVICE;
        if (hipStreamWaitEvent(s, f.join[i], 0) != hipSuccess) return COVT_ERR_DEVICE;
    }
    return st;
}

}  // namespace

// ================================================================================================
// C-ABI
// ================================================================================================
namespace {

// Pageable caller memory for the D2H: fault its pages in on host threads (MADV_POPULATE_WRITE) while
// the device runs H2D + decode, so the copy itself meets resident pages.  Started
// before the H2D is queued and joined just before the output D2H.  covt_plan_options.host_prefault = 0
// turns it off.  Kernels without MADV_POPULATE_WRITE (< 5.14) touch each page.
struct Prefault {
    std::vector<std::thread> th;
    Prefault(uint8_t* p, size_t n, bool on, int threads) {
        if (!on || n < (64u << 20)) return;
#ifdef MADV_POPULATE_WRITE
        const uintptr_t pg = 4096, lo = ((uintptr_t)p + pg - 1) & ~(pg - 1), hi = ((uintptr_t)p + n) & ~(pg - 1);
        if (hi <= lo) return;
        const size_t len = hi - lo;
        const unsigned hw = std::thread::hardware_concurrency();
        // (fresh pages are zeroed by the kernel on first touch: ~2.5 us a page on one thread)
        const size_t nthr = std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), hw ? hw : 1));
        for (size_t k = 0; k < nthr; ++k) {
            const uintptr_t a = lo + ((len * k / nthr) & ~(pg - 1));
            const uintptr_t b = k + 1 == nthr ? hi : lo + ((len * (k + 1) / nthr) & ~(pg - 1));
            th.emplace_back([=] {
                if (madvise((void*)a, b - a, MADV_POPULATE_WRITE) == 0) return;
                // older kernels: write each page's first byte back to itself (the copy overwrites it)
                for (uintptr_t q = a; q < b; q += pg) {
                    volatile uint8_t* v = (volatile uint8_t*)q;
                    *v = *v;
                }
            });
        }
#else
        (void)p;
        (void)threads;
#endif
    }
    void join() {
        for (auto& t : th) t.join();
        th.clear();
    }
    ~Prefault() { join(); }
};

}  // namespace

// One shard of a plan for the host entry points: a contiguous tile range, its descriptor table
// rebased to that range (built once), and the device buffers, kept on the plan across calls.
struct HostShard {
    int device = -1;
    bool prefault = true;
    int prefault_threads = 8;
    uint64_t in_lo = 0, in_len = 0;  // caller bytes [in_lo, in_lo + in_len) -> d_in
    int64_t out_lo = 0, out_len = 0; // plan output bytes [out_lo, out_lo + out_len) <- d_out
    std::vector<covt_stream_desc> descs;  // launch order, offsets rebased
    std::vector<int64_t> stream;          // plan-order stream index of each descriptor
    int64_t fam[COVT_NUM_FAMILIES] = {};
    std::vector<covt_stream_result> res;
    hipStream_t s = nullptr;
    uint8_t *d_in = nullptr, *d_out = nullptr;
    covt_stream_desc* d_desc = nullptr;
    covt_stream_result* d_res = nullptr;

    ~HostShard() {
        if (device < 0) return;
        int cur = 0;
        const bool have = hipGetDevice(&cur) == hipSuccess;
        (void)hipSetDevice(device);
        if (s) (void)hipStreamSynchronize(s);
        for (void* q : {(void*)d_in, (void*)d_out, (void*)d_desc, (void*)d_res})
            if (q) (void)hipFree(q);
        if (s) (void)hipStreamDestroy(s);
        if (have) (void)hipSetDevice(cur);
    }

    // device buffers + the descriptor upload, once per shard (on the calling thread's device)
    int open() {
        if (s) return COVT_OK;
        if (hipSetDevice(device) != hipSuccess) return COVT_ERR_DEVICE;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return COVT_ERR_DEVICE;
        const size_t nd = descs.size();
        if (hipMalloc(&d_in, in_len + COVT_INPUT_PADDING) != hipSuccess ||
            hipMalloc(&d_out, (size_t)std::max<int64_t>(out_len, 16)) != hipSuccess ||
            hipMalloc(&d_desc, std::max<size_t>(nd, 1) * sizeof(covt_stream_desc)) != hipSuccess ||
            hipMalloc(&d_res, std::max<size_t>(nd, 1) * sizeof(covt_stream_result)) != hipSuccess)
            return COVT_ERR_DEVICE;
        if ((uintptr_t)d_in & 15) return COVT_ERR_DEVICE;
        // the read-ahead tail past the last tile byte is defined (zero); the H2D never overwrites it
        if (hipMemsetAsync(d_in + in_len, 0, COVT_INPUT_PADDING, s) != hipSuccess) return COVT_ERR_DEVICE;
        if (nd && hipMemcpyAsync(d_desc, descs.data(), nd * sizeof(covt_stream_desc), hipMemcpyHostToDevice, s) !=
                      hipSuccess)
            return COVT_ERR_DEVICE;
        return hipStreamSynchronize(s) == hipSuccess ? COVT_OK : COVT_ERR_DEVICE;
    }

    // one H2D of the shard's tile bytes, one grouped launch, one D2H straight into the caller's buffer.
    // The shard's device is selected on every call, not only when open() creates the buffers: a later
    // call may run on a fresh host thread (current device 0) and launch_grouped takes its auxiliary
    // streams from the current device.
    int run(const uint8_t* bytes, uint8_t* host_out, covt_stream_result* host_res) {
        if (device < 0 || hipSetDevice(device) != hipSuccess) return COVT_ERR_DEVICE;
        int st = open();
        if (st) return st;
        if (descs.empty()) return COVT_OK;
        auto chk = [&](hipError_t e) { if (e != hipSuccess && st == COVT_OK) st = COVT_ERR_DEVICE; };
        Prefault pf(host_out + out_lo, (size_t)out_len, prefault, prefault_threads);
        if (in_len) chk(hipMemcpyAsync(d_in, bytes + in_lo, in_len, hipMemcpyHostToDevice, s));
        if (st == COVT_OK) st = launch_grouped(d_in, d_desc, fam, d_out, d_res, s);
        if (st == COVT_OK) chk(hipMemcpyAsync(res.data(), d_res, res.size() * sizeof(covt_stream_result),
                                              hipMemcpyDeviceToHost, s));
        pf.join();
        if (st == COVT_OK && out_len)
            chk(hipMemcpyAsync(host_out + out_lo, d_out, (size_t)out_len, hipMemcpyDeviceToHost, s));
        chk(hipStreamSynchronize(s));
        if (st == COVT_OK)
            for (size_t k = 0; k < stream.size(); ++k)
                if (stream[k] >= 0) host_res[(size_t)stream[k]] = res[k];
        return st;
    }
};

struct covt_plan {
    covt_plan_options opts{};  // resolved options the plan was made with
    int32_t n_tiles = 0;
    std::vector<int32_t> tile_status;
    std::vector<uint64_t> tile_off, tile_size;
    std::vector<covt_stream_info> info;   // tile order
    std::vector<covt_stream_desc> descs;  // launch order: grouped by family, largest first
    std::vector<int64_t> desc_stream;     // plan-order stream of each descriptor
    int64_t fam_counts[COVT_NUM_FAMILIES] = {};
    int64_t out_bytes = 0, in_bytes = 0, out_payload = 0, vertices = 0;
    int32_t format = COVT_FORMAT_GENC;
    std::vector<covt_geom_info> ginfo;   // geometry columns, tile order
    std::vector<covt_geom_desc> gdescs;  // launch order: largest first
    int64_t asm_bytes = 0;
    std::vector<covt_prop_info> pinfo;   // property (sub)columns, tile order
    std::vector<uint16_t> pflags;        // their COVT_PROP_* flags
    std::vector<covt_prop_desc> pdescs;  // launch order: largest first
    int64_t prop_bytes = 0;
    // host entry points (covt_plan_decode_host*): shards with device buffers kept across calls
    mutable std::mutex host_mu;
    mutable std::vector<int32_t> host_devs;
    mutable std::vector<std::unique_ptr<HostShard>> host_shards;
};

namespace {

// Geometry columns of a plan: one record per (tile, layer) geometry column,
// its source streams located in the decode output, and an assembly-output slice sized by
// data-independent bounds (every point part/ring consumes one source vertex, every line part one
// partOffsets entry, every polygon ring one ringOffsets entry):
//   parts <= Vs + n_po, rings <= Vs + n_po + n_ro, coordinates <= Vs (+ n_ro closing vertices).
void plan_geometry(covt_plan* p, int32_t nthr) {
    const size_t ns = p->info.size();
    // the column starting at stream i (the streams of one (tile, layer) geometry column are adjacent);
    // its record with assembly offsets from `off`, which it advances
    auto column = [&](size_t i, size_t& j, int64_t& off) {
        const covt_stream_info& s0 = p->info[i];
        covt_geom_info g{};
        g.tile = s0.tile;
        g.layer = s0.layer;
        g.column_type = s0.column_type;
        for (int k = 0; k < 6; ++k) g.stream[k] = -1;
        int64_t len[6] = {0, 0, 0, 0, 0, 0};
        j = i;
        for (; j < ns && p->info[j].tile == s0.tile && p->info[j].layer == s0.layer && p->info[j].column_kind == 1; ++j) {
            const covt_stream_info& s = p->info[j];
            const int k = s.stream_type - ST_GEOMETRY_TYPES;
            if (k < 0 || k > 5) continue;
            g.stream[k] = (int32_t)j;
            len[k] = k == 5 ? s.out_elems / 2 : s.out_elems;  // vertexBuffer: x,y pairs
            if (k == 5) g.column_type = s.column_type;
        }
        g.n_features = (int32_t)len[0];
        const int64_t vs = g.stream[4] >= 0 ? len[4] : len[5];
        const int64_t pcap = vs + len[2], rcap = vs + len[2] + len[3];
        g.flags = (p->format == COVT_FORMAT_GENC && (g.column_type == CT_ICE || g.column_type == CT_ICE_MORTON))
                      ? COVT_GEOM_CLOSED_IN_STREAM : 0;
        const int64_t ccap = vs + ((g.flags & COVT_GEOM_CLOSED_IN_STREAM) ? 0 : len[3]);
        const bool fits = rcap <= COVT_GEOM_MAX_CAP && ccap <= COVT_GEOM_MAX_CAP && len[0] <= COVT_GEOM_MAX_CAP;
        g.part_cap = fits ? (int32_t)pcap : 0;
        g.ring_cap = fits ? (int32_t)rcap : 0;
        g.coord_cap = fits ? (int32_t)ccap : 0;
        if (!fits) g.flags |= COVT_GEOM_TOO_LARGE;
        const int64_t nf = fits ? len[0] : 0;
        const int64_t bytes[6] = {4 * (nf + 1), 4 * ((int64_t)g.part_cap + 1), 4 * ((int64_t)g.ring_cap + 1),
                                  8 * (int64_t)g.coord_cap, 4 * (int64_t)g.part_cap, 4 * (int64_t)g.ring_cap};
        for (int k = 0; k < 6; ++k) {
            g.out_off[k] = off;
            off = align16(off + bytes[k]);
        }
        return g;
    };
    // stream ranges, one per thread, starting at column boundaries; each range's columns with assembly
    // offsets local to the range (16-byte aligned slices), rebased and concatenated in order
    const int64_t nt = std::max<int64_t>(1, std::min<int64_t>(nthr, (int64_t)ns / 4096 + 1));
    std::vector<size_t> cut((size_t)nt + 1);
    for (int64_t k = 0; k <= nt; ++k) {
        size_t i = (size_t)((int64_t)ns * k / nt);
        while (i > 0 && i < ns && p->info[i].column_kind == 1 && p->info[i - 1].column_kind == 1 &&
               p->info[i].tile == p->info[i - 1].tile && p->info[i].layer == p->info[i - 1].layer)
            ++i;  // (inside a column: move to its end)
        cut[(size_t)k] = k == nt ? ns : std::max(i, k ? cut[(size_t)k - 1] : (size_t)0);
    }
    std::vector<std::vector<covt_geom_info>> part((size_t)nt);
    std::vector<int64_t> part_off((size_t)nt);
    par_for((int32_t)nt, nt, [&](int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; ++k) {
            int64_t off = 0;
            for (size_t i = cut[(size_t)k]; i < cut[(size_t)k + 1];) {
                if (p->info[i].column_kind != 1) { ++i; continue; }
                size_t j;
                part[(size_t)k].push_back(column(i, j, off));
                i = j;
            }
            part_off[(size_t)k] = off;
        }
    });
    int64_t off = 0;
    size_t nc = 0;
    std::vector<int64_t> base((size_t)nt);
    std::vector<size_t> first((size_t)nt);
    for (int64_t k = 0; k < nt; ++k) {
        base[(size_t)k] = off;
        first[(size_t)k] = nc;
        off += part_off[(size_t)k];
        nc += part[(size_t)k].size();
    }
    p->asm_bytes = off;
    p->ginfo.resize(nc);
    std::vector<SortKey> order(nc);  // largest (coordinates + features) first, ties in tile order
    par_for((int32_t)nt, nt, [&](int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; ++k)
            for (size_t q = 0; q < part[(size_t)k].size(); ++q) {
                covt_geom_info g = part[(size_t)k][q];
                for (int m = 0; m < 6; ++m) g.out_off[m] += base[(size_t)k];
                const size_t c = first[(size_t)k] + q;
                p->ginfo[c] = g;
                order[c] = SortKey{(1ull << 40) - (uint64_t)((int64_t)g.coord_cap + g.n_features), (uint32_t)c};
            }
    });
    radix_sort(order);
    p->gdescs.resize(nc);
    par_for(nthr, (int64_t)nc, [&](int64_t k0, int64_t k1) {
        for (int64_t kk = k0; kk < k1; ++kk) {
            const size_t k = (size_t)kk;
            covt_geom_info& g = p->ginfo[order[k].i];
            covt_geom_desc d{};
            for (int m = 0; m < 6; ++m) {
                const int32_t si = g.stream[m];
                d.in_off[m] = si >= 0 ? p->info[(size_t)si].out_off : -1;
                d.in_len[m] = si >= 0 ? (int32_t)(m == 5 ? p->info[(size_t)si].out_elems / 2 : p->info[(size_t)si].out_elems) : 0;
                d.in_res[m] = si >= 0 ? p->info[(size_t)si].desc_index : -1;  // its decode status gates the column
                d.out_off[m] = g.out_off[m];
            }
            d.part_cap = g.part_cap;
            d.ring_cap = g.ring_cap;
            d.coord_cap = g.coord_cap;
            d.flags = (int32_t)g.flags;
            g.desc_index = (int32_t)k;
            p->gdescs[k] = d;
        }
    });
}

// Property (sub)columns (include/covt.h "Property columns"; CovtParser.decodePropertyColumn
// :276-354): their present / data / length streams join the decode launch as column_kind 2, and a
// record remembers where the materialization finds them.  Unsupported shapes get a flag instead of
// streams, in the order Java would throw: before anything (type, missing streams) or after the
// present stream was decoded (data encodings, non-dictionary strings).
// Stream / property records of a range of tiles, built by one host thread with output offsets and
// stream indices local to the range; covt_plan_create_ex rebases and concatenates the parts.
struct PlanPart {
    std::vector<covt_stream_info> info;
    std::vector<covt_prop_info> pinfo;
    std::vector<uint16_t> pflags;
    int64_t out_off = 0, in_bytes = 0, out_payload = 0, vertices = 0;
};
void plan_property(PlanPart* p, int32_t t, int64_t tile_off, const PropRaw& q, int id_mode, int64_t& out_off) {
    covt_prop_info pi = prop_info_of(q, t, tile_off);
    PropStreams ps;
    prop_streams(q, id_mode, ps);  // covt_props_plan.h: the same rule as the device plan
    for (int role = 0; role < 3; ++role) {
        if (!(ps.has >> role & 1u)) continue;
        const int64_t n = ps.count[role];
        const int elem = ps.elem[role];
        covt_stream_info si{};
        si.tile = t;
        si.layer = q.layer;
        si.column_kind = 2;
        si.stream_type = role;
        si.encoding = q.s_enc[role];
        si.column_type = q.ctype;
        si.num_values = q.s_nv[role];
        si.byte_length = q.s_bl[role];
        si.op = ps.op[role];
        si.elem_bytes = elem;
        si.in_off = tile_off + q.s_off[role];
        si.out_elems = n;
        si.out_off = out_off;
        out_off = align_out(out_off + n * elem);
        p->out_payload += n * elem;
        si.desc_index = (int32_t)n;  // temporarily: values to decode
        pi.stream[role] = (int32_t)p->info.size();
        p->info.push_back(si);
    }
    p->in_bytes += ps.in_bytes;
    p->pinfo.push_back(pi);
    p->pflags.push_back(ps.flags);
}

// Output slices of the property columns and the launch-ordered descriptors (after the decode
// streams got their launch rows).  A localized column's sub-columns share the owner's dictionary.
void plan_property_layout(covt_plan* p) {
    int64_t off = 0;
    const size_t np = p->pinfo.size();
    std::vector<int64_t> in_float(np), in_dict(np);
    size_t owner = 0;
    for (size_t k = 0; k < np; ++k) {
        covt_prop_info& pi = p->pinfo[k];
        in_float[k] = pi.out_off[1];
        in_dict[k] = pi.out_off[3];
        const bool own = (p->pflags[k] & COVT_PROP_DICT_OWNER) != 0;
        int64_t sz[4];
        prop_layout_sizes(pi, own, sz);  // covt_props_plan.h
        pi.out_off[0] = off;
        pi.out_off[1] = off + sz[0];
        off += sz[0] + sz[1];
        if (pi.type == COVT_PROP_STRING && own) {
            owner = k;
            pi.out_off[2] = off;
            pi.out_off[3] = off + sz[2];
            off += sz[2] + sz[3];
        } else if (pi.type == COVT_PROP_STRING && pi.lang > 0 && owner < k && p->pinfo[owner].tile == pi.tile &&
                   p->pinfo[owner].layer == pi.layer && p->pinfo[owner].column == pi.column) {
            pi.out_off[2] = p->pinfo[owner].out_off[2];
            pi.out_off[3] = p->pinfo[owner].out_off[3];
        } else {
            pi.out_off[2] = pi.out_off[3] = -1;
        }
    }
    p->prop_bytes = off;
    std::vector<SortKey> korder(np);  // largest (features + dictionary entries) first, ties in tile order
    for (size_t k = 0; k < np; ++k)
        korder[k] = SortKey{prop_order_key(p->pinfo[k]), (uint32_t)k};
    radix_sort(korder);
    std::vector<size_t> order(np);
    for (size_t k = 0; k < np; ++k) order[k] = korder[k].i;
    p->pdescs.resize(np);
    for (size_t k = 0; k < np; ++k) {
        covt_prop_info& pi = p->pinfo[order[k]];
        covt_prop_desc d{};
        auto s_out = [&](int role) { return pi.stream[role] >= 0 ? p->info[(size_t)pi.stream[role]].out_off : -1; };
        d.present_off = s_out(0);
        d.data_off = pi.type == COVT_PROP_FLOAT ? in_float[order[k]] : s_out(1);
        d.length_off = s_out(2);
        d.dict_in_off = pi.type == COVT_PROP_STRING ? in_dict[order[k]] : -1;
        for (int m = 0; m < 4; ++m) d.out_off[m] = pi.out_off[m];
        for (int m = 0; m < 3; ++m) d.res[m] = pi.stream[m] >= 0 ? p->info[(size_t)pi.stream[m]].desc_index : -1;
        d.n_features = pi.n_features;
        d.n_data = pi.n_data;
        d.n_dict = pi.n_dict;
        d.dict_bytes = pi.dict_bytes;
        d.type = (int16_t)pi.type;
        d.flags = (int16_t)p->pflags[order[k]];
        pi.desc_index = (int32_t)k;
        p->pdescs[k] = d;
    }
}

}  // namespace

extern "C" {

#ifndef COVT_BUILD_ID
#define COVT_BUILD_ID "unknown"
#endif
const char* covt_version(void) { return "covt-mi355x 0.4 (gfx950) src:" COVT_BUILD_ID; }

int covt_device_count(int32_t* n) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    if (n) *n = c;
    return COVT_OK;
}

int covt_decode_varint(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t n, int32_t* out) {
    return stream_call(buf, buf_len, pos, COVT_OP_VARINT_I32, n, 0, out, 4, (size_t)std::max(n, 0));
}
int covt_decode_zigzag_varint(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t n, int32_t* out) {
    return stream_call(buf, buf_len, pos, COVT_OP_VARINT_ZZ_I32, n, 0, out, 4, (size_t)std::max(n, 0));
}
int covt_decode_zigzag_delta_varint(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t n, int32_t* out) {
    return stream_call(buf, buf_len, pos, COVT_OP_VARINT_ZZ_DELTA_I32, n, 0, out, 4, (size_t)std::max(n, 0));
}
int covt_decode_zigzag_delta_varint_coordinates(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t n,
                                                int32_t* out) {
    return stream_call(buf, buf_len, pos, COVT_OP_VARINT_ZZ_DELTA_XY, n, 0, out, 4, (size_t)std::max(n, 0));
}
int covt_decode_rle(const uint8_t* buf, size_t buf_len, int32_t n, int32_t* pos, int32_t is_signed, int64_t* out) {
    return stream_call(buf, buf_len, pos, is_signed ? COVT_OP_RLE_S64 : COVT_OP_RLE_U64, n, 0, out, 8,
                       (size_t)std::max(n, 0));
}
int covt_decode_byte_rle(const uint8_t* buf, size_t buf_len, int32_t n, int32_t* pos, int32_t byte_length,
                         uint8_t* out) {
    if (!pos) return COVT_ERR_INVALID_ARG;
    const int32_t p0 = *pos;
    // the GeometryType range check belongs to decodeGeometryColumn, not to this method: raw bytes
    int st = stream_call(buf, buf_len, pos, COVT_OP_BYTE_RLE_RAW, n, 0, out, 1, (size_t)std::max(n, 0));
    // decodeByteRle(..., byteLength) advances by the metadata byteLength (DecodingUtils.java:286)
    if (!st) *pos = p0 + byte_length;
    return st;
}
// decodeByteRle(byte[], int, IntWrapper) (DecodingUtils.java:290-306) advances by the length of the
// values' re-encoding (getByteRleChunkSize :312-314 -> EncodingUtils.encodeByteRle, i.e. ORC
// RunLengthByteWriter): decoded on the GPU like :275, then the writer's output length is computed
// here from the decoded bytes (the Java code re-encodes them on the host as well).
int covt_decode_byte_rle_reencode(const uint8_t* buf, size_t buf_len, int32_t n, int32_t* pos, uint8_t* out) {
    if (!pos) return COVT_ERR_INVALID_ARG;
    const int32_t p0 = *pos;
    int st = stream_call(buf, buf_len, pos, COVT_OP_BYTE_RLE_RAW, n, 0, out, 1, (size_t)std::max(n, 0));
    if (st) return st;
    *pos = p0 + (int32_t)orc_byte_rle_length(out, n);
    return COVT_OK;
}
// decodeFloatsLE(byte[], IntWrapper, int) (DecodingUtils.java:446-453): a little-endian view of
// numValues*4 bytes (no decode arithmetic; the batch path reads float columns in place on the GPU).
int covt_decode_floats_le(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t n, float* out) {
    if (!pos || n < 0 || (!buf && buf_len) || (!out && n)) return COVT_ERR_INVALID_ARG;
    if (*pos < 0 || (size_t)*pos + 4 * (size_t)n > buf_len) return COVT_ERR_TRUNCATED;  // ByteBuffer.wrap bounds
    if (n) std::memcpy(out, buf + *pos, 4 * (size_t)n);
    *pos += 4 * n;
    return COVT_OK;
}
// decodeString(byte[], IntWrapper) (DecodingUtils.java:21-26): a 4-byte-capped varint length
// (decodeVarint(src, pos) :189-194), then that many UTF-8 bytes; returns where they are.
int covt_decode_string(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t* str_off, int32_t* str_len) {
    if (!pos || !str_off || !str_len || (!buf && buf_len)) return COVT_ERR_INVALID_ARG;
    if (*pos < 0) return COVT_ERR_TRUNCATED;
    size_t q = (size_t)*pos;
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {  // Java's cap: the 4th byte is always the last
        if (q >= buf_len) return COVT_ERR_TRUNCATED;
        const uint8_t b = buf[q++];
        v |= (uint32_t)(b & 0x7f) << (7 * k);
        if (!(b & 0x80)) break;
    }
    const int32_t len = (int32_t)v;
    if (len < 0 || q + (size_t)len > buf_len) return COVT_ERR_TRUNCATED;  // new String(...) bounds
    *str_off = (int32_t)q;
    *str_len = len;
    *pos = (int32_t)q + len;
    return COVT_OK;
}
int covt_decode_fastpfor_zigzag_delta(const uint8_t* buf, size_t buf_len, int32_t n, int32_t byte_length,
                                      int32_t* pos, int32_t* out) {
    return fpf_call(buf, buf_len, pos, COVT_OP_FPF_ZZ_DELTA_I32, n, byte_length, 0, out, (size_t)std::max(n, 0));
}
int covt_decode_fastpfor_delta_coordinates(const uint8_t* buf, size_t buf_len, int32_t n, int32_t byte_length,
                                           int32_t* pos, int32_t* out) {
    return fpf_call(buf, buf_len, pos, COVT_OP_FPF_ZZ_DELTA_XY, n, byte_length, 0, out, (size_t)std::max(n, 0));
}
int covt_decode_delta_varint_morton_codes(const uint8_t* buf, size_t buf_len, int32_t* pos, int32_t n_vertices,
                                          int32_t num_bits, int32_t* out) {
    if (num_bits < 0 || num_bits > 255) return COVT_ERR_INVALID_ARG;
    return stream_call(buf, buf_len, pos, COVT_OP_VARINT_DELTA_MORTON, n_vertices, num_bits, out, 4,
                       2 * (size_t)std::max(n_vertices, 0));
}
int covt_decode_fastpfor_delta_morton_codes(const uint8_t* buf, size_t buf_len, int32_t n_vertices,
                                            int32_t byte_length, int32_t* pos, int32_t num_bits, int32_t* out) {
    if (num_bits < 0 || num_bits > 255) return COVT_ERR_INVALID_ARG;
    return fpf_call(buf, buf_len, pos, COVT_OP_FPF_DELTA_MORTON, n_vertices, byte_length, num_bits, out,
                    2 * (size_t)std::max(n_vertices, 0));
}

// Test hook (not in covt.h): the plan's FastPFOR chunk start states for one stream, nch x 42 int32
// (the slots of pads [2..7], covt_internal.h kFpfStateSlots), as fpf_chunk_states computes them.
int covt_debug_fpf_chunk_states(const uint8_t* stream, int32_t byte_length, int32_t num_values, int64_t unit,
                                int64_t nch, int32_t* out);

int covt_plan_create(const uint8_t* bytes, const uint64_t* tile_offsets, const uint64_t* tile_sizes,
                     int32_t n_tiles, int32_t format, int32_t id_mode, covt_plan** out) {
    return covt_plan_create_ex(bytes, tile_offsets, tile_sizes, n_tiles, format, id_mode, 0u, out);
}

}  // extern "C"

namespace {
// Chunks of a long ORC RLE v1 stream for the split kernel: a host walk of its group headers (orc-core
// RunLengthIntegerReader / RunLengthByteReader framing: run = header, [delta,] base varint or byte;
// literal = header + 256 - h varints or bytes) cut at group starts every `unit` of cost (bytes +
// output bytes / 4).  Each chunk: {first byte, end byte, first value, values}; `consumed` = the bytes
// the one-wave decode reads (through the group that reaches num_values).  Empty when the stream does
// not frame num_values values in byte_length bytes: its one-wave decode then reports the error.
struct RleChunk {
    int32_t s, e, v0, nv;
};
std::vector<RleChunk> rle_chunks(const uint8_t* b, int32_t len, int op, int32_t n, int32_t elem, int64_t unit,
                                 int32_t& consumed) {
    const bool byte_rle = op == COVT_OP_BYTE_RLE_U8 || op == COVT_OP_BYTE_RLE_RAW;
    std::vector<RleChunk> ch;
    int32_t pos = 0, v = 0, cs = 0, cv = 0;
    auto varint = [&]() {
        do {
            if (pos >= len) return false;
        } while (b[pos++] & 0x80);
        return true;
    };
    while (v < n) {
        if (pos >= len) return {};
        if ((int64_t)(pos - cs) + (int64_t)(v - cv) * elem / 4 >= unit) {  // cut before this group
            ch.push_back(RleChunk{cs, pos, cv, v - cv});
            cs = pos;
            cv = v;
        }
        const uint8_t h = b[pos];
        if (h < 0x80) {
            if (byte_rle) {
                if (pos + 2 > len) return {};
                pos += 2;
            } else {
                pos += 2;
                if (pos > len || !varint()) return {};
            }
            v += h + 3;
        } else {
            const int32_t cnt = 256 - h;
            ++pos;
            if (byte_rle) {
                if (pos + cnt > len) return {};
                pos += cnt;
            } else {
                for (int32_t k = 0; k < cnt; ++k)
                    if (!varint()) return {};
            }
            v += cnt;
        }
    }
    ch.push_back(RleChunk{cs, pos, cv, n - cv});
    consumed = pos;
    if (ch.size() < 2) ch.clear();
    return ch;
}

// FastPFOR split chunks: each chunk's state at its first block, from a host walk of the page directories
// and block headers (JavaFastPFOR FastPFOR.decodePage framing, read exactly as run_fastpfor's pre-walk
// does): the container offset of the block's header, its packed-word index and the exception cursor of
// every dataTobePacked array.  The chunk then skips walking up to 255 headers before its range (the
// critical path of BASELINE config 3).  Stored in the chunk's pads [2..7], seven int32 slots each (all
// fields but op / num_bits / flags; covt_fpf_state_slot): [0] 1 = present, [1] the page's first value,
// [2] header offset, [3] packed word, [4 + k] cursor of array k (k = 0..32).  Where the walk cannot
// follow the framing it stops: later chunks get no state and walk (and report the error) on the device.
void fpf_chunk_states(const uint8_t* b, int32_t byte_length, int32_t n, int64_t unit, int64_t nch,
                      std::vector<int32_t>& st) {
    st.assign((size_t)nch * kFpfStateSlots, 0);
    const int64_t nw = byte_length / 4;
    if (nw <= 0 || unit % 256) return;
    auto W = [&](int64_t i) -> uint32_t {
        return ((uint32_t)b[4 * i] << 24) | ((uint32_t)b[4 * i + 1] << 16) | ((uint32_t)b[4 * i + 2] << 8) | b[4 * i + 3];
    };
    int32_t L = (int32_t)W(0);
    if (L < 0) return;
    L -= L % 256;
    if (L > n) return;
    int64_t p = 1;
    int32_t done = 0;
    while (done < L) {
        const int32_t thissize = std::min<int32_t>(L - done, 65536);
        const int64_t p0 = p;
        if (p0 >= nw) return;
        int64_t ie = p0 + (int32_t)W(p0);
        if (ie < 0 || ie >= nw) return;
        const int32_t bytesize = (int32_t)W(ie++);
        if (bytesize < 0 || bytesize > 3 * 65536 / 256 + 65536) return;
        const int64_t bcw = (bytesize + 3) / 4, bc = ie;
        if (bc + bcw >= nw) return;
        ie += bcw;
        uint32_t bm = W(ie++) & ~1u;  // (bc + bcw < nw)
        while (bm) {
            const int32_t k = __builtin_ctz(bm) + 1;
            bm &= bm - 1;
            if (ie >= nw) return;
            const int32_t size = (int32_t)W(ie++);
            if (size < 0) return;
            const int64_t groups = ((int64_t)size + 31) / 32;
            ie += groups * k - ((groups * 32 - size) * k) / 32;
        }
        const int32_t bclen = (int32_t)(bcw * 4), nblk = thissize / 256;
        auto cb = [&](int32_t q) -> uint32_t { return b[4 * bc + (q ^ 3)]; };  // container byte q
        int32_t cur = 0, xc[33] = {};
        int64_t pk = p0 + 1;
        for (int32_t j = 0; j < nblk; ++j) {
            const int64_t v = (int64_t)done + (int64_t)j * 256;
            if (j > 0 && v % unit == 0 && v / unit < nch) {  // chunk v / unit starts at block j of this page
                int32_t* s = st.data() + (size_t)(v / unit) * kFpfStateSlots;
                s[0] = 1;
                s[1] = done;
                s[2] = cur;
                s[3] = (int32_t)pk;
                for (int k = 0; k <= 32; ++k) s[4 + k] = xc[k];
            }
            if (cur + 3 > bclen + 1) return;  // (the device reads the header word through its window)
            const int32_t hb = (int32_t)(int8_t)cb(cur), ce = (int32_t)cb(cur + 1);
            const int32_t idx = ce > 0 && cur + 2 < bclen ? (int32_t)(int8_t)cb(cur + 2) - hb : 0;
            pk += 8 * hb;
            if (ce > 0 && idx >= 2 && idx <= 32) xc[idx] += ce;
            cur += ce > 0 ? 3 + ce : 2;
            if (cur > bclen) return;
        }
        done += thissize;
        p = ie;
    }
}
}  // namespace

extern "C" {

}  // extern "C"

bool covt_resolve_options(const covt_plan_options* in, covt_plan_options& o) {
    covt_plan_options d;
    if (!in) {
        covt_plan_options_init(&d);
        in = &d;
    }
    if (in->size != sizeof(covt_plan_options)) return false;
    o = *in;
    const bool props = (o.flags & COVT_PLAN_PROPERTIES) != 0;
    if (o.lane_max_bytes == 0) o.lane_max_bytes = props ? COVT_LANE_MAX_BYTES_PROPS : COVT_LANE_MAX_BYTES;
    if (o.lane_max_values == 0) o.lane_max_values = props ? COVT_LANE_MAX_VALUES_PROPS : COVT_LANE_MAX_VALUES;
    return o.lane_max_bytes <= 65535 && o.lane_max_values > 0 && o.lane_max_values <= 32767 && o.split_ratio >= 0 && o.split_chunk >= 64 && o.split_values >= 256 && o.split_values % 256 == 0 &&
           o.fpf_split_weight >= 1 && o.lane_min_streams >= 0 && o.split_max_streams >= 0 && (o.split_grow == 0 || o.split_grow == 1) && o.plan_threads >= 0 && o.prefault_threads >= 1 &&
           o.device_walk >= 0 && o.device_walk <= 256 && (o.host_prefault == 0 || o.host_prefault == 1);
}

extern "C" {

void covt_plan_options_init(covt_plan_options* o) {
    if (!o) return;
    *o = covt_plan_options{};
    o->size = (uint32_t)sizeof(covt_plan_options);
    o->flags = 0;
    o->split_min = COVT_SPLIT_MIN;
    o->split_ratio = COVT_SPLIT_RATIO;
    o->split_chunk = COVT_SPLIT_CHUNK;
    o->split_values = COVT_SPLIT_VALUES;
    o->fpf_split_weight = 1;
    o->lane_max_bytes = 0;   // auto: COVT_LANE_MAX_BYTES, or COVT_LANE_MAX_BYTES_PROPS with property columns
    o->lane_max_values = 0;  // auto: COVT_LANE_MAX_VALUES, or COVT_LANE_MAX_VALUES_PROPS
    o->lane_min_streams = COVT_LANE_MIN_STREAMS;
    o->plan_threads = 0;
    o->host_prefault = 1;
    o->prefault_threads = 8;
    o->device_walk = 0;
    o->split_max_streams = COVT_SPLIT_MAX_STREAMS;
    o->split_grow = 1;
}

int covt_plan_create_ex(const uint8_t* bytes, const uint64_t* tile_offsets, const uint64_t* tile_sizes,
                        int32_t n_tiles, int32_t format, int32_t id_mode, uint32_t flags, covt_plan** out) {
    covt_plan_options o;
    covt_plan_options_init(&o);
    o.flags = flags;
    return covt_plan_create_opts(bytes, tile_offsets, tile_sizes, n_tiles, format, id_mode, &o, out);
}

int covt_plan_create_opts(const uint8_t* bytes, const uint64_t* tile_offsets, const uint64_t* tile_sizes,
                          int32_t n_tiles, int32_t format, int32_t id_mode, const covt_plan_options* opts,
                          covt_plan** out) {
    covt_plan_options o;
    if (!covt_resolve_options(opts, o)) return COVT_ERR_INVALID_ARG;
    const uint32_t flags = o.flags;
    if (!out || n_tiles < 0 || (n_tiles && (!bytes || !tile_offsets || !tile_sizes))) return COVT_ERR_INVALID_ARG;
    if (flags & ~COVT_PLAN_PROPERTIES) return COVT_ERR_INVALID_ARG;
    if (format != COVT_FORMAT_GENC && format != COVT_FORMAT_GEND) return COVT_ERR_INVALID_ARG;
    auto* p = new covt_plan();
    p->opts = o;
    p->n_tiles = n_tiles;
    p->format = format;
    p->tile_status.assign((size_t)n_tiles, 0);
    p->tile_off.assign(tile_offsets, tile_offsets + n_tiles);
    p->tile_size.assign(tile_sizes, tile_sizes + n_tiles);
    // 1. container walks, tiles split over host threads (metadata only, independent per tile)
    struct Chunk {
        int32_t t0 = 0, t1 = 0;
        std::vector<RawStream> rs;
        std::vector<PropRaw> props;
        std::vector<int32_t> rs_end, props_end;  // per tile of the chunk: end index in rs / props
    };
    const int32_t n_thr = (int32_t)std::max<int64_t>(
        1, std::min<int64_t>({o.plan_threads > 0 ? (int64_t)o.plan_threads
                                                 : std::min<int64_t>(std::thread::hardware_concurrency(), 16),
                              ((int64_t)n_tiles + 63) / 64}));
    std::vector<Chunk> chunks((size_t)n_thr);
    auto walk_chunk = [&](Chunk* c) {
        c->rs.reserve((size_t)(c->t1 - c->t0) * 64);  // ~43 Id/Geometry streams per tile
        c->rs_end.reserve((size_t)(c->t1 - c->t0));
        c->props_end.reserve((size_t)(c->t1 - c->t0));
        for (int32_t t = c->t0; t < c->t1; ++t) {
            const uint8_t* tile = bytes + tile_offsets[t];
            const size_t r0 = c->rs.size(), q0 = c->props.size();
            std::vector<PropRaw>* pp = (flags & COVT_PLAN_PROPERTIES) ? &c->props : nullptr;
            const int st = format == COVT_FORMAT_GENC ? walk_genc(tile, (size_t)tile_sizes[t], c->rs, pp)
                                                      : walk_gend(tile, (size_t)tile_sizes[t], c->rs, pp);
            p->tile_status[(size_t)t] = st;
            if (st) {  // a failed tile contributes nothing
                c->rs.resize(r0);
                c->props.resize(q0);
            }
            c->rs_end.push_back((int32_t)c->rs.size());
            c->props_end.push_back((int32_t)c->props.size());
        }
    };
    {
        std::vector<std::thread> th;
        for (int32_t k = 0; k < n_thr; ++k) {
            chunks[(size_t)k].t0 = (int32_t)((int64_t)n_tiles * k / n_thr);
            chunks[(size_t)k].t1 = (int32_t)((int64_t)n_tiles * (k + 1) / n_thr);
            if (k + 1 < n_thr) th.emplace_back(walk_chunk, &chunks[(size_t)k]);
        }
        walk_chunk(&chunks[(size_t)n_thr - 1]);
        for (auto& x : th) x.join();
    }
    // 2. stream records and output slices in tile order: each thread builds its tiles' records with
    // output offsets and stream indices local to its range (every slice is 16-byte aligned, so a range's
    // layout does not depend on where it starts), then the parts are rebased and concatenated
    std::vector<PlanPart> parts((size_t)n_thr);
    par_for(n_thr, n_thr, [&](int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; ++k) {
            const Chunk& c = chunks[(size_t)k];
            PlanPart& pp = parts[(size_t)k];
            pp.info.reserve(c.rs.size());
            int32_t r = 0, q = 0;
            for (int32_t t = c.t0; t < c.t1; ++t) {
                const int32_t re = c.rs_end[(size_t)(t - c.t0)], qe = c.props_end[(size_t)(t - c.t0)];
                for (; r < re; ++r) {
                    const RawStream& s = c.rs[(size_t)r];
                    int op, elem;
                    int64_t nvals, out_elems;
                    choose_op(s, id_mode, op, nvals, elem, out_elems);
                    covt_stream_info si{};
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
                    si.in_off = (int64_t)tile_offsets[t] + s.off;
                    si.out_elems = op == COVT_OP_NONE ? 0 : out_elems;
                    si.out_off = pp.out_off;
                    pp.out_off = align_out(pp.out_off + si.out_elems * elem);
                    pp.in_bytes += s.bl;
                    pp.out_payload += si.out_elems * elem;
                    if (s.kind == 1 && s.type == ST_VERTEX_BUFFER)
                        pp.vertices += (s.ctype == CT_ICE || s.ctype == CT_ICE_MORTON) ? s.nv : s.nv / 2;
                    si.desc_index = (int32_t)nvals;  // temporarily: values to decode
                    pp.info.push_back(si);
                }
                for (; q < qe; ++q) plan_property(&pp, t, (int64_t)tile_offsets[t], c.props[(size_t)q], id_mode, pp.out_off);
            }
        }
    });
    {
        std::vector<int64_t> out_base((size_t)n_thr), info_base((size_t)n_thr), pinfo_base((size_t)n_thr);
        int64_t ob = 0, ib = 0, pb = 0;
        for (int32_t k = 0; k < n_thr; ++k) {
            const PlanPart& pp = parts[(size_t)k];
            out_base[(size_t)k] = ob;
            info_base[(size_t)k] = ib;
            pinfo_base[(size_t)k] = pb;
            ob += pp.out_off;
            ib += (int64_t)pp.info.size();
            pb += (int64_t)pp.pinfo.size();
            p->in_bytes += pp.in_bytes;
            p->out_payload += pp.out_payload;
            p->vertices += pp.vertices;
        }
        p->out_bytes = ob;
        p->info.resize((size_t)ib);
        p->pinfo.resize((size_t)pb);
        p->pflags.resize((size_t)pb);
        par_for(n_thr, n_thr, [&](int64_t k0, int64_t k1) {
            for (int64_t k = k0; k < k1; ++k) {
                PlanPart& pp = parts[(size_t)k];
                const int64_t o = out_base[(size_t)k], i0 = info_base[(size_t)k], q0 = pinfo_base[(size_t)k];
                for (size_t i = 0; i < pp.info.size(); ++i) {
                    covt_stream_info si = pp.info[i];
                    si.out_off += o;
                    p->info[(size_t)i0 + i] = si;
                }
                for (size_t i = 0; i < pp.pinfo.size(); ++i) {
                    covt_prop_info pi = pp.pinfo[i];
                    for (int m = 0; m < 3; ++m)
                        if (pi.stream[m] >= 0) pi.stream[m] += (int32_t)i0;
                    p->pinfo[(size_t)q0 + i] = pi;
                    p->pflags[(size_t)q0 + i] = pp.pflags[i];
                }
                PlanPart().info.swap(pp.info);  // free as we go
            }
        });
    }
    // 3. launch order: grouped by family (the lane family also by op, for op-uniform waves), largest
    // streams first inside a family so the long poles start early (launch_key, covt_internal.h); one
    // precomputed key per stream, ties in tile order
    const size_t ns = p->info.size();
    std::vector<SortKey> keys(ns);
    // split a stream only where one wave decoding it would outlast the launch.  A stream's cost is its
    // bytes + output bytes / 4 (the launch-order key below; FastPFOR and RLE time follows the values as
    // much as the bytes): split above COVT_SPLIT_MIN and above the batch's total cost /
    // COVT_SPLIT_RATIO (a wave decodes ~0.35 GB/s, the launch ~500 GB/s: a stream over ~1/1400 of the
    // batch is a long pole).  Big batches are throughput-bound and split nothing; single tiles and
    // small batches split their long streams.
    auto stream_cost = [](const covt_stream_info& s) {
        return (int64_t)s.byte_length + s.out_elems * s.elem_bytes / 4;
    };
    int64_t split_min = o.split_min;
    const int64_t split_ratio = o.split_ratio;
    int32_t lane_max = lane_limits(o.lane_max_bytes, o.lane_max_values);
    int64_t grow = 1;
    {
        // batch totals: cost (split threshold) and the streams the lane kernel would take (it decodes 64
        // streams per wave, each serially: a wave of 100-250-value streams takes ~80-110 us, worth it only
        // where tiny RLE streams outnumber the wave slots; in smaller batches every RLE stream gets a wave)
        std::atomic<int64_t> tot_cost{0}, tot_lane{0};
        par_for(n_thr, (int64_t)ns, [&](int64_t i0, int64_t i1) {
            int64_t cst = 0, nl = 0;
            for (int64_t i = i0; i < i1; ++i) {
                const auto& si = p->info[(size_t)i];
                cst += stream_cost(si);
                nl += lane_stream(si.op, si.desc_index, si.byte_length, lane_max);
            }
            tot_cost += cst;
            tot_lane += nl;
        });
        const int64_t total = tot_cost.load(), n_lane = tot_lane.load();
        if (split_min >= 0 && split_ratio > 0) split_min = std::max<int64_t>(split_min, total / split_ratio);
        if (o.split_max_streams > 0 && (int64_t)ns > o.split_max_streams) split_min = -1;
        if (n_lane < o.lane_min_streams) lane_max = -1;
        grow = split_grow_factor(total, o.split_grow);
    }
    const int64_t split_chunk = o.split_chunk * grow;
    const int64_t split_values = o.split_values * grow;  // FastPFOR: whole blocks
    // long RLE streams: chunk boundaries from the host walk (stream index -> chunks, consumed)
    std::unordered_map<size_t, std::pair<std::vector<RleChunk>, int32_t>> rle_split;
    if (split_min >= 0) {
        for (size_t i = 0; i < ns; ++i) {
            const auto& s = p->info[i];
            if (!split_rle_op(s.op) || stream_cost(s) <= split_min || s.desc_index <= 0) continue;
            int32_t consumed = 0;
            auto ch = rle_chunks(bytes + s.in_off, s.byte_length, s.op, s.desc_index, s.elem_bytes, split_chunk,
                                 consumed);
            if (!ch.empty()) rle_split.emplace(i, std::make_pair(std::move(ch), consumed));
        }
    }
    const int64_t fpf_w = o.fpf_split_weight;
    // descriptors per stream: 1, or COVT_SPLIT_SLOTS per chunk of a split stream
    std::vector<int32_t> ndesc(ns);
    par_for(n_thr, (int64_t)ns, [&](int64_t i0, int64_t i1) {
        for (int64_t ii = i0; ii < i1; ++ii) {
            const size_t i = (size_t)ii;
            const auto& s = p->info[i];
            const bool lane = lane_stream(s.op, s.desc_index, s.byte_length, lane_max);
            const auto rs = rle_split.empty() ? rle_split.end() : rle_split.find(i);
            const bool rsplit = rs != rle_split.end();
            // (FastPFOR: a wave's time follows the blocks, i.e. the values: their output counts fpf_w times)
            const int64_t scost = split_fpf_op(s.op) ? stream_cost(s) + (fpf_w - 1) * (s.out_elems * s.elem_bytes / 4)
                                                     : stream_cost(s);
            const bool split = split_stream(s.op, s.desc_index, scost, split_min, split_values) || rsplit;
            const uint64_t fam = split ? (uint64_t)(split_fpf_op(s.op) ? COVT_FAMILY_SPLIT_FPF
                                                    : rsplit           ? COVT_FAMILY_SPLIT_RLE
                                                                       : COVT_FAMILY_SPLIT)
                                 : lane ? (uint64_t)COVT_FAMILY_LANE : (uint64_t)covt_op_family_of(s.op);
#ifdef COVT_EXACT_ORDER  // (A/B: the exact cost-descending order of rounds 1-4)
            const uint64_t cost = std::min<uint64_t>((uint64_t)stream_cost(s), (1ull << 48) - 1);
            keys[i] = SortKey{(fam << 60) | ((lane ? (uint64_t)s.op : 0ull) << 52) | ((1ull << 48) - 1 - cost),
                              (uint32_t)i};
#else
            keys[i] = SortKey{launch_key((uint32_t)fam, fam == COVT_FAMILY_LANE, s.op, stream_cost(s)), (uint32_t)i};
#endif
            int64_t nd = 1;
            if (rsplit) {
                nd = (int64_t)rs->second.first.size() * COVT_SPLIT_SLOTS;
            } else if (split) {
                const bool fpf = fam == COVT_FAMILY_SPLIT_FPF;
                const int64_t unit = fpf ? split_values : split_chunk, tot = fpf ? s.desc_index : s.byte_length;
                nd = (tot + unit - 1) / unit * COVT_SPLIT_SLOTS;
            }
            ndesc[i] = (int32_t)nd;
        }
    });
    radix_sort(keys);  // stable: ties in tile order
    // 4. descriptors in launch order: offsets by a prefix sum over the sorted streams, filled in parallel
    std::vector<int64_t> dpos(ns + 1);
    dpos[0] = 0;
    for (size_t k = 0; k < ns; ++k) {
        dpos[k + 1] = dpos[k] + ndesc[keys[k].i];
        p->fam_counts[key_family(keys[k].k)] += ndesc[keys[k].i];
    }
    p->descs.resize((size_t)dpos[ns]);
    p->desc_stream.resize((size_t)dpos[ns]);
    par_for(n_thr, (int64_t)ns, [&](int64_t k0, int64_t k1) {
        for (int64_t kk = k0; kk < k1; ++kk) {
            const size_t k = (size_t)kk;
            const size_t i = keys[k].i;
            covt_stream_info& si = p->info[i];
            const int fam = key_family(keys[k].k);
            size_t o = (size_t)dpos[k];
            covt_stream_desc d{};
            d.in_off = (uint64_t)si.in_off;
            d.out_off = (uint64_t)si.out_off;
            d.avail = si.byte_length;
            d.num_values = si.desc_index;
            d.op = (uint8_t)si.op;
            d.num_bits = (uint8_t)si.num_bits;
            d.byte_length = si.byte_length;
            d.flags = fam == COVT_FAMILY_LANE ? COVT_DESC_LANE : 0;
            si.desc_index = (int32_t)o;
            for (int64_t q = 0; q < ndesc[i]; ++q) p->desc_stream[o + (size_t)q] = (int64_t)i;
            if (fam != COVT_FAMILY_SPLIT && fam != COVT_FAMILY_SPLIT_FPF && fam != COVT_FAMILY_SPLIT_RLE) {
                p->descs[o] = d;
                continue;
            }
            // RLE: the host walk's chunks
            auto rs = rle_split.find(i);
            if (rs != rle_split.end()) {
                const auto& ch = rs->second.first;
                for (size_t c = 0; c < ch.size(); ++c) {
                    covt_stream_desc cd = d;
                    cd.flags = COVT_DESC_SPLIT | COVT_DESC_SPLIT_RLE;
                    cd.avail = (int32_t)c;
                    p->descs[o++] = cd;
                    for (int q = 1; q < COVT_SPLIT_SLOTS; ++q) {
                        covt_stream_desc pd{};
                        pd.flags = COVT_DESC_SPLIT_PAD | COVT_DESC_SPLIT_RLE;
                        if (q == 1) pd.in_off = (uint64_t)ch[c].s, pd.out_off = (uint64_t)ch[c].e;
                        if (q == 2) pd.in_off = (uint64_t)ch[c].v0, pd.out_off = (uint64_t)ch[c].nv;
                        if (q == 3) pd.in_off = (uint64_t)rs->second.second;
                        p->descs[o++] = pd;
                    }
                }
                continue;
            }
            // chunk c: bytes [c * split_chunk, min((c + 1) * split_chunk, byte_length)) of a varint stream,
            // values [c * split_values, min((c + 1) * split_values, num_values)) of a FastPFOR stream
            const bool fpf = fam == COVT_FAMILY_SPLIT_FPF;
            const uint16_t fflag = fpf ? COVT_DESC_SPLIT_FPF : 0;
            const int64_t unit = fpf ? split_values : split_chunk, total = fpf ? d.num_values : d.byte_length;
            const int64_t nch = (total + unit - 1) / unit;
            std::vector<int32_t> fst;
            if (fpf) fpf_chunk_states(bytes + si.in_off, si.byte_length, d.num_values, unit, nch, fst);
            for (int64_t c = 0; c < nch; ++c) {
                covt_stream_desc cd = d;
                cd.flags = COVT_DESC_SPLIT | fflag;
                cd.avail = (int32_t)c;
                p->descs[o++] = cd;
                for (int q = 1; q < COVT_SPLIT_SLOTS; ++q) {
                    covt_stream_desc pd{};
                    pd.flags = COVT_DESC_SPLIT_PAD | fflag;
                    if (q == 1) {
                        pd.in_off = (uint64_t)(c * unit);
                        pd.out_off = (uint64_t)std::min<int64_t>((c + 1) * unit, total);
                    }
                    if (fpf && q >= 2)
                        for (int k = 0; k < 7; ++k)
                            std::memcpy((uint8_t*)&pd + covt_fpf_state_byte(k), &fst[(size_t)c * kFpfStateSlots + (size_t)(q - 2) * 7 + (size_t)k],
                                        4);
                    p->descs[o++] = pd;
                }
            }
        }
    });
    plan_geometry(p, n_thr);
    plan_property_layout(p);
    *out = p;
    return COVT_OK;
}

void covt_plan_destroy(covt_plan* plan) { delete plan; }
int64_t covt_plan_num_streams(const covt_plan* p) { return p ? (int64_t)p->info.size() : 0; }
int64_t covt_plan_output_bytes(const covt_plan* p) { return p ? p->out_bytes : 0; }
int covt_plan_totals(const covt_plan* p, int64_t* in_bytes, int64_t* out_bytes, int64_t* vertices) {
    if (!p) return COVT_ERR_INVALID_ARG;
    if (in_bytes) *in_bytes = p->in_bytes;
    if (out_bytes) *out_bytes = p->out_payload;
    if (vertices) *vertices = p->vertices;
    return COVT_OK;
}
int covt_plan_streams(const covt_plan* p, covt_stream_info* out) {
    if (!p || (!out && !p->info.empty())) return COVT_ERR_INVALID_ARG;
    if (!p->info.empty()) std::memcpy(out, p->info.data(), p->info.size() * sizeof(covt_stream_info));
    return COVT_OK;
}
int64_t covt_plan_num_descs(const covt_plan* p) { return p ? (int64_t)p->descs.size() : 0; }
int covt_plan_desc_streams(const covt_plan* p, int64_t* out) {
    if (!p || (!out && !p->desc_stream.empty())) return COVT_ERR_INVALID_ARG;
    if (!p->desc_stream.empty()) std::memcpy(out, p->desc_stream.data(), p->desc_stream.size() * sizeof(int64_t));
    return COVT_OK;
}
int covt_plan_descs(const covt_plan* p, covt_stream_desc* out) {
    if (!p || (!out && !p->descs.empty())) return COVT_ERR_INVALID_ARG;
    if (!p->descs.empty()) std::memcpy(out, p->descs.data(), p->descs.size() * sizeof(covt_stream_desc));
    return COVT_OK;
}
int covt_plan_tile_status(const covt_plan* p, int32_t* out) {
    if (!p || (!out && p->n_tiles)) return COVT_ERR_INVALID_ARG;
    if (p->n_tiles) std::memcpy(out, p->tile_status.data(), sizeof(int32_t) * (size_t)p->n_tiles);
    return COVT_OK;
}

int covt_decode_streams_device(const uint8_t* d_in, const covt_stream_desc* d_desc, int64_t n_streams,
                               uint8_t* d_out, covt_stream_result* d_res, void* hip_stream) {
    if (n_streams < 0 || (n_streams && (!d_in || !d_desc || !d_res))) return COVT_ERR_INVALID_ARG;
    if ((uintptr_t)d_in & 15) return COVT_ERR_INVALID_ARG;
    for (int f = 0; f < COVT_NUM_FAMILIES; ++f) {  // any order: each family kernel skips the others
        if (f >= COVT_FAMILY_SPLIT) continue;  // split chunks need the grouped launch
        const int st = covt_launch_family(f, d_in, d_desc, n_streams, d_out, d_res, (hipStream_t)hip_stream);
        if (st) return st;
    }
    return COVT_OK;
}

int covt_plan_family_counts(const covt_plan* p, int64_t counts[COVT_NUM_FAMILIES]) {
    if (!p || !counts) return COVT_ERR_INVALID_ARG;
    for (int f = 0; f < COVT_NUM_FAMILIES; ++f) counts[f] = p->fam_counts[f];
    return COVT_OK;
}

int covt_decode_streams_device_grouped(const uint8_t* d_in, const covt_stream_desc* d_desc,
                                       const int64_t family_counts[COVT_NUM_FAMILIES], uint8_t* d_out,
                                       covt_stream_result* d_res, void* hip_stream) {
    if (!family_counts || ((uintptr_t)d_in & 15)) return COVT_ERR_INVALID_ARG;
    return launch_grouped(d_in, d_desc, family_counts, d_out, d_res, (hipStream_t)hip_stream);
}

int covt_decode_streams_device_grouped_mode(const uint8_t* d_in, const covt_stream_desc* d_desc,
                                            const int64_t family_counts[COVT_NUM_FAMILIES], uint8_t* d_out,
                                            covt_stream_result* d_res, void* hip_stream, int32_t launch_mode) {
    if (!family_counts || ((uintptr_t)d_in & 15)) return COVT_ERR_INVALID_ARG;
    return launch_grouped(d_in, d_desc, family_counts, d_out, d_res, (hipStream_t)hip_stream, launch_mode);
}

}  // extern "C"

namespace {

// Tile ranges of the shards: contiguous in tile order (so each shard's inputs and, the plan's output
// layout being in tile order, its outputs are single byte ranges), cut where the running weight
// (stream bytes + output bytes) crosses k/n of the total.  For 10k tiles the imbalance is at most
// one tile (~0.01 %).
std::vector<std::pair<int32_t, int32_t>> shard_ranges(const covt_plan* p, int32_t n) {
    std::vector<double> w((size_t)p->n_tiles + 1, 0.0);
    for (const auto& si : p->info) w[(size_t)si.tile + 1] += (double)si.byte_length + (double)(si.out_elems * si.elem_bytes);
    for (int32_t t = 0; t < p->n_tiles; ++t) w[(size_t)t + 1] += w[(size_t)t];
    const double tot = w[(size_t)p->n_tiles];
    std::vector<std::pair<int32_t, int32_t>> r;
    int32_t t0 = 0;
    for (int32_t k = 0; k < n; ++k) {
        int32_t t1 = p->n_tiles;
        if (k + 1 < n) {
            const double cut = tot * (k + 1) / n;
            t1 = (int32_t)(std::lower_bound(w.begin() + t0, w.end(), cut) - w.begin());
            t1 = std::max(t0, std::min(t1, p->n_tiles));
        }
        r.emplace_back(t0, t1);
        t0 = t1;
    }
    return r;
}

}  // namespace

namespace {

void build_shards(const covt_plan* p, const std::vector<int32_t>& devs, std::vector<std::unique_ptr<HostShard>>& out) {
    out.clear();
    const auto rng = shard_ranges(p, (int32_t)devs.size());
    std::vector<int32_t> shard_of_tile((size_t)p->n_tiles, 0);
    for (size_t g = 0; g < rng.size(); ++g) {
        auto h = std::make_unique<HostShard>();
        h->device = devs[g];
        h->prefault = p->opts.host_prefault != 0;
        h->prefault_threads = p->opts.prefault_threads;
        const int32_t t0 = rng[g].first, t1 = rng[g].second;
        uint64_t lo = UINT64_MAX, hi = 0;
        for (int32_t t = t0; t < t1; ++t) {
            shard_of_tile[(size_t)t] = (int32_t)g;
            lo = std::min<uint64_t>(lo, p->tile_off[(size_t)t]);
            hi = std::max<uint64_t>(hi, p->tile_off[(size_t)t] + p->tile_size[(size_t)t]);
        }
        if (t1 > t0) {
            h->in_lo = lo & ~(uint64_t)15;  // keeps every stream's 16-byte window alignment
            h->in_len = hi - h->in_lo;
        }
        h->out_lo = INT64_MAX;
        out.push_back(std::move(h));
    }
    for (const auto& si : p->info) {  // output range of each shard (tile order = output order)
        HostShard& h = *out[(size_t)shard_of_tile[(size_t)si.tile]];
        h.out_lo = std::min<int64_t>(h.out_lo, si.out_off);
        h.out_len = std::max<int64_t>(h.out_len, si.out_off + si.out_elems * si.elem_bytes);
    }
    for (auto& h : out) {
        if (h->out_lo == INT64_MAX) h->out_lo = h->out_len = 0;
        else h->out_len -= h->out_lo;
    }
    for (size_t k = 0; k < p->descs.size(); ++k) {  // launch order restricted to each shard stays grouped
        const int64_t i = p->desc_stream[k];
        const covt_stream_info& si = p->info[(size_t)i];
        HostShard& h = *out[(size_t)shard_of_tile[(size_t)si.tile]];
        covt_stream_desc d = p->descs[k];
        if (!(d.flags & COVT_DESC_SPLIT_PAD)) {  // pads carry stream-relative chunk ranges
            d.in_off -= h.in_lo;
            d.out_off -= (uint64_t)h.out_lo;
        }
        h.fam[desc_family(d)]++;
        h.stream.push_back(si.desc_index == (int32_t)k ? i : -1);  // only a stream's own entry is its result
        h.descs.push_back(d);
    }
    for (auto& h : out) h->res.resize(h->descs.size());
}

int decode_host_shards(const covt_plan* p, const uint8_t* bytes, uint64_t n_bytes, const std::vector<int32_t>& devs,
                       uint8_t* host_out, covt_stream_result* host_res);

// argument checks of the host entry points, before anything touches the device
bool host_args_ok(const covt_plan* p, const uint8_t* bytes, uint64_t n_bytes, const uint8_t* host_out,
                  const covt_stream_result* host_res) {
    if (!p || (!host_res && !p->info.empty()) || (!host_out && p->out_bytes) || (!bytes && n_bytes)) return false;
    for (int32_t t = 0; t < p->n_tiles; ++t)  // the caller's buffer must hold every tile the plan names
        if (p->tile_off[(size_t)t] + p->tile_size[(size_t)t] > n_bytes) return false;
    return true;
}

}  // namespace

extern "C" {

int covt_plan_decode_host(const covt_plan* p, const uint8_t* bytes, uint64_t n_bytes, uint8_t* host_out,
                          covt_stream_result* host_res) {
    if (!host_args_ok(p, bytes, n_bytes, host_out, host_res)) return COVT_ERR_INVALID_ARG;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return COVT_ERR_DEVICE;
    return decode_host_shards(p, bytes, n_bytes, std::vector<int32_t>{dev}, host_out, host_res);
}

int covt_plan_decode_host_multi(const covt_plan* p, const uint8_t* bytes, uint64_t n_bytes, int32_t n_gpus,
                                uint8_t* host_out, covt_stream_result* host_res) {
    if (n_gpus < 1 || !host_args_ok(p, bytes, n_bytes, host_out, host_res)) return COVT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return COVT_ERR_DEVICE;
    std::vector<int32_t> devs((size_t)std::min(n_gpus, ndev));
    std::iota(devs.begin(), devs.end(), 0);
    return decode_host_shards(p, bytes, n_bytes, devs, host_out, host_res);
}

int covt_plan_decode_host_shards(const covt_plan* p, const uint8_t* bytes, uint64_t n_bytes, int32_t n_shards,
                                 const int32_t* shard_devices, uint8_t* host_out, covt_stream_result* host_res) {
    if (n_shards < 1 || !shard_devices || !host_args_ok(p, bytes, n_bytes, host_out, host_res))
        return COVT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return COVT_ERR_DEVICE;
    for (int32_t g = 0; g < n_shards; ++g)
        if (shard_devices[g] < 0 || shard_devices[g] >= ndev) return COVT_ERR_INVALID_ARG;
    return decode_host_shards(p, bytes, n_bytes, std::vector<int32_t>(shard_devices, shard_devices + n_shards),
                              host_out, host_res);
}

int covt_plan_release_device(const covt_plan* p) {
    if (!p) return COVT_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(p->host_mu);
    p->host_shards.clear();
    p->host_devs.clear();
    return COVT_OK;
}

}  // extern "C"

namespace {

int decode_host_shards(const covt_plan* p, const uint8_t* bytes, uint64_t n_bytes, const std::vector<int32_t>& devs,
                       uint8_t* host_out, covt_stream_result* host_res) {
    std::lock_guard<std::mutex> g(p->host_mu);  // one call per plan at a time; plans are independent
    int cur = 0;
    const bool have_cur = hipGetDevice(&cur) == hipSuccess;
    if (p->host_devs != devs) {
        p->host_shards.clear();
        build_shards(p, devs, p->host_shards);
        p->host_devs = devs;
    }
    const size_t n = p->host_shards.size();
    std::vector<int> st(n, COVT_OK);
    if (n == 1) {
        st[0] = p->host_shards[0]->run(bytes, host_out, host_res);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 0; k < n; ++k)
            th.emplace_back([&, k] { st[k] = p->host_shards[k]->run(bytes, host_out, host_res); });
        for (auto& t : th) t.join();
    }
    if (have_cur) (void)hipSetDevice(cur);
    for (int x : st)
        if (x) return x;
    return COVT_OK;
}

}  // namespace

extern "C" {

int64_t covt_plan_num_geometry_columns(const covt_plan* p) { return p ? (int64_t)p->ginfo.size() : 0; }
int64_t covt_plan_assembly_bytes(const covt_plan* p) { return p ? p->asm_bytes : 0; }
int covt_plan_geometry_columns(const covt_plan* p, covt_geom_info* out) {
    if (!p || (!out && !p->ginfo.empty())) return COVT_ERR_INVALID_ARG;
    if (!p->ginfo.empty()) std::memcpy(out, p->ginfo.data(), p->ginfo.size() * sizeof(covt_geom_info));
    return COVT_OK;
}
int covt_plan_geometry_descs(const covt_plan* p, covt_geom_desc* out) {
    if (!p || (!out && !p->gdescs.empty())) return COVT_ERR_INVALID_ARG;
    if (!p->gdescs.empty()) std::memcpy(out, p->gdescs.data(), p->gdescs.size() * sizeof(covt_geom_desc));
    return COVT_OK;
}

// Whole plan on the current device: the caller's tile bytes [0, n_bytes) go to the device as they
// lie (the plan's offsets index them), then decode, assembly and the copies back on one stream.
int covt_plan_assemble_host(const covt_plan* p, const uint8_t* bytes, uint64_t n_bytes, uint8_t* host_asm,
                            covt_geom_result* host_gres) {
    if (!p || (!bytes && n_bytes) || (!host_asm && p->asm_bytes) || (!host_gres && !p->ginfo.empty()))
        return COVT_ERR_INVALID_ARG;
    for (int32_t t = 0; t < p->n_tiles; ++t)
        if (p->tile_off[(size_t)t] + p->tile_size[(size_t)t] > n_bytes) return COVT_ERR_INVALID_ARG;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return COVT_ERR_DEVICE;
    const size_t nd = p->descs.size(), nc = p->gdescs.size();
    uint8_t *d_in = nullptr, *d_out = nullptr, *d_asm = nullptr;
    covt_stream_desc* d_desc = nullptr;
    covt_stream_result* d_res = nullptr;
    covt_geom_desc* d_gdesc = nullptr;
    covt_geom_result* d_gres = nullptr;
    int st = COVT_OK;
    auto chk = [&](hipError_t e) { if (e != hipSuccess && st == COVT_OK) st = COVT_ERR_DEVICE; };
    chk(hipMalloc(&d_in, (size_t)n_bytes + COVT_INPUT_PADDING));
    chk(hipMalloc(&d_out, (size_t)std::max<int64_t>(p->out_bytes, 16)));
    chk(hipMalloc(&d_asm, (size_t)std::max<int64_t>(p->asm_bytes, 16)));
    chk(hipMalloc(&d_desc, std::max<size_t>(nd, 1) * sizeof(covt_stream_desc)));
    chk(hipMalloc(&d_res, std::max<size_t>(nd, 1) * sizeof(covt_stream_result)));
    chk(hipMalloc(&d_gdesc, std::max<size_t>(nc, 1) * sizeof(covt_geom_desc)));
    chk(hipMalloc(&d_gres, std::max<size_t>(nc, 1) * sizeof(covt_geom_result)));
    std::vector<covt_geom_result> gres(nc);
    if (st == COVT_OK) {
        if (n_bytes) chk(hipMemcpyAsync(d_in, bytes, (size_t)n_bytes, hipMemcpyHostToDevice, s));
        chk(hipMemsetAsync(d_in + n_bytes, 0, COVT_INPUT_PADDING, s));
        if (nd) chk(hipMemcpyAsync(d_desc, p->descs.data(), nd * sizeof(covt_stream_desc), hipMemcpyHostToDevice, s));
        if (nc)
            chk(hipMemcpyAsync(d_gdesc, p->gdescs.data(), nc * sizeof(covt_geom_desc), hipMemcpyHostToDevice, s));
        if (st == COVT_OK && ((uintptr_t)d_in & 15)) st = COVT_ERR_DEVICE;
        if (st == COVT_OK) st = launch_grouped(d_in, d_desc, p->fam_counts, d_out, d_res, s);
        if (st == COVT_OK)
            st = covt_assemble_geometry_device(d_out, d_res, d_gdesc, (int64_t)nc, d_asm, d_gres, s);
        if (st == COVT_OK && p->asm_bytes)
            chk(hipMemcpyAsync(host_asm, d_asm, (size_t)p->asm_bytes, hipMemcpyDeviceToHost, s));
        if (st == COVT_OK && nc)
            chk(hipMemcpyAsync(gres.data(), d_gres, nc * sizeof(covt_geom_result), hipMemcpyDeviceToHost, s));
        chk(hipStreamSynchronize(s));
    }
    if (st == COVT_OK)
        for (size_t k = 0; k < nc; ++k) host_gres[k] = gres[(size_t)p->ginfo[k].desc_index];
    for (void* q : {(void*)d_in, (void*)d_out, (void*)d_asm, (void*)d_desc, (void*)d_res, (void*)d_gdesc, (void*)d_gres})
        if (q) (void)hipFree(q);
    (void)hipStreamDestroy(s);
    return st;
}

int64_t covt_plan_num_property_columns(const covt_plan* p) { return p ? (int64_t)p->pinfo.size() : 0; }
int64_t covt_plan_property_bytes(const covt_plan* p) { return p ? p->prop_bytes : 0; }
int covt_plan_property_columns(const covt_plan* p, covt_prop_info* out) {
    if (!p || (!out && !p->pinfo.empty())) return COVT_ERR_INVALID_ARG;
    if (!p->pinfo.empty()) std::memcpy(out, p->pinfo.data(), p->pinfo.size() * sizeof(covt_prop_info));
    return COVT_OK;
}
int covt_plan_property_descs(const covt_plan* p, covt_prop_desc* out) {
    if (!p || (!out && !p->pdescs.empty())) return COVT_ERR_INVALID_ARG;
    if (!p->pdescs.empty()) std::memcpy(out, p->pdescs.data(), p->pdescs.size() * sizeof(covt_prop_desc));
    return COVT_OK;
}

// Whole plan on the current device: tile bytes H2D as they lie, decode, property materialization,
// copies back on one stream.
int covt_plan_properties_host(const covt_plan* p, const uint8_t* bytes, uint64_t n_bytes, uint8_t* host_props,
                              covt_prop_result* host_pres) {
    if (!p || (!bytes && n_bytes) || (!host_props && p->prop_bytes) || (!host_pres && !p->pinfo.empty()))
        return COVT_ERR_INVALID_ARG;
    for (int32_t t = 0; t < p->n_tiles; ++t)
        if (p->tile_off[(size_t)t] + p->tile_size[(size_t)t] > n_bytes) return COVT_ERR_INVALID_ARG;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return COVT_ERR_DEVICE;
    const size_t nd = p->descs.size(), nc = p->pdescs.size();
    uint8_t *d_in = nullptr, *d_out = nullptr, *d_props = nullptr;
    covt_stream_desc* d_desc = nullptr;
    covt_stream_result* d_res = nullptr;
    covt_prop_desc* d_pdesc = nullptr;
    covt_prop_result* d_pres = nullptr;
    int st = COVT_OK;
    auto chk = [&](hipError_t e) { if (e != hipSuccess && st == COVT_OK) st = COVT_ERR_DEVICE; };
    chk(hipMalloc(&d_in, (size_t)n_bytes + COVT_INPUT_PADDING));
    chk(hipMalloc(&d_out, (size_t)std::max<int64_t>(p->out_bytes, 16)));
    chk(hipMalloc(&d_props, (size_t)std::max<int64_t>(p->prop_bytes, 16)));
    chk(hipMalloc(&d_desc, std::max<size_t>(nd, 1) * sizeof(covt_stream_desc)));
    chk(hipMalloc(&d_res, std::max<size_t>(nd, 1) * sizeof(covt_stream_result)));
    chk(hipMalloc(&d_pdesc, std::max<size_t>(nc, 1) * sizeof(covt_prop_desc)));
    chk(hipMalloc(&d_pres, std::max<size_t>(nc, 1) * sizeof(covt_prop_result)));
    std::vector<covt_prop_result> pres(nc);
    if (st == COVT_OK) {
        if (n_bytes) chk(hipMemcpyAsync(d_in, bytes, (size_t)n_bytes, hipMemcpyHostToDevice, s));
        chk(hipMemsetAsync(d_in + n_bytes, 0, COVT_INPUT_PADDING, s));
        if (nd) chk(hipMemcpyAsync(d_desc, p->descs.data(), nd * sizeof(covt_stream_desc), hipMemcpyHostToDevice, s));
        if (nc)
            chk(hipMemcpyAsync(d_pdesc, p->pdescs.data(), nc * sizeof(covt_prop_desc), hipMemcpyHostToDevice, s));
        if (st == COVT_OK && ((uintptr_t)d_in & 15)) st = COVT_ERR_DEVICE;
        if (st == COVT_OK) st = launch_grouped(d_in, d_desc, p->fam_counts, d_out, d_res, s);
        if (st == COVT_OK)
            st = covt_materialize_properties_device(d_in, d_out, d_res, d_pdesc, (int64_t)nc, d_props, d_pres, s);
        if (st == COVT_OK && p->prop_bytes)
            chk(hipMemcpyAsync(host_props, d_props, (size_t)p->prop_bytes, hipMemcpyDeviceToHost, s));
        if (st == COVT_OK && nc)
            chk(hipMemcpyAsync(pres.data(), d_pres, nc * sizeof(covt_prop_result), hipMemcpyDeviceToHost, s));
        chk(hipStreamSynchronize(s));
    }
    if (st == COVT_OK)
        for (size_t k = 0; k < nc; ++k) host_pres[k] = pres[(size_t)p->pinfo[k].desc_index];
    for (void* q : {(void*)d_in, (void*)d_out, (void*)d_props, (void*)d_desc, (void*)d_res, (void*)d_pdesc,
                    (void*)d_pres})
        if (q) (void)hipFree(q);
    (void)hipStreamDestroy(s);
    return st;
}

}  // extern "C"

extern "C" int covt_debug_fpf_chunk_states(const uint8_t* stream, int32_t byte_length, int32_t num_values, int64_t unit,
                                           int64_t nch, int32_t* out) {
    if (!out || nch < 0 || byte_length < 0 || (!stream && byte_length)) return COVT_ERR_INVALID_ARG;
    std::vector<int32_t> st;
    fpf_chunk_states(stream, byte_length, num_values, unit, nch, st);
    std::copy(st.begin(), st.end(), out);
    return COVT_OK;
}
