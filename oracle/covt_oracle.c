/*
 * covt_oracle.c -- TEST INFRASTRUCTURE ONLY (see covt_oracle.h).
 *
 * Plain-C restatement of the reference's Id/Geometry stream decode path with
 * Java integer semantics.  Every function cites the reference line it follows:
 *   DecodingUtils.java   = evaluation/java/src/main/java/com/covt/decoder/DecodingUtils.java
 *   CovtParser.java      = evaluation/java/src/main/java/com/covt/decoder/CovtParser.java
 *   GeometryUtils.java   = evaluation/java/src/main/java/com/covt/converter/GeometryUtils.java
 *   EncodingUtils.java   = evaluation/java/src/main/java/com/covt/converter/EncodingUtils.java
 * Third-party arithmetic (not vendored in the reference; restated from the published
 * algorithms):
 *   orc-core 1.8.1   RunLengthIntegerReader/Writer, RunLengthByteReader/Writer, SerializationUtils
 *   JavaFastPFOR 0.1.12  FastPFOR (BLOCK_SIZE 256, pageSize 65536), VariableByte, Composition
 */
#include "covt_oracle.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Java-semantics helpers                                                    */
/* ------------------------------------------------------------------------ */
static inline int32_t jzigzag(int32_t e) { /* DecodingUtils.java:252-254 */
    return (int32_t)(((uint32_t)e >> 1) ^ (uint32_t)(-(e & 1)));
}
static inline int32_t jadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t jshl(int32_t v, int32_t s) { return (int32_t)((uint32_t)v << (s & 31)); }

/* DecodingUtils.java:157-186: protobuf varint capped at 4 bytes; the 4th byte always ends it. */
static int jvarint(const uint8_t* src, size_t avail, int32_t* off, int32_t* value) {
    int32_t o = *off;
    if (o < 0) return ORC_ERR_ARG;
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) {
        if ((size_t)o >= avail) return ORC_ERR_TRUNCATED;
        uint8_t b = src[o++];
        v |= (uint32_t)(b & 0x7f) << (7 * i);
        if (i < 3 && (b & 0x80) == 0) break;
    }
    *off = o;
    *value = (int32_t)v;
    return ORC_OK;
}

/* orc SerializationUtils.readVulong: unbounded LEB128 into a long (shift masked to 6 bits). */
static int vulong(const uint8_t* src, size_t avail, int32_t* off, uint64_t* value) {
    int32_t o = *off;
    uint64_t r = 0;
    int shift = 0;
    uint8_t b;
    do {
        if (o < 0 || (size_t)o >= avail) return ORC_ERR_TRUNCATED;
        b = src[o++];
        r |= (uint64_t)(b & 0x7f) << (shift & 63);
        shift += 7;
    } while (b >= 0x80);
    *off = o;
    *value = r;
    return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* DecodingUtils varint family                                               */
/* ------------------------------------------------------------------------ */
int oracle_decode_varint(const uint8_t* src, size_t avail, int32_t* pos, int32_t n, int32_t* out) {
    if (n < 0) return ORC_ERR_ARG;
    for (int32_t i = 0; i < n; i++) { /* :38-42 */
        int st = jvarint(src, avail, pos, &out[i]);
        if (st) return st;
    }
    return ORC_OK;
}

int oracle_decode_zigzag_varint(const uint8_t* src, size_t avail, int32_t* pos, int32_t n, int32_t* out) {
    if (n < 0) return ORC_ERR_ARG;
    for (int32_t i = 0; i < n; i++) { /* :48-50 -> :247-250 */
        int32_t v;
        int st = jvarint(src, avail, pos, &v);
        if (st) return st;
        out[i] = jzigzag(v);
    }
    return ORC_OK;
}

int oracle_decode_zigzag_delta_varint(const uint8_t* src, size_t avail, int32_t* pos, int32_t n, int32_t* out) {
    if (n < 0) return ORC_ERR_ARG;
    int32_t prev = 0;
    for (int32_t i = 0; i < n; i++) { /* :58-63 */
        int32_t v;
        int st = jvarint(src, avail, pos, &v);
        if (st) return st;
        prev = jadd(prev, jzigzag(v));
        out[i] = prev;
    }
    return ORC_OK;
}

int oracle_decode_zigzag_delta_varint_coordinates(const uint8_t* src, size_t avail, int32_t* pos, int32_t n,
                                                  int32_t* out) {
    if (n < 0) return ORC_ERR_ARG;
    int32_t px = 0, py = 0;
    for (int32_t i = 0; i < n; i += 2) { /* :99-109 */
        int32_t dx, dy;
        int st = jvarint(src, avail, pos, &dx);
        if (st) return st;
        st = jvarint(src, avail, pos, &dy);
        if (st) return st;
        px = jadd(px, jzigzag(dx));
        py = jadd(py, jzigzag(dy));
        out[i] = px;
        if (i + 1 >= n) return ORC_ERR_COUNT; /* Java: values[i+1] -> ArrayIndexOutOfBounds */
        out[i + 1] = py;
    }
    return ORC_OK;
}

int oracle_decode_varint_u64(const uint8_t* src, size_t avail, int32_t* pos, int32_t n, uint64_t* out) {
    if (n < 0) return ORC_ERR_ARG;
    for (int32_t i = 0; i < n; i++) {
        int32_t start = *pos;
        int st = vulong(src, avail, pos, &out[i]);
        if (st) return st;
        if (*pos - start > 10) return ORC_ERR_HEADER; /* not a valid 64-bit LEB128 */
    }
    return ORC_OK;
}

/* GeometryUtils.java:34-47 */
static int32_t morton_axis(int32_t code, int32_t num_bits) {
    int32_t coordinate = 0;
    int64_t c = (int64_t)code; /* int promoted to long (sign-extended) for `code & (1L << 2i)` */
    for (int32_t i = 0; i < num_bits; i++) {
        int sh = (2 * i) & 63;
        int64_t bit = c & ((int64_t)1 << sh);
        coordinate = (int32_t)((int64_t)coordinate | (bit >> (i & 63))); /* `|=` narrows to int */
    }
    return coordinate;
}
void oracle_decode_morton(int32_t code, int32_t num_bits, int32_t* x, int32_t* y) {
    int32_t tile_extent = (int32_t)(2u << ((num_bits - 2) & 31));
    int32_t half = tile_extent / 2;
    *x = (int32_t)((uint32_t)morton_axis(code, num_bits) - (uint32_t)half);
    *y = (int32_t)((uint32_t)morton_axis(code >> 1, num_bits) - (uint32_t)half);
}

int oracle_decode_delta_varint_morton_codes(const uint8_t* src, size_t avail, int32_t* pos, int32_t n_vertices,
                                            int32_t num_bits, int32_t* out) {
    if (n_vertices < 0) return ORC_ERR_ARG;
    int32_t prev = 0;
    for (int32_t i = 0; i < n_vertices; i++) { /* :397-406: no zigzag */
        int32_t d;
        int st = jvarint(src, avail, pos, &d);
        if (st) return st;
        prev = jadd(prev, d);
        oracle_decode_morton(prev, num_bits, &out[2 * i], &out[2 * i + 1]);
    }
    return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* ORC RLE v1 (orc-core 1.8.1)                                               */
/* ------------------------------------------------------------------------ */
/* RunLengthIntegerReader.readValues/next.  Reads exactly as the Java reader does:
 * every literal group is read whole when it is entered. */
static int rle_read(const uint8_t* src, size_t avail, int32_t start, int32_t n, int is_signed, int64_t* out,
                    int32_t* end) {
    int32_t o = start;
    int32_t done = 0;
    while (done < n) {
        if (o < 0 || (size_t)o >= avail) return ORC_ERR_TRUNCATED; /* EOFException */
        int control = src[o++];
        if (control < 0x80) {
            int cnt = control + 3; /* MIN_REPEAT_SIZE */
            if ((size_t)o >= avail) return ORC_ERR_TRUNCATED;
            int delta = (int8_t)src[o++];
            uint64_t base;
            int st = vulong(src, avail, &o, &base);
            if (st) return st;
            int64_t b = is_signed ? (int64_t)((base >> 1) ^ (uint64_t)(-(int64_t)(base & 1))) : (int64_t)base;
            for (int i = 0; i < cnt && done < n; i++) /* literals[0] + used * delta */
                out[done++] = (int64_t)((uint64_t)b + (uint64_t)(int64_t)(int32_t)(i * delta));
        } else {
            int cnt = 0x100 - control;
            for (int i = 0; i < cnt; i++) {
                uint64_t v;
                int st = vulong(src, avail, &o, &v);
                if (st) return st;
                int64_t x = is_signed ? (int64_t)((v >> 1) ^ (uint64_t)(-(int64_t)(v & 1))) : (int64_t)v;
                if (done < n) out[done++] = x;
            }
        }
    }
    *end = o;
    return ORC_OK;
}

/* orc SerializationUtils.writeVulong */
typedef struct { uint8_t* p; int64_t n, cap; } wbuf;
static void wput(wbuf* w, uint8_t b) {
    if (w->n < w->cap) w->p[w->n] = b;
    w->n++;
}
static void wvulong(wbuf* w, uint64_t v) {
    while (1) {
        if ((v & ~(uint64_t)0x7f) == 0) { wput(w, (uint8_t)v); return; }
        wput(w, (uint8_t)(0x80 | (v & 0x7f)));
        v >>= 7;
    }
}

/* RunLengthIntegerWriter (MIN_REPEAT_SIZE 3, MAX_REPEAT_SIZE 130, MAX_LITERAL_SIZE 128,
 * MIN_DELTA -128, MAX_DELTA 127). */
typedef struct {
    wbuf w;
    int is_signed, repeat, num_literals, tail_run;
    int64_t delta;
    int64_t literals[128];
} rle_writer;
static void rle_put_value(rle_writer* r, int64_t v) {
    if (r->is_signed) wvulong(&r->w, ((uint64_t)v << 1) ^ (uint64_t)(v >> 63));
    else wvulong(&r->w, (uint64_t)v);
}
static void rle_write_values(rle_writer* r) {
    if (r->num_literals != 0) {
        if (r->repeat) {
            wput(&r->w, (uint8_t)(r->num_literals - 3));
            wput(&r->w, (uint8_t)(int8_t)r->delta);
            rle_put_value(r, r->literals[0]);
        } else {
            wput(&r->w, (uint8_t)(-r->num_literals));
            for (int i = 0; i < r->num_literals; i++) rle_put_value(r, r->literals[i]);
        }
        r->repeat = 0;
        r->num_literals = 0;
        r->tail_run = 0;
    }
}
static void rle_write(rle_writer* r, int64_t value) {
    if (r->num_literals == 0) {
        r->literals[r->num_literals++] = value;
        r->tail_run = 1;
    } else if (r->repeat) {
        if (value == (int64_t)((uint64_t)r->literals[0] + (uint64_t)r->delta * (uint64_t)r->num_literals)) {
            r->num_literals += 1;
            if (r->num_literals == 130) rle_write_values(r);
        } else {
            rle_write_values(r);
            r->literals[r->num_literals++] = value;
            r->tail_run = 1;
        }
    } else {
        if (r->tail_run == 1) {
            r->delta = (int64_t)((uint64_t)value - (uint64_t)r->literals[r->num_literals - 1]);
            r->tail_run = (r->delta < -128 || r->delta > 127) ? 1 : 2;
        } else if (value == (int64_t)((uint64_t)r->literals[r->num_literals - 1] + (uint64_t)r->delta)) {
            r->tail_run += 1;
        } else {
            r->delta = (int64_t)((uint64_t)value - (uint64_t)r->literals[r->num_literals - 1]);
            r->tail_run = (r->delta < -128 || r->delta > 127) ? 1 : 2;
        }
        if (r->tail_run == 3) {
            if (r->num_literals + 1 == 3) {
                r->repeat = 1;
                r->num_literals += 1;
            } else {
                r->num_literals -= 2;
                int64_t base = r->literals[r->num_literals];
                rle_write_values(r);
                r->literals[0] = base;
                r->repeat = 1;
                r->num_literals = 3;
            }
        } else {
            r->literals[r->num_literals++] = value;
            if (r->num_literals == 128) rle_write_values(r);
        }
    }
}

int64_t oracle_encode_rle(const int64_t* v, int64_t n, int is_signed, uint8_t* dst, int64_t cap) {
    rle_writer r;
    memset(&r, 0, sizeof r);
    r.w.p = dst;
    r.w.cap = dst ? cap : 0;
    r.is_signed = is_signed;
    for (int64_t i = 0; i < n; i++) rle_write(&r, v[i]);
    rle_write_values(&r); /* flush */
    if (dst && r.w.n > cap) return ORC_ERR_ARG;
    return r.w.n;
}

/* RunLengthByteWriter */
int64_t oracle_encode_byte_rle(const uint8_t* v, int64_t n, uint8_t* dst, int64_t cap) {
    wbuf w = {dst, 0, dst ? cap : 0};
    uint8_t lit[128];
    int num = 0, repeat = 0, tail = 0;
#define BRLE_FLUSH()                                                    \
    do {                                                                \
        if (num) {                                                      \
            if (repeat) {                                               \
                wput(&w, (uint8_t)(num - 3));                           \
                wput(&w, lit[0]);                                       \
            } else {                                                    \
                wput(&w, (uint8_t)(-num));                              \
                for (int q = 0; q < num; q++) wput(&w, lit[q]);         \
            }                                                           \
            repeat = 0;                                                 \
            num = 0;                                                    \
            tail = 0;                                                   \
        }                                                               \
    } while (0)
    for (int64_t i = 0; i < n; i++) {
        uint8_t value = v[i];
        if (num == 0) {
            lit[num++] = value;
            tail = 1;
        } else if (repeat) {
            if (value == lit[0]) {
                num += 1;
                if (num == 130) BRLE_FLUSH();
            } else {
                BRLE_FLUSH();
                lit[num++] = value;
                tail = 1;
            }
        } else {
            tail = (value == lit[num - 1]) ? tail + 1 : 1;
            if (tail == 3) {
                if (num + 1 == 3) {
                    repeat = 1;
                    num += 1;
                } else {
                    num -= 2;
                    BRLE_FLUSH();
                    lit[0] = value;
                    repeat = 1;
                    num = 3;
                }
            } else {
                lit[num++] = value;
                if (num == 128) BRLE_FLUSH();
            }
        }
    }
    BRLE_FLUSH();
#undef BRLE_FLUSH
    if (dst && w.n > cap) return ORC_ERR_ARG;
    return w.n;
}

int oracle_decode_rle(const uint8_t* src, size_t avail, int32_t n, int32_t* pos, int is_signed, int64_t* out,
                      int32_t* consumed) {
    if (n < 0) return ORC_ERR_ARG;
    int32_t end;
    int st = rle_read(src, avail, *pos, n, is_signed, out, &end);
    if (st) return st;
    if (consumed) *consumed = end - *pos;
    /* :268-270 getRleChunkSize -> EncodingUtils.encodeRle(values, signed).length */
    int64_t size = oracle_encode_rle(out, n, is_signed, NULL, 0);
    *pos = (int32_t)(*pos + size);
    return ORC_OK;
}

/* RunLengthByteReader + decodeByteRle(..., byteLength) DecodingUtils.java:275-288 */
int oracle_decode_byte_rle(const uint8_t* src, size_t avail, int32_t n, int32_t* pos, int32_t byte_length,
                           uint8_t* out, int32_t* consumed) {
    if (n < 0) return ORC_ERR_ARG;
    int32_t o = *pos, done = 0;
    while (done < n) {
        if (o < 0 || (size_t)o >= avail) return ORC_ERR_TRUNCATED;
        int control = src[o++];
        if (control < 0x80) {
            int cnt = control + 3;
            if ((size_t)o >= avail) return ORC_ERR_TRUNCATED;
            uint8_t b = src[o++];
            for (int i = 0; i < cnt && done < n; i++) out[done++] = b;
        } else {
            int cnt = 0x100 - control;
            if ((size_t)o + (size_t)cnt > avail) return ORC_ERR_TRUNCATED;
            for (int i = 0; i < cnt; i++) {
                if (done < n) out[done++] = src[o];
                o++;
            }
        }
    }
    if (consumed) *consumed = o - *pos;
    *pos += byte_length;
    return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* JavaFastPFOR 0.1.12: Composition(FastPFOR, VariableByte)                  */
/* ------------------------------------------------------------------------ */
#define FPF_BLOCK 256
#define FPF_PAGE 65536
#define FPF_BC_CAP (3 * FPF_PAGE / FPF_BLOCK + FPF_PAGE) /* byteContainer capacity */

typedef struct {
    const uint8_t* src;
    size_t avail;
    int32_t pos;
    int32_t nw;
} words;
/* DecodingUtils.java:317-327: Arrays.copyOfRange (zero-padded past the array) viewed as
 * big-endian ints; ceil(byteLength / 4) with integer division = floor. */
static inline uint32_t wget(const words* w, int64_t i) {
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
        int64_t b = (int64_t)w->pos + 4 * i + k;
        uint8_t x = (b >= 0 && (uint64_t)b < w->avail) ? w->src[b] : 0;
        v = (v << 8) | x;
    }
    return v;
}
/* BitPacking.fastunpack: value r of a 32-value group = bits [r*b, r*b+b) of the LSB-first
 * concatenation of b words starting at word `base`.  Words at index >= limit read as 0. */
static inline uint32_t unpack_at(const words* w, int64_t base, int32_t r, int32_t b, int64_t limit) {
    if (b == 0) return 0;
    int64_t bit = (int64_t)r * b;
    int64_t wi = base + (bit >> 5);
    int off = (int)(bit & 31);
    uint64_t lo = (wi < limit) ? wget(w, wi) : 0;
    uint64_t hi = (off + b > 32 && wi + 1 < limit) ? wget(w, wi + 1) : 0;
    uint64_t cat = lo | (hi << 32);
    uint64_t mask = (b == 32) ? 0xffffffffull : ((1ull << b) - 1);
    return (uint32_t)((cat >> off) & mask);
}

int oracle_fastpfor_uncompress(const uint8_t* src, size_t avail, int32_t pos, int32_t byte_length, int32_t n,
                               uint32_t* raw, int32_t* decoded) {
    if (n < 0 || byte_length < 0 || pos < 0) return ORC_ERR_ARG;
    memset(raw, 0, sizeof(uint32_t) * (size_t)n);
    words W = {src, avail, pos, byte_length / 4};
    const int64_t nw = W.nw;
    *decoded = 0;
    if (nw == 0) return ORC_OK; /* Composition.uncompress: inlength == 0 */
    /* FastPFOR.uncompress: header = number of FastPFOR-coded values */
    int32_t L = (int32_t)wget(&W, 0);
    if (L < 0) return ORC_ERR_HEADER;
    L -= L % FPF_BLOCK; /* Util.greatestMultiple */
    if (L > n) return ORC_ERR_COUNT;
    int64_t p = 1;
    int32_t done = 0;
    static const int32_t kmax = 33;
    while (done < L) {
        int32_t thissize = (L - done < FPF_PAGE) ? (L - done) : FPF_PAGE;
        /* decodePage */
        int64_t p0 = p;
        if (p0 >= nw) return ORC_ERR_TRUNCATED;
        int64_t inexcept = p0 + (int32_t)wget(&W, p0);
        if (inexcept < 0 || inexcept >= nw) return ORC_ERR_TRUNCATED;
        int32_t bytesize = (int32_t)wget(&W, inexcept++);
        if (bytesize < 0 || bytesize > FPF_BC_CAP) return ORC_ERR_HEADER;
        int64_t bc_words = (bytesize + 3) / 4;
        if (inexcept + bc_words > nw) return ORC_ERR_TRUNCATED;
        int64_t bc_base = inexcept;
        inexcept += bc_words;
        if (inexcept >= nw) return ORC_ERR_TRUNCATED;
        uint32_t bitmap = wget(&W, inexcept++);
        int64_t xstart[33];
        int32_t xsize[33], xptr[33];
        for (int k = 0; k < kmax; k++) { xstart[k] = 0; xsize[k] = -1; xptr[k] = 0; }
        for (int k = 2; k <= 32; k++) {
            if (bitmap & (1u << (k - 1))) {
                if (inexcept >= nw) return ORC_ERR_TRUNCATED;
                int32_t size = (int32_t)wget(&W, inexcept++);
                if (size < 0) return ORC_ERR_HEADER;
                int64_t groups = ((int64_t)size + 31) / 32;
                xstart[k] = inexcept;
                xsize[k] = size;
                inexcept += groups * k;
                inexcept -= ((groups * 32 - size) * k) / 32; /* overflow * k / 32 */
            }
        }
        /* the byte container: LE bytes of the BE words at bc_base */
        int64_t bc = 0;
        const int64_t bc_limit = bc_words * 4;
#define BC_GET(dst)                                                                     \
    do {                                                                                \
        if (bc >= bc_limit) return ORC_ERR_HEADER;                                      \
        uint32_t w_ = wget(&W, bc_base + (bc >> 2));                                    \
        (dst) = (uint8_t)(w_ >> (8 * (bc & 3)));                                        \
        bc++;                                                                           \
    } while (0)
        int64_t tmpinpos = p0 + 1;
        for (int32_t run = 0; run < thissize / FPF_BLOCK; run++) {
            uint8_t bb, cc;
            BC_GET(bb);
            BC_GET(cc);
            int32_t b = (int8_t)bb;
            int32_t cexcept = cc;
            if (b < 0 || b > 32) return ORC_ERR_HEADER; /* fastunpack: unsupported bit width */
            uint32_t* o = raw + done + run * FPF_BLOCK;
            for (int mb = 0; mb < 8; mb++) {
                if (tmpinpos + b > nw) return ORC_ERR_TRUNCATED;
                for (int r = 0; r < 32; r++) o[mb * 32 + r] = unpack_at(&W, tmpinpos, r, b, nw);
                tmpinpos += b;
            }
            if (cexcept > 0) {
                uint8_t mbits;
                BC_GET(mbits);
                int32_t index = (int8_t)mbits - b;
                if (index == 1) {
                    for (int k = 0; k < cexcept; k++) {
                        uint8_t pp;
                        BC_GET(pp);
                        o[pp] |= (uint32_t)1 << (b & 31);
                    }
                } else {
                    if (index < 2 || index > 32 || xsize[index] < 0) return ORC_ERR_HEADER;
                    for (int k = 0; k < cexcept; k++) {
                        uint8_t pp;
                        BC_GET(pp);
                        int32_t i = xptr[index]++;
                        if (i >= xsize[index]) return ORC_ERR_HEADER;
                        /* dataTobePacked[index][i]: words past the stream read as 0 */
                        uint32_t ex = unpack_at(&W, xstart[index] + (int64_t)(i / 32) * index, i % 32, index, nw);
                        o[pp] |= ex << (b & 31);
                    }
                }
            }
        }
#undef BC_GET
        done += thissize;
        p = inexcept;
    }
    /* VariableByte.uncompress over the remaining words */
    int32_t outpos = L;
    int s = 0;
    int32_t v = 0, shift = 0;
    for (int64_t q = p; q < nw;) {
        uint32_t val = wget(&W, q);
        int32_t c = (int8_t)(uint8_t)(val >> s);
        s += 8;
        q += s >> 5;
        s &= 31;
        v = jadd(v, jshl(c & 127, shift));
        if ((c & 128) == 128) {
            if (outpos >= n) return ORC_ERR_COUNT; /* out[tmpoutpos++] past numValues */
            raw[outpos++] = (uint32_t)v;
            v = 0;
            shift = 0;
        } else {
            shift += 7;
        }
    }
    *decoded = outpos;
    return ORC_OK;
}

static int fpf_prologue(const uint8_t* src, size_t avail, int32_t n, int32_t byte_length, int32_t* pos,
                        uint32_t** raw) {
    if (n < 0 || byte_length < 0) return ORC_ERR_ARG;
    *raw = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    if (!*raw) return ORC_ERR_ARG;
    int32_t dec;
    int st = oracle_fastpfor_uncompress(src, avail, *pos, byte_length, n, *raw, &dec);
    if (st) {
        free(*raw);
        *raw = NULL;
    }
    return st;
}

int oracle_decode_fastpfor_zigzag_delta(const uint8_t* src, size_t avail, int32_t n, int32_t byte_length,
                                        int32_t* pos, int32_t* out) {
    uint32_t* raw;
    int st = fpf_prologue(src, avail, n, byte_length, pos, &raw);
    if (st) return st;
    int32_t prev = 0;
    for (int32_t i = 0; i < n; i++) { /* :337-343 */
        prev = jadd(prev, jzigzag((int32_t)raw[i]));
        out[i] = prev;
    }
    free(raw);
    *pos += byte_length; /* :345 */
    return ORC_OK;
}

int oracle_decode_fastpfor_delta_coordinates(const uint8_t* src, size_t avail, int32_t n, int32_t byte_length,
                                             int32_t* pos, int32_t* out) {
    uint32_t* raw;
    int st = fpf_prologue(src, avail, n, byte_length, pos, &raw);
    if (st) return st;
    *pos += byte_length; /* :374 */
    int32_t px = 0, py = 0;
    for (int32_t i = 0; i < n; i += 2) { /* :369-389 */
        if (i + 1 >= n) { free(raw); return ORC_ERR_COUNT; }
        px = jadd(px, jzigzag((int32_t)raw[i]));
        py = jadd(py, jzigzag((int32_t)raw[i + 1]));
        out[i] = px;
        out[i + 1] = py;
    }
    free(raw);
    return ORC_OK;
}

int oracle_decode_fastpfor_delta_morton_codes(const uint8_t* src, size_t avail, int32_t n_vertices,
                                              int32_t byte_length, int32_t* pos, int32_t num_bits, int32_t* out) {
    uint32_t* raw;
    int st = fpf_prologue(src, avail, n_vertices, byte_length, pos, &raw);
    if (st) return st;
    *pos += byte_length; /* :430 */
    int32_t prev = 0;
    for (int32_t i = 0; i < n_vertices; i++) { /* :434-441 */
        prev = jadd(prev, (int32_t)raw[i]);
        oracle_decode_morton(prev, num_bits, &out[2 * i], &out[2 * i + 1]);
    }
    free(raw);
    return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* encoders for synthetic streams                                            */
/* ------------------------------------------------------------------------ */
int64_t oracle_encode_varints_u64(const uint64_t* v, int64_t n, uint8_t* dst, int64_t cap) {
    /* EncodingUtils.putVarInt :105-114 */
    wbuf w = {dst, 0, dst ? cap : 0};
    for (int64_t i = 0; i < n; i++) {
        uint64_t x = v[i];
        do {
            uint64_t bits = x & 0x7f;
            x >>= 7;
            wput(&w, (uint8_t)(bits + (x != 0 ? 0x80 : 0)));
        } while (x != 0);
    }
    if (dst && w.n > cap) return ORC_ERR_ARG;
    return w.n;
}

static int bits_of(uint32_t v) { return v ? 32 - __builtin_clz(v) : 0; }

/* BitPacking.fastpack (masking): LSB-first concatenation of 32 b-bit values into b words */
static void pack32(const uint32_t* in, uint32_t* outw, int b) {
    for (int k = 0; k < b; k++) outw[k] = 0;
    if (b == 0) return;
    uint64_t mask = (b == 32) ? 0xffffffffull : ((1ull << b) - 1);
    for (int r = 0; r < 32; r++) {
        uint64_t val = in[r] & mask;
        int64_t bit = (int64_t)r * b;
        int wi = (int)(bit >> 5), off = (int)(bit & 31);
        outw[wi] |= (uint32_t)(val << off);
        if (off + b > 32) outw[wi + 1] |= (uint32_t)(val >> (32 - off));
    }
}

typedef struct { uint32_t* p; int64_t n, cap; } ibuf;
static void iput(ibuf* b, uint32_t v) {
    if (b->n < b->cap) b->p[b->n] = v;
    b->n++;
}

/* FastPFOR.encodePage + getBestBFromData (overheadofeachexcept = 8) */
static void fpf_encode_page(const uint32_t* in, int32_t thissize, ibuf* out) {
    int64_t headerpos = out->n;
    iput(out, 0);
    uint8_t* bcont = (uint8_t*)malloc(FPF_BC_CAP + 8);
    int64_t bcn = 0;
    uint32_t* xdata[33];
    int32_t xptr[33] = {0};
    for (int k = 0; k < 33; k++) xdata[k] = (uint32_t*)calloc((size_t)thissize + 32, sizeof(uint32_t));
    for (int32_t blk = 0; blk < thissize; blk += FPF_BLOCK) {
        const uint32_t* v = in + blk;
        int freqs[33] = {0};
        for (int k = 0; k < FPF_BLOCK; k++) freqs[bits_of(v[k])]++;
        int bestb = 32;
        while (freqs[bestb] == 0) bestb--;
        int maxb = bestb;
        int bestcost = bestb * FPF_BLOCK;
        int cexcept = 0, bestc = 0;
        for (int b = bestb - 1; b >= 0; --b) {
            cexcept += freqs[b + 1];
            if (cexcept == FPF_BLOCK) break;
            int thiscost = cexcept * 8 + cexcept * (maxb - b) + b * FPF_BLOCK + 8;
            if (maxb - b == 1) thiscost -= cexcept;
            if (thiscost < bestcost) {
                bestcost = thiscost;
                bestb = b;
                bestc = cexcept;
            }
        }
        bcont[bcn++] = (uint8_t)bestb;
        bcont[bcn++] = (uint8_t)bestc;
        if (bestc > 0) {
            bcont[bcn++] = (uint8_t)maxb;
            int index = maxb - bestb;
            for (int k = 0; k < FPF_BLOCK; k++) {
                if ((bestb == 32 ? 0u : (v[k] >> bestb)) != 0) {
                    bcont[bcn++] = (uint8_t)k;
                    xdata[index][xptr[index]++] = v[k] >> bestb;
                }
            }
        }
        for (int k = 0; k < FPF_BLOCK; k += 32) {
            uint32_t tmp[32];
            pack32(v + k, tmp, bestb);
            for (int q = 0; q < bestb; q++) iput(out, tmp[q]);
        }
    }
    if (out->n > headerpos && headerpos < out->cap) out->p[headerpos] = (uint32_t)(out->n - headerpos);
    int64_t bytesize = bcn;
    while (bcn & 3) bcont[bcn++] = 0;
    iput(out, (uint32_t)bytesize);
    for (int64_t i = 0; i < bcn; i += 4) /* byteContainer (LITTLE_ENDIAN) -> ints */
        iput(out, (uint32_t)bcont[i] | ((uint32_t)bcont[i + 1] << 8) | ((uint32_t)bcont[i + 2] << 16) |
                      ((uint32_t)bcont[i + 3] << 24));
    uint32_t bitmap = 0;
    for (int k = 2; k <= 32; k++)
        if (xptr[k] != 0) bitmap |= 1u << (k - 1);
    iput(out, bitmap);
    for (int k = 2; k <= 32; k++) {
        if (xptr[k] == 0) continue;
        iput(out, (uint32_t)xptr[k]);
        int64_t j = 0;
        for (; j < xptr[k]; j += 32) {
            uint32_t tmp[32];
            pack32(xdata[k] + j, tmp, k);
            for (int q = 0; q < k; q++) iput(out, tmp[q]);
        }
        int64_t overflow = j - xptr[k];
        out->n -= overflow * k / 32;
    }
    for (int k = 0; k < 33; k++) free(xdata[k]);
    free(bcont);
}

int64_t oracle_encode_fastpfor(const uint32_t* v, int64_t n, uint8_t* dst, int64_t cap) {
    int64_t wcap = n * 2 + 4096;
    ibuf out = {(uint32_t*)malloc(sizeof(uint32_t) * (size_t)wcap), 0, wcap};
    if (n > 0) { /* Composition.compress: nothing at all for an empty input */
        int64_t L = n - n % FPF_BLOCK;
        iput(&out, (uint32_t)L); /* FastPFOR header (Composition writes 0 when FastPFOR wrote nothing) */
        for (int64_t done = 0; done < L;) {
            int32_t ts = (int32_t)((L - done) < FPF_PAGE ? (L - done) : FPF_PAGE);
            fpf_encode_page(v + done, ts, &out);
            done += ts;
        }
        /* VariableByte.compress of the tail */
        int64_t tn = n - L;
        if (tn > 0) {
            uint8_t* vb = (uint8_t*)malloc((size_t)tn * 5 + 8);
            int64_t m = 0;
            for (int64_t i = L; i < n; i++) {
                uint64_t x = v[i];
                while (x >= 128) {
                    vb[m++] = (uint8_t)(x & 127);
                    x >>= 7;
                }
                vb[m++] = (uint8_t)(x | 128);
            }
            while (m & 3) vb[m++] = 0;
            for (int64_t i = 0; i < m; i += 4)
                iput(&out, (uint32_t)vb[i] | ((uint32_t)vb[i + 1] << 8) | ((uint32_t)vb[i + 2] << 16) |
                               ((uint32_t)vb[i + 3] << 24));
            free(vb);
        }
    }
    int64_t nbytes = out.n * 4;
    if (out.n > out.cap || (dst && nbytes > cap)) {
        free(out.p);
        return ORC_ERR_ARG;
    }
    if (dst) /* EncodingUtils.encodeFastPfor128 :172-186: big-endian bytes */
        for (int64_t i = 0; i < out.n; i++) {
            uint32_t w = out.p[i];
            dst[4 * i] = (uint8_t)(w >> 24);
            dst[4 * i + 1] = (uint8_t)(w >> 16);
            dst[4 * i + 2] = (uint8_t)(w >> 8);
            dst[4 * i + 3] = (uint8_t)w;
        }
    free(out.p);
    return nbytes;
}

/* ------------------------------------------------------------------------ */
/* Container walkers                                                         */
/* ------------------------------------------------------------------------ */
static int rd_u64(const uint8_t* t, size_t len, int64_t* o, uint64_t* v) {
    if (*o < 0 || *o > 0x7fffffff) return ORC_ERR_TRUNCATED;
    int32_t oo = (int32_t)*o;
    int st = vulong(t, len, &oo, v);
    *o = oo;
    return st;
}
static int rd_j32(const uint8_t* t, size_t len, int64_t* o, int32_t* v) {
    if (*o < 0 || *o > 0x7fffffff) return ORC_ERR_TRUNCATED;
    int32_t oo = (int32_t)*o;
    int st = jvarint(t, len, &oo, v);
    *o = oo;
    return st;
}
static int nlz32(uint32_t x) { return x ? __builtin_clz(x) : 32; }

enum { ST_PRESENT = 0, ST_DATA = 1, ST_LENGTH, ST_DICTIONARY, ST_GEOMETRY_TYPES, ST_GEOMETRY_OFFSETS,
       ST_PART_OFFSETS, ST_RING_OFFSETS, ST_VERTEX_OFFSETS, ST_VERTEX_BUFFER, ST_Z, ST_M };

static int genc_stream_type(const uint8_t* s, uint64_t n) {
    static const char* names[] = {"present", "data", "length", "dictionary", "geometry_types",
                                  "geometry_offsets", "part_offsets", "ring_offsets", "vertex_offsets",
                                  "vertex_buffer"};
    for (int i = 0; i < 10; i++)
        if (strlen(names[i]) == n && memcmp(names[i], s, n) == 0) return i;
    return -1;
}

typedef struct { int32_t type, enc, nv, bl; } smeta;

static int emit(oracle_stream* out, int32_t max_out, int32_t* cnt, const oracle_stream* s) {
    if (out && *cnt < max_out) out[*cnt] = *s;
    (*cnt)++;
    return ORC_OK;
}

/* Gen C (all committed fixtures), SURVEY Appendix A.1 */
static int walk_genc(const uint8_t* t, size_t len, oracle_stream* out, int32_t max_out, int32_t* n_out) {
    int64_t o = 0;
    uint64_t version, nlayers;
    int st;
    int32_t cnt = 0;
    if ((st = rd_u64(t, len, &o, &version))) return st;
    if ((st = rd_u64(t, len, &o, &nlayers))) return st;
    if (version != 1) return ORC_ERR_HEADER;
    for (uint64_t L = 0; L < nlayers; L++) {
        uint64_t nl, extent, nfeat, ncols;
        if ((st = rd_u64(t, len, &o, &nl))) return st;
        if ((uint64_t)o + nl > len) return ORC_ERR_TRUNCATED;
        o += (int64_t)nl;
        if ((st = rd_u64(t, len, &o, &extent))) return st;
        if ((st = rd_u64(t, len, &o, &nfeat))) return st;
        if ((st = rd_u64(t, len, &o, &ncols))) return st;
        if (ncols > 4096) return ORC_ERR_HEADER;
        /* column metadata */
        typedef struct { int kind, dtype, ctype, ns; smeta s[256]; } cmeta;
        cmeta* cols = (cmeta*)calloc(ncols ? ncols : 1, sizeof(cmeta));
        for (uint64_t c = 0; c < ncols; c++) {
            uint64_t cn, ns;
            if ((st = rd_u64(t, len, &o, &cn))) goto fail;
            if ((uint64_t)o + cn + 2 > len) { st = ORC_ERR_TRUNCATED; goto fail; }
            const uint8_t* cname = t + o;
            o += (int64_t)cn;
            cols[c].dtype = t[o++];
            cols[c].ctype = t[o++];
            cols[c].kind = (cn == 2 && memcmp(cname, "id", 2) == 0) ? 0
                           : ((cn == 8 && memcmp(cname, "geometry", 8) == 0) || cols[c].dtype == 6) ? 1 : 2;
            if ((st = rd_u64(t, len, &o, &ns))) goto fail;
            if (ns > 256) { st = ORC_ERR_HEADER; goto fail; }
            cols[c].ns = (int)ns;
            for (uint64_t s = 0; s < ns; s++) {
                uint64_t sn, nv, bl;
                if ((st = rd_u64(t, len, &o, &sn))) goto fail;
                if ((uint64_t)o + sn > len) { st = ORC_ERR_TRUNCATED; goto fail; }
                cols[c].s[s].type = genc_stream_type(t + o, sn);
                o += (int64_t)sn;
                if ((st = rd_u64(t, len, &o, &nv))) goto fail;
                if ((st = rd_u64(t, len, &o, &bl))) goto fail;
                if ((uint64_t)o >= len) { st = ORC_ERR_TRUNCATED; goto fail; }
                cols[c].s[s].enc = t[o++];
                if (nv > 0x7fffffff || bl > 0x7fffffff) { st = ORC_ERR_HEADER; goto fail; }
                cols[c].s[s].nv = (int32_t)nv;
                cols[c].s[s].bl = (int32_t)bl;
            }
        }
        /* layer data */
        for (uint64_t c = 0; c < ncols; c++) {
            cmeta* cm = &cols[c];
            if (cm->kind == 1) {
                /* geometry streams are laid out in StreamType order whatever the metadata order */
                for (int type = ST_GEOMETRY_TYPES; type <= ST_VERTEX_BUFFER; type++) {
                    for (int s = 0; s < cm->ns; s++) {
                        if (cm->s[s].type != type) continue;
                        oracle_stream os = {(int32_t)L, 1, type, cm->s[s].enc, cm->ctype, cm->s[s].nv, cm->s[s].bl,
                                            32 - nlz32((uint32_t)extent), o, (int32_t)extent, (int32_t)nfeat};
                        emit(out, max_out, &cnt, &os);
                        o += cm->s[s].bl;
                    }
                }
                for (int s = 0; s < cm->ns; s++) /* unknown stream kinds after the known ones */
                    if (cm->s[s].type < ST_GEOMETRY_TYPES || cm->s[s].type > ST_VERTEX_BUFFER) o += cm->s[s].bl;
            } else {
                for (int s = 0; s < cm->ns; s++) {
                    if (cm->kind == 0 && cm->s[s].type == ST_DATA) {
                        oracle_stream os = {(int32_t)L, 0, ST_DATA, cm->s[s].enc, cm->ctype, cm->s[s].nv, cm->s[s].bl,
                                            32 - nlz32((uint32_t)extent), o, (int32_t)extent, (int32_t)nfeat};
                        emit(out, max_out, &cnt, &os);
                    }
                    o += cm->s[s].bl;
                }
            }
            if ((uint64_t)o > len) { st = ORC_ERR_TRUNCATED; goto fail; }
        }
        free(cols);
        continue;
    fail:
        free(cols);
        return st;
    }
    if ((uint64_t)o != len) return ORC_ERR_HEADER; /* the walk must end exactly at EOF */
    *n_out = cnt;
    return ORC_OK;
}

/* Gen D property columns carry an implicit present stream: the writer puts its bytes first in the column
 * but no metadata for it (CovtConverter.addNamedColumnMetadata skips StreamType.PRESENT, :452-458), and
 * decodePropertyColumn reads it with the 3-argument decodeByteRle (CovtParser.java:296): ceil(numFeatures/8)
 * bytes, advancing by the length of their re-encoding (DecodingUtils.java:290-306).  BOOLEAN columns have
 * none (:280-291).  Gen D ColumnDataType: BOOLEAN = 0 (converter/ColumnDataType.java). */
int oracle_gend_present_length(const uint8_t* t, size_t len, int64_t off, int32_t n_features, int32_t* length) {
    const int32_t nb = (int32_t)(((int64_t)(n_features > 0 ? n_features : 0) + 7) / 8);
    if (off < 0 || (uint64_t)off > len) return ORC_ERR_TRUNCATED;
    uint8_t* v = (uint8_t*)malloc((size_t)nb + 1);
    int32_t pos = 0, cons = 0;
    int st = oracle_decode_byte_rle(t + off, len - (size_t)off, nb, &pos, 0, v, &cons);
    if (!st) *length = (int32_t)oracle_encode_byte_rle(v, nb, NULL, 0); /* getByteRleChunkSize */
    free(v);
    return st;
}

/* Gen D: CovtParser.decodeLayerMetadata :574-652 + the column loop of decodeCovt :56-85 */
static int walk_gend(const uint8_t* t, size_t len, oracle_stream* out, int32_t max_out, int32_t* n_out) {
    int64_t o = 0;
    int32_t cnt = 0, layer = 0;
    int st;
    while ((uint64_t)o < len) {
        int hdr = t[o++];
        int optimized = hdr & 1;
        int32_t v, extent, nfeat, ncols;
        if (optimized) {
            if ((st = rd_j32(t, len, &o, &v))) return st; /* layerId */
        } else {
            if ((st = rd_j32(t, len, &o, &v))) return st; /* decodeString: length + UTF-8 */
            if (v < 0 || (uint64_t)o + (uint64_t)v > len) return ORC_ERR_TRUNCATED;
            o += v;
        }
        if ((st = rd_j32(t, len, &o, &extent))) return st;
        if ((st = rd_j32(t, len, &o, &nfeat))) return st;
        if ((st = rd_j32(t, len, &o, &ncols))) return st;
        if (ncols < 0 || ncols > 4096) return ORC_ERR_HEADER;
        typedef struct { int kind, dtype, ctype; smeta s[12]; int have[12]; } dmeta;
        dmeta* cols = (dmeta*)calloc(ncols ? (size_t)ncols : 1, sizeof(dmeta));
        for (int32_t c = 0; c < ncols; c++) {
            if (optimized || c == 0) {
                int32_t cid;
                if ((st = rd_j32(t, len, &o, &cid))) goto fail;
                cols[c].kind = cid == 0 ? 0 : cid == 1 ? 1 : 2;
            } else {
                int32_t sl;
                if ((st = rd_j32(t, len, &o, &sl))) goto fail;
                if (sl < 0 || (uint64_t)o + (uint64_t)sl > len) { st = ORC_ERR_TRUNCATED; goto fail; }
                cols[c].kind = (sl == 2 && memcmp(t + o, "id", 2) == 0) ? 0
                               : (sl == 8 && memcmp(t + o, "geometry", 8) == 0) ? 1 : 2;
                o += sl;
            }
            if ((uint64_t)o >= len) { st = ORC_ERR_TRUNCATED; goto fail; }
            int desc = t[o++];
            cols[c].dtype = (desc >> 3) & 0xF;
            cols[c].ctype = desc & 0x7;
            if (cols[c].ctype > 4) { st = ORC_ERR_HEADER; goto fail; }
            for (;;) {
                if ((uint64_t)o >= len) { st = ORC_ERR_TRUNCATED; goto fail; }
                int sd = t[o++];
                int type = sd >> 4, enc = sd & 0xF;
                if (type > ST_M || enc > 9) { st = ORC_ERR_HEADER; goto fail; }
                int32_t nv, bl;
                if ((st = rd_j32(t, len, &o, &nv))) goto fail;
                if ((st = rd_j32(t, len, &o, &bl))) goto fail;
                cols[c].s[type] = (smeta){type, enc, nv, bl}; /* TreeMap.put: last one wins */
                cols[c].have[type] = 1;
                if (cols[c].dtype == 8 && type == ST_VERTEX_BUFFER) break;
                if (type == ST_DATA && cols[c].ctype == 0) break;
                if (type == ST_DICTIONARY) break;
            }
        }
        for (int32_t c = 0; c < ncols; c++) {
            dmeta* cm = &cols[c];
            if (cm->kind == 2 && cm->dtype != 0) { /* implicit present stream (oracle_gend_present_length) */
                int32_t pl = 0;
                if ((st = oracle_gend_present_length(t, len, o, nfeat, &pl))) goto fail;
                o += pl;
            }
            for (int type = 0; type < 12; type++) { /* TreeMap<StreamType> order */
                if (!cm->have[type] || (cm->kind == 2 && type == ST_PRESENT)) continue;
                int is_hot = (cm->kind == 0 && type == ST_DATA) ||
                             (cm->kind == 1 && type >= ST_GEOMETRY_TYPES && type <= ST_VERTEX_BUFFER);
                if (is_hot) {
                    oracle_stream os = {layer, cm->kind, type, cm->s[type].enc, cm->ctype, cm->s[type].nv,
                                        cm->s[type].bl, 32 - nlz32((uint32_t)extent), o, extent, nfeat};
                    emit(out, max_out, &cnt, &os);
                }
                if (cm->s[type].bl < 0) { st = ORC_ERR_HEADER; goto fail; }
                o += cm->s[type].bl;
            }
            if ((uint64_t)o > len) { st = ORC_ERR_TRUNCATED; goto fail; }
        }
        free(cols);
        layer++;
        continue;
    fail:
        free(cols);
        return st;
    }
    *n_out = cnt;
    return ORC_OK;
}

int oracle_walk_tile(const uint8_t* tile, size_t len, int format, oracle_stream* out, int32_t max_out,
                     int32_t* n_out) {
    if (format == ORACLE_FMT_GENC) return walk_genc(tile, len, out, max_out, n_out);
    if (format == ORACLE_FMT_GEND) return walk_gend(tile, len, out, max_out, n_out);
    return ORC_ERR_ARG;
}

/* ------------------------------------------------------------------------ */
/* Stream dispatch (CovtParser.decodeGeometryColumn :392-511, decodedIds :552-572) */
/* ------------------------------------------------------------------------ */
enum { ENC_VARINT = 1, ENC_VARINT_DELTA_ZZ = 4, ENC_RLE = 5, ENC_FPF_ZZ = 9 };

int oracle_stream_output(const oracle_stream* s, int id_mode, int32_t* elem_bytes, int64_t* n_elems) {
    int64_t n = s->num_values;
    (void)id_mode;
    if (s->column_kind == 0) {
        *elem_bytes = 8;
        *n_elems = n;
        return ORC_OK;
    }
    switch (s->stream_type) {
    case ST_GEOMETRY_TYPES: *elem_bytes = 1; *n_elems = n; return ORC_OK;
    case ST_VERTEX_BUFFER:
        *elem_bytes = 4;
        /* ICE_MORTON: numValues = vertices -> 2n ints; ICE (Q4): build rule decodes 2n ints */
        *n_elems = (s->column_type == 4 || s->column_type == 3) ? 2 * n : n;
        return ORC_OK;
    default: *elem_bytes = 4; *n_elems = n; return ORC_OK;
    }
}

int oracle_decode_stream(const uint8_t* tile, size_t len, const oracle_stream* s, int id_mode, void* out,
                         int32_t* consumed) {
    if (s->offset < 0 || (uint64_t)s->offset + (uint64_t)s->byte_length > len) return ORC_ERR_TRUNCATED;
    const uint8_t* p = tile + s->offset;
    size_t avail = (size_t)s->byte_length; /* reads bounded by the stream (strict) */
    int32_t pos = 0, n = s->num_values;
    int st;
    *consumed = 0;
    if (s->column_kind == 0) {
        int64_t* o64 = (int64_t*)out;
        int enc = s->encoding;
        if (enc == ENC_RLE || (enc == ENC_VARINT_DELTA_ZZ && id_mode == ORACLE_ID_FORMAT)) {
            int32_t c;
            st = oracle_decode_rle(p, avail, n, &pos, 0, o64, &c);
            if (!st) *consumed = c;
            return st;
        }
        if (enc == ENC_VARINT) {
            if (id_mode == ORACLE_ID_FORMAT) {
                st = oracle_decode_varint_u64(p, avail, &pos, n, (uint64_t*)o64);
            } else {
                int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
                st = oracle_decode_varint(p, avail, &pos, n, tmp);
                for (int32_t i = 0; !st && i < n; i++) o64[i] = tmp[i];
                free(tmp);
            }
            if (!st) *consumed = pos;
            return st;
        }
        if (enc == ENC_VARINT_DELTA_ZZ) { /* Java mode */
            int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
            st = oracle_decode_zigzag_delta_varint(p, avail, &pos, n, tmp);
            for (int32_t i = 0; !st && i < n; i++) o64[i] = tmp[i];
            free(tmp);
            if (!st) *consumed = pos;
            return st;
        }
        return ORC_ERR_UNSUPPORTED;
    }
    int32_t* o32 = (int32_t*)out;
    switch (s->stream_type) {
    case ST_GEOMETRY_TYPES: {
        int32_t c;
        st = oracle_decode_byte_rle(p, avail, n, &pos, s->byte_length, (uint8_t*)out, &c);
        if (st) return st;
        for (int32_t i = 0; i < n; i++) /* GeometryType.values()[b] */
            if (((uint8_t*)out)[i] > 5) return ORC_ERR_HEADER;
        *consumed = c;
        return ORC_OK;
    }
    case ST_GEOMETRY_OFFSETS:
    case ST_PART_OFFSETS:
    case ST_RING_OFFSETS:
        if (s->encoding == ENC_RLE) {
            int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
            int32_t c;
            st = oracle_decode_rle(p, avail, n, &pos, 0, tmp, &c);
            for (int32_t i = 0; !st && i < n; i++) o32[i] = (int32_t)tmp[i]; /* (int) i */
            free(tmp);
            if (!st) *consumed = c;
            return st;
        }
        if (s->encoding == ENC_FPF_ZZ) {
            st = oracle_decode_fastpfor_zigzag_delta(p, avail, n, s->byte_length, &pos, o32);
            if (!st) *consumed = s->byte_length;
            return st;
        }
        return ORC_ERR_UNSUPPORTED;
    case ST_VERTEX_OFFSETS:
        if (s->encoding == ENC_VARINT_DELTA_ZZ) {
            st = oracle_decode_zigzag_delta_varint(p, avail, &pos, n, o32);
            if (!st) *consumed = pos;
            return st;
        }
        if (s->encoding == ENC_FPF_ZZ) {
            st = oracle_decode_fastpfor_zigzag_delta(p, avail, n, s->byte_length, &pos, o32);
            if (!st) *consumed = s->byte_length;
            return st;
        }
        return ORC_ERR_UNSUPPORTED;
    case ST_VERTEX_BUFFER:
        if (s->column_type == 4) {
            if (s->encoding == ENC_VARINT_DELTA_ZZ) {
                st = oracle_decode_delta_varint_morton_codes(p, avail, &pos, n, s->num_bits, o32);
                if (!st) *consumed = pos;
                return st;
            }
            if (s->encoding == ENC_FPF_ZZ) {
                st = oracle_decode_fastpfor_delta_morton_codes(p, avail, n, s->byte_length, &pos, s->num_bits, o32);
                if (!st) *consumed = s->byte_length;
                return st;
            }
            return ORC_ERR_UNSUPPORTED;
        } else {
            int32_t nv = s->column_type == 3 ? 2 * n : n;
            if (s->encoding == ENC_VARINT_DELTA_ZZ) {
                st = oracle_decode_zigzag_delta_varint_coordinates(p, avail, &pos, nv, o32);
                if (!st) *consumed = pos;
                return st;
            }
            if (s->encoding == ENC_FPF_ZZ) {
                st = oracle_decode_fastpfor_delta_coordinates(p, avail, nv, s->byte_length, &pos, o32);
                if (!st) *consumed = s->byte_length;
                return st;
            }
            return ORC_ERR_UNSUPPORTED;
        }
    default: return ORC_ERR_UNSUPPORTED;
    }
}

/* ------------------------------------------------------------------------ */
/* Multi-threaded CPU baseline                                               */
/* ------------------------------------------------------------------------ */
typedef struct {
    const uint8_t* bytes;
    const uint64_t* offsets;
    const uint64_t* sizes;
    int32_t n_tiles, format, id_mode;
    atomic_int next;
    atomic_int status;
    atomic_llong in_bytes, out_bytes, vertices;
} mt_job;

static void* mt_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    int32_t cap_s = 256;
    oracle_stream* ss = (oracle_stream*)malloc(sizeof(oracle_stream) * (size_t)cap_s);
    size_t cap_o = 1 << 20;
    uint8_t* scratch = (uint8_t*)malloc(cap_o);
    long long ib = 0, ob = 0, vx = 0;
    for (;;) {
        int t = atomic_fetch_add(&j->next, 1);
        if (t >= j->n_tiles) break;
        const uint8_t* tile = j->bytes + j->offsets[t];
        size_t len = (size_t)j->sizes[t];
        int32_t n;
        int st = oracle_walk_tile(tile, len, j->format, ss, cap_s, &n);
        if (!st && n > cap_s) {
            cap_s = n;
            ss = (oracle_stream*)realloc(ss, sizeof(oracle_stream) * (size_t)cap_s);
            st = oracle_walk_tile(tile, len, j->format, ss, cap_s, &n);
        }
        if (st) { atomic_store(&j->status, st); continue; }
        for (int32_t i = 0; i < n; i++) {
            int32_t eb;
            int64_t ne;
            oracle_stream_output(&ss[i], j->id_mode, &eb, &ne);
            size_t need = (size_t)(eb * ne) + 16;
            if (need > cap_o) {
                cap_o = need * 2;
                scratch = (uint8_t*)realloc(scratch, cap_o);
            }
            int32_t consumed;
            st = oracle_decode_stream(tile, len, &ss[i], j->id_mode, scratch, &consumed);
            if (st) atomic_store(&j->status, st);
            ib += ss[i].byte_length;
            ob += (long long)eb * ne;
            if (ss[i].column_kind == 1 && ss[i].stream_type == ST_VERTEX_BUFFER)
                vx += (ss[i].column_type == 3 || ss[i].column_type == 4) ? ss[i].num_values : ss[i].num_values / 2;
        }
    }
    atomic_fetch_add(&j->in_bytes, ib);
    atomic_fetch_add(&j->out_bytes, ob);
    atomic_fetch_add(&j->vertices, vx);
    free(ss);
    free(scratch);
    return NULL;
}

int oracle_decode_tiles_mt(const uint8_t* bytes, const uint64_t* offsets, const uint64_t* sizes, int32_t n_tiles,
                           int format, int id_mode, int32_t n_threads, int64_t* in_bytes, int64_t* out_bytes,
                           int64_t* vertices) {
    mt_job j;
    j.bytes = bytes;
    j.offsets = offsets;
    j.sizes = sizes;
    j.n_tiles = n_tiles;
    j.format = format;
    j.id_mode = id_mode;
    atomic_init(&j.next, 0);
    atomic_init(&j.status, 0);
    atomic_init(&j.in_bytes, 0);
    atomic_init(&j.out_bytes, 0);
    atomic_init(&j.vertices, 0);
    if (n_threads < 1) n_threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    for (int i = 1; i < n_threads; i++) pthread_create(&th[i], NULL, mt_worker, &j);
    mt_worker(&j);
    for (int i = 1; i < n_threads; i++) pthread_join(th[i], NULL);
    free(th);
    if (in_bytes) *in_bytes = atomic_load(&j.in_bytes);
    if (out_bytes) *out_bytes = atomic_load(&j.out_bytes);
    if (vertices) *vertices = atomic_load(&j.vertices);
    return atomic_load(&j.status);
}

/* ------------------------------------------------------------------------ */
/* Geometry assembly: CovtParser.convertGeometryColumn (CovtParser.java:135-274)               */
/* ------------------------------------------------------------------------ */
typedef struct {
    const int32_t *go, *po, *ro, *vo, *vb;
    int32_t n_go, n_po, n_ro, n_vo, n_vb, closed;
    int32_t gi, pi, ri, vi;              /* geometryOffsetsCounter, partOffsetCounter, ringOffsetsCounter,
                                            vertexBufferOffset / vertexOffsetsOffset (in vertices) */
    int32_t np, nr, nc, pcap, rcap, ccap; /* emitted parts / rings / coordinates and capacities */
    int32_t *part_off, *ring_off, *coords;
    int st;
} asm_state;

static int32_t asm_count(asm_state* a, const int32_t* s, int32_t n, int32_t* i) {
    if (*i >= n || !s) { a->st = ORC_ERR_COUNT; return 0; }
    const int32_t c = s[(*i)++];
    if (c < 0) { a->st = ORC_ERR_COUNT; return 0; }
    return c;
}
/* one source vertex: getLineString (:522-534) reads vertexBuffer[vertexBufferOffset + 2i],
 * getICELineString (:537-550) reads vertexBuffer[vertexOffsets[vertexOffset + i] * 2] */
static void asm_vertex(asm_state* a, int32_t src) {
    if (a->st) return;
    int32_t idx = src;
    if (a->vo) {
        if (src >= a->n_vo) { a->st = ORC_ERR_COUNT; return; }
        idx = a->vo[src];
    } else if (src >= a->n_vb) {
        a->st = ORC_ERR_COUNT;
        return;
    }
    if (idx < 0 || idx >= a->n_vb) { a->st = ORC_ERR_TRUNCATED; return; }
    if (a->nc >= a->ccap) { a->st = ORC_ERR_COUNT; return; }
    a->coords[2 * a->nc] = a->vb[2 * (int64_t)idx];
    a->coords[2 * a->nc + 1] = a->vb[2 * (int64_t)idx + 1];
    a->nc++;
}
/* a ring / line of nv source vertices; poly: a LinearRing, closed once (getLinearRing :513-516) */
static void asm_ring(asm_state* a, int32_t nv, int poly) {
    if (a->st) return;
    if (a->nr >= a->rcap) { a->st = ORC_ERR_COUNT; return; }
    a->ring_off[a->nr++] = a->nc;
    const int32_t first = a->vi;
    for (int32_t k = 0; k < nv && !a->st; ++k) asm_vertex(a, a->vi++);
    if (poly && !a->closed && nv > 0) asm_vertex(a, first);
}
static void asm_part_begin(asm_state* a) {
    if (a->st) return;
    if (a->np >= a->pcap) { a->st = ORC_ERR_COUNT; return; }
    a->part_off[a->np++] = a->nr;
}

int oracle_assemble_geometry(const uint8_t* types, int32_t n, const int32_t* go, int32_t n_go, const int32_t* po,
                             int32_t n_po, const int32_t* ro, int32_t n_ro, const int32_t* vo, int32_t n_vo,
                             const int32_t* vb, int32_t n_vb, int closed_in_stream, int32_t part_cap,
                             int32_t ring_cap, int32_t coord_cap, int32_t* geo_off, int32_t* part_off,
                             int32_t* ring_off, int32_t* coords, int32_t* n_parts, int32_t* n_rings,
                             int32_t* n_coords) {
    asm_state a = {go, po, ro, vo, vb, n_go, n_po, n_ro, n_vo, n_vb, closed_in_stream ? 1 : 0,
                   0, 0, 0, 0, 0, 0, 0, part_cap, ring_cap, coord_cap, part_off, ring_off, coords, ORC_OK};
    for (int32_t f = 0; f < n && !a.st; ++f) { /* for(var geometryType : geometryTypes) :152 */
        geo_off[f] = a.np;
        switch (types[f]) {
        case 0: /* POINT :153-167 */
            asm_part_begin(&a);
            asm_ring(&a, 1, 0);
            break;
        case 1: /* LINESTRING :168-181 */
            asm_part_begin(&a);
            asm_ring(&a, asm_count(&a, po, n_po, &a.pi), 0);
            break;
        case 2: { /* POLYGON :182-206: numRings from partOffsets, each ring's vertices from ringOffsets */
            const int32_t nrings = asm_count(&a, po, n_po, &a.pi);
            asm_part_begin(&a);
            for (int32_t r = 0; r < nrings && !a.st; ++r) asm_ring(&a, asm_count(&a, ro, n_ro, &a.ri), 1);
            break;
        }
        case 3: { /* MULTIPOINT: rejected by Java (:270); format truth = a count of points */
            const int32_t k = asm_count(&a, go, n_go, &a.gi);
            for (int32_t i = 0; i < k && !a.st; ++i) {
                asm_part_begin(&a);
                asm_ring(&a, 1, 0);
            }
            break;
        }
        case 4: { /* MULTILINESTRING :207-230 */
            const int32_t k = asm_count(&a, go, n_go, &a.gi);
            for (int32_t i = 0; i < k && !a.st; ++i) {
                const int32_t nv = asm_count(&a, po, n_po, &a.pi);
                asm_part_begin(&a);
                asm_ring(&a, nv, 0);
            }
            break;
        }
        case 5: { /* MULTIPOLYGON :231-268 (without the Q7 accumulation / rings[i] / offset bugs) */
            const int32_t k = asm_count(&a, go, n_go, &a.gi);
            for (int32_t i = 0; i < k && !a.st; ++i) {
                const int32_t nrings = asm_count(&a, po, n_po, &a.pi);
                asm_part_begin(&a);
                for (int32_t r = 0; r < nrings && !a.st; ++r) asm_ring(&a, asm_count(&a, ro, n_ro, &a.ri), 1);
            }
            break;
        }
        default: a.st = ORC_ERR_HEADER; /* GeometryType.values()[b] / :270-272 */
        }
    }
    if (!a.st) {
        geo_off[n] = a.np;
        part_off[a.np] = a.nr;
        ring_off[a.nr] = a.nc;
    }
    *n_parts = a.np;
    *n_rings = a.nr;
    *n_coords = a.nc;
    return a.st;
}
