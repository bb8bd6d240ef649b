/* mvt_decode.c -- CPU Mapbox Vector Tile (MVT 2.1, protobuf) decoder for the MVT-vs-COVT decode
 * benchmark (the reference's side-by-side is parser/js/test/benchmark/
 * decodingPerformance.ts:37-55 with @mapbox/vector-tile, and the Java readers in
 * evaluation/java/src/main/java/com/covt/converter/mvt/MvtUtils.java:27-89 use
 * mapbox-vector-tile-java / java-vector-tile).  BENCHMARK INFRASTRUCTURE, not part of the product:
 * it restates the published MVT 2.1 decoding (vector_tile.proto fields; geometry command integers
 * id & 0x7 / count >> 3 with zigzag parameter deltas, spec §4.3) and produces the same flat output a
 * COVT Id + Geometry decode produces: feature ids, geometry types, and per feature its vertices as
 * int32 (x, y) pairs with part / ring counts -- no JTS objects, so the comparison is decoder against
 * decoder.  Properties (tags + values) are walked and their values decoded when `with_props` is set. */
#include <stdint.h>
#include <string.h>

typedef struct {
    const uint8_t* p;
    const uint8_t* e;
    int err;
} pb;

static uint64_t pb_varint(pb* b) {
    uint64_t v = 0;
    int s = 0;
    while (b->p < b->e) {
        const uint8_t c = *b->p++;
        v |= (uint64_t)(c & 0x7f) << s;
        if (!(c & 0x80)) return v;
        s += 7;
        if (s > 63) break;
    }
    b->err = 1;
    return 0;
}
static pb pb_sub(pb* b) {
    pb s;
    const uint64_t n = pb_varint(b);
    if (b->err || n > (uint64_t)(b->e - b->p)) {
        b->err = 1;
        s.p = s.e = b->p;
        s.err = 1;
        return s;
    }
    s.p = b->p;
    s.e = b->p + n;
    s.err = 0;
    b->p += n;
    return s;
}
static void pb_skip(pb* b, int wt) {
    switch (wt) {
    case 0: pb_varint(b); break;
    case 1: if (b->e - b->p < 8) b->err = 1; else b->p += 8; break;
    case 2: (void)pb_sub(b); break;
    case 5: if (b->e - b->p < 4) b->err = 1; else b->p += 4; break;
    default: b->err = 1;
    }
}

typedef struct {
    int64_t features, vertices, parts, values;
    uint64_t checksum; /* keeps every decoded number live */
    int32_t* xy;       /* scratch for one feature's vertices (2 * cap ints) */
    int64_t cap;
} mvt_acc;

/* geometry command stream (packed uint32) -> vertices; returns 0 or an error */
static int decode_geometry(pb g, mvt_acc* a) {
    int32_t x = 0, y = 0;
    int64_t nv = 0;
    while (g.p < g.e) {
        const uint32_t ci = (uint32_t)pb_varint(&g);
        if (g.err) return 1;
        const uint32_t id = ci & 7u, cnt = ci >> 3;
        if (id == 7) { /* ClosePath: closes the ring */
            a->parts++;
            continue;
        }
        if (id != 1 && id != 2) return 1;
        if (id == 1) a->parts++;
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t dx = (uint32_t)pb_varint(&g), dy = (uint32_t)pb_varint(&g);
            if (g.err) return 1;
            x += (int32_t)((dx >> 1) ^ (0u - (dx & 1u)));
            y += (int32_t)((dy >> 1) ^ (0u - (dy & 1u)));
            if (nv < a->cap) {
                a->xy[2 * nv] = x;
                a->xy[2 * nv + 1] = y;
            }
            nv++;
        }
    }
    a->vertices += nv;
    for (int64_t i = 0; i < nv && i < a->cap; i += 16) a->checksum += (uint32_t)a->xy[2 * i] ^ (uint32_t)a->xy[2 * i + 1];
    return 0;
}

static int decode_value(pb v, mvt_acc* a) {
    while (v.p < v.e) {
        const uint64_t key = pb_varint(&v);
        if (v.err) return 1;
        const int f = (int)(key >> 3), wt = (int)(key & 7);
        if (f == 1 && wt == 2) {
            pb s = pb_sub(&v);
            a->checksum += (uint64_t)(s.e - s.p);
        } else if (f == 2 && wt == 5) {
            float x;
            memcpy(&x, v.p, 4);
            v.p += 4;
            a->checksum += (uint64_t)(int64_t)x;
        } else if (f == 3 && wt == 1) {
            double x;
            memcpy(&x, v.p, 8);
            v.p += 8;
            a->checksum += (uint64_t)(int64_t)x;
        } else if ((f == 4 || f == 5 || f == 7) && wt == 0) {
            a->checksum += pb_varint(&v);
        } else if (f == 6 && wt == 0) {
            const uint64_t z = pb_varint(&v);
            a->checksum += (z >> 1) ^ (0ull - (z & 1ull));
        } else {
            pb_skip(&v, wt);
        }
        if (v.err) return 1;
        a->values++;
    }
    return 0;
}

static int decode_layer(pb l, mvt_acc* a, int with_props) {
    while (l.p < l.e) {
        const uint64_t key = pb_varint(&l);
        if (l.err) return 1;
        const int f = (int)(key >> 3), wt = (int)(key & 7);
        if (f == 2 && wt == 2) { /* Feature */
            pb ft = pb_sub(&l);
            a->features++;
            while (ft.p < ft.e) {
                const uint64_t k2 = pb_varint(&ft);
                if (ft.err) return 1;
                const int f2 = (int)(k2 >> 3), w2 = (int)(k2 & 7);
                if (f2 == 1 && w2 == 0) {
                    a->checksum += pb_varint(&ft); /* id */
                } else if (f2 == 3 && w2 == 0) {
                    a->checksum += pb_varint(&ft); /* type */
                } else if (f2 == 4 && w2 == 2) {
                    if (decode_geometry(pb_sub(&ft), a)) return 1;
                } else if (f2 == 2 && w2 == 2 && with_props) {
                    pb t = pb_sub(&ft); /* packed (key index, value index) pairs */
                    while (t.p < t.e) a->checksum += pb_varint(&t);
                    if (t.err) return 1;
                } else {
                    pb_skip(&ft, w2);
                }
                if (ft.err) return 1;
            }
        } else if (f == 4 && wt == 2 && with_props) {
            if (decode_value(pb_sub(&l), a)) return 1;
        } else {
            pb_skip(&l, wt);
        }
        if (l.err) return 1;
    }
    return 0;
}

/* Decodes one tile.  out4 (optional) receives features, vertices, parts, property values; the
 * returned value is 0 or 1 (malformed).  `xy` is caller scratch of 2 * cap int32. */
int mvt_decode_tile(const uint8_t* tile, int64_t len, int with_props, int32_t* xy, int64_t cap, int64_t* out4,
                    uint64_t* checksum) {
    pb t = {tile, tile + len, 0};
    mvt_acc a;
    memset(&a, 0, sizeof a);
    a.xy = xy;
    a.cap = cap;
    while (t.p < t.e) {
        const uint64_t key = pb_varint(&t);
        if (t.err) return 1;
        if ((key >> 3) == 3 && (key & 7) == 2) {
            if (decode_layer(pb_sub(&t), &a, with_props)) return 1;
        } else {
            pb_skip(&t, (int)(key & 7));
        }
        if (t.err) return 1;
    }
    if (out4) {
        out4[0] = a.features;
        out4[1] = a.vertices;
        out4[2] = a.parts;
        out4[3] = a.values;
    }
    if (checksum) *checksum = a.checksum;
    return 0;
}
