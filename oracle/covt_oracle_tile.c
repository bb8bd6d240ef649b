/* covt_oracle_tile.c -- TEST INFRASTRUCTURE (CPU restatement, never on the product path).
 *
 * One whole tile decoded the way CovtParser.decodeCovt does it (evaluation/java/src/main/java/com/covt/
 * decoder/CovtParser.java:53-133), single-threaded, for the BASELINE configs[0] CPU figure ("single z5
 * tile (16,20) full decode on Java CPU reference"): the metadata walk (:574-652 / Gen C Appendix A.1),
 * every Id and Geometry stream decoded (decodedIds :552-572, decodeGeometryColumn :392-511), every
 * geometry column assembled (convertGeometryColumn :135-274, here oracle_assemble_geometry's nested
 * offsets) and every property column decoded (decodePropertyColumn :276-354).  Parity for each piece is
 * pinned elsewhere (tests/test_oracle.py, test_props_oracle.py, test_assembly_oracle.py); this file only
 * chains them so bench.py's cpu_baseline leg can time a whole tile without Python in the loop.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "covt_oracle.h"

#define NSTREAM_TYPES 10 /* StreamType ordinals 0..9; geometry streams are 4..9 */

static void* xmalloc(size_t n) { return malloc(n ? n : 1); }

int oracle_decode_tile_full(const uint8_t* tile, size_t len, int format, int id_mode, int64_t counts[4]) {
    int32_t cap = 256, n = 0;
    oracle_stream* ss = (oracle_stream*)xmalloc(sizeof(oracle_stream) * (size_t)cap);
    int st = oracle_walk_tile(tile, len, format, ss, cap, &n);
    if (!st && n > cap) {
        cap = n;
        ss = (oracle_stream*)realloc(ss, sizeof(oracle_stream) * (size_t)cap);
        st = oracle_walk_tile(tile, len, format, ss, cap, &n);
    }
    if (st) {
        free(ss);
        return st;
    }
    void** arr = (void**)calloc((size_t)(n ? n : 1), sizeof(void*));
    int64_t* nel = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
    int64_t c_streams = 0, c_vertices = 0, c_coords = 0, c_props = 0;
    for (int32_t i = 0; i < n && !st; i++) {
        int32_t eb, consumed;
        int64_t ne;
        oracle_stream_output(&ss[i], id_mode, &eb, &ne);
        arr[i] = xmalloc((size_t)(eb * ne) + 16);
        nel[i] = ne;
        st = oracle_decode_stream(tile, len, &ss[i], id_mode, arr[i], &consumed);
        c_streams++;
        if (ss[i].column_kind == 1 && ss[i].stream_type == 9)
            c_vertices += (ss[i].column_type == 3 || ss[i].column_type == 4) ? ss[i].num_values : ss[i].num_values / 2;
    }
    /* geometry columns: the streams of one layer's geometry column, by StreamType */
    for (int32_t i = 0; i < n && !st;) {
        if (ss[i].column_kind != 1) {
            i++;
            continue;
        }
        const int32_t layer = ss[i].layer;
        int32_t idx[NSTREAM_TYPES];
        for (int k = 0; k < NSTREAM_TYPES; k++) idx[k] = -1;
        int32_t ctype = ss[i].column_type, nf = ss[i].num_features;
        for (; i < n && ss[i].column_kind == 1 && ss[i].layer == layer; i++) {
            if (ss[i].stream_type >= 4 && ss[i].stream_type < NSTREAM_TYPES) idx[ss[i].stream_type] = i;
            if (ss[i].stream_type == 9) ctype = ss[i].column_type;
        }
        const uint8_t* types = idx[4] >= 0 ? (const uint8_t*)arr[idx[4]] : NULL;
        const int32_t nt = idx[4] >= 0 ? (int32_t)nel[idx[4]] : 0;
#define A(k) (idx[k] >= 0 ? (const int32_t*)arr[idx[k]] : NULL)
#define N(k) (idx[k] >= 0 ? (int32_t)nel[idx[k]] : 0)
        /* capacities: every part / ring consumes a count entry or a source vertex, every coordinate a
         * source vertex or a ring's closing copy */
        const int32_t nvb = idx[9] >= 0 ? (int32_t)(nel[idx[9]] / 2) : 0;
        const int64_t src = (int64_t)N(8) + nvb;
        const int64_t pc = (int64_t)nt + N(5) + N(6) + N(7) + src + 16;
        const int64_t cc = src + pc + 16;
        if (pc > (1 << 28) || cc > (1 << 28)) {
            st = ORC_ERR_COUNT;
            break;
        }
        int32_t* geo = (int32_t*)xmalloc(sizeof(int32_t) * (size_t)(nt + 1));
        int32_t* part = (int32_t*)xmalloc(sizeof(int32_t) * (size_t)(pc + 1));
        int32_t* ring = (int32_t*)xmalloc(sizeof(int32_t) * (size_t)(pc + 1));
        int32_t* coords = (int32_t*)xmalloc(sizeof(int32_t) * (size_t)(2 * cc));
        int32_t np, nr, ncd;
        const int closed = format == 0 && (ctype == 3 || ctype == 4); /* SURVEY Q6 */
        (void)nf;
        st = oracle_assemble_geometry(types, nt, A(5), N(5), A(6), N(6), A(7), N(7), A(8), N(8), A(9), nvb, closed,
                                      (int32_t)pc, (int32_t)pc, (int32_t)cc, geo, part, ring, coords, &np, &nr, &ncd);
        c_coords += ncd;
        free(geo);
        free(part);
        free(ring);
        free(coords);
#undef A
#undef N
    }
    /* property columns */
    if (!st) {
        int32_t pcap = 256, np2 = 0;
        oracle_prop* ps = (oracle_prop*)xmalloc(sizeof(oracle_prop) * (size_t)pcap);
        st = oracle_walk_properties(tile, len, format, ps, pcap, &np2);
        if (!st && np2 > pcap) {
            pcap = np2;
            ps = (oracle_prop*)realloc(ps, sizeof(oracle_prop) * (size_t)pcap);
            st = oracle_walk_properties(tile, len, format, ps, pcap, &np2);
        }
        for (int32_t c = 0; c < np2 && !st; c++) {
            if (ps[c].type < 0) continue; /* a data type Java rejects: not decoded */
            int64_t sz[4];
            oracle_property_sizes(&ps[c], sz);
            uint8_t* b[4];
            for (int k = 0; k < 4; k++) b[k] = (uint8_t*)xmalloc((size_t)sz[k] + 16);
            int32_t nv;
            const int ps_st = oracle_decode_property(tile, len, &ps[c], id_mode, b[0], b[1], (int32_t*)b[2], b[3], &nv);
            (void)ps_st; /* columns Java rejects keep their status; the tile's time still counts them */
            c_props++;
            for (int k = 0; k < 4; k++) free(b[k]);
        }
        free(ps);
    }
    for (int32_t i = 0; i < n; i++) free(arr[i]);
    free(arr);
    free(nel);
    free(ss);
    if (counts) {
        counts[0] = c_streams;
        counts[1] = c_vertices;
        counts[2] = c_coords;
        counts[3] = c_props;
    }
    return st;
}
