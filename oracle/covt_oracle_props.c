/*
 * covt_oracle_props.c -- TEST INFRASTRUCTURE ONLY (see covt_oracle.h).
 *
 * CPU restatement of the property-column half of the reference decoder:
 *   CovtParser.decodePropertyColumn   evaluation/java/.../decoder/CovtParser.java:276-354
 *   CovtParser.getStringDictionary    CovtParser.java:367-377
 *   DecodingUtils.decodeByteRle(3-arg) DecodingUtils.java:290-306 (present streams),
 *   DecodingUtils.decodeFloatsLE      DecodingUtils.java:446-453
 * restated into the Arrow-style column layout that include/covt.h defines for the GPU path
 * (validity bitmap + values at feature positions + dictionary offsets/bytes), so the GPU result
 * can be compared byte for byte.  The container walk for property columns follows SURVEY.md
 * Appendix A.1 (Gen C: streams in metadata order) and A.2 (Gen D: TreeMap<StreamType> order,
 * CovtParser.java:600-647).
 */
#include <stdlib.h>
#include <string.h>

#include "covt_oracle.h"

enum { P_ST_PRESENT = 0, P_ST_DATA = 1, P_ST_LENGTH = 2, P_ST_DICTIONARY = 3 };
enum { P_ENC_PLAIN = 0, P_ENC_VARINT_ZZ = 2, P_ENC_VARINT_DELTA_ZZ = 4, P_ENC_RLE = 5 };

static int rdv(const uint8_t* t, size_t len, int64_t* o, uint64_t* v) { /* 64-bit LEB128 */
    *v = 0;
    for (int i = 0; i < 10; i++) {
        if ((uint64_t)*o >= len) return ORC_ERR_TRUNCATED;
        uint8_t b = t[(*o)++];
        *v |= (uint64_t)(b & 0x7f) << (7 * i);
        if (!(b & 0x80)) return ORC_OK;
    }
    return ORC_ERR_HEADER;
}
static int rdj(const uint8_t* t, size_t len, int64_t* o, int32_t* v) { /* DecodingUtils.decodeVarint */
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        if ((uint64_t)*o >= len) return ORC_ERR_TRUNCATED;
        uint8_t b = t[(*o)++];
        r |= (uint32_t)(b & 0x7f) << (7 * i);
        if (i < 3 && !(b & 0x80)) break;
    }
    *v = (int32_t)r;
    return ORC_OK;
}

static void set_stream(oracle_prop* p, int role, int64_t off, int32_t nv, int32_t bl, int32_t enc) {
    p->s_off[role] = off;
    p->s_nv[role] = nv;
    p->s_bl[role] = bl;
    p->s_enc[role] = enc;
}
static void prop_init(oracle_prop* p, int32_t layer, int32_t column, int32_t nf) {
    memset(p, 0, sizeof *p);
    p->layer = layer;
    p->column = column;
    p->n_features = nf;
    p->lang = -1;
    p->name_off = p->lang_off = -1;
    for (int r = 0; r < 4; r++) p->s_off[r] = -1;
}
static void put(oracle_prop* out, int32_t max_out, int32_t* cnt, const oracle_prop* p) {
    if (out && *cnt < max_out) out[*cnt] = *p;
    (*cnt)++;
}

/* Gen C ColumnDataType (evaluation/file/ColumnDataType.java) -> ORACLE_PROP_* (-1: not decodable) */
static int genc_prop_type(int dtype) {
    switch (dtype) {
    case 0: return ORACLE_PROP_STRING;
    case 1: return ORACLE_PROP_FLOAT;
    case 3: return ORACLE_PROP_INT64;
    case 5: return ORACLE_PROP_BOOLEAN;
    default: return -1; /* DOUBLE, UINT_64: "Data type not supported" (CovtParser.java:352) */
    }
}
/* Gen D ColumnDataType (converter/ColumnDataType.java) */
static int gend_prop_type(int dtype) {
    switch (dtype) {
    case 0: return ORACLE_PROP_BOOLEAN;
    case 3: return ORACLE_PROP_INT64;
    case 5: return ORACLE_PROP_FLOAT;
    case 7: return ORACLE_PROP_STRING;
    default: return -1;
    }
}

static int name_is(const uint8_t* t, int64_t off, int32_t len, const char* s) {
    return (size_t)len == strlen(s) && memcmp(t + off, s, (size_t)len) == 0;
}

static int walk_props_genc(const uint8_t* t, size_t len, oracle_prop* out, int32_t max_out, int32_t* n_out) {
    int64_t o = 0;
    uint64_t version, nlayers;
    int st;
    int32_t cnt = 0;
    if ((st = rdv(t, len, &o, &version)) || (st = rdv(t, len, &o, &nlayers))) return st;
    if (version != 1) return ORC_ERR_HEADER;
    typedef struct { int64_t name_off, off; int32_t name_len, nv, bl, enc; } sm;
    typedef struct { int64_t name_off; int32_t name_len, dtype, ctype, ns, first; } cm;
    for (uint64_t L = 0; L < nlayers; L++) {
        uint64_t nl, extent, nfeat, ncols;
        if ((st = rdv(t, len, &o, &nl))) return st;
        if ((uint64_t)o + nl > len) return ORC_ERR_TRUNCATED;
        o += (int64_t)nl;
        if ((st = rdv(t, len, &o, &extent)) || (st = rdv(t, len, &o, &nfeat)) || (st = rdv(t, len, &o, &ncols)))
            return st;
        if (ncols > 4096 || nfeat > 0x7fffffff) return ORC_ERR_HEADER;
        cm* cols = (cm*)calloc(ncols ? ncols : 1, sizeof(cm));
        sm* ss = NULL;
        int64_t nss = 0;
        for (uint64_t c = 0; c < ncols; c++) {
            uint64_t cn, ns;
            if ((st = rdv(t, len, &o, &cn))) goto fail;
            if ((uint64_t)o + cn + 2 > len) { st = ORC_ERR_TRUNCATED; goto fail; }
            cols[c].name_off = o;
            cols[c].name_len = (int32_t)cn;
            o += (int64_t)cn;
            cols[c].dtype = t[o++];
            cols[c].ctype = t[o++];
            if ((st = rdv(t, len, &o, &ns))) goto fail;
            if (ns > 256) { st = ORC_ERR_HEADER; goto fail; }
            cols[c].ns = (int32_t)ns;
            cols[c].first = (int32_t)nss;
            ss = (sm*)realloc(ss, sizeof(sm) * (size_t)(nss + (int64_t)ns + 1));
            for (uint64_t s = 0; s < ns; s++, nss++) {
                uint64_t sn, nv, bl;
                if ((st = rdv(t, len, &o, &sn))) goto fail;
                if ((uint64_t)o + sn > len) { st = ORC_ERR_TRUNCATED; goto fail; }
                ss[nss].name_off = o;
                ss[nss].name_len = (int32_t)sn;
                o += (int64_t)sn;
                if ((st = rdv(t, len, &o, &nv)) || (st = rdv(t, len, &o, &bl))) goto fail;
                if ((uint64_t)o >= len) { st = ORC_ERR_TRUNCATED; goto fail; }
                ss[nss].enc = t[o++];
                if (nv > 0x7fffffff || bl > 0x7fffffff) { st = ORC_ERR_HEADER; goto fail; }
                ss[nss].nv = (int32_t)nv;
                ss[nss].bl = (int32_t)bl;
            }
        }
        /* payload offsets: non-geometry columns lay out their streams in metadata order (a geometry
           column's streams are reordered, but only its total matters here) */
        for (uint64_t c = 0; c < ncols; c++)
            for (int32_t s = 0; s < cols[c].ns; s++) {
                ss[cols[c].first + s].off = o;
                o += ss[cols[c].first + s].bl;
            }
        if ((uint64_t)o > len) { st = ORC_ERR_TRUNCATED; goto fail; }
        for (uint64_t c = 0; c < ncols; c++) {
            const cm* col = &cols[c];
            if (name_is(t, col->name_off, col->name_len, "id") || name_is(t, col->name_off, col->name_len, "geometry") ||
                col->dtype == 6)
                continue;
            oracle_prop p;
            prop_init(&p, (int32_t)L, (int32_t)c, (int32_t)nfeat);
            p.name_off = col->name_off;
            p.name_len = col->name_len;
            p.type = genc_prop_type(col->dtype);
            p.column_type = col->ctype;
            const sm* cs = ss + col->first;
            if (p.type == ORACLE_PROP_STRING && col->ctype == 2) {
                /* LOCALIZED_DICTIONARY (Gen C only): (present_<lang>, <lang>)* then the shared
                   length + dictionary streams; one sub-column per language */
                int32_t li = -1, di = -1;
                for (int32_t s = 0; s < col->ns; s++) {
                    if (name_is(t, cs[s].name_off, cs[s].name_len, "length")) li = s;
                    else if (name_is(t, cs[s].name_off, cs[s].name_len, "dictionary")) di = s;
                }
                int32_t lang = 0;
                for (int32_t s = 0; s < col->ns; s++) {
                    if (cs[s].name_len <= 8 || memcmp(t + cs[s].name_off, "present_", 8)) continue;
                    const int32_t ll = cs[s].name_len - 8;
                    int32_t d = -1;
                    for (int32_t k = 0; k < col->ns; k++)
                        if (cs[k].name_len == ll && !memcmp(t + cs[k].name_off, t + cs[s].name_off + 8, (size_t)ll)) d = k;
                    oracle_prop q = p;
                    q.lang = lang++;
                    q.lang_off = cs[s].name_off + 8;
                    q.lang_len = ll;
                    set_stream(&q, P_ST_PRESENT, cs[s].off, cs[s].nv, cs[s].bl, cs[s].enc);
                    if (d >= 0) set_stream(&q, P_ST_DATA, cs[d].off, cs[d].nv, cs[d].bl, cs[d].enc);
                    if (li >= 0) set_stream(&q, P_ST_LENGTH, cs[li].off, cs[li].nv, cs[li].bl, cs[li].enc);
                    if (di >= 0) set_stream(&q, P_ST_DICTIONARY, cs[di].off, cs[di].nv, cs[di].bl, cs[di].enc);
                    put(out, max_out, &cnt, &q);
                }
                continue;
            }
            static const char* roles[4] = {"present", "data", "length", "dictionary"};
            for (int32_t s = 0; s < col->ns; s++)
                for (int r = 0; r < 4; r++)
                    if (name_is(t, cs[s].name_off, cs[s].name_len, roles[r]))
                        set_stream(&p, r, cs[s].off, cs[s].nv, cs[s].bl, cs[s].enc);
            put(out, max_out, &cnt, &p);
        }
        free(cols);
        free(ss);
        continue;
    fail:
        free(cols);
        free(ss);
        return st;
    }
    if ((uint64_t)o != len) return ORC_ERR_HEADER;
    *n_out = cnt;
    return ORC_OK;
}

static int walk_props_gend(const uint8_t* t, size_t len, oracle_prop* out, int32_t max_out, int32_t* n_out) {
    int64_t o = 0;
    int32_t cnt = 0, layer = 0;
    int st;
    typedef struct {
        int kind, dtype, ctype, have[12];
        int32_t enc[12], nv[12], bl[12], name_len;
        int64_t name_off;
    } dm;
    while ((uint64_t)o < len) {
        const int optimized = t[o++] & 1;
        int32_t v, extent, nfeat, ncols;
        if ((st = rdj(t, len, &o, &v))) return st;
        if (!optimized) {
            if (v < 0 || (uint64_t)o + (uint64_t)v > len) return ORC_ERR_TRUNCATED;
            o += v;
        }
        if ((st = rdj(t, len, &o, &extent)) || (st = rdj(t, len, &o, &nfeat)) || (st = rdj(t, len, &o, &ncols)))
            return st;
        if (ncols < 0 || ncols > 4096 || nfeat < 0) return ORC_ERR_HEADER;
        dm* cols = (dm*)calloc(ncols ? (size_t)ncols : 1, sizeof(dm));
        for (int32_t c = 0; c < ncols; c++) {
            cols[c].name_off = -1;
            if (optimized || c == 0) {
                int32_t cid;
                if ((st = rdj(t, len, &o, &cid))) goto fail;
                cols[c].kind = cid == 0 ? 0 : cid == 1 ? 1 : 2;
            } else {
                int32_t sl;
                if ((st = rdj(t, len, &o, &sl))) goto fail;
                if (sl < 0 || (uint64_t)o + (uint64_t)sl > len) { st = ORC_ERR_TRUNCATED; goto fail; }
                cols[c].kind = name_is(t, o, sl, "id") ? 0 : name_is(t, o, sl, "geometry") ? 1 : 2;
                cols[c].name_off = o;
                cols[c].name_len = sl;
                o += sl;
            }
            if ((uint64_t)o >= len) { st = ORC_ERR_TRUNCATED; goto fail; }
            const int desc = t[o++];
            cols[c].dtype = (desc >> 3) & 0xF;
            cols[c].ctype = desc & 0x7;
            if (cols[c].ctype > 4) { st = ORC_ERR_HEADER; goto fail; }
            for (;;) {
                if ((uint64_t)o >= len) { st = ORC_ERR_TRUNCATED; goto fail; }
                const int sd = t[o++];
                const int type = sd >> 4, enc = sd & 0xF;
                if (type > 11 || enc > 9) { st = ORC_ERR_HEADER; goto fail; }
                int32_t nv, bl;
                if ((st = rdj(t, len, &o, &nv)) || (st = rdj(t, len, &o, &bl))) goto fail;
                cols[c].have[type] = 1;
                cols[c].enc[type] = enc;
                cols[c].nv[type] = nv;
                cols[c].bl[type] = bl;
                if (cols[c].dtype == 8 && type == 9) break;
                if (type == P_ST_DATA && cols[c].ctype == 0) break;
                if (type == P_ST_DICTIONARY) break;
            }
        }
        for (int32_t c = 0; c < ncols; c++) {
            const dm* cm = &cols[c];
            oracle_prop p;
            prop_init(&p, layer, c, nfeat);
            p.name_off = cm->name_off;
            p.name_len = cm->name_len;
            p.type = gend_prop_type(cm->dtype);
            p.column_type = cm->ctype;
            if (cm->kind == 2 && cm->dtype != 0) { /* implicit present stream: no metadata (see covt_oracle.h) */
                int32_t pl = 0;
                if ((st = oracle_gend_present_length(t, len, o, nfeat, &pl))) goto fail;
                set_stream(&p, P_ST_PRESENT, o, nfeat, pl, 7);
                o += pl;
            }
            for (int type = 0; type < 12; type++) { /* TreeMap<StreamType> order */
                if (!cm->have[type] || (cm->kind == 2 && type == P_ST_PRESENT)) continue;
                if (cm->bl[type] < 0) { st = ORC_ERR_HEADER; goto fail; }
                if (type <= P_ST_DICTIONARY) set_stream(&p, type, o, cm->nv[type], cm->bl[type], cm->enc[type]);
                o += cm->bl[type];
            }
            if ((uint64_t)o > len) { st = ORC_ERR_TRUNCATED; goto fail; }
            if (cm->kind != 2) continue;
            put(out, max_out, &cnt, &p);
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

int oracle_walk_properties(const uint8_t* tile, size_t len, int format, oracle_prop* out, int32_t max_out,
                           int32_t* n_out) {
    *n_out = 0;
    if (format == ORACLE_FMT_GENC) return walk_props_genc(tile, len, out, max_out, n_out);
    if (format == ORACLE_FMT_GEND) return walk_props_gend(tile, len, out, max_out, n_out);
    return ORC_ERR_ARG;
}

/* ---- decode ----------------------------------------------------------------------------- */
static int byte_rle_bits(const uint8_t* tile, size_t len, int64_t off, int32_t bl, int32_t nbytes, uint8_t* dst) {
    if (off < 0 || bl < 0 || (uint64_t)off + (uint64_t)bl > len) return ORC_ERR_TRUNCATED;
    int32_t pos = 0, cons = 0;
    return oracle_decode_byte_rle(tile + off, (size_t)bl, nbytes, &pos, bl, dst, &cons);
}
static inline int bit(const uint8_t* b, int32_t i) { return (b[i >> 3] >> (i & 7)) & 1; }

void oracle_property_sizes(const oracle_prop* p, int64_t sizes[4]) {
    const int64_t n = p->n_features > 0 ? p->n_features : 0, nb = (n + 7) / 8;
    const int64_t nd = p->s_nv[P_ST_DICTIONARY] > 0 ? p->s_nv[P_ST_DICTIONARY] : 0;
    sizes[0] = nb;
    sizes[1] = p->type == ORACLE_PROP_BOOLEAN ? nb : p->type == ORACLE_PROP_INT64 ? 8 * n : 4 * n;
    sizes[2] = p->type == ORACLE_PROP_STRING ? 4 * (nd + 1) : 0;
    sizes[3] = p->type == ORACLE_PROP_STRING && p->s_bl[P_ST_DICTIONARY] > 0 ? p->s_bl[P_ST_DICTIONARY] : 0;
}

int oracle_decode_property(const uint8_t* tile, size_t len, const oracle_prop* p, int mode, uint8_t* validity,
                           void* values, int32_t* dict_offsets, uint8_t* dict_bytes, int32_t* n_valid) {
    const int32_t n = p->n_features;
    const int32_t nbytes = (int32_t)(((int64_t)n + 7) / 8);
    int st;
    *n_valid = 0;
    if (n < 0) return ORC_ERR_HEADER;
    if (p->type < 0 || p->s_off[P_ST_DATA] < 0) return ORC_ERR_UNSUPPORTED;
    if (p->type != ORACLE_PROP_BOOLEAN && p->s_off[P_ST_PRESENT] < 0) return ORC_ERR_UNSUPPORTED;
    /* validity: the present stream's bitset (BitSet.valueOf: LSB first), or all set (Gen D BOOLEAN) */
    if (p->s_off[P_ST_PRESENT] >= 0) {
        if ((st = byte_rle_bits(tile, len, p->s_off[P_ST_PRESENT], p->s_bl[P_ST_PRESENT], nbytes, validity))) return st;
    } else {
        memset(validity, 0xff, (size_t)nbytes);
    }
    if (n & 7) validity[nbytes - 1] &= (uint8_t)((1u << (n & 7)) - 1u);
    int32_t nv = 0;
    for (int32_t i = 0; i < n; i++) nv += bit(validity, i);
    *n_valid = nv;
    const int64_t doff = p->s_off[P_ST_DATA];
    const int32_t dbl = p->s_bl[P_ST_DATA], dn = p->s_nv[P_ST_DATA];
    if (dbl < 0 || dn < 0) return ORC_ERR_HEADER;
    if ((uint64_t)doff + (uint64_t)dbl > len) return ORC_ERR_TRUNCATED;
    const uint8_t* dp = tile + doff;
    if (p->type == ORACLE_PROP_BOOLEAN) {
        uint8_t* v = (uint8_t*)values;
        if (p->s_off[P_ST_PRESENT] < 0) { /* decodeByteRle(numBytes, byteLength) + BitSet (:280-291) */
            if ((st = byte_rle_bits(tile, len, doff, dbl, nbytes, v))) return st;
            if (n & 7) v[nbytes - 1] &= (uint8_t)((1u << (n & 7)) - 1u);
            return ORC_OK;
        }
        /* Gen C with a present stream: the data bitset holds the present values only (numValues bits) */
        const int32_t db = (int32_t)(((int64_t)dn + 7) / 8);
        uint8_t* dense = (uint8_t*)calloc((size_t)db + 1, 1);
        st = byte_rle_bits(tile, len, doff, dbl, db, dense);
        if (!st && nv > dn) st = ORC_ERR_COUNT;
        memset(v, 0, (size_t)nbytes);
        for (int32_t i = 0, j = 0; !st && i < n; i++)
            if (bit(validity, i)) {
                v[i >> 3] |= (uint8_t)(bit(dense, j) << (i & 7));
                j++;
            }
        free(dense);
        return st;
    }
    /* Java decodes the data stream first; a present bit without a data value then fails in the
       feature loop (decodedDataColumn[j++] past its end): statuses in that order */
    if (p->type == ORACLE_PROP_INT64) {
        int64_t* dense = (int64_t*)malloc(sizeof(int64_t) * (size_t)(dn > 0 ? dn : 1));
        int32_t pos = 0, cons = 0;
        const int enc = p->s_enc[P_ST_DATA];
        if (enc == P_ENC_RLE) {
            st = oracle_decode_rle(dp, (size_t)dbl, dn, &pos, 1, dense, &cons);
        } else if (enc == P_ENC_VARINT_ZZ || enc == P_ENC_VARINT_DELTA_ZZ) {
            if (mode == ORACLE_ID_JAVA) { /* int decode, then mapToLong (:304-312) */
                int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(dn > 0 ? dn : 1));
                st = enc == P_ENC_VARINT_ZZ ? oracle_decode_zigzag_varint(dp, (size_t)dbl, &pos, dn, tmp)
                                            : oracle_decode_zigzag_delta_varint(dp, (size_t)dbl, &pos, dn, tmp);
                for (int32_t i = 0; !st && i < dn; i++) dense[i] = tmp[i];
                free(tmp);
            } else { /* format truth: 64-bit zigzag varints (EncodingUtils.encodeVarints(data, true, delta)) */
                st = oracle_decode_varint_u64(dp, (size_t)dbl, &pos, dn, (uint64_t*)dense);
                uint64_t acc = 0;
                for (int32_t i = 0; !st && i < dn; i++) {
                    const uint64_t u = (uint64_t)dense[i];
                    const uint64_t z = (u >> 1) ^ (0ull - (u & 1ull));
                    acc = enc == P_ENC_VARINT_DELTA_ZZ ? acc + z : z;
                    dense[i] = (int64_t)acc;
                }
            }
        } else {
            st = ORC_ERR_UNSUPPORTED; /* "The specified encoding for the long data stream is not supported." */
        }
        if (!st && nv > dn) st = ORC_ERR_COUNT;
        int64_t* v = (int64_t*)values;
        for (int32_t i = 0, j = 0; !st && i < n; i++) v[i] = bit(validity, i) ? dense[j++] : 0;
        free(dense);
        return st;
    }
    if (p->type == ORACLE_PROP_FLOAT) { /* decodeFloatsLE (:446-453) */
        if ((int64_t)dn * 4 > dbl) return ORC_ERR_TRUNCATED;
        if (nv > dn) return ORC_ERR_COUNT;
        uint32_t* v = (uint32_t*)values;
        for (int32_t i = 0, j = 0; i < n; i++) {
            uint32_t w = 0;
            if (bit(validity, i)) memcpy(&w, dp + 4 * (int64_t)j++, 4);
            v[i] = w;
        }
        return ORC_OK;
    }
    /* STRING: DICTIONARY (Java, :319-345) or LOCALIZED_DICTIONARY (Gen C format truth) */
    if (p->column_type != 1 && p->column_type != 2) return ORC_ERR_UNSUPPORTED;
    if (p->s_off[P_ST_LENGTH] < 0 || p->s_off[P_ST_DICTIONARY] < 0) return ORC_ERR_UNSUPPORTED;
    if (p->s_enc[P_ST_DATA] != P_ENC_RLE) return ORC_ERR_UNSUPPORTED;
    const int32_t nd = p->s_nv[P_ST_DICTIONARY];
    if (nd < 0) return ORC_ERR_HEADER;
    int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (size_t)(dn > 0 ? dn : 1));
    int64_t* lens = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nd > 0 ? nd : 1));
    int32_t pos = 0, cons = 0;
    st = oracle_decode_rle(dp, (size_t)dbl, dn, &pos, 0, idx, &cons);
    if (!st) {
        const int64_t lo = p->s_off[P_ST_LENGTH];
        const int32_t lbl = p->s_bl[P_ST_LENGTH];
        if (lbl < 0 || (uint64_t)lo + (uint64_t)lbl > len) st = ORC_ERR_TRUNCATED;
        else {
            pos = 0;
            st = oracle_decode_rle(tile + lo, (size_t)lbl, nd, &pos, 0, lens, &cons);
        }
    }
    if (!st) { /* getStringDictionary: (int) lengths, decodeString back to back; a negative length
                  fails (COUNT), then strings running past the dictionary stream (TRUNCATED) */
        int64_t acc = 0;
        dict_offsets[0] = 0;
        for (int32_t i = 0; i < nd && !st; i++)
            if ((int32_t)lens[i] < 0) st = ORC_ERR_COUNT;
        for (int32_t i = 0; i < nd && !st; i++) {
            acc += (int32_t)lens[i];
            dict_offsets[i + 1] = (int32_t)acc;
        }
        if (!st && acc > p->s_bl[P_ST_DICTIONARY]) st = ORC_ERR_TRUNCATED;
        if (!st) {
            const int64_t so = p->s_off[P_ST_DICTIONARY];
            if ((uint64_t)so + (uint64_t)p->s_bl[P_ST_DICTIONARY] > len) st = ORC_ERR_TRUNCATED;
            else memcpy(dict_bytes, tile + so, (size_t)p->s_bl[P_ST_DICTIONARY]);
        }
    }
    if (!st && nv > dn) st = ORC_ERR_COUNT;
    int32_t* v = (int32_t*)values;
    for (int32_t i = 0, j = 0; !st && i < n; i++) {
        if (bit(validity, i)) {
            const int32_t k = (int32_t)idx[j++]; /* (int) data[dataCounter++] */
            if (k < 0 || k >= nd) st = ORC_ERR_COUNT; /* dictionaryData[index] out of bounds */
            v[i] = k;
        } else {
            v[i] = 0;
        }
    }
    free(idx);
    free(lens);
    return st;
}
