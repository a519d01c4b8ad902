/*
 * packos_oracle.c — CPU ORACLE (test infrastructure only; see packos_oracle.h).
 *
 * Plain-C restatement of quickwritereader/PackOS (Go).  Each function cites
 * the reference file:line it follows.  Used only by tests/, smoke() and the
 * bench cpu_baseline leg; never linked into libpackos.so.
 */
#include "packos_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* typetags/types.go:44-50                                                  */
/* ------------------------------------------------------------------------ */
uint16_t or_encode_header(int64_t offset, int tag) {
    /* uint16(offset<<3) | (uint16(typeID) & 0x07): high bits silently lost */
    return (uint16_t)(((uint64_t)offset << 3) & 0xFFFFu) | (uint16_t)(tag & 7);
}
uint16_t or_encode_end(int64_t offset) { return (uint16_t)(((uint64_t)offset << 3) & 0xFFFFu); }

static inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline void wr16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
static inline int ovf(int64_t off) { return off >= 8192 || off < 0; }

/* ------------------------------------------------------------------------ */
/* PutAccess (access/put.go:46-702)                                         */
/* ------------------------------------------------------------------------ */
static void grow(uint8_t** b, size_t* cap, size_t need) {
    if (need <= *cap) return;
    size_t nc = *cap ? *cap : 256;
    while (nc < need) nc *= 2;
    *b = (uint8_t*)realloc(*b, nc);
    *cap = nc;
}
void or_put_init(or_put* p) { memset(p, 0, sizeof(*p)); }
void or_put_free(or_put* p) { free(p->buf); free(p->offs); memset(p, 0, sizeof(*p)); }
/* GetPutAccess: buf[:0], offsets[:0], position 0 (put.go:25-31) */
void or_put_reset(or_put* p) { p->len = 0; p->olen = 0; p->position = 0; p->overflow = 0; }

static void put_hdr(or_put* p, int64_t off, int tag) {
    grow(&p->offs, &p->ocap, p->olen + 2);
    if (ovf(off)) p->overflow = 1;
    wr16(p->offs + p->olen, or_encode_header(off, tag));
    p->olen += 2;
}
/* Add* / AppendTagAndValue (put.go:69-81, 296-301): the header records the
 * current position, the payload is appended, position = len(buf).          */
void or_put_add(or_put* p, int tag, const uint8_t* bytes, size_t n) {
    put_hdr(p, p->position, tag);
    grow(&p->buf, &p->cap, p->len + n);
    if (n) memcpy(p->buf + p->len, bytes, n);
    p->len += n;
    p->position = (int64_t)p->len;
}
/* AddNullable*(nil): header only, position unchanged (put.go:191-292) */
void or_put_add_nil(or_put* p, int tag) { put_hdr(p, p->position, tag); }
/* BeginTuple / BeginMap (put.go:687-698) */
void or_put_begin(or_put* parent, int tag) { put_hdr(parent, parent->position, tag); }

/* PackAppend (put.go:637-652): End, h0 rewrite, headers then payload */
static void put_pack_append(or_put* p, uint8_t** dst, size_t* dlen, size_t* dcap) {
    put_hdr(p, p->position, 0); /* EncodeEnd(position) */
    size_t hsz = p->olen;
    int tag0 = p->offs[0] & 7;
    if (ovf((int64_t)hsz)) p->overflow = 1;
    wr16(p->offs, or_encode_header((int64_t)hsz, tag0));
    grow(dst, dcap, *dlen + hsz + p->len);
    memcpy(*dst + *dlen, p->offs, hsz);
    if (p->len) memcpy(*dst + *dlen + hsz, p->buf, p->len);
    *dlen += hsz + p->len;
}
/* EndNested -> appendAndReleaseNested (put.go:609-615, 700-702) */
void or_put_end(or_put* parent, or_put* child) {
    put_pack_append(child, &parent->buf, &parent->len, &parent->cap);
    if (child->overflow) parent->overflow = 1;
    parent->position = (int64_t)parent->len;
}
size_t or_put_pack_size(const or_put* p) { return p->olen + p->len + 2; } /* put.go:655-658 */
/* Pack (put.go:619-635) */
size_t or_put_pack(or_put* p, uint8_t* out) {
    put_hdr(p, p->position, 0);
    size_t hsz = p->olen;
    int tag0 = p->offs[0] & 7;
    if (ovf((int64_t)hsz)) p->overflow = 1;
    wr16(p->offs, or_encode_header((int64_t)hsz, tag0));
    memcpy(out, p->offs, hsz);
    if (p->len) memcpy(out + hsz, p->buf, p->len);
    return hsz + p->len;
}

/* ------------------------------------------------------------------------ */
/* schema node helpers                                                      */
/* ------------------------------------------------------------------------ */
#define NK(s, n) ((s)->nodes[4 * (n)])
#define NA(s, n) ((s)->nodes[4 * (n) + 1])
#define NB(s, n) ((s)->nodes[4 * (n) + 2])
#define NC(s, n) ((s)->nodes[4 * (n) + 3])

static int is_container(int k) { return k == ORN_TUPLE || k == ORN_MAP; }
static int nchild(const or_schema* s, int n) { return is_container(NK(s, n)) ? NB(s, n) : 0; }

static int prep_rec(or_schema* s, int n) {
    if (n >= s->n_nodes || n >= 512) return -1;
    int k = nchild(s, n);
    int c = n + 1;
    for (int j = 0; j < k; j++) {
        int nx = prep_rec(s, c);
        if (nx < 0) return -1;
        c = nx;
    }
    s->next_sibling[n] = c;
    return c;
}
static int children(const or_schema* s, int n, int* out);
/* columns are numbered in emission (wire) order: pre-order with sorted map
 * pairs already in key order                                                */
static void number_cols(or_schema* s, int n, int* col) {
    s->col_of_node[n] = NK(s, n) != ORN_MATCH ? (*col)++ : -1;
    int kids[256];
    int k = children(s, n, kids);
    for (int j = 0; j < k; j++) number_cols(s, kids[j], col);
}
int or_schema_prepare(or_schema* s) {
    int col = 0, c = 0;
    if (s->n_top > 256) return -1;
    for (int t = 0; t < s->n_top; t++) {
        s->top_nodes[t] = c;
        c = prep_rec(s, c);
        if (c < 0) return -1;
    }
    if (c != s->n_nodes) return -1;
    for (int t = 0; t < s->n_top; t++) number_cols(s, s->top_nodes[t], &col);
    s->n_cols = col;
    return 0;
}
/* top-level fields an encode writes: EncodeValueNamed walks FieldNames
 * (schema.go:976), so a SchemaNamedChain with fewer names than schemas
 * writes only the first len(FieldNames) of them                              */
static int enc_top(const or_schema* s) {
    return s->chain_names > 0 && s->chain_names < s->n_top ? s->chain_names : s->n_top;
}

static int leaf_tag(int k) {
    switch (k) {
        case ORN_INT: case ORN_UINT: return 1;
        case ORN_FLOAT: return 3;
        case ORN_BOOL: return 5;
        case ORN_STRING: case ORN_BYTES: case ORN_MATCH: return 6;
        case ORN_TUPLE: return 4;
        case ORN_MAP: return 7;
    }
    return 0;
}

static const uint8_t* lit_ptr(const or_schema* s, int li, size_t* len) {
    *len = (size_t)(s->lit_off[li + 1] - s->lit_off[li]);
    return s->lit + s->lit_off[li];
}

/* value checks (schema.go:1172-1364 Range, 2188-2250 SDateRange, 1070-1158
 * CheckFunc Prefix/Suffix, 270-286 DefaultDecodeValue) */
enum { X_MIN = 1, X_MAX = 2, X_DATE = 4, X_PREFIX = 8, X_SUFFIX = 16, X_DEFAULT = 32 };
static int64_t xflags(const or_schema* s, int n) { return s->ext ? s->ext[4 * n] : 0; }
static const uint8_t* xlit(const or_schema* s, int n, int which, size_t* len) {
    int64_t li = which ? ((s->ext[4 * n + 3] >> 32) & 0xFFFFFFFF) - 1 : (s->ext[4 * n + 3] & 0xFFFFFFFF) - 1;
    if (li < 0) { *len = 0; return (const uint8_t*)""; }
    return lit_ptr(s, (int)li, len);
}
/* CheckIntRange on the LE value of width w (sign-extended) */
static int range_bad(const or_schema* s, int n, const uint8_t* p, int w) {
    int64_t f = xflags(s, n);
    uint64_t u = 0;
    for (int b = 0; b < w; b++) u |= (uint64_t)p[b] << (8 * b);
    int sh = 64 - 8 * w;
    int64_t v = (int64_t)(u << sh) >> sh;
    return ((f & X_MIN) && v < s->ext[4 * n + 1]) || ((f & X_MAX) && v > s->ext[4 * n + 2]);
}
/* strings.HasPrefix / HasSuffix */
static int str_bad(const or_schema* s, int n, const uint8_t* p, size_t len) {
    size_t L;
    const uint8_t* lit = xlit(s, n, 0, &L);
    if (len < L) return 1;
    const uint8_t* at = (xflags(s, n) & X_PREFIX) ? p : p + len - L;
    return L && memcmp(at, lit, L) != 0;
}

/* children of a container in emission order; sorted maps order key/value
 * pairs by key bytes (utils.SortKeys = sort.Strings, utils/utils.go:7-14). */
static int children(const or_schema* s, int n, int* out) {
    int k = nchild(s, n), c = n + 1;
    for (int j = 0; j < k; j++) { out[j] = c; c = s->next_sibling[c]; }
    if (NK(s, n) == ORN_MAP && NA(s, n)) {
        int np = k / 2;
        for (int a = 1; a < np; a++) {  /* insertion sort on pairs */
            int kk = out[2 * a], vv = out[2 * a + 1];
            size_t la; const uint8_t* pa = lit_ptr(s, NA(s, kk), &la);
            int b = a - 1;
            while (b >= 0) {
                size_t lb; const uint8_t* pb = lit_ptr(s, NA(s, out[2 * b]), &lb);
                size_t m = la < lb ? la : lb;
                int cmp = memcmp(pb, pa, m);
                if (cmp < 0 || (cmp == 0 && lb <= la)) break;
                out[2 * b + 2] = out[2 * b]; out[2 * b + 3] = out[2 * b + 1];
                b--;
            }
            out[2 * b + 2] = kk; out[2 * b + 3] = vv;
        }
    }
    return k;
}

static int col_valid(const packos_column* c, size_t i) { return !c->valid || c->valid[i]; }

/* leaf payload for blob i: pointer + length (nil -> returns 0 with *nil=1) */
static const uint8_t* leaf_bytes(const or_schema* s, const packos_column* cols, size_t i, int n,
                                 size_t* len, int* nil, uint8_t* tmp) {
    int k = NK(s, n);
    *nil = 0;
    if (k == ORN_MATCH) return lit_ptr(s, NA(s, n), len);
    const packos_column* c = &cols[s->col_of_node[n]];
    if (k == ORN_STRING || k == ORN_BYTES) {
        if (NA(s, n) > 0) { *len = (size_t)NA(s, n); return (const uint8_t*)c->data + i * (size_t)NA(s, n); }
        *len = c->offsets[i + 1] - c->offsets[i];
        return (const uint8_t*)c->data + c->offsets[i];
    }
    int w = NA(s, n);
    *len = (size_t)w;
    if (NB(s, n) && !col_valid(c, i)) { *nil = 1; return NULL; }
    const uint8_t* p = (const uint8_t*)c->data + i * (size_t)w;
    if (k == ORN_BOOL) { tmp[0] = p[0] != 0; return tmp; } /* AddBool writes 0/1 (put.go:179-189) */
    return p;
}

/* ------------------------------------------------------------------------ */
/* schema.EncodeValue through PutAccess (schema/schema.go:912-941,           */
/* 594-829, 270-326, 416-457, 1636-1680)                                     */
/* ------------------------------------------------------------------------ */
static void put_node(const or_schema* s, const packos_column* cols, size_t i, int n, or_put* p,
                     or_put* pool, int depth) {
    int k = NK(s, n);
    if (is_container(k)) {
        int nullable = (k == ORN_MAP) ? 1 : NA(s, n);
        const packos_column* c = &cols[s->col_of_node[n]];
        if (nullable && !col_valid(c, i)) { or_put_add_nil(p, leaf_tag(k)); return; } /* AddAnyTuple(nil)/AddMapAny(nil) */
        or_put* ch = &pool[depth];
        or_put_reset(ch);
        or_put_begin(p, leaf_tag(k));
        int kids[256];
        int nk = children(s, n, kids);
        for (int j = 0; j < nk; j++) put_node(s, cols, i, kids[j], ch, pool, depth + 1);
        or_put_end(p, ch);
        return;
    }
    size_t len; int nil; uint8_t tmp[8];
    const uint8_t* b = leaf_bytes(s, cols, i, n, &len, &nil, tmp);
    if (nil) or_put_add_nil(p, leaf_tag(k));
    else or_put_add(p, leaf_tag(k), b, len);
}

/* ------------------------------------------------------------------------ */
/* packable two-pass encode (packable/pack.go:17-67,                          */
/* packable_mapPackables.go:13-53, packable_nullables.go)                    */
/* ------------------------------------------------------------------------ */
static int64_t pk_value_size(const or_schema* s, const packos_column* cols, size_t i, int n) {
    int k = NK(s, n);
    if (is_container(k)) {
        int nullable = (k == ORN_MAP) ? 1 : NA(s, n);
        if (nullable && !col_valid(&cols[s->col_of_node[n]], i)) return 0;
        int kids[256];
        int nk = children(s, n, kids);
        if (nk == 0) return 0;
        int64_t sz = 0;
        for (int j = 0; j < nk; j++) sz += pk_value_size(s, cols, i, kids[j]);
        return sz + 2 * (int64_t)nk + 2;
    }
    size_t len; int nil; uint8_t tmp[8];
    leaf_bytes(s, cols, i, n, &len, &nil, tmp);
    return (int64_t)len; /* nullable ValueSize reports full width even for nil */
}

static int64_t pk_write(const or_schema* s, const packos_column* cols, size_t i, int n, uint8_t* buf,
                        int64_t pos, int* overflow) {
    int k = NK(s, n);
    if (is_container(k)) {
        int nullable = (k == ORN_MAP) ? 1 : NA(s, n);
        if (nullable && !col_valid(&cols[s->col_of_node[n]], i)) return pos;
        int kids[256];
        int nk = children(s, n, kids);
        if (nk == 0) return pos;
        int64_t hsz = 2 * (int64_t)nk + 2, posH = pos;
        pos += hsz;
        int64_t delta = pos;
        for (int j = 0; j < nk; j++) {
            int64_t off = j == 0 ? hsz : pos - delta;
            if (ovf(off)) *overflow = 1;
            wr16(buf + posH, or_encode_header(off, leaf_tag(NK(s, kids[j]))));
            posH += 2;
            pos = pk_write(s, cols, i, kids[j], buf, pos, overflow);
        }
        if (ovf(pos - delta)) *overflow = 1;
        wr16(buf + posH, or_encode_header(pos - delta, 0));
        return pos;
    }
    size_t len; int nil; uint8_t tmp[8];
    const uint8_t* b = leaf_bytes(s, cols, i, n, &len, &nil, tmp);
    if (nil) return pos; /* WriteNullable*(nil) writes nothing */
    if (len) memcpy(buf + pos, b, len);
    return pos + (int64_t)len;
}

/* ------------------------------------------------------------------------ */
/* ADR-001 extended containers (PACKOS_MODE_EXTENDED).  NOT reference code:  */
/* PackOS reserves tag 2 (typetags/types.go:11) and names the ADR            */
/* (README.md:34) without a format; this restates the format this build      */
/* defines (include/packos.h).  Written independently of or_put / pk_write   */
/* (bottom-up: a container's payload is built first, then its header block   */
/* in 16-bit or extended form) so the two checks cross-validate: with no     */
/* payload over 8191 bytes both must give the reference bytes.              */
/* ------------------------------------------------------------------------ */
typedef struct xbuf { uint8_t* p; size_t len, cap; } xbuf;
static void xput(xbuf* b, const void* src, size_t n) {
    grow(&b->p, &b->cap, b->len + n + 1);
    if (n) memcpy(b->p + b->len, src, n);
    b->len += n;
}
static void xput16(xbuf* b, uint16_t v) { uint8_t t[2] = {(uint8_t)v, (uint8_t)(v >> 8)}; xput(b, t, 2); }
static void xput32(xbuf* b, uint32_t v) {
    uint8_t t[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
    xput(b, t, 4);
}
static int x_field(const or_schema* s, const packos_column* cols, size_t i, int n, int mode, xbuf* b,
                   int64_t* slack);
/* container of nk fields (kids) appended to b; returns 1 when written extended */
static int x_container(const or_schema* s, const packos_column* cols, size_t i, const int* kids, int nk,
                       int own_tag, int mode, xbuf* b, int64_t* slack) {
    if (nk == 0) {
        if (mode == PACKOS_MODE_PUTACCESS) xput16(b, or_encode_header(2, 0)); /* Q3: 10 00 */
        return 0;
    }
    xbuf pay = {0};
    int64_t* st = (int64_t*)malloc(sizeof(int64_t) * (size_t)nk);
    int* tg = (int*)calloc((size_t)nk, sizeof(int));
    for (int j = 0; j < nk; j++) {
        st[j] = (int64_t)pay.len;
        tg[j] = x_field(s, cols, i, kids[j], mode, &pay, slack);
    }
    int ext = pay.len > 8191;
    if (ext) {
        xput16(b, or_encode_header(0, PACKOS_TAG_EXTENDED));
        xput16(b, (uint16_t)own_tag);
        xput32(b, (uint32_t)((4 + 4 * (nk + 1)) << 3) | (uint32_t)tg[0]);
        for (int j = 1; j < nk; j++) xput32(b, (uint32_t)(st[j] << 3) | (uint32_t)tg[j]);
        xput32(b, (uint32_t)(pay.len << 3));
    } else {
        xput16(b, or_encode_header(2 * (nk + 1), tg[0]));
        for (int j = 1; j < nk; j++) xput16(b, or_encode_header(st[j], tg[j]));
        xput16(b, or_encode_end((int64_t)pay.len));
    }
    xput(b, pay.p, pay.len);
    free(pay.p); free(st); free(tg);
    return ext;
}
/* one field appended to b; returns the tag its parent entry carries */
static int x_field(const or_schema* s, const packos_column* cols, size_t i, int n, int mode, xbuf* b,
                   int64_t* slack) {
    int k = NK(s, n);
    if (is_container(k)) {
        int nullable = (k == ORN_MAP) ? 1 : NA(s, n);
        if (nullable && !col_valid(&cols[s->col_of_node[n]], i)) return leaf_tag(k); /* nil: 0 bytes */
        int kids[256];
        int nk = children(s, n, kids);
        return x_container(s, cols, i, kids, nk, leaf_tag(k), mode, b, slack) ? PACKOS_TAG_EXTENDED : leaf_tag(k);
    }
    size_t len; int nil; uint8_t tmp[8];
    const uint8_t* p = leaf_bytes(s, cols, i, n, &len, &nil, tmp);
    if (nil) { *slack += (int64_t)len; return leaf_tag(k); }   /* packable: ValueSize keeps the width */
    xput(b, p, len);
    return leaf_tag(k);
}
/* whole blob in extended mode: the chain as a tuple (+ packable slack) */
static int64_t x_encode(const or_schema* s, const packos_column* cols, size_t i, int mode, xbuf* b) {
    b->len = 0;
    int64_t slack = 0;
    if (mode == PACKOS_MODE_PACKABLE && enc_top(s) == 0) return 0;   /* Pack() with no args */
    x_container(s, cols, i, s->top_nodes, enc_top(s), PACKOS_TAG_TUPLE, mode, b, &slack);
    if (mode == PACKOS_MODE_PACKABLE && slack) {
        grow(&b->p, &b->cap, b->len + (size_t)slack + 1);
        memset(b->p + b->len, 0, (size_t)slack);
        b->len += (size_t)slack;
    }
    return (int64_t)b->len;
}

int64_t or_encoded_size_one(const or_schema* s, const packos_column* cols, size_t i, int mode) {
    if (mode & PACKOS_MODE_EXTENDED) {
        xbuf b = {0};
        int64_t r = x_encode(s, cols, i, mode & ~PACKOS_MODE_EXTENDED, &b);
        free(b.p);
        return r;
    }
    const int nt = enc_top(s);
    if (mode == PACKOS_MODE_PACKABLE) {
        if (nt == 0) return 0;
        int64_t sz = 0;
        for (int t = 0; t < nt; t++) sz += pk_value_size(s, cols, i, s->top_nodes[t]);
        return sz + 2 * (int64_t)nt + 2;
    }
    or_put p, pool[16];
    or_put_init(&p);
    for (int d = 0; d < 16; d++) or_put_init(&pool[d]);
    for (int t = 0; t < nt; t++) put_node(s, cols, i, s->top_nodes[t], &p, pool, 0);
    int64_t sz = (int64_t)or_put_pack_size(&p);
    or_put_free(&p);
    for (int d = 0; d < 16; d++) or_put_free(&pool[d]);
    return sz;
}

/* EncodeFunc value checks in emission order: the ErrorCode of the first
 * failing top-level field (Range -> ErrOutOfRange, SDateRange ->
 * ErrDateOutOfRange, CheckFunc -> ErrEncode; a present TupleSchemaNamed whose
 * FieldNames and Schemas differ in length -> ErrConstraintViolated,
 * schema.go:1808-1810), 0 if every value passes.  A tuple or map wraps its
 * child's error as ErrInvalidFormat (schema.go:1671-1673, 1859-1861,
 * 444-449).  Nil containers and nil values are not encoded, so not checked
 * (schema.go:1203-1214, 2227-2246, 1110-1124, 1804-1806).                    */
static int has_names_bad(const or_schema* s) {
    for (int n = 0; n < s->n_nodes; n++) {
        if (NK(s, n) == ORN_TUPLE && (NC(s, n) & ORT_NAMES_BAD)) return 1;
        if (NK(s, n) == ORN_MAP && (NB(s, n) % 2) != 0) return 1;   /* odd SMap */
    }
    return 0;
}

static int enc_check(const or_schema* s, const packos_column* cols, size_t i, int n) {
    int k = NK(s, n);
    if (is_container(k)) {
        int nullable = (k == ORN_MAP) ? 1 : NA(s, n);
        if (nullable && !col_valid(&cols[s->col_of_node[n]], i)) return 0;
        if (k == ORN_TUPLE && (NC(s, n) & ORT_NAMES_BAD)) return 3;
        int kids[256];
        int nk = children(s, n, kids);
        /* SchemaMap.Encode of a present value with an odd schema count:
         * SizeExact -> ErrConstraintViolated (schema.go:417-429)             */
        if (k == ORN_MAP && (nk % 2) != 0) return 3;
        for (int j = 0; j < nk; j++) {
            if (enc_check(s, cols, i, kids[j])) return 1;
        }
        return 0;
    }
    int64_t f = xflags(s, n);
    if (f & (X_MIN | X_MAX)) {
        size_t len; int nil; uint8_t tmp[8];
        const uint8_t* b = leaf_bytes(s, cols, i, n, &len, &nil, tmp);
        if (nil) return 0;
        if (range_bad(s, n, b, (int)len)) return (f & X_DATE) ? PACKOS_ERR_DATE_OUT_OF_RANGE : PACKOS_ERR_OUT_OF_RANGE;
    } else if (f & (X_PREFIX | X_SUFFIX)) {
        size_t len; int nil; uint8_t tmp[8];
        const uint8_t* b = leaf_bytes(s, cols, i, n, &len, &nil, tmp);
        if (str_bad(s, n, b, len)) return PACKOS_ERR_ENCODE;
    }
    return 0;
}

typedef struct enc_tls { or_put p; or_put pool[16]; } enc_tls;

static int64_t encode_one_tls(const or_schema* s, const packos_column* cols, size_t i, int mode,
                              uint8_t* out, size_t cap, int* overflow, enc_tls* t) {
    *overflow = 0;
    if (mode & PACKOS_MODE_EXTENDED) {
        xbuf b = {0};
        int64_t r = x_encode(s, cols, i, mode & ~PACKOS_MODE_EXTENDED, &b);
        if ((size_t)r > cap) r = -1;
        else if (r > 0) memcpy(out, b.p, (size_t)r);
        free(b.p);
        return r;
    }
    const int nt = enc_top(s);
    if (mode == PACKOS_MODE_PACKABLE) {
        /* packable.Pack: buffer of ValueSize() bytes, zero filled (pack.go:59-67) */
        if (nt == 0) return 0;
        int64_t size = 0;
        for (int k = 0; k < nt; k++) size += pk_value_size(s, cols, i, s->top_nodes[k]);
        size += 2 * (int64_t)nt + 2;
        if (size < 0 || (size_t)size > cap) return -1;
        memset(out, 0, (size_t)size);
        int64_t hsz = 2 * (int64_t)nt + 2, posH = 0, pos = hsz, delta = hsz;
        for (int k = 0; k < nt; k++) {
            int n = s->top_nodes[k];
            int64_t off = k == 0 ? hsz : pos - delta;
            if (ovf(off)) *overflow = 1;
            wr16(out + posH, or_encode_header(off, leaf_tag(NK(s, n))));
            posH += 2;
            pos = pk_write(s, cols, i, n, out, pos, overflow);
        }
        if (ovf(pos - delta)) *overflow = 1;
        wr16(out + posH, or_encode_header(pos - delta, 0));
        return size;
    }
    or_put_reset(&t->p);
    for (int k = 0; k < nt; k++) put_node(s, cols, i, s->top_nodes[k], &t->p, t->pool, 0);
    size_t need = or_put_pack_size(&t->p);
    if (need > cap) return -1;
    size_t got = or_put_pack(&t->p, out);
    *overflow = t->p.overflow;
    return (int64_t)got;
}

int64_t or_encode_one(const or_schema* s, const packos_column* cols, size_t i, int mode, uint8_t* out,
                      size_t cap, int* overflow) {
    enc_tls t;
    or_put_init(&t.p);
    for (int d = 0; d < 16; d++) or_put_init(&t.pool[d]);
    int64_t r = encode_one_tls(s, cols, i, mode, out, cap, overflow, &t);
    or_put_free(&t.p);
    for (int d = 0; d < 16; d++) or_put_free(&t.pool[d]);
    return r;
}

/* batch calls use up to this many threads (every core of a large host) */
#define OR_MAX_THREADS 1024

typedef struct enc_job {
    const or_schema* s; const packos_column* cols; int mode;
    uint8_t* out; uint64_t* offs; uint32_t* status; size_t lo, hi;
} enc_job;

static void* enc_worker(void* arg) {
    enc_job* j = (enc_job*)arg;
    enc_tls t;
    or_put_init(&t.p);
    for (int d = 0; d < 16; d++) or_put_init(&t.pool[d]);
    for (size_t i = j->lo; i < j->hi; i++) {
        int o = 0;
        size_t cap = (size_t)(j->offs[i + 1] - j->offs[i]);
        encode_one_tls(j->s, j->cols, i, j->mode, j->out + j->offs[i], cap, &o, &t);
        if (j->status) {
            uint32_t sv = o ? PACKOS_STATUS_OVERFLOW13 : 0u;
            const int more_names = j->s->chain_names > j->s->n_top;
            const int chk = j->s->ext != NULL || has_names_bad(j->s) || more_names;
            int failed = 0;
            for (int tp = 0; chk && tp < enc_top(j->s); tp++) {
                int inner = enc_check(j->s, j->cols, i, j->s->top_nodes[tp]);
                if (inner) {
                    /* SchemaError(ErrEncode, ChainName, "", -1, err): position -1 (schema.go:919-936) */
                    sv |= (uint32_t)PACKOS_ERR_ENCODE | ((uint32_t)inner << 24);
                    failed = 1;
                    break;
                }
            }
            /* EncodeValueNamed with more FieldNames than Schemas: every schema's
             * field written, the next name indexes chain.Schemas[len(Schemas)]
             * (schema.go:976-987) -- a Go runtime panic, no bytes              */
            if (more_names && !failed) sv = PACKOS_STATUS_PANIC;
            j->status[i] = sv;
        }
    }
    or_put_free(&t.p);
    for (int d = 0; d < 16; d++) or_put_free(&t.pool[d]);
    return NULL;
}

typedef struct size_job { const or_schema* s; const packos_column* cols; int mode; uint64_t* offs; size_t lo, hi; } size_job;
static void* size_worker(void* arg) {
    size_job* j = (size_job*)arg;
    for (size_t i = j->lo; i < j->hi; i++) j->offs[i + 1] = (uint64_t)or_encoded_size_one(j->s, j->cols, i, j->mode);
    return NULL;
}

/* total encoded bytes of a batch (size pass only), nthreads workers */
int64_t or_encoded_total(const or_schema* s, const packos_column* cols, size_t n, int mode, uint64_t* offs_scratch,
                         int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > OR_MAX_THREADS) nthreads = OR_MAX_THREADS;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    size_job* sj = (size_job*)malloc(sizeof(size_job) * (size_t)nthreads);
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        size_t lo = (size_t)t * per, hi = lo + per > n ? n : lo + per;
        if (lo > hi) lo = hi;
        sj[t] = (size_job){s, cols, mode, offs_scratch, lo, hi};
        pthread_create(&th[t], NULL, size_worker, &sj[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th); free(sj);
    int64_t tot = 0;
    for (size_t i = 0; i < n; i++) tot += (int64_t)offs_scratch[i + 1];
    return tot;
}

int64_t or_encode_batch(const or_schema* s, const packos_column* cols, size_t n, int mode, uint8_t* out,
                        size_t cap, uint64_t* out_offsets, uint32_t* status, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > OR_MAX_THREADS) nthreads = OR_MAX_THREADS;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    size_job* sj = (size_job*)malloc(sizeof(size_job) * (size_t)nthreads);
    enc_job* ej = (enc_job*)malloc(sizeof(enc_job) * (size_t)nthreads);
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    out_offsets[0] = 0;
    for (int t = 0; t < nthreads; t++) {
        size_t lo = (size_t)t * per, hi = lo + per > n ? n : lo + per;
        if (lo > hi) lo = hi;
        sj[t] = (size_job){s, cols, mode, out_offsets, lo, hi};
        pthread_create(&th[t], NULL, size_worker, &sj[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    for (size_t i = 0; i < n; i++) out_offsets[i + 1] += out_offsets[i];
    if (out_offsets[n] > cap) { free(th); free(sj); free(ej); return -1; }
    for (int t = 0; t < nthreads; t++) {
        size_t lo = (size_t)t * per, hi = lo + per > n ? n : lo + per;
        if (lo > hi) lo = hi;
        ej[t] = (enc_job){s, cols, mode, out, out_offsets, status, lo, hi};
        pthread_create(&th[t], NULL, enc_worker, &ej[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th); free(sj); free(ej);
    return (int64_t)out_offsets[n];
}

/* ------------------------------------------------------------------------ */
/* SeqGetAccess (access/seqget.go:22-154)                                    */
/* ------------------------------------------------------------------------ */
int or_seq_init(or_seq* s, const uint8_t* buf, int64_t len) {
    if (len < 4) return 1;                     /* "insufficient header" */
    uint16_t h0 = rd16(buf);
    int64_t base = h0 >> 3;
    if (len < base) return 1;
    uint16_t h1 = rd16(buf + 2);
    s->buf = buf; s->len = len;
    s->base = base; s->count = base / 2; s->pos = 0;
    s->cur_off = base; s->cur_type = h0 & 7;
    s->next_off = (h1 >> 3) + base; s->next_type = h1 & 7;
    s->xw = 0;
    return 0;
}
static uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
/* ADR-001 extended container (this build's format, include/packos.h) */
int or_seq_init_ext(or_seq* s, const uint8_t* buf, int64_t len, int xkind) {
    if (len < 12 || rd16(buf) != or_encode_header(0, PACKOS_TAG_EXTENDED) || rd16(buf + 2) != xkind) return 1;
    uint32_t e0 = rd32(buf + 4);
    int64_t base = e0 >> 3;
    if (base < 12 || (base & 3) || len < base) return 1;
    uint32_t e1 = rd32(buf + 8);
    s->buf = buf; s->len = len;
    s->base = base; s->count = (base - 4) / 4; s->pos = 0;
    s->cur_off = base; s->cur_type = e0 & 7;
    s->next_off = (int64_t)(e1 >> 3) + base; s->next_type = e1 & 7;
    s->xw = 1;
    return 0;
}
int or_seq_peek(const or_seq* s, int* typ, int64_t* width) {
    if (s->pos >= s->count) return 1;
    *typ = s->cur_type;
    if (s->next_off > s->len) { *width = -1; return 1; }
    *width = s->next_off - s->cur_off;
    return 0;
}
/* returns 0 ok, 1 "out of bounds" error, 2 = Go runtime panic: the header
 * read binary.LittleEndian.Uint16(s.buf[(s.pos+1)*2:]) is not bounds
 * checked (seqget.go:95) and panics when fewer than 2 bytes remain.         */
int or_seq_advance(or_seq* s) {
    if (s->pos + 2 > s->count) return 1;
    s->pos++;
    s->cur_off = s->next_off;
    s->cur_type = s->next_type;
    if (s->cur_type != 0 && s->xw) {   /* extended: a short buffer is an error, not a panic */
        if (4 + (s->pos + 1) * 4 + 4 > s->len) return 1;
        uint32_t h = rd32(s->buf + 4 + (s->pos + 1) * 4);
        s->next_off = (int64_t)(h >> 3) + s->base;
        s->next_type = h & 7;
        return 0;
    }
    if (s->cur_type != 0) {
        if ((s->pos + 1) * 2 + 2 > s->len) return 2;
        uint16_t h = rd16(s->buf + (s->pos + 1) * 2);
        s->next_off = (h >> 3) + s->base;
        s->next_type = h & 7;
    }
    return 0;
}
int or_seq_next(or_seq* s, int64_t* start, int64_t* width, int* typ) {
    int64_t w;
    if (or_seq_peek(s, typ, &w)) return 1;
    if (w < 0 || s->cur_off + w > s->len) return 1;
    *start = s->cur_off; *width = w;
    return or_seq_advance(s) ? 1 : 0;
}
int or_seq_peek_nested(const or_seq* s, or_seq* nested) {
    if (s->cur_type != 7 && s->cur_type != 4) return 1;
    int64_t w = s->next_off - s->cur_off;
    if (w <= 0 || s->next_off > s->len) return 1;
    return or_seq_init(nested, s->buf + s->cur_off, w);
}

/* ------------------------------------------------------------------------ */
/* schema decode (schema/schema.go:893-910, 997-1052, 594-829, 270-326,      */
/* 383-414, 1591-1633, 1062-1130 Match)                                       */
/* ------------------------------------------------------------------------ */
typedef struct dec_ctx {
    const or_schema* s; packos_column* cols; size_t i; uint64_t blob_base;
    int ext;   /* PACKOS_MODE_EXTENDED: tag-2 fields are extended containers */
    int val;   /* ValidateBuffer (schema.go:880-891): Validate rules, no outputs */
} dec_ctx;

#define DEC_PANIC 0x100
#define DEC_POS0 0x200   /* the error carries position 0, not the field's */

/* precheck (schema.go:997-1013): 0 ok, else ErrConstraintViolated */
static int precheck(const or_seq* q, int tag, int64_t hint, int nullable, int64_t* w) {
    int typ; int64_t width;
    if (or_seq_peek(q, &typ, &width)) return 3;
    if (typ != tag) return 3;
    if (!nullable && hint != 0 && width != hint) return 3;
    *w = width;
    return 0;
}

/* validatePrimitiveAndGetPayload (schema.go:1031-1052): returns code,
 * *ps = payload start (-1 = nil payload), *w = width                        */
static int prim(or_seq* q, int tag, int64_t hint, int nullable, int64_t* ps, int64_t* w) {
    int e = precheck(q, tag, hint, nullable, w);
    if (e) return e;
    *ps = -1;
    if (*w > 0) {
        if (q->cur_off + *w > q->len) return 1;
        *ps = q->cur_off;
    }
    int a = or_seq_advance(q);
    if (a == 2) return DEC_PANIC;
    if (a) return 2;
    return 0;
}

static int dec_node(dec_ctx* c, int n, or_seq* q, uint64_t sub_base) {
    const or_schema* s = c->s;
    int k = NK(s, n);
    packos_column* col = !c->val && s->col_of_node[n] >= 0 ? &c->cols[s->col_of_node[n]] : NULL;
    int64_t ps, w;
    switch (k) {
        case ORN_INT: case ORN_UINT: case ORN_FLOAT: case ORN_BOOL: {
            int W = NA(s, n), nul = NB(s, n);
            int e = prim(q, leaf_tag(k), W, nul, &ps, &w);
            if (e) return e;
            if (c->val) {
                /* Validate: SBool..SFloat64 only run validatePrimitive, which never
                 * reads the payload (schema.go:596-715), so a short nullable payload
                 * passes; Range / SDateRange ValidateFuncs read it like their
                 * DecodeFuncs (:1177-1188, :2198-2212) and panic alike          */
                if (ps < 0 || !(xflags(s, n) & (X_MIN | X_MAX | X_DATE))) return 0;
                if (w < W) return DEC_PANIC;
                if ((xflags(s, n) & (X_MIN | X_MAX)) && range_bad(s, n, q->buf + ps, W))
                    return (xflags(s, n) & X_DATE) ? PACKOS_ERR_DATE_OUT_OF_RANGE : PACKOS_ERR_OUT_OF_RANGE;
                return 0;
            }
            if (ps < 0) { if (col->valid) col->valid[c->i] = 0; return 0; }
            if (w < W) return DEC_PANIC; /* binary.LittleEndian.UintXX on a short slice panics */
            uint8_t* dst = (uint8_t*)col->data + c->i * (size_t)W;
            if (k == ORN_BOOL) dst[0] = q->buf[ps] != 0;
            else memcpy(dst, q->buf + ps, (size_t)W);
            if (col->valid) col->valid[c->i] = 1;
            /* Range / SDateRange: CheckIntRange after the Advance */
            if ((xflags(s, n) & (X_MIN | X_MAX)) && range_bad(s, n, q->buf + ps, W))
                return (xflags(s, n) & X_DATE) ? PACKOS_ERR_DATE_OUT_OF_RANGE : PACKOS_ERR_OUT_OF_RANGE;
            return 0;
        }
        case ORN_STRING: case ORN_BYTES: {
            int W = NA(s, n);
            int e = prim(q, 6, W, W <= 0, &ps, &w);
            if (e) return e;
            size_t have = ps < 0 ? 0 : (size_t)w, dl = 0;
            const uint8_t* dp = (xflags(s, n) & X_DEFAULT) ? xlit(s, n, 1, &dl) : NULL;
            int dflt = have == 0 && dl > 0;   /* DefaultDecodeVal replaces an empty payload */
            if (c->val) {
                /* SchemaString/SchemaBytes.Validate = validatePrimitive (schema.go:275-277,
                 * 304-306); CheckFunc's ValidateFunc passes an empty string of a nullable
                 * receiver before the test (:1085-1087), the default applied first   */
                if (!(xflags(s, n) & (X_PREFIX | X_SUFFIX))) return 0;
                if (W <= 0 && (dflt ? dl : have) == 0) return 0;
                if (str_bad(s, n, dflt ? dp : q->buf + (ps < 0 ? 0 : ps), dflt ? dl : have))
                    return (xflags(s, n) & X_PREFIX) ? PACKOS_ERR_STRING_PREFIX : PACKOS_ERR_STRING_SUFFIX;
                return 0;
            }
            if (W > 0) {
                memcpy((uint8_t*)col->data + c->i * (size_t)W, q->buf + ps, (size_t)W);
            } else {
                /* aliasing view like GetStringUnsafe: absolute payload start, 0 for nil */
                col->start[c->i] = dflt ? PACKOS_VIEW_DEFAULT : ps < 0 ? 0u : sub_base + (uint64_t)ps;
                col->length[c->i] = dflt ? (uint32_t)dl : (uint32_t)have;
            }
            if ((xflags(s, n) & (X_PREFIX | X_SUFFIX)) &&
                str_bad(s, n, dflt ? dp : q->buf + (ps < 0 ? 0 : ps), dflt ? dl : have))
                return (xflags(s, n) & X_PREFIX) ? PACKOS_ERR_STRING_PREFIX : PACKOS_ERR_STRING_SUFFIX;
            return 0;
        }
        case ORN_MATCH: {
            /* SString.Match(expected): CheckFunc DecodeFunc (schema.go:1092-1108);
             * the hint is the receiver SchemaString's Width (b)               */
            int e = prim(q, 6, NB(s, n), NB(s, n) <= 0, &ps, &w);
            if (e) return e;
            size_t ll; const uint8_t* lp = lit_ptr(s, NA(s, n), &ll);
            size_t have = ps < 0 ? 0 : (size_t)w, dl = 0;
            const uint8_t* dp = (xflags(s, n) & X_DEFAULT) ? xlit(s, n, 1, &dl) : NULL;
            const uint8_t* vp = q->buf + (ps < 0 ? 0 : ps);
            if (have == 0 && dl > 0) { vp = dp; have = dl; }
            if (c->val && NB(s, n) <= 0 && have == 0) return 0;   /* ValidateFunc (schema.go:1085-1087) */
            if (have != ll || (ll && memcmp(vp, lp, ll) != 0)) return PACKOS_ERR_STRING_MATCH;
            return 0;
        }
        case ORN_TUPLE: case ORN_MAP: {
            /* TupleSchemaNamed.Decode: len(FieldNames) != len(Schemas) fails first,
             * ErrConstraintViolated at position 0 (schema.go:1754-1756)            */
            if (k == ORN_TUPLE && (NC(s, n) & ORT_NAMES_BAD)) return 3 | DEC_POS0;
            int nul = (k == ORN_MAP) ? 1 : NA(s, n);
            int xc = c->ext && q->cur_type == PACKOS_TAG_EXTENDED;
            int e = precheck(q, xc ? PACKOS_TAG_EXTENDED : leaf_tag(k), -1, nul, &w);
            if (e) return e;
            int kids[256];
            int nk = children(s, n, kids);
            /* SizeExact: Decode only (schema.go:369-377); SchemaMap.Validate has no
             * such check and validates the schemas in sequence (:336-359)    */
            if (k == ORN_MAP && (nk % 2) != 0 && !c->val) return 3;
            if (w != 0) {
                or_seq sub;
                if (xc) {
                    if (q->next_off - q->cur_off <= 0 || q->next_off > q->len) return 1;
                    if (or_seq_init_ext(&sub, q->buf + q->cur_off, q->next_off - q->cur_off, leaf_tag(k))) return 1;
                } else if (or_seq_peek_nested(q, &sub)) {
                    return 1;
                }
                /* arg count: TupleSchema.Decode checks it only when argCount > 0
                 * (schema.go:1607), TupleSchemaNamed.Decode always (:1773)       */
                if (k == ORN_TUPLE && !(NC(s, n) & ORT_VARIABLE) && (nk > 0 || (NC(s, n) & ORT_NAMED)) &&
                    (sub.count - 1) != nk)
                    return 3;
                uint64_t nb = sub_base + (uint64_t)q->cur_off;
                for (int j = 0; j < nk; j++) {
                    int ce = dec_node(c, kids[j], &sub, nb);
                    if (ce == DEC_PANIC) return DEC_PANIC;
                    if (ce) return 1; /* wrapped as ErrInvalidFormat */
                }
            }
            if (col && col->valid) col->valid[c->i] = w != 0;
            int a = or_seq_advance(q);
            if (a == 2) return DEC_PANIC;
            if (a) return 2;
            return 0;
        }
    }
    return 1;
}

static uint32_t decode_one(const or_schema* s, const uint8_t* blob, int64_t len, uint64_t base,
                           packos_column* cols, size_t i, int ext, int val) {
    or_seq q;
    if (ext && len >= 2 && rd16(blob) == or_encode_header(0, PACKOS_TAG_EXTENDED)) {
        if (or_seq_init_ext(&q, blob, len, PACKOS_TAG_TUPLE)) return (uint32_t)PACKOS_ERR_INVALID_FORMAT;
    } else if (or_seq_init(&q, blob, len)) {
        return (uint32_t)PACKOS_ERR_INVALID_FORMAT; /* pos -1 */
    }
    /* DecodeBufferNamed (schema.go:948-956): NewSeqGetAccess first, then the
     * length check fails every blob -- ErrConstraintViolated, position -1.
     * ValidateBuffer takes the plain SchemaChain (val): no such check.       */
    if (s->chain_names && !val) return (uint32_t)PACKOS_ERR_CONSTRAINT_VIOLATED;
    dec_ctx c = {s, cols, i, base, ext, val};
    for (int t = 0; t < s->n_top; t++) {
        int e = dec_node(&c, s->top_nodes[t], &q, base);
        if (e == DEC_PANIC) return PACKOS_STATUS_PANIC | ((uint32_t)(t + 1) << 8);
        if (e & DEC_POS0) return (uint32_t)(e & 0xFF) | (1u << 8);
        if (e) return (uint32_t)e | ((uint32_t)(t + 1) << 8);
    }
    return 0;
}

typedef struct dec_job {
    const or_schema* s; const uint8_t* arena; const uint64_t* offs; uint64_t stride;
    packos_column* cols; uint32_t* status; size_t lo, hi; int ext, val;
} dec_job;
static void* dec_worker(void* arg) {
    dec_job* j = (dec_job*)arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        uint64_t a = j->offs ? j->offs[i] : i * j->stride;
        uint64_t b = j->offs ? j->offs[i + 1] : (i + 1) * j->stride;
        j->status[i] = decode_one(j->s, j->arena + a, (int64_t)(b - a), a, j->cols, i, j->ext, j->val);
    }
    return NULL;
}
int or_decode_batch(const or_schema* s, const uint8_t* arena, const uint64_t* offsets, uint64_t stride,
                    size_t n, packos_column* cols, uint32_t* status, int nthreads) {
    return or_decode_batch_mode(s, arena, offsets, stride, n, cols, status, nthreads, 0);
}
static int dec_run(const or_schema* s, const uint8_t* arena, const uint64_t* offsets, uint64_t stride,
                   size_t n, packos_column* cols, uint32_t* status, int nthreads, int mode, int val);
int or_decode_batch_mode(const or_schema* s, const uint8_t* arena, const uint64_t* offsets, uint64_t stride,
                         size_t n, packos_column* cols, uint32_t* status, int nthreads, int mode) {
    return dec_run(s, arena, offsets, stride, n, cols, status, nthreads, mode, 0);
}
/* ValidateBuffer (schema/schema.go:880-891) per blob: the status word
 * DecodeBuffer's would be under the Validate methods' rules (no outputs)    */
int or_validate_batch(const or_schema* s, const uint8_t* arena, const uint64_t* offsets, uint64_t stride,
                      size_t n, uint32_t* status, int nthreads, int mode) {
    return dec_run(s, arena, offsets, stride, n, NULL, status, nthreads, mode, 1);
}
static int dec_run(const or_schema* s, const uint8_t* arena, const uint64_t* offsets, uint64_t stride,
                   size_t n, packos_column* cols, uint32_t* status, int nthreads, int mode, int val) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > OR_MAX_THREADS) nthreads = OR_MAX_THREADS;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    dec_job* dj = (dec_job*)malloc(sizeof(dec_job) * (size_t)nthreads);
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        size_t lo = (size_t)t * per, hi = lo + per > n ? n : lo + per;
        if (lo > hi) lo = hi;
        dj[t] = (dec_job){s, arena, offsets, stride, cols, status, lo, hi, (mode & PACKOS_MODE_EXTENDED) != 0, val};
        pthread_create(&th[t], NULL, dec_worker, &dj[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th); free(dj);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* GetAccess (access/get.go:19-58, 60-375, 492-501)                          */
/* ------------------------------------------------------------------------ */
int or_get_init(or_get* g, const uint8_t* buf, int64_t len) {
    if (len < 2) return 0;
    int64_t base = rd16(buf) >> 3;
    if (len < base) return 0;
    g->buf = buf; g->len = len; g->base = base; g->arg_count = base / 2 - 1;
    g->xw = 0; g->xmode = 0;
    return 1;
}
/* ADR-001 extended container as a GetAccess (this build's format,
 * include/packos.h): lead 02 00 | kind (4 or 7; top level: 4) | u32 entries */
static int get_init_ext(or_get* g, const uint8_t* buf, int64_t len, int top) {
    if (len < 12 || rd16(buf) != or_encode_header(0, PACKOS_TAG_EXTENDED)) return 0;
    int kind = rd16(buf + 2);
    if (kind != PACKOS_TAG_TUPLE && (top || kind != PACKOS_TAG_MAP)) return 0;
    int64_t base = rd32(buf + 4) >> 3;
    if (base < 12 || (base & 3) || len < base) return 0;
    g->buf = buf; g->len = len; g->base = base; g->arg_count = (base - 4) / 4 - 1;
    g->xw = 1; g->xmode = 1;
    return 1;
}
void or_get_range(const or_get* g, int64_t pos, int* tp, int64_t* start, int64_t* end) {
    if (pos >= g->arg_count) { *tp = 0; *start = -2; *end = -1; return; }
    if (g->xw) {
        uint32_t e1 = rd32(g->buf + 4 + pos * 4), e2 = rd32(g->buf + 4 + (pos + 1) * 4);
        *start = e1 >> 3; *tp = e1 & 7;
        *end = (int64_t)(e2 >> 3) + g->base;
        if (pos > 0) *start += g->base;
        if (*end > g->len) *end = -1;
        return;
    }
    uint16_t h1 = rd16(g->buf + pos * 2), h2 = rd16(g->buf + (pos + 1) * 2);
    *start = h1 >> 3; *tp = h1 & 7;
    *end = (h2 >> 3) + g->base;
    if (pos > 0) *start += g->base;
    if (*end > g->len) *end = -1;
}
int or_get_fixed(const or_get* g, int64_t pos, int tag, int width, int64_t* start) {
    int tp; int64_t st, en;
    or_get_range(g, pos, &tp, &st, &en);
    if (tp != tag || en - st != width) return 1;
    *start = st;
    return 0;
}
int or_get_nullable(const or_get* g, int64_t pos, int tag, int width, int64_t* start) {
    int tp; int64_t st, en;
    or_get_range(g, pos, &tp, &st, &en);
    if (en - st == 0) return 2;
    if (tp != tag || en - st != width) return 1;
    *start = st;
    return 0;
}
int or_get_span(const or_get* g, int64_t pos, int64_t* start, int64_t* end) {
    int tp; int64_t st, en;
    or_get_range(g, pos, &tp, &st, &en);
    if (tp != 6 || en < st) return 1;
    *start = st; *end = en;
    return 0;
}
int or_get_nested(const or_get* g, int64_t pos, or_get* nested, int* tp) {
    int64_t st, en;
    or_get_range(g, pos, tp, &st, &en);
    const int x = g->xmode && *tp == PACKOS_TAG_EXTENDED;
    if (en < st || (*tp != 7 && *tp != 4 && !x)) return 1;
    if (en == st) return 2;
    if (x) return get_init_ext(nested, g->buf + st, en - st, 0) ? 0 : 1;   /* malformed: decode error */
    if (!or_get_init(nested, g->buf + st, en - st)) return 3; /* nil accessor: later use panics */
    nested->xmode = g->xmode;
    return 0;
}
/* top-level accessor; xmode: a blob starting 02 00 is extended */
static int get_open(or_get* g, const uint8_t* buf, int64_t len, int xmode) {
    if (xmode && len >= 2 && rd16(buf) == or_encode_header(0, PACKOS_TAG_EXTENDED)) return get_init_ext(g, buf, len, 1);
    if (!or_get_init(g, buf, len)) return 0;
    g->xmode = xmode;
    return 1;
}

int or_get_field_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n,
                       const int32_t* path, int depth, int want_tag, int want_width,
                       uint64_t* out_start, uint32_t* out_len, uint8_t* out_tag, uint8_t* status) {
    for (size_t i = 0; i < n; i++) {
        uint64_t a = offsets ? offsets[i] : i * stride;
        uint64_t b = offsets ? offsets[i + 1] : (i + 1) * stride;
        or_get g;
        out_start[i] = 0; out_len[i] = 0; out_tag[i] = 0;
        if (!or_get_init(&g, arena + a, (int64_t)(b - a))) { status[i] = 3; continue; }
        uint64_t base = a;
        int st = 0;
        for (int d = 0; d < depth - 1 && !st; d++) {
            or_get nx; int tp;
            int r = or_get_nested(&g, path[d], &nx, &tp);
            if (r) { st = r; break; }
            base += (uint64_t)(nx.buf - g.buf);
            g = nx;
        }
        if (st) { status[i] = (uint8_t)st; continue; }
        int tp; int64_t s0, e0;
        or_get_range(&g, path[depth - 1], &tp, &s0, &e0);
        out_tag[i] = (uint8_t)tp;
        if (want_width >= 0) {
            if (tp != want_tag || e0 - s0 != want_width) { status[i] = 1; continue; }
        } else {
            if (tp != want_tag || e0 < s0) { status[i] = 1; continue; }
        }
        out_start[i] = base + (uint64_t)s0;
        out_len[i] = (uint32_t)(e0 - s0);
        status[i] = 0;
    }
    return 0;
}

/* packos_get_batch contract (include/packos.h).  Each getter restates the
 * matching Get* family of access/get.go:
 *   FIXED     Get{Bool,Int8..64,Uint8..64,Float32/64}: tag and exact width
 *             (get.go:60-66, 80-94, 173-226, 287-305); value = the LE bytes,
 *             a Bool normalised to 0/1 (g.buf[start] != 0)
 *   NULLABLE  GetNullable*: width 0 -> (nil, nil) BEFORE the tag check
 *             (get.go:68-78, 96-118, 214-284, 307-333)
 *   SPAN      GetBytes / GetString(Unsafe): tag and end >= start (get.go:335-375)
 *   INT       GetInt: tag Integer first, then width 0 -> nil, 1/2/4/8 ->
 *             int8..int64 (sign-extended to 8 bytes), else error (get.go:120-146)
 *   FLOAT     GetFloating: tag Floating first, then 0 -> nil, 4/8 -> raw bits
 *             (8-byte slot, float32 bits low), else error (get.go:148-170)
 * status: 0 ok, 1 decode error, 2 nil nested accessor, 3 nil accessor (the
 * reference dereferences nil: panic), 4 nil value (no error). */
int or_get_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n,
                 const int32_t* path, int depth, int getter, int want_tag, int want_width,
                 uint8_t* out_values, uint32_t value_width, uint64_t* out_start, uint32_t* out_len,
                 uint8_t* out_tag, uint8_t* status) {
    const int xmode = (getter & PACKOS_GET_EXTENDED) != 0;
    getter &= ~PACKOS_GET_EXTENDED;
    for (size_t i = 0; i < n; i++) {
        uint64_t a = offsets ? offsets[i] : i * stride;
        uint64_t b = offsets ? offsets[i + 1] : (i + 1) * stride;
        or_get g;
        out_start[i] = 0; out_len[i] = 0; out_tag[i] = 0;
        if (out_values) memset(out_values + i * value_width, 0, value_width);
        if (!get_open(&g, arena + a, (int64_t)(b - a), xmode)) { status[i] = 3; continue; }
        uint64_t base = a;
        int st = 0;
        for (int d = 0; d < depth - 1 && !st; d++) {
            or_get nx; int tp;
            int r = or_get_nested(&g, path[d], &nx, &tp);
            if (r) { st = r; break; }
            base += (uint64_t)(nx.buf - g.buf);
            g = nx;
        }
        if (st) { status[i] = (uint8_t)st; continue; }
        int tp; int64_t s0, e0;
        or_get_range(&g, path[depth - 1], &tp, &s0, &e0);
        out_tag[i] = (uint8_t)tp;
        const int64_t w = e0 - s0;
        int r = 0;
        switch (getter) {
            case PACKOS_GET_NULLABLE:
                if (w == 0) { r = 4; break; }
                /* fall through */
            case PACKOS_GET_FIXED:
                if (tp != want_tag || w != want_width) r = 1;
                break;
            case PACKOS_GET_SPAN:
                if (tp != want_tag || e0 < s0) r = 1;
                break;
            case PACKOS_GET_INT:
                if (tp != PACKOS_TAG_INTEGER) r = 1;
                else if (w == 0) r = 4;
                else if (w != 1 && w != 2 && w != 4 && w != 8) r = 1;
                break;
            case PACKOS_GET_FLOAT:
                if (tp != PACKOS_TAG_FLOATING) r = 1;
                else if (w == 0) r = 4;
                else if (w != 4 && w != 8) r = 1;
                break;
            case PACKOS_GET_ANY:   /* GetTypeAndValue (get.go:504-510) */
                /* past argCount rangeAt gives (End, -2, -1): end >= start, and
                 * g.buf[-2:-1] is a Go runtime panic */
                r = s0 < 0 ? 3 : e0 < s0 ? 1 : 0;
                break;
            default:
                r = 1;
        }
        status[i] = (uint8_t)r;
        if (r) continue;
        out_start[i] = base + (uint64_t)s0;
        out_len[i] = (uint32_t)w;
        if (!out_values || getter == PACKOS_GET_SPAN || getter == PACKOS_GET_ANY) continue;
        const uint8_t* src = g.buf + s0;
        uint8_t* dst = out_values + i * value_width;
        if (getter == PACKOS_GET_INT) {
            uint64_t v = 0;
            for (int k = 0; k < w; k++) v |= (uint64_t)src[k] << (8 * k);
            if (w < 8 && (v >> (8 * w - 1)) & 1) v |= ~0ull << (8 * w);   /* int8..int32 -> int64 */
            for (int k = 0; k < 8 && k < (int)value_width; k++) dst[k] = (uint8_t)(v >> (8 * k));
        } else if (tp == PACKOS_TAG_BOOL && w == 1) {
            dst[0] = src[0] != 0;
        } else {
            for (int64_t k = 0; k < w && k < (int64_t)value_width; k++) dst[k] = src[k];
        }
    }
    return 0;
}

/* GetMapStr / GetMapAny (access/get.go:412-490) over every blob, the
 * packos_get_map_batch contract (include/packos.h).  The recursion of
 * GetMapAny -> GetAny -> GetMapAny (get.go:377-430) is restated directly. */
#define OR_MAP_MAX_DEPTH 32
/* GetAny (get.go:377-410) of value position pos of map accessor m: 0 ok, 1
 * error, 3 panic, 6 too deep; a non-empty nested map is walked (depth+1). */
static int map_walk(const or_get* m, int any, int depth);
static int get_any_value(const or_get* m, int64_t pos, int any, int depth) {
    int tp; int64_t st, en;
    if (!any) {   /* GetString (get.go:359-365) */
        or_get_range(m, pos, &tp, &st, &en);
        return (en < st || tp != PACKOS_TAG_STRING) ? 1 : 0;
    }
    /* GetAny reads the header at pos (the End header when pos == argCount);
     * every getter it calls re-reads through rangeAt, which fails there */
    if (pos >= m->arg_count) return 1;
    or_get_range(m, pos, &tp, &st, &en);
    const int64_t w = en - st;
    switch (tp) {
        case PACKOS_TAG_INTEGER: return (w == 0 || w == 1 || w == 2 || w == 4 || w == 8) ? 0 : 1;   /* GetInt :120-146 */
        case PACKOS_TAG_FLOATING: return (w == 0 || w == 4 || w == 8) ? 0 : 1;                      /* GetFloating :148-170 */
        case PACKOS_TAG_STRING: return en < st ? 1 : 0;                                              /* GetString */
        case PACKOS_TAG_MAP: case PACKOS_TAG_EXTENDED: {                                            /* GetMapAny :412-436 */
            const int x = tp == PACKOS_TAG_EXTENDED;
            if (x && !m->xmode) return 1;
            if (en < st) return 1;
            if (en == st) return 0;   /* nil map */
            or_get nm;
            if (x) {
                if (!get_init_ext(&nm, m->buf + st, en - st, 0) || rd16(nm.buf + 2) != PACKOS_TAG_MAP) return 1;
            } else if (!or_get_init(&nm, m->buf + st, en - st)) {
                return 3;   /* NewGetAccess nil -> nested.argCount panics */
            } else {
                nm.xmode = m->xmode;
            }
            if (depth + 1 >= OR_MAP_MAX_DEPTH) return 6;
            return map_walk(&nm, any, depth + 1);
        }
        default: return 1;   /* "GetAny: unsupported type tag" */
    }
}
static int map_walk(const or_get* m, int any, int depth) {
    for (int64_t j = 0; j < m->arg_count; j += 2) {
        int tp; int64_t st, en;
        or_get_range(m, j, &tp, &st, &en);   /* key: GetString */
        if (en < st || tp != PACKOS_TAG_STRING) return 1;
        const int r = get_any_value(m, j + 1, any, depth);
        if (r) return r;
    }
    return 0;
}
int or_get_map_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n,
                     const int32_t* path, int depth, int flags, uint32_t max_pairs, uint32_t* out_pairs,
                     uint64_t* key_start, uint32_t* key_len, uint64_t* val_start, uint32_t* val_len,
                     uint8_t* val_tag, uint8_t* status) {
    const int xmode = (flags & PACKOS_GET_EXTENDED) != 0;
    const int any = (flags & ~PACKOS_GET_EXTENDED) == PACKOS_MAP_ANY;
    for (size_t i = 0; i < n; i++) {
        uint64_t a = offsets ? offsets[i] : i * stride;
        uint64_t b = offsets ? offsets[i + 1] : (i + 1) * stride;
        out_pairs[i] = 0;
        for (uint32_t j = 0; j < max_pairs; j++) {
            const size_t k = i * (size_t)max_pairs + j;
            key_start[k] = 0; key_len[k] = 0; val_start[k] = 0; val_len[k] = 0; val_tag[k] = 0;
        }
        or_get g;
        if (!get_open(&g, arena + a, (int64_t)(b - a), xmode)) { status[i] = 3; continue; }
        uint64_t base = a;
        int st = 0;
        for (int d = 0; d < depth - 1 && !st; d++) {
            or_get nx; int tp;
            int r = or_get_nested(&g, path[d], &nx, &tp);
            if (r) { st = r; break; }
            base += (uint64_t)(nx.buf - g.buf);
            g = nx;
        }
        if (st) { status[i] = (uint8_t)st; continue; }
        int tp; int64_t s0, e0;
        or_get_range(&g, path[depth - 1], &tp, &s0, &e0);
        const int x = xmode && tp == PACKOS_TAG_EXTENDED;
        if (e0 < s0 || (tp != PACKOS_TAG_MAP && !x)) { status[i] = 1; continue; }   /* get.go:414-416 */
        if (e0 == s0) { status[i] = 4; continue; }                                    /* nil map */
        or_get m;
        if (x) {
            if (!get_init_ext(&m, g.buf + s0, e0 - s0, 0) || rd16(m.buf + 2) != PACKOS_TAG_MAP) { status[i] = 1; continue; }
        } else if (!or_get_init(&m, g.buf + s0, e0 - s0)) {
            status[i] = 3;
            continue;
        } else {
            m.xmode = xmode;
        }
        const uint64_t mb = base + (uint64_t)s0;
        int r = 0;
        uint32_t pairs = 0;
        for (int64_t j = 0; j < m.arg_count && !r; j += 2, pairs++) {
            int kt; int64_t ks, ke;
            or_get_range(&m, j, &kt, &ks, &ke);
            if (ke < ks || kt != PACKOS_TAG_STRING) { r = 1; break; }
            r = get_any_value(&m, j + 1, any, 0);
            if (r) break;
            if (pairs < max_pairs) {
                int vt; int64_t vs, ve;
                or_get_range(&m, j + 1, &vt, &vs, &ve);
                const size_t k = i * (size_t)max_pairs + pairs;
                key_start[k] = mb + (uint64_t)ks; key_len[k] = (uint32_t)(ke - ks);
                val_start[k] = mb + (uint64_t)vs; val_len[k] = (uint32_t)(ve - vs); val_tag[k] = (uint8_t)vt;
            }
        }
        if (r) {   /* a failing call returns no map */
            status[i] = (uint8_t)r;
            for (uint32_t j = 0; j < max_pairs; j++) {
                const size_t k = i * (size_t)max_pairs + j;
                key_start[k] = 0; key_len[k] = 0; val_start[k] = 0; val_len[k] = 0; val_tag[k] = 0;
            }
            continue;
        }
        out_pairs[i] = pairs;
        status[i] = pairs > max_pairs ? 5 : 0;
    }
    return 0;
}

uint64_t or_splitmix64(uint64_t* state) {
    uint64_t z = (*state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
