// compile.cpp — host schema compiler: SchemaJSON -> encode / fixed-layout /
// decode programs.  No GPU needed.
//
// Replaces schema.BuildSchema (schema/schemabuilder_json.go:124-300) for the
// fixed-schema subset and resolves, once per schema, everything the reference
// recomputes per blob: map key order (utils.SortKeys, utils/utils.go:7-14),
// header-block sizes (access/put.go:619-627, packable/pack.go:36) and, for
// fixed-size schemas, every header word of the blob.
#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "json_lite.hpp"
#include "schema_impl.h"

using namespace packos;

namespace {

thread_local std::string g_err;

struct CompileError {
    int code;
    std::string msg;
};

[[noreturn]] void fail(int code, const std::string& m) { throw CompileError{code, m}; }

int tag_of(int kind) {
    switch (kind) {
        case K_INT: case K_UINT: return PACKOS_TAG_INTEGER;
        case K_FLOAT: return PACKOS_TAG_FLOATING;
        case K_BOOL: return PACKOS_TAG_BOOL;
        case K_STRING: case K_BYTES: case K_MATCH: return PACKOS_TAG_STRING;
        case K_TUPLE: return PACKOS_TAG_TUPLE;
        case K_MAP: return PACKOS_TAG_MAP;
    }
    return 0;
}

// uint16(offset<<3) | tag (typetags/types.go:44-46): silently truncating
uint16_t enc_header(int64_t off, int tag) { return (uint16_t)((((uint64_t)off) << 3) & 0xFFFFu) | (uint16_t)(tag & 7); }

struct Builder {
    packos_schema* s;

    int new_node() {
        s->nodes.emplace_back();
        return (int)s->nodes.size() - 1;
    }

    static int width_of(const char* t) {
        if (!strcmp(t, "8")) return 1;
        if (!strcmp(t, "16")) return 2;
        if (!strcmp(t, "32")) return 4;
        if (!strcmp(t, "64")) return 8;
        return 0;
    }

    static std::string str_field(const JVal& j, const char* k) {
        const JVal* v = j.get(k);
        return (v && v->kind == JVal::STR) ? v->str : std::string();
    }
    static bool bool_field(const JVal& j, const char* k, bool dflt = false) {
        const JVal* v = j.get(k);
        return v ? v->truthy() : dflt;
    }
    static int int_field(const JVal& j, const char* k) {
        const JVal* v = j.get(k);
        return (v && v->kind == JVal::NUM) ? (int)v->num : 0;
    }

    // SchemaJSON Min/Max are *int64 (schemabuilder_json.go:18-19): an exact
    // integer literal, or absent / null
    static bool int64_field(const JVal& j, const char* k, int64_t* out) {
        const JVal* v = j.get(k);
        if (!v || v->kind == JVal::NUL) return false;
        if (v->kind != JVal::NUM || v->str.find_first_of(".eE") != std::string::npos)
            fail(PACKOS_E_SCHEMA, std::string("'") + k + "' must be an integer");
        errno = 0;
        char* end = nullptr;
        long long x = strtoll(v->str.c_str(), &end, 10);
        if (errno || !end || *end) fail(PACKOS_E_SCHEMA, std::string("'") + k + "' is not an int64");
        *out = (int64_t)x;
        return true;
    }

    // time.Parse(time.RFC3339, s).Unix(); the builder drops the parse error
    // (schemabuilder_json.go:169-170), so a bad string is the zero Time,
    // whose Unix() is -62135596800.
    static int64_t rfc3339_unix(const std::string& t) {
        const int64_t zero = -62135596800LL;
        auto dig = [&](size_t at, int n, int* v) {
            if (at + n > t.size()) return false;
            int x = 0;
            for (int k = 0; k < n; k++) {
                char c = t[at + k];
                if (c < '0' || c > '9') return false;
                x = 10 * x + (c - '0');
            }
            *v = x;
            return true;
        };
        int Y, M, D, h, m, sec;
        if (!dig(0, 4, &Y) || t.size() < 20 || t[4] != '-' || !dig(5, 2, &M) || t[7] != '-' || !dig(8, 2, &D) ||
            t[10] != 'T' || !dig(11, 2, &h) || t[13] != ':' || !dig(14, 2, &m) || t[16] != ':' || !dig(17, 2, &sec))
            return zero;
        size_t p = 19;
        if (p < t.size() && t[p] == '.') {   // fractional seconds: dropped by Unix()
            size_t q = p + 1;
            while (q < t.size() && t[q] >= '0' && t[q] <= '9') q++;
            if (q == p + 1) return zero;
            p = q;
        }
        int64_t tz = 0;
        if (p < t.size() && t[p] == 'Z') {
            p++;
        } else if (p < t.size() && (t[p] == '+' || t[p] == '-')) {
            int th, tm;
            if (!dig(p + 1, 2, &th) || p + 3 >= t.size() || t[p + 3] != ':' || !dig(p + 4, 2, &tm) || th > 23 || tm > 59)
                return zero;
            tz = (t[p] == '-' ? -1 : 1) * (int64_t)(th * 3600 + tm * 60);
            p += 6;
        } else {
            return zero;
        }
        if (p != t.size()) return zero;
        static const int mdays[12] = {31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
        const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
        if (M < 1 || M > 12 || D < 1 || D > mdays[M - 1] || (M == 2 && D == 29 && !leap) || h > 23 || m > 59 || sec > 59)
            return zero;
        // days from civil (proleptic Gregorian)
        const int y = Y - (M <= 2);
        const int era = (y >= 0 ? y : y - 399) / 400;
        const int yoe = y - era * 400;
        const int doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
        const int doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
        const int64_t days = (int64_t)era * 146097 + doe - 719468;
        return days * 86400 + h * 3600 + m * 60 + sec - tz;
    }

    // BuildSchema (schemabuilder_json.go:124-300), compiled subset
    int node(const JVal& j, int parent, int depth, int top, const std::string& name) {
        if (j.kind != JVal::OBJ) fail(PACKOS_E_SCHEMA, "schema node must be an object");
        if (depth >= kMaxDepth - 1) fail(PACKOS_E_UNSUPPORTED, "nesting deeper than supported");
        std::string t = str_field(j, "type");
        int id = new_node();
        {
            Node& n = s->nodes[id];
            n.parent = parent;
            n.depth = depth;
            n.top = top;
            n.name = name;
        }
        bool nullable = bool_field(j, "nullable");
        auto unsupported_keys = [&](std::initializer_list<const char*> keys) {
            for (const char* k : keys)
                if (j.get(k) && !(j.get(k)->kind == JVal::STR && j.get(k)->str.empty()))
                    fail(PACKOS_E_UNSUPPORTED, std::string("'") + k + "' on a " + t +
                                                   " node is outside the compiled subset");
        };
        if (t == "bool") {
            Node& n = s->nodes[id];
            n.kind = K_BOOL; n.width = 1; n.nullable = nullable;
        } else if (t.rfind("int", 0) == 0 && width_of(t.c_str() + 3)) {
            Node& n = s->nodes[id];
            n.kind = K_INT; n.width = width_of(t.c_str() + 3); n.nullable = nullable;
            // int16/32/64 with Min or Max -> s.Range(min, max), whose precheck
            // is never nullable (schema.go:1175-1364); int8 ignores them
            // (schemabuilder_json.go:133-137)
            int64_t lo = 0, hi = 0;
            const bool has_lo = int64_field(j, "min", &lo), has_hi = int64_field(j, "max", &hi);
            if (n.width > 1 && (has_lo || has_hi)) {
                n.nullable = false;
                n.check = (has_lo ? CHK_MIN : 0u) | (has_hi ? CHK_MAX : 0u);
                n.rmin = lo;
                n.rmax = hi;
            }
        } else if (t == "date") {
            // SDateRange(nullable, from, to): int64 payload, bounds only when
            // both dates are given (schemabuilder_json.go:166-173, schema.go:2188-2250)
            Node& n = s->nodes[id];
            n.kind = K_INT; n.width = 8; n.nullable = nullable;
            n.check = CHK_DATE;
            const std::string from = str_field(j, "dateFrom"), to = str_field(j, "dateTo");
            if (!from.empty() && !to.empty()) {
                n.check |= CHK_RANGE;
                n.rmin = rfc3339_unix(from);
                n.rmax = rfc3339_unix(to);
            }
        } else if (t.rfind("uint", 0) == 0 && width_of(t.c_str() + 4)) {
            unsupported_keys({"min", "max"});
            Node& n = s->nodes[id];
            n.kind = K_UINT; n.width = width_of(t.c_str() + 4); n.nullable = nullable;
        } else if (t == "float32" || t == "float64") {
            Node& n = s->nodes[id];
            n.kind = K_FLOAT; n.width = t == "float32" ? 4 : 8; n.nullable = nullable;
        } else if (t == "string") {
            // SString / Optional() (Width -1) / WithWidth(n), then
            // DefaultDecodeValue, then the first of exact / prefix / suffix /
            // pattern (schemabuilder_json.go:184-208)
            int w = 0;
            if (nullable) w = -1;
            else if (int_field(j, "width") > 0) w = int_field(j, "width");
            Node& n = s->nodes[id];
            n.width = w;
            n.nullable = w <= 0;
            n.dflt = str_field(j, "decodeDefault");
            if (!n.dflt.empty()) n.check |= CHK_DEFAULT;
            const std::string exact = str_field(j, "exact"), prefix = str_field(j, "prefix"),
                              suffix = str_field(j, "suffix"), pattern = str_field(j, "pattern");
            if (!exact.empty()) {
                n.kind = K_MATCH;
                n.literal = exact;
            } else {
                n.kind = K_STRING;
                if (!prefix.empty()) {
                    n.check |= CHK_PREFIX;
                    n.check_lit = prefix;
                } else if (!suffix.empty()) {
                    n.check |= CHK_SUFFIX;
                    n.check_lit = suffix;
                } else if (!pattern.empty()) {
                    fail(PACKOS_E_UNSUPPORTED, "'pattern' (regexp) strings are outside the compiled subset");
                }
            }
        } else if (t == "bytes") {
            int w = int_field(j, "width");
            Node& n = s->nodes[id];
            n.kind = K_BYTES; n.width = w > 0 ? w : -1; n.nullable = n.width <= 0;
        } else if (t == "tuple") {
            // "flatten" (with variableLength: STupleValFlatten / STupleNamedValFlattened,
            // schemabuilder_json.go:247-258) only changes how SRepeatSchema
            // children encode and decode (schema.go:1616-1623,1649-1664,1781-1790,
            // 1816); repeat is rejected below, so a flattened tuple is compiled
            // exactly as the plain one
            const JVal* sch = j.get("schema");
            const JVal* names = j.get("fieldNames");
            {
                Node& n = s->nodes[id];
                n.kind = K_TUPLE;
                // every STuple* constructor sets Nullable: true and BuildSchema
                // never reads the key for tuples (schemabuilder_json.go:244-260,
                // schema.go:1551-1552)
                n.nullable = true;
                n.variable = bool_field(j, "variableLength");
                // BuildSchema makes a TupleSchemaNamed of a non-empty fieldNames
                // (schemabuilder_json.go:245-253); "named" (a key of this build,
                // which Go's json ignores) marks STupleNamed(nil, ...) / an empty
                // name list, which the reference JSON cannot express
                const size_t nn = names && names->kind == JVal::ARR ? names->arr.size() : 0;
                n.named = nn > 0 || bool_field(j, "named");
                const size_t ns = sch && sch->kind == JVal::ARR ? sch->arr.size() : 0;
                n.names_bad = n.named && nn != ns;
            }
            if (sch && sch->kind == JVal::ARR) {
                for (size_t k = 0; k < sch->arr.size(); k++) {
                    std::string nm;
                    if (names && names->kind == JVal::ARR && k < names->arr.size() &&
                        names->arr[k].kind == JVal::STR)
                        nm = names->arr[k].str;
                    std::string path = name.empty() ? nm : (nm.empty() ? name : name + "." + nm);
                    int kid = node(sch->arr[k], id, depth + 1, top, path);
                    s->nodes[id].kids.push_back(kid);
                }
            }
        } else if (t == "map") {
            const JVal* sch = j.get("schema");
            {
                Node& n = s->nodes[id];
                n.kind = K_MAP;
                n.width = -1;
                n.nullable = true;  // SchemaMap.IsNullable: Width <= 0
                n.sorted = bool_field(j, "sorted");
            }
            if (sch && sch->kind == JVal::ARR) {
                // an odd schema count compiles: Encode fails a present value and
                // Decode every non-nil map with SizeExact (schema.go:369-377,
                // 422-429), but Validate has no such check (:336-359)
                for (size_t k = 0; k < sch->arr.size(); k++) {
                    int kid = node(sch->arr[k], id, depth + 1, top, name);
                    int kk = s->nodes[kid].kind;
                    if (k % 2 == 0 && kk != K_MATCH && kk != K_STRING)
                        fail(PACKOS_E_SCHEMA, "map keys must be strings");
                    s->nodes[id].kids.push_back(kid);
                }
            }
            Node& n = s->nodes[id];
            if (n.sorted) {
                size_t np = n.kids.size() / 2;
                std::vector<std::pair<int, int>> pairs;
                for (size_t p = 0; p < np; p++) {
                    if (s->nodes[n.kids[2 * p]].kind != K_MATCH)
                        fail(PACKOS_E_SCHEMA, "sorted maps need exact (constant) keys");
                    pairs.emplace_back(n.kids[2 * p], n.kids[2 * p + 1]);
                }
                // sort.Strings order = bytewise (utils/utils.go:7-14)
                std::stable_sort(pairs.begin(), pairs.end(), [&](auto& a, auto& b) {
                    return s->nodes[a.first].literal < s->nodes[b.first].literal;
                });
                std::vector<int> k2;
                for (auto& p : pairs) { k2.push_back(p.first); k2.push_back(p.second); }
                if (n.kids.size() % 2) k2.push_back(n.kids.back());   // odd count: the unpaired key stays last
                n.kids = k2;
            }
        } else {
            fail(PACKOS_E_UNSUPPORTED, "schema type '" + t + "' is outside the compiled subset");
        }
        return id;
    }

    void assign_columns(int id) {
        Node& n = s->nodes[id];
        if (n.kind != K_MATCH && n.kind != K_ROOT) {
            n.col = (int)s->col_node.size();
            s->col_node.push_back(id);
        }
        for (int k : s->nodes[id].kids) assign_columns(k);
    }

    // ---------------------------------------------------------- encode ----
    int emit_container(int id, int cont_id) {
        Node& n = s->nodes[id];
        int nk = (int)n.kids.size();
        EncItem hdr{};
        hdr.type = IT_HDR;
        hdr.cont = (int16_t)cont_id;
        hdr.col = -1;
        hdr.size = nk ? (uint32_t)(2 * (nk + 1)) : (s->mode == PACKOS_MODE_PUTACCESS ? 2u : 0u);
        int hdr_item = (int)s->items.size();
        s->items.push_back(hdr);
        s->conts[cont_id].hdr_item = (uint16_t)hdr_item;
        s->conts[cont_id].n_kids = (uint16_t)nk;
        std::vector<int> kid_start, kid_cont;
        for (int k : n.kids) {
            kid_start.push_back((int)s->items.size());
            const int k_kind = s->nodes[k].kind;
            kid_cont.push_back(k_kind == K_TUPLE || k_kind == K_MAP ? (int)s->conts.size() + 1 : 0);
            emit_node(k, cont_id);
        }
        int end_item = (int)s->items.size();
        s->conts[cont_id].end_item = (uint16_t)end_item;
        s->conts[cont_id].tag = (uint8_t)(n.kind == K_MAP ? tag_of(K_MAP) : tag_of(K_TUPLE));
        if (nk == 0) {
            if (s->mode == PACKOS_MODE_PUTACCESS) {
                // BeginX/EndNested (or Pack() of an empty accessor) appends End(0)
                // and rewrites h0 as EncodeHeader(2, 0) = 0x0010 (put.go:619-652)
                EncHdr h{};
                h.hdr_item = (uint16_t)hdr_item; h.cont = (uint16_t)cont_id;
                h.relative = 0; h.j = 0; h.value = enc_header(2, 0); h.tag = 0;
                s->hdrs.push_back(h);
            }
            return end_item;
        }
        for (int j = 0; j <= nk; j++) {
            EncHdr h{};
            h.hdr_item = (uint16_t)hdr_item;
            h.cont = (uint16_t)cont_id;
            h.j = (uint16_t)j;
            h.child = j < nk ? (uint16_t)kid_cont[j] : (uint16_t)0;
            if (j == 0) {
                int64_t hs = 2 * (int64_t)(nk + 1);
                h.relative = 0;
                h.tag = (uint8_t)tag_of(s->nodes[n.kids[0]].kind);
                h.value = enc_header(hs, h.tag);
                h.ovf = hs >= 8192;
            } else if (j < nk) {
                h.relative = 1;
                h.target = (uint16_t)kid_start[j];
                h.tag = (uint8_t)tag_of(s->nodes[n.kids[j]].kind);
            } else {
                h.relative = 1;
                h.target = (uint16_t)end_item;
                h.tag = 0;
            }
            s->hdrs.push_back(h);
        }
        return end_item;
    }

    void emit_node(int id, int cont_id) {
        Node& n = s->nodes[id];
        EncItem it{};
        it.cont = (int16_t)cont_id;
        it.col = (int16_t)n.col;
        switch (n.kind) {
            case K_INT: case K_UINT: case K_FLOAT: case K_BOOL:
                it.type = IT_FIXED;
                it.size = (uint32_t)n.width;
                it.nullable = n.nullable;
                it.is_bool = n.kind == K_BOOL;
                s->items.push_back(it);
                if (n.nullable) s->has_nullable = true;
                add_check(n, cont_id);
                return;
            case K_STRING: case K_BYTES:
                if (n.width > 0) {
                    it.type = IT_FIXED;
                    it.size = (uint32_t)n.width;
                } else {
                    it.type = IT_VAR;
                    s->has_var = true;
                }
                s->items.push_back(it);
                add_check(n, cont_id);
                return;
            case K_MATCH:
                it.type = IT_CONST;
                it.col = -1;
                it.size = (uint32_t)n.literal.size();
                it.lit = (uint32_t)s->lits.size();
                s->lits.insert(s->lits.end(), n.literal.begin(), n.literal.end());
                s->items.push_back(it);
                return;
            case K_TUPLE: case K_MAP: {
                if ((int)s->conts.size() >= kMaxConts) fail(PACKOS_E_UNSUPPORTED, "too many nested containers");
                EncCont c{};
                c.parent = (int16_t)cont_id;
                bool can_nil = n.kind == K_MAP || n.nullable;
                c.valid_col = can_nil ? (int16_t)n.col : (int16_t)-1;
                if (can_nil) s->has_nullable = true;
                int cid = (int)s->conts.size();
                s->conts.push_back(c);
                if ((n.kind == K_TUPLE && n.names_bad) || (n.kind == K_MAP && (n.kids.size() & 1))) {
                    // TupleSchemaNamed.Encode of a present value fails before writing
                    // anything (schema.go:1808-1810), so does SchemaMap.Encode with an
                    // odd schema count (:422-429); a parent tuple / map wraps it as
                    // ErrInvalidFormat
                    EncCheck k{};
                    k.col = n.col;
                    k.cont = cid;
                    k.top = n.top;
                    k.flags = CHK_FAIL;
                    k.inner = cont_id == 0 ? PACKOS_ERR_CONSTRAINT_VIOLATED : PACKOS_ERR_INVALID_FORMAT;
                    s->echk.push_back(k);
                }
                emit_container(id, cid);
                return;
            }
        }
        fail(PACKOS_E_SCHEMA, "bad node");
    }

    // EncodeFunc value checks, in emission order (EncodeValue stops at the
    // first failing field): Range -> ErrOutOfRange (schema.go:1205-1212),
    // SDateRange -> ErrDateOutOfRange (:2231-2246), CheckFunc Prefix/Suffix ->
    // ErrEncode (:1110-1124)
    void add_check(const Node& n, int cont_id) {
        const uint32_t f = n.check & (CHK_RANGE | CHK_STR);
        if (!f) return;
        EncCheck c{};
        c.col = n.col;
        c.cont = cont_id;
        c.top = n.top;
        c.flags = n.check;
        c.width = n.width > 0 ? (uint32_t)n.width : 0u;
        c.rmin = n.rmin;
        c.rmax = n.rmax;
        if (f & CHK_STR) {
            c.lit = (uint32_t)s->lits.size();
            c.lit_len = (uint32_t)n.check_lit.size();
            s->lits.insert(s->lits.end(), n.check_lit.begin(), n.check_lit.end());
            c.inner = PACKOS_ERR_ENCODE;
        } else {
            c.inner = (n.check & CHK_DATE) ? PACKOS_ERR_DATE_OUT_OF_RANGE : PACKOS_ERR_OUT_OF_RANGE;
        }
        // a leaf inside a tuple / map: the container wraps its error as
        // ErrInvalidFormat (schema.go:1671-1673, 1859-1861, 444-449)
        if (cont_id != 0) c.inner = PACKOS_ERR_INVALID_FORMAT;
        s->echk.push_back(c);
    }

    void build_encode() {
        s->items.clear(); s->hdrs.clear(); s->conts.clear(); s->lits.clear(); s->echk.clear();
        EncCont root{};
        root.parent = -1;
        root.valid_col = -1;
        s->conts.push_back(root);
        if (s->mode == PACKOS_MODE_PACKABLE && s->nodes[0].kids.empty()) {
            // packable.Pack() with no args: empty slice (pack.go:59-67)
            s->conts[0].hdr_item = 0;
            return;
        }
        {
            // EncodeValueNamed walks FieldNames (schema.go:976): a SchemaNamedChain
            // with fewer names than schemas writes only the first len(FieldNames)
            std::vector<int> top = s->nodes[0].kids;
            if (s->chain_names > 0 && (size_t)s->chain_names < top.size()) s->nodes[0].kids.resize(s->chain_names);
            emit_container(0, 0);
            s->nodes[0].kids = top;
            if (s->chain_names > 0 && (size_t)s->chain_names > top.size()) {
                // ... and with more names it indexes chain.Schemas[len(Schemas)] once
                // every schema's field is written (:976-987): a Go panic for every
                // blob whose fields all encode (k_encode_checks, CHK_PANIC last)
                EncCheck k{};
                k.col = -1;
                k.cont = 0;
                k.top = -1;
                k.flags = CHK_PANIC;
                s->echk.push_back(k);
            }
        }
        if (s->items.size() > 65000) fail(PACKOS_E_UNSUPPORTED, "schema too large");
        // per-item kernel aux data: var slot, staging region, divide magic
        int nv = 0, nr = 0;
        s->ipk.clear();
        for (EncItem& it : s->items) {
            it.vslot = it.type == IT_VAR ? (uint8_t)std::min(nv++, 255) : 0;
            it.reg = it.type == IT_FIXED ? (uint8_t)std::min(nr++, 255) : 255;
            it.magic = it.size > 1 ? (uint32_t)(((1ull << 32) + it.size - 1) / it.size) : 0u;
            const uint32_t vs = it.type == IT_VAR ? it.vslot : 255u;
            s->ipk.push_back((std::min<uint32_t>(it.size, 0xFFFFu)) | (vs << 16));
        }
        // header entries of each header item: contiguous, j ascending (emit_container)
        s->ihr.assign(s->items.size(), 0u);
        for (size_t h = 0; h < s->hdrs.size(); h++) {
            const EncHdr& e = s->hdrs[h];
            uint32_t& r = s->ihr[e.hdr_item];
            if ((r >> 16) == 0) r = (uint32_t)h;
            if ((r & 0xFFFFu) + (r >> 16) != h || e.j != (r >> 16) || h > 0xFFFF)
                fail(PACKOS_E_UNSUPPORTED, "internal: header entries not contiguous");
            r += 1u << 16;
        }
    }

    // All-present blob layout for schemas without var leaves.
    void build_fixed() {
        s->fix_ok = false;
        s->all_present_size = -1;
        if (s->has_var) return;
        size_t ni = s->items.size();
        std::vector<int64_t> pos(ni + 1, 0);
        for (size_t i = 0; i < ni; i++) pos[i + 1] = pos[i] + s->items[i].size;
        int64_t B = pos[ni];
        s->all_present_size = B;
        // byte map: -1 const, else (col, off) packed
        struct BM { int col; int off; uint8_t val; bool is_bool; };
        std::vector<BM> bm((size_t)B, BM{-1, 0, 0, false});
        bool ovf = false;
        for (size_t i = 0; i < ni; i++) {
            const EncItem& it = s->items[i];
            if (it.type == IT_CONST)
                for (uint32_t k = 0; k < it.size; k++) bm[pos[i] + k].val = s->lits[it.lit + k];
            else if (it.type == IT_FIXED)
                for (uint32_t k = 0; k < it.size; k++) bm[pos[i] + k] = BM{it.col, (int)k, 0, it.is_bool != 0};
        }
        for (const EncHdr& h : s->hdrs) {
            const EncItem& hi = s->items[h.hdr_item];
            int64_t payload = pos[h.hdr_item] + hi.size;
            uint16_t v;
            if (h.relative) {
                int64_t off = pos[h.target] - payload;
                if (off >= 8192) ovf = true;
                v = enc_header(off, h.tag);
            } else {
                v = h.value;
                if (h.ovf) ovf = true;
            }
            int64_t at = pos[h.hdr_item] + 2 * h.j;
            bm[at].val = (uint8_t)(v & 0xFF);
            bm[at + 1].val = (uint8_t)(v >> 8);
        }
        s->all_present_overflow = ovf;
        if (B <= 0 || B > 1024) return;  // large fixed blobs use the general kernel
        // a SchemaNamedChain whose names and schemas differ: the tile tables
        // cover every column, the encode layout only the named fields (rare:
        // the general kernel takes it)
        if (s->chain_names) return;

        // tile size: T blobs (multiple of 16 so tile in/out are whole 16-B chunks)
        // ~16 KiB of output per tile (env PACKOS_TILE_BYTES overrides, tuning only)
        int64_t tile_bytes = 16384;
        if (const char* e = getenv("PACKOS_TILE_BYTES"))   // read once, at compile
            tile_bytes = std::min<int64_t>(16384, std::max<int64_t>(1024, atoll(e)));  // staging plan holds <= 16 KiB
        int T = (int)((tile_bytes / B) / 16 * 16);
        if (T < 16) T = 16;
        if (T > 1024) T = 1024;
        s->fix_T = T;
        // LDS regions per fixed column (16-B guards on both sides)
        s->fcols.clear();
        std::vector<int> lds_of_col(s->col_node.size(), -1);
        uint32_t lds = 16, chunks = 0;
        for (size_t c = 0; c < s->col_node.size(); c++) {
            const Node& n = s->nodes[s->col_node[c]];
            bool fixed_leaf = (n.kind >= K_INT && n.kind <= K_BOOL) ||
                              ((n.kind == K_STRING || n.kind == K_BYTES) && n.width > 0);
            if (!fixed_leaf) continue;
            FixCol fc{};
            fc.col = (int)c;
            fc.width = (uint32_t)n.width;
            fc.lds_off = lds;
            fc.chunk_begin = chunks;
            fc.flags = n.kind == K_BOOL ? 1u : 0u;
            lds_of_col[c] = (int)lds;
            uint32_t bytes = (uint32_t)T * fc.width;
            chunks += bytes / 16;
            lds += bytes;  // regions back to back in chunk order (T*w % 16 == 0): chunk k
                           // of a tile sits at 16 + 16k, the layout one LDS-DMA wave
                           // instruction (1 KiB, lane-linear) fills
            s->fcols.push_back(fc);
        }
        s->fix_lds = (int)lds + 32;  // tail guard (read-past of the last region, dummy slot)
        s->fix_chunks = (int)chunks;
        // decode fast path tables: per-dword constant check, per-column
        // blob offset, canonical blob (payload bytes zero)
        s->dchk.clear();
        s->canon.assign((size_t)B, 0);
        for (int64_t q = 0; q < (B + 3) / 4; q++) {
            uint32_t cm = 0, cv = 0;
            for (int b = 0; b < 4; b++)
                if (4 * q + b < B && bm[4 * q + b].col < 0) {
                    cm |= 0xFFu << (8 * b);
                    cv |= (uint32_t)bm[4 * q + b].val << (8 * b);
                    s->canon[4 * q + b] = bm[4 * q + b].val;
                }
            if (cm) {   // compact: only the dwords that hold constant bytes
                s->dchk.push_back((uint32_t)q);
                s->dchk.push_back(cm);
                s->dchk.push_back(cv);
            }
        }
        s->dfix.clear();
        for (const FixCol& fc : s->fcols) {
            DecFix df{};
            df.col = fc.col;
            df.width = fc.width;
            df.blob_off = UINT32_MAX;
            for (int64_t q = 0; q < B; q++)
                if (bm[q].col == fc.col && bm[q].off == 0) { df.blob_off = (uint32_t)q; break; }
            if (df.blob_off == UINT32_MAX) fail(PACKOS_E_SCHEMA, "internal: fixed column not in layout");
            df.flags = bm[df.blob_off].is_bool ? 1u : 0u;
            df.magic = fc.width > 1 ? (uint32_t)(((1ull << 32) + fc.width - 1) / fc.width) : 0u;
            s->dfix.push_back(df);
        }
        s->dvchk.clear();
        for (const EncCheck& c : s->echk) {
            if (c.flags & (CHK_FAIL | CHK_PANIC)) continue;   // no value to check (the decoder fails the blob itself)
            DecChk v{};
            for (const DecFix& df : s->dfix)
                if (df.col == c.col) v.blob_off = df.blob_off;
            v.width = (uint32_t)s->nodes[s->col_node[c.col]].width;
            v.flags = c.flags;
            v.lit = c.lit;
            v.lit_len = c.lit_len;
            v.rmin = c.rmin;
            v.rmax = c.rmax;
            s->dvchk.push_back(v);
        }
        if (s->fix_lds > 60 * 1024) return;
        // segments for each dword r of a 4-blob period
        s->fsegs.clear();
        s->fseg_index.assign((size_t)B + 1, 0);
        for (int64_t r = 0; r < B; r++) {
            s->fseg_index[r] = (uint32_t)s->fsegs.size();
            uint32_t cmask = 0, cval = 0;
            int b = 0;
            while (b < 4) {
                int64_t pb = 4 * r + b;
                int d = (int)(pb / B);
                int64_t q = pb % B;
                const BM& m = bm[q];
                if (m.col < 0) {
                    cmask |= 0xFFu << (8 * b);
                    cval |= (uint32_t)m.val << (8 * b);
                    b++;
                    continue;
                }
                // extend the run: same column, same blob, consecutive source bytes
                int b1 = b + 1;
                while (b1 < 4) {
                    int64_t pb1 = 4 * r + b1;
                    int d1 = (int)(pb1 / B);
                    const BM& m1 = bm[pb1 % B];
                    if (m1.col != m.col || d1 != d || m1.off != m.off + (b1 - b) || m.is_bool) break;
                    b1++;
                }
                FixSeg sg{};
                uint32_t w = (uint32_t)s->nodes[s->col_node[m.col]].width;
                sg.a = lds_of_col[m.col] + d * (int)w + m.off - b;
                sg.stride4 = 4 * w;
                uint32_t mask = 0;
                for (int x = b; x < b1; x++) mask |= 0xFFu << (8 * x);
                sg.mask = mask;
                sg.cval = m.is_bool ? 1u : 0u;
                s->fsegs.push_back(sg);
                b = b1;
            }
            if (cmask) {
                FixSeg sg{};
                sg.a = 0; sg.stride4 = 0; sg.mask = cmask; sg.cval = cval;
                s->fsegs.push_back(sg);
            }
        }
        s->fseg_index[B] = (uint32_t)s->fsegs.size();
        // lane-invariant per-dword descriptors (blob-relative; B % 4 == 0 means
        // no dword straddles two blobs)
        s->fdw.clear();
        s->fix_maxseg = 0;
        if (B % 4 == 0) {
            for (int64_t q = 0; q < B / 4; q++) {
                DwDesc dd{};
                int b = 0;
                while (b < 4) {
                    const BM& m = bm[4 * q + b];
                    if (m.col < 0) {
                        dd.cval |= (uint32_t)m.val << (8 * b);
                        b++;
                        continue;
                    }
                    int b1 = b + 1;
                    while (b1 < 4) {
                        const BM& m1 = bm[4 * q + b1];
                        if (m1.col != m.col || m1.off != m.off + (b1 - b) || m.is_bool) break;
                        b1++;
                    }
                    DwSeg sg{};
                    sg.a = lds_of_col[m.col] + m.off - b;
                    sg.w = (uint32_t)s->nodes[s->col_node[m.col]].width;
                    for (int x = b; x < b1; x++) sg.mask |= 0xFFu << (8 * x);
                    sg.flags = m.is_bool ? 1u : 0u;
                    dd.seg[dd.nseg++] = sg;
                    b = b1;
                }
                s->fdw.push_back(dd);
                s->fix_maxseg = std::max<int>(s->fix_maxseg, (int)dd.nseg);
            }
            // single-source form for k_encode_fixed_tile: X dwords (several
            // runs, or a bool byte to normalise) get a slot in the X region
            s->ftdw = s->fdw;
            s->fxdw.clear();
            s->fxq.clear();
            for (int64_t q = 0; q < B / 4; q++) {
                const DwDesc& d = s->fdw[q];
                bool x = d.nseg > 1;
                for (uint32_t g = 0; g < d.nseg; g++) x = x || (d.seg[g].flags & 1u);
                if (x) { s->fxq.push_back((uint32_t)q); s->fxdw.push_back(d); }
            }
            const uint32_t nx = (uint32_t)s->fxq.size();
            s->fix_x_lds = (s->fix_lds + 15) / 16 * 16;
            s->fix_tile_lds = s->fix_x_lds + (int)(T * nx * 4) + 16;
            for (uint32_t k = 0; k < nx; k++) {
                DwDesc& t = s->ftdw[s->fxq[k]];
                uint32_t cm = 0;
                for (uint32_t g = 0; g < t.nseg; g++) cm |= t.seg[g].mask;
                DwSeg sg{};
                sg.a = s->fix_x_lds + (int32_t)(4 * k);
                sg.w = 4 * nx;
                sg.mask = cm;
                sg.flags = 0;
                t.seg[0] = sg;
                for (int g = 1; g < 4; g++) t.seg[g] = DwSeg{};
                t.nseg = 1;
            }
            // a constant-only dword still issues the (masked) LDS read in the
            // branch-free kernels: point it at a source another lane of the
            // same 32-lane LDS group reads, so it broadcasts instead of
            // adding a bank conflict
            const int64_t Q4 = B / 4;
            for (int64_t q = 0; q < Q4; q++) {
                if (s->fdw[q].nseg) continue;
                int64_t best = -1;
                for (int64_t d = 1; d < Q4 && best < 0; d++)
                    for (int64_t c : {q + d, q - d})
                        if (c >= 0 && c < Q4 && c / 32 == q / 32 && s->fdw[c].nseg && best < 0) best = c;
                if (best >= 0) {
                    s->fdw[q].seg[0] = s->fdw[best].seg[0];
                    s->fdw[q].seg[0].mask = 0;
                    s->fdw[q].seg[0].flags = 0;
                    s->ftdw[q].seg[0] = s->ftdw[best].seg[0];
                    s->ftdw[q].seg[0].mask = 0;
                    s->ftdw[q].seg[0].flags = 0;
                }
            }
        }
        // tile + descriptor tables must fit the 64 KiB dynamic LDS of one launch
        size_t lds_total = (size_t)s->fix_lds + ((size_t)(B + 1) * 4 + 15) / 16 * 16 + s->fsegs.size() * sizeof(FixSeg);
        s->fix_ok = lds_total <= 64 * 1024;
    }

    // ---------------------------------------------------------- decode ----
    void build_decode() {
        s->dnodes.assign(s->nodes.size(), DecNode{});
        s->dkids.clear();
        for (size_t i = 0; i < s->nodes.size(); i++) {
            const Node& n = s->nodes[i];
            DecNode& d = s->dnodes[i];
            d.kind = n.kind;
            d.width = n.width;
            d.col = n.col;
            d.nkids = (int)n.kids.size();
            d.kid0 = (int)s->dkids.size();
            for (int k : n.kids) s->dkids.push_back(k);
            d.tag = (uint8_t)tag_of(n.kind);
            d.variable = (uint8_t)((n.variable ? DT_VARIABLE : 0) | (n.named ? DT_NAMED : 0) |
                                   (n.names_bad ? DT_NAMES_BAD : 0));
            switch (n.kind) {
                case K_STRING: case K_BYTES: case K_MATCH: d.nullable = n.width <= 0; break;
                case K_MAP: d.nullable = 1; break;
                default: d.nullable = n.nullable;
            }
            if (n.kind == K_MATCH) {
                d.lit = (uint32_t)s->lits.size();
                d.lit_len = (uint32_t)n.literal.size();
                s->lits.insert(s->lits.end(), n.literal.begin(), n.literal.end());
            } else if (n.check & CHK_STR) {
                d.lit = (uint32_t)s->lits.size();
                d.lit_len = (uint32_t)n.check_lit.size();
                s->lits.insert(s->lits.end(), n.check_lit.begin(), n.check_lit.end());
            }
            d.check = n.check;
            d.rmin = n.rmin;
            d.rmax = n.rmax;
            if (n.check & CHK_DEFAULT) {
                d.dlit = (uint32_t)s->lits.size();
                d.dlit_len = (uint32_t)n.dflt.size();
                s->lits.insert(s->lits.end(), n.dflt.begin(), n.dflt.end());
            }
        }
    }

    void build_info() {
        s->col_info.clear();
        for (size_t c = 0; c < s->col_node.size(); c++) {
            const Node& n = s->nodes[s->col_node[c]];
            packos_column_info ci{};
            switch (n.kind) {
                case K_INT: ci.kind = PACKOS_KIND_INT; break;
                case K_UINT: ci.kind = PACKOS_KIND_UINT; break;
                case K_FLOAT: ci.kind = PACKOS_KIND_FLOAT; break;
                case K_BOOL: ci.kind = PACKOS_KIND_BOOL; break;
                case K_STRING: ci.kind = PACKOS_KIND_STRING; break;
                case K_BYTES: ci.kind = PACKOS_KIND_BYTES; break;
                case K_TUPLE: ci.kind = PACKOS_KIND_TUPLE; break;
                case K_MAP: ci.kind = PACKOS_KIND_MAP; break;
            }
            bool scalar = n.kind >= K_INT && n.kind <= K_BOOL;
            ci.width = scalar ? n.width : ((n.kind == K_STRING || n.kind == K_BYTES) && n.width > 0 ? n.width : 0);
            ci.nullable = scalar ? n.nullable : (n.kind == K_MAP ? 1 : (n.kind == K_TUPLE ? n.nullable : 0));
            ci.tag = tag_of(n.kind);
            ci.top_index = n.top;
            ci.depth = n.depth - 1;
            snprintf(ci.name, sizeof(ci.name), "%s", n.name.c_str());
            s->col_info.push_back(ci);
        }
    }

    void build_describe() {
        std::ostringstream o;
        o << "mode=" << s->mode << " cols=" << s->col_node.size() << " items=" << s->items.size()
          << " hdrs=" << s->hdrs.size() << " conts=" << s->conts.size() << " var=" << s->has_var
          << " nullable=" << s->has_nullable << " B=" << s->all_present_size << " fix=" << s->fix_ok
          << " T=" << s->fix_T << " lds=" << s->fix_lds << " segs=" << s->fsegs.size() << "\n";
        const char* tn[] = {"HDR", "FIXED", "VAR", "CONST"};
        for (size_t i = 0; i < s->items.size(); i++) {
            const EncItem& it = s->items[i];
            o << "item " << i << " " << tn[it.type] << " cont=" << it.cont << " col=" << it.col
              << " size=" << it.size << (it.nullable ? " nullable" : "") << (it.is_bool ? " bool" : "") << "\n";
        }
        for (const EncCheck& c : s->echk)
            o << "check col=" << c.col << " cont=" << c.cont << " top=" << c.top << " flags=" << c.flags
              << " min=" << c.rmin << " max=" << c.rmax << " lit_len=" << c.lit_len << " inner=" << c.inner << "\n";
        for (const EncHdr& h : s->hdrs)
            o << "hdr cont=" << h.cont << " j=" << h.j << " tag=" << (int)h.tag
              << (h.relative ? " rel target=" : " const=") << (h.relative ? h.target : h.value) << "\n";
        s->describe = o.str();
    }
};

}  // namespace

namespace packos {
void set_error(const std::string& m) { g_err = m; }

void read_tune(Tune& t) {
    if (const char* e = getenv("PACKOS_VAR_PER")) {
        t.var_per = std::max(0, std::min(256, atoi(e)));
        t.var_per_set = true;
    }
    t.sizes_scan = getenv("PACKOS_SIZES_SCAN") != nullptr;
    t.decode_generic = getenv("PACKOS_DECODE_GENERIC") != nullptr;
    if (const char* e = getenv("PACKOS_DEC_TILE_BYTES")) t.dec_tile_bytes = std::min(49152, std::max(1024, atoi(e)));
    if (const char* e = getenv("PACKOS_ENC_FLAT")) t.enc_flat = atoi(e);
}

// Same rule as the device's ext_layout_wave (kernels.hip): containers in
// reverse pre-order (children before their parent), payload = the sizes of
// the items between its header item and its end item, so a nested container
// already written extended counts with its grown header block.
uint64_t ext_layout_host(const packos_schema* s, std::vector<int64_t>& sz) {
    uint64_t xm = 0;
    for (int c = (int)s->conts.size() - 1; c >= 0; c--) {
        const EncCont& ct = s->conts[c];
        if (ct.n_kids == 0 || ct.hdr_item >= sz.size()) continue;
        int64_t pay = 0;
        for (uint32_t k = ct.hdr_item + 1u; k < ct.end_item; k++) pay += sz[k];
        if (pay > (int64_t)kExtMaxPayload) {
            sz[ct.hdr_item] = ext_hdr_bytes(ct.n_kids);
            if (c < 64) xm |= 1ull << c;
        }
    }
    return xm;
}

int64_t ext_overhead(const packos_schema* s) {
    int64_t x = 0;
    for (const EncCont& ct : s->conts)
        if (ct.n_kids) x += (int64_t)ext_hdr_bytes(ct.n_kids) - 2 * ((int64_t)ct.n_kids + 1);
    return x;
}
}  // namespace packos

extern "C" {

const char* packos_last_error(void) { return g_err.c_str(); }
int packos_abi_version(void) { return PACKOS_ABI_VERSION; }

const char* packos_strerror(int code) {
    switch (code) {
        case PACKOS_OK: return "ok";
        case PACKOS_E_INVALID: return "invalid argument";
        case PACKOS_E_SCHEMA: return "schema rejected";
        case PACKOS_E_UNSUPPORTED: return "schema feature outside the compiled subset";
        case PACKOS_E_ALIGN: return "fixed-width column or output not 16-byte aligned";
        case PACKOS_E_WORKSPACE: return "workspace too small";
        case PACKOS_E_CAPACITY: return "output arena too small";
        case PACKOS_E_HIP: return "HIP runtime error";
        case PACKOS_E_NODEVICE: return "no GPU visible";
    }
    return "unknown error";
}

int packos_schema_compile(const char* schema_json, int mode, packos_schema** out) {
    const int base_mode = mode & ~PACKOS_MODE_EXTENDED;
    if (!schema_json || !out || (base_mode != PACKOS_MODE_PUTACCESS && base_mode != PACKOS_MODE_PACKABLE)) {
        g_err = "packos_schema_compile: bad argument";
        return PACKOS_E_INVALID;
    }
    *out = nullptr;
    auto* s = new packos_schema();
    s->mode = base_mode;
    s->ext = (mode & PACKOS_MODE_EXTENDED) != 0;
    try {
        std::string txt(schema_json);
        JVal j = JParser(txt).parse();
        Builder b{s};
        int root = b.new_node();
        s->nodes[root].kind = K_ROOT;
        const JVal* list = nullptr;
        const JVal* names = nullptr;
        JVal single;
        if (j.kind == JVal::ARR) {
            list = &j;
        } else if (j.kind == JVal::OBJ && Builder::str_field(j, "type") == "chain") {
            list = j.get("schema");
            names = j.get("fieldNames");
            if (!list || list->kind != JVal::ARR) fail(PACKOS_E_SCHEMA, "chain needs a schema array");
            // SchemaNamedChain whose FieldNames and Schemas differ in length:
            // DecodeBufferNamed fails every blob, EncodeValueNamed writes only
            // len(FieldNames) fields or indexes past Schemas (schema.go:953-956,
            // 975-994): build_encode, k_encode_checks (CHK_PANIC) and
            // packos_decode_batch (k_decode_chain_names) follow chain_names
            if (names && names->kind == JVal::ARR && !names->arr.empty() && names->arr.size() != list->arr.size())
                s->chain_names = (int)names->arr.size();
        } else if (j.kind == JVal::OBJ) {
            single.kind = JVal::ARR;
            single.arr.push_back(j);
            list = &single;
        } else {
            fail(PACKOS_E_SCHEMA, "top level must be an array or an object");
        }
        for (size_t t = 0; t < list->arr.size(); t++) {
            std::string nm;
            if (names && names->kind == JVal::ARR && t < names->arr.size() && names->arr[t].kind == JVal::STR)
                nm = names->arr[t].str;
            int id = b.node(list->arr[t], root, 1, (int)t, nm);
            s->nodes[root].kids.push_back(id);
        }
        s->n_top = (int)list->arr.size();
        b.assign_columns(root);
        if ((int)s->col_node.size() > kMaxCols) fail(PACKOS_E_UNSUPPORTED, "more than 64 columns");
        read_tune(s->tune);
        b.build_encode();
        {   // static prefix read by the decoder's per-blob window
            int64_t pre = 0;
            bool var = false, tail = false;
            for (const EncItem& it : s->items) {
                if (it.type == IT_VAR) var = true;
                else if (var) tail = true;
                if (!var) pre += it.size;
            }
            s->dec_prefix = pre;
            s->dec_tail_fixed = tail;
            // ValidateBuffer reads header words, literals (Match) and the
            // payloads of Range / date / prefix / suffix leaves only: the bytes
            // up to the last of those before the first var item, when none
            // follows it (else the whole window, as decode)
            int64_t p = 0, need = 0;
            bool v = false, after = false;
            for (const EncItem& it : s->items) {
                bool reads = it.type == IT_HDR || it.type == IT_CONST;
                if ((it.type == IT_FIXED || it.type == IT_VAR) && it.col >= 0) {
                    const Node& nd = s->nodes[s->col_node[it.col]];
                    reads = (nd.check & (CHK_RANGE | CHK_DATE | CHK_STR)) != 0;
                }
                if (it.type == IT_VAR) v = true;
                if (reads && v) after = true;
                if (!v) {
                    p += it.size;
                    if (reads) need = p;
                }
            }
            s->val_win = after || s->ext ? 0 : need;
        }
        b.build_fixed();
        b.build_decode();
        // (the fixed-layout decoder follows the ENCODE layout, which a
        // SchemaNamedChain with fewer names than schemas cuts short)
        s->dec_fast = !s->chain_names && canonical_decodes(s) ? 1 : 0;
        b.build_info();
        b.build_describe();
    } catch (const CompileError& e) {
        g_err = e.msg;
        delete s;
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        delete s;
        return PACKOS_E_SCHEMA;
    }
    *out = s;
    return PACKOS_OK;
}

int packos_schema_num_columns(const packos_schema* s) { return s ? (int)s->col_node.size() : -1; }
int packos_schema_num_top_fields(const packos_schema* s) { return s ? s->n_top : -1; }

int packos_schema_column_info(const packos_schema* s, int col, packos_column_info* out) {
    if (!s || !out || col < 0 || col >= (int)s->col_info.size()) return PACKOS_E_INVALID;
    *out = s->col_info[col];
    return PACKOS_OK;
}

int packos_schema_decode_fast(const packos_schema* s) { return s && s->dec_fast == 1 ? 1 : 0; }
int packos_schema_has_checks(const packos_schema* s) { return s && !s->echk.empty() ? 1 : 0; }

int64_t packos_schema_fixed_blob_size(const packos_schema* s) {
    if (!s || s->has_var) return -1;
    if (s->ext && s->all_present_size > (int64_t)kExtMaxPayload) return -1;   // may hold extended containers
    return s->all_present_size;
}

int64_t packos_schema_ext_overhead(const packos_schema* s) {
    if (!s) return -1;
    return s->ext ? packos::ext_overhead(s) : 0;
}

int64_t packos_schema_column_default(const packos_schema* s, int col, char* buf, size_t cap) {
    if (!s || col < 0 || col >= (int)s->col_node.size()) return -1;
    const Node& n = s->nodes[s->col_node[col]];
    if (!(n.check & CHK_DEFAULT)) return 0;
    if (buf && cap) memcpy(buf, n.dflt.data(), std::min(cap, n.dflt.size()));
    return (int64_t)n.dflt.size();
}

size_t packos_schema_describe(const packos_schema* s, char* buf, size_t cap) {
    if (!s) return 0;
    size_t need = s->describe.size() + 1;
    if (buf && cap) {
        size_t n = std::min(cap - 1, s->describe.size());
        memcpy(buf, s->describe.data(), n);
        buf[n] = 0;
    }
    return need;
}

int64_t packos_schema_blob_size_host(const packos_schema* s, const uint32_t* widths, const uint8_t* valid) {
    if (!s) return -1;
    size_t nc = s->conts.size();
    std::vector<char> present(nc, 0);
    for (size_t c = 0; c < nc; c++) {
        const EncCont& ct = s->conts[c];
        bool p = ct.parent < 0 ? true : present[ct.parent] != 0;
        if (p && ct.valid_col >= 0 && valid) p = valid[ct.valid_col] != 0;
        present[c] = p;
    }
    int64_t tot = 0, slack = 0;
    std::vector<int64_t> sz(s->items.size(), 0);
    for (size_t k = 0; k < s->items.size(); k++) {
        const EncItem& it = s->items[k];
        if (!present[it.cont]) continue;
        switch (it.type) {
            case IT_HDR: case IT_CONST: sz[k] = it.size; break;
            case IT_FIXED:
                if (it.nullable && valid && !valid[it.col]) slack += it.size;
                else sz[k] = it.size;
                break;
            case IT_VAR: sz[k] = widths ? widths[it.col] : 0; break;
        }
    }
    if (s->ext) packos::ext_layout_host(s, sz);
    for (int64_t z : sz) tot += z;
    if (s->mode == PACKOS_MODE_PACKABLE) tot += slack;
    return tot;
}

void packos_schema_free(packos_schema* s);  // defined with the device tables (kernels.hip)

}  // extern "C"
