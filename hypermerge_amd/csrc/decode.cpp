// decode.cpp — the host front of the merge path, native and multi-threaded: hypercore blocks
// -> Change objects -> the columnar rows of include/hypermerge_amd.h.
//
//   Block.unpack   (src/Block.ts:18-29)   '{"' raw JSON | 'BR' + brotli(JSON), else a throw
//   JsonBuffer.parse (src/JsonBuffer.ts:1-4) JSON.parse(buffer.toString())
//   Actor.parseBlock (src/Actor.ts:137-141) one Change per block, no validation
//   then the host encoder (hypermerge_amd/js/columnar.js DocEncoder, the Node drop-in's)
//   row for row: actor ranks in JS string (UTF-16) order, object / register ids in order of
//   first appearance, per-document content ids (Immutable `equals` classes: maps compared
//   order-insensitively, numbers by value), one string pool over the batch in document order.
//
// Documents decode in parallel (one thread per document range); the string pool is merged
// afterwards in document order, so the rows are identical whatever the thread count.
// Brotli blocks use the system libbrotlidec (loaded on first use); without it a 'BR' block is
// an undecodable block.  An undecodable block (the reference's Block.unpack / JSON.parse
// throw) marks its document HM_ERR_INVALID with no rows; other documents are unaffected.
#include <dlfcn.h>
#include <algorithm>
#include <cctype>
#include <emmintrin.h>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <chrono>
#include <cstdio>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>
#include "../../include/hypermerge_amd.h"

namespace {

// ---------------- brotli (system libbrotlidec, streaming API) ----------------
struct Brotli {
    void *(*create)(void *, void *, void *) = nullptr;
    int (*stream)(void *, size_t *, const uint8_t **, size_t *, uint8_t **, size_t *) = nullptr;
    void (*destroy)(void *) = nullptr;
    bool ok = false;
};
Brotli &brotli() {
    static Brotli B;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("libbrotlidec.so.1", RTLD_NOW);
        if (!h) return;
        *(void **)&B.create = dlsym(h, "BrotliDecoderCreateInstance");
        *(void **)&B.stream = dlsym(h, "BrotliDecoderDecompressStream");
        *(void **)&B.destroy = dlsym(h, "BrotliDecoderDestroyInstance");
        B.ok = B.create && B.stream && B.destroy;
    });
    return B;
}
bool brotli_decompress(const uint8_t *in, size_t n, std::string &out) {
    Brotli &B = brotli();
    if (!B.ok) return false;
    void *st = B.create(nullptr, nullptr, nullptr);
    if (!st) return false;
    out.clear();
    size_t avail_in = n;
    const uint8_t *next_in = in;
    int r;
    do {
        uint8_t buf[1 << 14];
        size_t avail_out = sizeof buf;
        uint8_t *next_out = buf;
        r = B.stream(st, &avail_in, &next_in, &avail_out, &next_out, nullptr);
        out.append((const char *)buf, sizeof buf - avail_out);
    } while (r == 3);                                      // NEEDS_MORE_OUTPUT
    B.destroy(st);
    return r == 1;                                         // SUCCESS
}

// ---------------- JSON (JSON.parse) ----------------
enum JT : uint8_t { J_NULL, J_FALSE, J_TRUE, J_NUM, J_STR, J_ARR, J_OBJ };
struct JV {
    JT t = J_NULL;
    double num = 0;
    std::string str;                                       // J_STR: UTF-8 text
    std::vector<JV> items;                                 // J_ARR
    std::vector<std::pair<std::string, JV>> fields;        // J_OBJ, in text order (last duplicate wins below)
    const JV *get(const char *k) const {
        const JV *r = nullptr;
        for (auto &f : fields) if (f.first == k) r = &f.second;    // JSON.parse: the last duplicate key wins
        return r;
    }
};

struct Parser {
    const char *p, *e;
    bool ok = true;
    void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
    bool lit(const char *s) {
        size_t n = strlen(s);
        if ((size_t)(e - p) < n || memcmp(p, s, n)) return false;
        p += n;
        return true;
    }
    static void utf8(std::string &o, uint32_t c) {
        if (c < 0x80) o += (char)c;
        else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 0x3F)); }
        else if (c < 0x10000) { o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F)); }
        else { o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 0x3F)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F)); }
    }
    int hex4(uint32_t &v) {
        if (e - p < 4) return 0;
        v = 0;
        for (int i = 0; i < 4; i++) {
            const char c = p[i];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else return 0;
        }
        p += 4;
        return 1;
    }
    bool string(std::string &o) {
        if (p >= e || *p != '"') return false;
        p++;
        o.clear();
        while (p < e && *p != '"') {
            const unsigned char c = (unsigned char)*p;
            if (c < 0x20) return false;
            if (c != '\\') { o += (char)c; p++; continue; }
            if (++p >= e) return false;
            const char x = *p++;
            switch (x) {
            case '"': o += '"'; break; case '\\': o += '\\'; break; case '/': o += '/'; break;
            case 'b': o += '\b'; break; case 'f': o += '\f'; break; case 'n': o += '\n'; break;
            case 'r': o += '\r'; break; case 't': o += '\t'; break;
            case 'u': {
                uint32_t v;
                if (!hex4(v)) return false;
                if (v >= 0xD800 && v < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                    const char *save = p;
                    p += 2;
                    uint32_t lo;
                    if (hex4(lo) && lo >= 0xDC00 && lo < 0xE000) v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
                    else p = save;
                }
                utf8(o, v);                                // (a lone surrogate keeps its code unit's UTF-8 form)
                break;
            }
            default: return false;
            }
        }
        if (p >= e) return false;
        p++;
        return true;
    }
    bool value(JV &v, int depth) {
        if (depth > 256) return false;
        ws();
        if (p >= e) return false;
        const char c = *p;
        if (c == '{') {
            p++;
            v.t = J_OBJ;
            ws();
            if (p < e && *p == '}') { p++; return true; }
            for (;;) {
                ws();
                std::string k;
                if (!string(k)) return false;
                ws();
                if (p >= e || *p != ':') return false;
                p++;
                v.fields.emplace_back(std::move(k), JV());
                if (!value(v.fields.back().second, depth + 1)) return false;
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == '}') { p++; return true; }
                return false;
            }
        }
        if (c == '[') {
            p++;
            v.t = J_ARR;
            ws();
            if (p < e && *p == ']') { p++; return true; }
            for (;;) {
                v.items.emplace_back();
                if (!value(v.items.back(), depth + 1)) return false;
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == ']') { p++; return true; }
                return false;
            }
        }
        if (c == '"') { v.t = J_STR; return string(v.str); }
        if (lit("null")) { v.t = J_NULL; return true; }
        if (lit("true")) { v.t = J_TRUE; return true; }
        if (lit("false")) { v.t = J_FALSE; return true; }
        // number (JSON grammar), converted as JS does (IEEE double, round to nearest)
        const char *s = p;
        if (p < e && *p == '-') p++;
        if (p >= e || !(*p >= '0' && *p <= '9')) return false;
        if (*p == '0') p++; else while (p < e && *p >= '0' && *p <= '9') p++;
        if (p < e && *p == '.') { p++; if (p >= e || !(*p >= '0' && *p <= '9')) return false; while (p < e && *p >= '0' && *p <= '9') p++; }
        if (p < e && (*p == 'e' || *p == 'E')) {
            p++;
            if (p < e && (*p == '+' || *p == '-')) p++;
            if (p >= e || !(*p >= '0' && *p <= '9')) return false;
            while (p < e && *p >= '0' && *p <= '9') p++;
        }
        v.t = J_NUM;
        char nb[64];
        const size_t nl = (size_t)(p - s);
        if (nl < sizeof nb) { memcpy(nb, s, nl); nb[nl] = 0; v.num = strtod(nb, nullptr); }
        else v.num = strtod(std::string(s, p).c_str(), nullptr);
        return true;
    }
};

bool parse_json(const char *s, size_t n, JV &out) {
    Parser P{s, s + n};
    if (!P.value(out, 0)) return false;
    P.ws();
    return P.p == P.e;
}

// ---------------- content identity (Immutable.fromJS(a).equals(b)) ----------------
void canon(const JV &v, std::string &o) {
    switch (v.t) {
    case J_NULL: o += "null"; break;
    case J_FALSE: o += "false"; break;
    case J_TRUE: o += "true"; break;
    case J_NUM: {
        char b[40];
        if (v.num == 0) snprintf(b, sizeof b, "0");                       // 0 and -0 are one value
        else snprintf(b, sizeof b, "%.17g", v.num);
        o += b;
        break;
    }
    case J_STR: o += '"'; for (char c : v.str) { if (c == '"' || c == '\\') o += '\\'; o += c; } o += '"'; break;
    case J_ARR: o += '['; for (size_t i = 0; i < v.items.size(); i++) { if (i) o += ','; canon(v.items[i], o); } o += ']'; break;
    case J_OBJ: {
        // keys sorted, the last duplicate of a key wins (JSON.parse)
        std::vector<std::pair<const std::string *, const JV *>> f;
        for (auto &x : v.fields) {
            bool dup = false;
            for (auto &y : f) if (*y.first == x.first) { y.second = &x.second; dup = true; }
            if (!dup) f.emplace_back(&x.first, &x.second);
        }
        std::sort(f.begin(), f.end(), [](const auto &a, const auto &b) { return *a.first < *b.first; });
        o += '{';
        for (size_t i = 0; i < f.size(); i++) {
            if (i) o += ',';
            o += '"'; o += *f[i].first; o += "\":";
            canon(*f[i].second, o);
        }
        o += '}';
        break;
    }
    }
}

// JS string order (UTF-16 code units) of two UTF-8 strings
std::u16string u16(const std::string &s) {
    std::u16string o;
    for (size_t i = 0; i < s.size();) {
        const unsigned char c = (unsigned char)s[i];
        uint32_t cp, n;
        if (c < 0x80) { cp = c; n = 1; }
        else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
        else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
        else { cp = c & 0x07; n = 4; }
        for (uint32_t k = 1; k < n && i + k < s.size(); k++) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
        i += n;
        if (cp >= 0x10000) { cp -= 0x10000; o += (char16_t)(0xD800 + (cp >> 10)); o += (char16_t)(0xDC00 + (cp & 0x3FF)); }
        else o += (char16_t)cp;
    }
    return o;
}

const char *ROOT_ID = "00000000-0000-0000-0000-000000000000";

int action_of(const std::string &a) {
    static const char *names[] = {"makeMap", "makeTable", "makeList", "makeText", "ins", "set", "del", "link", "inc"};
    for (int i = 0; i < 9; i++) if (a == names[i]) return i;
    return -1;
}

// JS Number.isInteger(v) && |v| < 2^53
bool js_int(double v) { return std::isfinite(v) && std::floor(v) == v && std::fabs(v) < 9007199254740992.0; }
// `${n}` of an integral JS number (the element counter of an elemId)
std::string js_num_text(double v) {
    char b[40];
    if (js_int(v)) snprintf(b, sizeof b, "%lld", (long long)v);
    else snprintf(b, sizeof b, "%.17g", v);
    return b;
}

// One document's rows, with string ids local to the document (remapped at the merge).
struct DocOut {
    int32_t status = HM_OK;
    std::vector<hm_change_row> ch;
    std::vector<hm_dep_row> dp;
    std::vector<hm_op_row> op;
    std::vector<uint8_t> op_str_key, op_str_val;            // per op: key / value is a local string id
    std::vector<std::string> strings;                        // local string ids -> text
    std::vector<std::string> actors;                         // rank -> actor id
    std::vector<std::string> objs;                           // object id -> uuid
    std::vector<std::pair<uint32_t, std::string>> regs;      // register -> (object, key | elemId)
    uint32_t n_regs = 0, n_objs = 1;
    uint16_t flags = 0;
};

// ---------------- the fast path: a streaming scan of one Change ----------------
// The reference parses each block with JSON.parse into objects; here one scan per block
// extracts exactly the fields the rows need (unescaped strings stay views into the block,
// escaped ones are decoded into an arena), and skips every other field without building
// it.  Names are interned as they are scanned (open-addressed tables reused across the
// documents a thread decodes, no per-change allocation).  The full JSON DOM above is built
// only for changes whose (actor, seq) repeats in the document, where content identity
// (Immutable `equals`) must be decided.
struct SV { const char *p = nullptr; uint32_t n = 0; bool operator==(const SV &o) const { return n == o.n && !memcmp(p, o.p, n); } };

inline uint64_t hash_bytes(const char *p, uint32_t n, uint64_t seed) {
    uint64_t h = seed ^ (0x9E3779B97F4A7C15ull * (n + 1));
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        h = (h ^ w) * 0xff51afd7ed558ccdull;
        h ^= h >> 32;
        p += 8; n -= 8;
    }
    uint64_t w = 0;
    memcpy(&w, p, n);
    h = (h ^ w) * 0xc4ceb9fe1a85ec53ull;
    return h ^ (h >> 29);
}

// (tag, name) -> dense id in first-insertion order; tag is 0 for plain names, the object
// id for register keys
struct Intern {
    struct K { SV s; uint32_t tag; uint64_t h; };
    std::vector<uint32_t> slot;                              // id + 1, 0 = empty
    std::vector<K> keys;
    uint32_t mask = 0;
    void reset(size_t expect) {
        size_t c = 64;
        while (c < expect * 2) c <<= 1;
        if (slot.size() != c) slot.assign(c, 0); else std::fill(slot.begin(), slot.end(), 0u);
        mask = (uint32_t)c - 1;
        keys.clear();
    }
    void grow() {
        slot.assign(slot.size() * 2, 0);
        mask = (uint32_t)slot.size() - 1;
        for (uint32_t id = 0; id < keys.size(); id++) {
            uint32_t i = (uint32_t)keys[id].h & mask;
            while (slot[i]) i = (i + 1) & mask;
            slot[i] = id + 1;
        }
    }
    uint32_t get(const SV &s, uint32_t tag, bool &fresh) {
        const uint64_t h = hash_bytes(s.p, s.n, tag);
        for (uint32_t i = (uint32_t)h & mask;; i = (i + 1) & mask) {
            const uint32_t v = slot[i];
            if (!v) {
                if ((keys.size() + 1) * 2 > slot.size()) { grow(); return get(s, tag, fresh); }
                slot[i] = (uint32_t)keys.size() + 1;
                keys.push_back({s, tag, h});
                fresh = true;
                return (uint32_t)keys.size() - 1;
            }
            const K &k = keys[v - 1];
            if (k.h == h && k.tag == tag && k.s == s) { fresh = false; return v - 1; }
        }
    }
};

struct ScanOp { int8_t action = -1; uint8_t datatype = 0; JT vt = J_NULL; bool has_value = false; SV obj, key, sval; double num = 0, elem = 0; bool has_key = false, has_elem = false; };
struct ScanChange { uint32_t actor = UINT32_MAX; double seq = 0; bool has_seq = false; uint32_t dep0 = 0, ndeps = 0, op0 = 0, nops = 0; const char *text; uint32_t len; };
struct ScanDep { uint32_t actor; double seq; };

// per-thread scratch, reused across documents
struct Ctx {
    std::deque<std::string> arena;                            // decoded blocks and escaped strings
    std::vector<ScanChange> cs;
    std::vector<ScanOp> ops;
    std::vector<ScanDep> deps;
    Intern actors, objs, strs, regs;
    std::vector<uint64_t> key_slot;                          // (rank, seq) + 1 -> first change, open-addressed
    std::vector<uint32_t> key_first;
    std::vector<uint64_t> ckey;
    std::vector<std::string> canon_of;
    std::vector<uint32_t> cid, rank;
    std::string el;
};

struct Scan {
    const char *p, *e;
    Ctx *cx;
    void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
    // advance p to the first '"', '\\' or control byte (16 bytes at a time)
    void run() {
        const __m128i q = _mm_set1_epi8('"'), b = _mm_set1_epi8('\\'), lo = _mm_set1_epi8((char)(0x20 ^ 0x80)),
                      f = _mm_set1_epi8((char)0x80);
        while (e - p >= 16) {
            const __m128i v = _mm_loadu_si128((const __m128i *)p);
            const __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, q), _mm_cmpeq_epi8(v, b)),
                                           _mm_cmplt_epi8(_mm_xor_si128(v, f), lo));
            const int bits = _mm_movemask_epi8(m);
            if (bits) { p += __builtin_ctz(bits); return; }
            p += 16;
        }
        while (p < e && *p != '"' && *p != '\\' && (unsigned char)*p >= 0x20) p++;
    }
    bool str(SV &out) {
        if (p >= e || *p != '"') return false;
        const char *s = ++p;
        run();
        if (p < e && (unsigned char)*p < 0x20) return false;
        if (p < e && *p == '"') { out.p = s; out.n = (uint32_t)(p - s); p++; return true; }
        // escapes: decode through the DOM parser's string routine into the arena
        Parser P{s - 1, e};
        cx->arena.emplace_back();
        if (!P.string(cx->arena.back())) return false;
        p = P.p;
        out.p = cx->arena.back().data(); out.n = (uint32_t)cx->arena.back().size();
        return true;
    }
    bool skip_str() {                                        // a JSON string, validated, not decoded
        if (p >= e || *p != '"') return false;
        p++;
        for (;;) {
            run();
            if (p >= e || *p == '"') break;
            const unsigned char c = (unsigned char)*p;
            if (c < 0x20) return false;
            if (c == '\\') {
                if (++p >= e) return false;
                const char x = *p;
                if (x == 'u') {
                    if (e - p < 5) return false;
                    for (int i = 1; i <= 4; i++) if (!isxdigit((unsigned char)p[i])) return false;
                    p += 4;
                } else if (!strchr("\"\\/bfnrt", x) || !x) return false;
            }
            p++;
        }
        if (p >= e) return false;
        p++;
        return true;
    }
    bool num(double &v) {
        // plain integers (the common case) directly; anything else through strtod
        const char *s = p;
        bool neg = false;
        if (p < e && *p == '-') { neg = true; p++; }
        if (p >= e || !(*p >= '0' && *p <= '9')) return false;
        uint64_t x = 0;
        int nd = 0;
        if (*p == '0') { p++; nd = 1; }
        else while (p < e && *p >= '0' && *p <= '9' && nd < 18) { x = x * 10 + (uint64_t)(*p - '0'); p++; nd++; }
        if (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E')) {
            p = s;
            Parser P{p, e};
            JV j;
            if (!P.value(j, 0) || j.t != J_NUM) return false;
            p = P.p; v = j.num;
            return true;
        }
        v = neg ? -(double)x : (double)x;
        return true;
    }
    bool skip(int depth = 0) {                               // any JSON value, validated, not built
        if (depth > 256) return false;
        ws();
        if (p >= e) return false;
        const char c = *p;
        if (c == '"') return skip_str();
        if (c == '{' || c == '[') {
            const char close = c == '{' ? '}' : ']';
            p++;
            ws();
            if (p < e && *p == close) { p++; return true; }
            for (;;) {
                ws();
                if (c == '{') {
                    if (!skip_str()) return false;
                    ws();
                    if (p >= e || *p != ':') return false;
                    p++;
                }
                if (!skip(depth + 1)) return false;
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == close) { p++; return true; }
                return false;
            }
        }
        if (c == 't') { if (e - p < 4 || memcmp(p, "true", 4)) return false; p += 4; return true; }
        if (c == 'f') { if (e - p < 5 || memcmp(p, "false", 5)) return false; p += 5; return true; }
        if (c == 'n') { if (e - p < 4 || memcmp(p, "null", 4)) return false; p += 4; return true; }
        double v;
        return num(v);
    }
    static bool is(const SV &k, const char *lit) { const size_t n = strlen(lit); return k.n == n && !memcmp(k.p, lit, n); }
    // value of an op field into the scan op (anything a field can hold)
    bool anyval(ScanOp &o) {
        ws();
        if (p >= e) return false;
        o.has_value = true;
        if (*p == '"') { o.vt = J_STR; return str(o.sval); }
        if (*p == 't') { if (e - p < 4 || memcmp(p, "true", 4)) return false; p += 4; o.vt = J_TRUE; return true; }
        if (*p == 'f') { if (e - p < 5 || memcmp(p, "false", 5)) return false; p += 5; o.vt = J_FALSE; return true; }
        if (*p == 'n') { if (e - p < 4 || memcmp(p, "null", 4)) return false; p += 4; o.vt = J_NULL; return true; }
        if (*p == '-' || (*p >= '0' && *p <= '9')) { o.vt = J_NUM; return num(o.num); }
        o.vt = J_OBJ;                                        // an object / array value: 'unsupported op value'
        return skip();
    }
    template <typename F> bool object(F &&field) {            // {"k": v, ...}; field(k) parses v
        ws();
        if (p >= e || *p != '{') return false;
        p++;
        ws();
        if (p < e && *p == '}') { p++; return true; }
        for (;;) {
            ws();
            SV k;
            if (!str(k)) return false;
            ws();
            if (p >= e || *p != ':') return false;
            p++;
            ws();
            if (!field(k)) return false;
            ws();
            if (p < e && *p == ',') { p++; continue; }
            if (p < e && *p == '}') { p++; return true; }
            return false;
        }
    }
    uint32_t actor_id(const SV &a) { bool f; return cx->actors.get(a, 0, f); }
    bool change(ScanChange &c) {
        auto &ops = cx->ops;
        auto &deps = cx->deps;
        c.op0 = (uint32_t)ops.size();
        c.dep0 = (uint32_t)deps.size();
        SV actor;
        bool ok = object([&](const SV &k) {
            if (is(k, "actor")) return ws(), str(actor);
            if (is(k, "seq")) { c.has_seq = true; return num(c.seq); }
            if (is(k, "deps")) {
                deps.resize(c.dep0);
                if (p < e && *p != '{') return skip();
                return object([&](const SV &a) {
                    double v = 0;
                    if (p < e && (*p == '-' || (*p >= '0' && *p <= '9'))) { if (!num(v)) return false; }
                    else if (!skip()) return false;
                    const uint32_t id = actor_id(a);
                    for (size_t i = c.dep0; i < deps.size(); i++)
                        if (deps[i].actor == id) { deps[i].seq = v; return true; }   // first position, last value
                    deps.push_back({id, v});
                    return true;
                });
            }
            if (is(k, "ops")) {
                ops.resize(c.op0);
                if (p >= e || *p != '[') return skip();
                p++;
                ws();
                if (p < e && *p == ']') { p++; return true; }
                for (;;) {
                    ScanOp o;
                    bool r = object([&](const SV &f) {
                        if (is(f, "action")) {
                            SV a;
                            if (p < e && *p != '"') { o.action = -1; return skip(); }
                            if (!str(a)) return false;
                            o.action = (int8_t)action_of(std::string(a.p, a.n));
                            return true;
                        }
                        if (is(f, "obj")) { if (p < e && *p == '"') return str(o.obj); o.obj = SV(); return skip(); }
                        if (is(f, "key")) { o.has_key = p < e && *p == '"'; if (!o.has_key) o.key = SV(); return o.has_key ? str(o.key) : skip(); }
                        if (is(f, "elem")) { o.has_elem = p < e && (*p == '-' || (*p >= '0' && *p <= '9')); return o.has_elem ? num(o.elem) : skip(); }
                        if (is(f, "value")) return anyval(o);
                        if (is(f, "datatype")) {
                            SV t;
                            if (p < e && *p == '"') { if (!str(t)) return false; o.datatype = is(t, "counter") ? HM_DT_COUNTER : (is(t, "timestamp") ? HM_DT_TIMESTAMP : 0); return true; }
                            o.datatype = 0;
                            return skip();
                        }
                        return skip();
                    });
                    if (!r) return false;
                    ops.push_back(o);
                    ws();
                    if (p < e && *p == ',') { p++; ws(); continue; }
                    if (p < e && *p == ']') { p++; return true; }
                    return false;
                }
            }
            return skip();
        });
        c.nops = (uint32_t)ops.size() - c.op0;
        c.ndeps = (uint32_t)deps.size() - c.dep0;
        ws();
        if (!ok || p != e || !actor.p || !c.has_seq) return false;
        c.actor = actor_id(actor);
        return true;
    }
};

bool decode_doc(const uint8_t *data, const uint64_t *block_off, uint32_t b0, uint32_t b1, DocOut &D, Ctx &cx) {
    const uint32_t n = b1 - b0;
    cx.arena.clear();
    cx.cs.assign(n, ScanChange());
    cx.ops.clear();
    cx.deps.clear();
    cx.actors.reset(16);
    size_t bytes = (size_t)(block_off[b1] - block_off[b0]);
    for (uint32_t i = 0; i < n; i++) {
        const char *s = (const char *)data + block_off[b0 + i];
        size_t len = (size_t)(block_off[b0 + i + 1] - block_off[b0 + i]);
        if (len >= 2 && s[0] == 'B' && s[1] == 'R') {
            cx.arena.emplace_back();
            if (!brotli_decompress((const uint8_t *)s + 2, len - 2, cx.arena.back())) return false;
            s = cx.arena.back().data(); len = cx.arena.back().size();
            bytes += len;
        } else if (!(len >= 2 && s[0] == '{' && s[1] == '"')) {
            return false;                                    // 'fail to unpack blocks - head is ...'
        }
        Scan S{s, s + len, &cx};
        cx.cs[i].text = s; cx.cs[i].len = (uint32_t)len;
        if (!S.change(cx.cs[i])) return false;
    }
    // actors (every change's actor and deps keys) ranked in JS string (UTF-16) order
    const auto &an = cx.actors.keys;
    const uint32_t na = (uint32_t)an.size();
    if (na > 0xFFFF) return false;
    std::vector<uint32_t> order(na);
    for (uint32_t i = 0; i < na; i++) order[i] = i;
    bool ascii = true;
    for (auto &k : an) for (uint32_t i = 0; i < k.s.n && ascii; i++) ascii = (unsigned char)k.s.p[i] < 0x80;
    if (ascii) std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
        const SV &a = an[x].s, &b = an[y].s;
        const int r = memcmp(a.p, b.p, std::min(a.n, b.n));
        return r ? r < 0 : a.n < b.n; });
    else {
        std::vector<std::u16string> k(na);
        for (uint32_t i = 0; i < na; i++) k[i] = u16(std::string(an[i].s.p, an[i].s.n));
        std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return k[x] < k[y]; });
    }
    cx.rank.resize(na);
    D.actors.reserve(na);
    for (uint32_t r = 0; r < na; r++) { cx.rank[order[r]] = r; D.actors.emplace_back(an[order[r]].s.p, an[order[r]].s.n); }

    const size_t nops = cx.ops.size();
    cx.objs.reset(8); cx.strs.reset(nops); cx.regs.reset(nops);
    bool fresh;
    cx.objs.get(SV{ROOT_ID, 36}, 0, fresh);
    D.objs.push_back(ROOT_ID);
    SV last_obj{ROOT_ID, 36};
    uint32_t last_obj_id = 0;
    auto obj = [&](const SV &u) {
        if (u == last_obj) return last_obj_id;
        const uint32_t id = cx.objs.get(u, 0, fresh);
        last_obj = u; last_obj_id = id;
        if (fresh) D.objs.emplace_back(u.p, u.n);
        return id;
    };
    auto reg = [&](uint32_t o, const SV &k) {
        const uint32_t id = cx.regs.get(k, o, fresh);
        if (fresh) D.regs.emplace_back(o, std::string(k.p, k.n));
        return id;
    };
    auto str = [&](const SV &v) {
        const uint32_t id = cx.strs.get(v, 0, fresh);
        if (fresh) D.strings.emplace_back(v.p, v.n);
        return id;
    };
    // content identity: equal content needs equal (actor, seq); only repeated keys are compared
    size_t kc = 64;
    while (kc < (size_t)n * 2) kc <<= 1;
    cx.key_slot.assign(kc, 0);
    cx.key_first.resize(kc);
    cx.ckey.resize(n);
    cx.cid.resize(n);
    cx.canon_of.assign(n, std::string());
    auto canon_text = [&](uint32_t i) -> const std::string & {
        if (cx.canon_of[i].empty()) {
            JV v;
            if (!parse_json(cx.cs[i].text, cx.cs[i].len, v)) cx.canon_of[i] = "?";
            else canon(v, cx.canon_of[i]);
        }
        return cx.canon_of[i];
    };
    uint32_t n_content = 0;
    D.ch.reserve(n); D.dp.reserve(cx.deps.size()); D.op.reserve(nops);
    D.op_str_key.reserve(nops); D.op_str_val.reserve(nops);
    for (uint32_t i = 0; i < n; i++) {
        const ScanChange &c = cx.cs[i];
        hm_change_row row = {};
        row.actor = (uint16_t)cx.rank[c.actor];
        row.seq = (uint32_t)(int64_t)c.seq;
        const uint64_t key = ((uint64_t)row.actor << 32) | row.seq;
        cx.ckey[i] = key;
        uint32_t id = UINT32_MAX;
        const uint64_t kh = (key + 1) * 0x9E3779B97F4A7C15ull;
        for (uint32_t s = (uint32_t)(kh >> 32) & (uint32_t)(kc - 1);; s = (s + 1) & (uint32_t)(kc - 1)) {
            if (!cx.key_slot[s]) { cx.key_slot[s] = key + 1; cx.key_first[s] = i; id = n_content++; break; }
            if (cx.key_slot[s] == key + 1) {
                // a repeated (actor, seq): compare content with every earlier change of the key
                for (uint32_t j = cx.key_first[s]; j < i && id == UINT32_MAX; j++)
                    if (cx.ckey[j] == key && canon_text(j) == canon_text(i)) id = cx.cid[j];
                if (id == UINT32_MAX) id = n_content++;
                break;
            }
        }
        cx.cid[i] = id;
        row.content_id = id;
        row.dep_off = (uint32_t)D.dp.size();
        for (uint32_t k = 0; k < c.ndeps; k++) {
            const ScanDep &d = cx.deps[c.dep0 + k];
            hm_dep_row r = {};
            r.actor = (uint16_t)cx.rank[d.actor];
            r.seq = (uint32_t)(int64_t)d.seq;
            D.dp.push_back(r);
        }
        row.n_deps = (uint16_t)c.ndeps;
        row.op_first = (uint32_t)D.op.size();
        for (uint32_t k = 0; k < c.nops; k++) {
            const ScanOp &o = cx.ops[c.op0 + k];
            const int a = o.action;
            if (a < 0 || !o.obj.p) return false;
            hm_op_row r = {};
            r.obj = obj(o.obj);
            r.reg = HM_NONE; r.parent = HM_NONE;
            uint8_t sk = 0, sv = 0;
            if (a == HM_INS) {
                if (!o.has_key || !o.has_elem) return false;
                r.elem = (uint32_t)(int64_t)o.elem;
                const std::string &an_ = D.actors[row.actor];
                cx.arena.emplace_back();
                std::string &el = cx.arena.back();
                el.reserve(an_.size() + 12);
                el.assign(an_);
                el += ':';
                el += js_num_text(o.elem);
                r.reg = reg(r.obj, SV{el.data(), (uint32_t)el.size()});
                r.parent = Scan::is(o.key, "_head") ? HM_HEAD : reg(r.obj, o.key);
            } else if (a >= HM_SET) {
                if (!o.has_key) return false;
                r.reg = reg(r.obj, o.key);
                r.key = str(o.key); sk = 1;
                if (a == HM_LINK) {
                    if (o.vt != J_STR) return false;
                    r.vtag = HM_V_OBJ; r.value = obj(o.sval);
                } else if (a != HM_DEL) {
                    if (!o.has_value || o.vt == J_NULL) r.vtag = HM_V_NULL;
                    else if (o.vt == J_TRUE) r.vtag = HM_V_TRUE;
                    else if (o.vt == J_FALSE) r.vtag = HM_V_FALSE;
                    else if (o.vt == J_NUM) {
                        if (js_int(o.num)) { r.vtag = HM_V_INT; r.value = (uint64_t)(int64_t)o.num; }
                        else { r.vtag = HM_V_FLOAT; memcpy(&r.value, &o.num, 8); }
                    } else if (o.vt == J_STR) { r.vtag = HM_V_STR; r.value = str(o.sval); sv = 1; }
                    else return false;                                        // 'unsupported op value'
                }
            }
            r.datatype = o.datatype;
            r.action = (uint8_t)a;
            if (a == HM_MAKE_LIST || a == HM_MAKE_TEXT) D.flags |= HM_DOC_HAS_LISTS;
            if (a == HM_INC || r.datatype == HM_DT_COUNTER) D.flags |= HM_DOC_HAS_COUNTERS;
            D.op.push_back(r);
            D.op_str_key.push_back(sk);
            D.op_str_val.push_back(sv);
        }
        row.n_ops = c.nops;
        D.ch.push_back(row);
    }
    (void)bytes;
    D.n_regs = (uint32_t)cx.regs.keys.size();
    D.n_objs = (uint32_t)cx.objs.keys.size();
    return true;
}

}  // namespace

// a table of POD rows written once by the decoder threads (no zero fill before they write it)
template <typename T> struct Rows {
    std::unique_ptr<T[]> p;
    size_t n = 0;
    void alloc(size_t k) { p.reset(k ? new T[k] : nullptr); n = k; }
    T *data() { return p.get(); }
    const T *data() const { return p.get(); }
    size_t size() const { return n; }
};

struct hm_decoded {
    std::vector<hm_doc_row> docs;
    Rows<hm_change_row> ch;
    Rows<hm_dep_row> dp;
    Rows<hm_op_row> op;
    std::vector<int32_t> status;
    std::vector<std::string> strings;
    std::vector<std::vector<std::string>> actors, objs;
    std::vector<std::vector<std::pair<uint32_t, std::string>>> regs;
    uint32_t a_stride = 1, max_changes = 0, max_ops = 0, max_regs = 0, max_objs = 0, max_deps = 0, doc_flags = 0;
};

extern "C" {

int hm_decode_blocks(const uint8_t *data, const uint64_t *block_off, const uint32_t *doc_block, uint32_t n_docs,
                     uint32_t a_stride, int threads, hm_decoded **out) {
    if (!out || (n_docs && (!block_off || !doc_block))) return HM_ERR_INVALID;
    *out = nullptr;
    try {
        const auto t_start = std::chrono::steady_clock::now();
        std::vector<DocOut> docs(n_docs);
        const int T = std::max(1, std::min(threads, 256));
        auto work = [&](uint32_t lo, uint32_t hi) {
            Ctx cx;
            for (uint32_t d = lo; d < hi; d++) {
                if (!decode_doc(data, block_off, doc_block[d], doc_block[d + 1], docs[d], cx)) {
                    docs[d] = DocOut();
                    docs[d].status = HM_ERR_INVALID;
                    docs[d].objs.push_back(ROOT_ID);
                }
            }
        };
        if (T == 1 || n_docs < 2) work(0, n_docs);
        else {
            std::vector<std::thread> th;
            for (int t = 0; t < T; t++) {
                const uint32_t lo = (uint32_t)((uint64_t)n_docs * t / T), hi = (uint32_t)((uint64_t)n_docs * (t + 1) / T);
                th.emplace_back(work, lo, hi);
            }
            for (auto &x : th) x.join();
        }
        const auto t_par = std::chrono::steady_clock::now();
        hm_decoded *D = new hm_decoded();
        std::unique_ptr<hm_decoded> own(D);
        // the batch's string pool, in document order (columnar.js StringPool over documents):
        // the one serial step; every document's local string ids -> pool ids in `remap`
        Intern pool;
        pool.reset(1024);
        std::vector<uint64_t> roff(n_docs + 1, 0);
        for (uint32_t d = 0; d < n_docs; d++) roff[d + 1] = roff[d] + docs[d].strings.size();
        std::vector<uint32_t> remap(roff[n_docs]);
        for (uint32_t d = 0; d < n_docs; d++) {
            DocOut &x = docs[d];
            for (size_t i = 0; i < x.strings.size(); i++) {
                bool fresh;
                const std::string &t = x.strings[i];
                remap[roff[d] + i] = pool.get(SV{t.data(), (uint32_t)t.size()}, 0, fresh);
                if (fresh) D->strings.push_back(t);
            }
        }
        // document rows and table offsets (prefix over documents), then the rows themselves are
        // copied by the threads, each into its documents' ranges
        D->docs.resize(n_docs);
        D->status.resize(n_docs); D->actors.resize(n_docs); D->objs.resize(n_docs); D->regs.resize(n_docs);
        uint64_t nc = 0, nd = 0, no = 0;
        uint32_t reg_off = 0, maxa = 1;
        for (uint32_t d = 0; d < n_docs; d++) {
            const DocOut &x = docs[d];
            hm_doc_row &r = D->docs[d];
            r = hm_doc_row{};
            r.change_off = (uint32_t)nc; r.n_changes = (uint32_t)x.ch.size();
            r.dep_off = (uint32_t)nd; r.n_deps = (uint32_t)x.dp.size();
            r.op_off = (uint32_t)no; r.n_ops = (uint32_t)x.op.size();
            r.reg_off = reg_off; r.n_regs = x.n_regs; r.n_objs = x.n_objs;
            r.n_actors = (uint16_t)x.actors.size(); r.flags = x.flags;
            nc += x.ch.size(); nd += x.dp.size(); no += x.op.size();
            reg_off += x.n_regs;
            D->status[d] = x.status;
            maxa = std::max<uint32_t>(maxa, r.n_actors);
            D->max_changes = std::max(D->max_changes, r.n_changes); D->max_ops = std::max(D->max_ops, r.n_ops);
            D->max_regs = std::max(D->max_regs, r.n_regs); D->max_objs = std::max(D->max_objs, r.n_objs);
            D->max_deps = std::max(D->max_deps, r.n_deps); D->doc_flags |= r.flags;
        }
        D->ch.alloc(nc); D->dp.alloc(nd); D->op.alloc(no);
        auto place = [&](uint32_t lo, uint32_t hi) {
            for (uint32_t d = lo; d < hi; d++) {
                DocOut &x = docs[d];
                const hm_doc_row &r = D->docs[d];
                hm_change_row *ch = D->ch.data() + r.change_off;
                for (size_t i = 0; i < x.ch.size(); i++) {
                    hm_change_row c = x.ch[i];
                    c.dep_off += r.dep_off; c.op_first += r.op_off;
                    ch[i] = c;
                }
                if (!x.dp.empty()) memcpy(D->dp.data() + r.dep_off, x.dp.data(), x.dp.size() * sizeof(hm_dep_row));
                hm_op_row *op = D->op.data() + r.op_off;
                const uint32_t *rm = remap.data() + roff[d];
                for (size_t i = 0; i < x.op.size(); i++) {
                    hm_op_row o = x.op[i];
                    if (x.op_str_key[i]) o.key = rm[o.key];
                    if (x.op_str_val[i]) o.value = rm[(size_t)o.value];
                    op[i] = o;
                }
                D->actors[d] = std::move(x.actors);
                D->objs[d] = std::move(x.objs);
                D->regs[d] = std::move(x.regs);
                DocOut().ch.swap(x.ch);
            }
        };
        if (T == 1 || n_docs < 2) place(0, n_docs);
        else {
            std::vector<std::thread> th;
            for (int t = 0; t < T; t++)
                th.emplace_back(place, (uint32_t)((uint64_t)n_docs * t / T), (uint32_t)((uint64_t)n_docs * (t + 1) / T));
            for (auto &x : th) x.join();
        }
        if (getenv("HM_DECODE_PROFILE")) {
            const auto t_end = std::chrono::steady_clock::now();
            fprintf(stderr, "[hm_decode] parallel %.3f ms  merge %.3f ms\n",
                    std::chrono::duration<double, std::milli>(t_par - t_start).count(),
                    std::chrono::duration<double, std::milli>(t_end - t_par).count());
        }
        D->a_stride = a_stride ? a_stride : maxa;
        if (D->a_stride < maxa)
            for (uint32_t d = 0; d < n_docs; d++)
                if (D->docs[d].n_actors > D->a_stride) D->status[d] = HM_ERR_INVALID;   // the merge rejects the row too
        *out = own.release();
        return HM_OK;
    } catch (...) {
        return HM_ERR_NOMEM;
    }
}

int hm_decoded_batch(const hm_decoded *d, hm_batch *b) {
    if (!d || !b) return HM_ERR_INVALID;
    memset(b, 0, sizeof *b);
    b->n_docs = (uint32_t)d->docs.size(); b->n_changes = (uint32_t)d->ch.size();
    b->n_deps = (uint32_t)d->dp.size(); b->n_ops = (uint32_t)d->op.size();
    uint64_t nr = 0;
    for (auto &r : d->docs) nr += r.n_regs;
    b->n_regs = (uint32_t)nr;
    b->a_stride = d->a_stride;
    b->max_changes = d->max_changes; b->max_ops = d->max_ops; b->max_regs = d->max_regs;
    b->max_objs = d->max_objs; b->max_deps = d->max_deps; b->doc_flags = d->doc_flags;
    b->docs = d->docs.data(); b->changes = d->ch.data(); b->deps = d->dp.data(); b->ops = d->op.data();
    b->min_clock = nullptr;
    return HM_OK;
}

const int32_t *hm_decoded_status(const hm_decoded *d) { return d ? d->status.data() : nullptr; }

uint32_t hm_decoded_n_strings(const hm_decoded *d) { return d ? (uint32_t)d->strings.size() : 0; }

const char *hm_decoded_string(const hm_decoded *d, uint32_t i, size_t *len) {
    if (!d || i >= d->strings.size()) return nullptr;
    if (len) *len = d->strings[i].size();
    return d->strings[i].data();
}

const char *hm_decoded_actor(const hm_decoded *d, uint32_t doc, uint32_t rank, size_t *len) {
    if (!d || doc >= d->actors.size() || rank >= d->actors[doc].size()) return nullptr;
    if (len) *len = d->actors[doc][rank].size();
    return d->actors[doc][rank].data();
}

const char *hm_decoded_obj(const hm_decoded *d, uint32_t doc, uint32_t obj, size_t *len) {
    if (!d || doc >= d->objs.size() || obj >= d->objs[doc].size()) return nullptr;
    if (len) *len = d->objs[doc][obj].size();
    return d->objs[doc][obj].data();
}

const char *hm_decoded_reg(const hm_decoded *d, uint32_t doc, uint32_t reg, uint32_t *obj, size_t *len) {
    if (!d || doc >= d->regs.size() || reg >= d->regs[doc].size()) return nullptr;
    if (obj) *obj = d->regs[doc][reg].first;
    if (len) *len = d->regs[doc][reg].second.size();
    return d->regs[doc][reg].second.data();
}

void hm_decoded_free(hm_decoded *d) { delete d; }

}  // extern "C"
