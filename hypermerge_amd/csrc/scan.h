// scan.h — the JSON side of the host decoder, shared by decode.cpp (hm_decode_blocks: stateless
// cold-load batches) and docset.cpp (hm_docset_*: per-document interners kept across rounds).
//   Block.unpack (src/Block.ts:18-29), JsonBuffer.parse (src/JsonBuffer.ts:1-4) and the
//   content identity Automerge decides with Immutable `equals`.
#pragma once
#include <dlfcn.h>
#include <algorithm>
#include <cctype>
#include <emmintrin.h>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <cstdio>
#include <mutex>
#include <string>
#include <utility>
#include <vector>
#include "../../include/hypermerge_amd.h"

namespace hmscan {
namespace {   // TU-local copies (decode.cpp, docset.cpp)

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

// JS Number.isInteger(v) && |v| < 2^53
bool js_int(double v) { return std::isfinite(v) && std::floor(v) == v && std::fabs(v) < 9007199254740992.0; }
// `${n}` of an integral JS number (the element counter of an elemId), written into b
// (>= 40 bytes); returns its length
uint32_t js_num_text(double v, char *b) {
    if (!js_int(v)) return (uint32_t)snprintf(b, 40, "%.17g", v);
    long long x = (long long)v;
    char t[24];
    int n = 0;
    const bool neg = x < 0;
    unsigned long long u = neg ? 0ull - (unsigned long long)x : (unsigned long long)x;
    do { t[n++] = (char)('0' + u % 10); u /= 10; } while (u);
    uint32_t k = 0;
    if (neg) b[k++] = '-';
    while (n) b[k++] = t[--n];
    b[k] = 0;
    return k;
}


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
    uint32_t get(const SV &s, uint32_t tag, bool &fresh) { return get_h(s, tag, hash_bytes(s.p, s.n, tag), fresh); }
    // with the name's hash_bytes(s, tag) already known (the batch pool re-interns names that a
    // document's table hashed before)
    uint32_t get_h(const SV &s, uint32_t tag, uint64_t h, bool &fresh) {
        for (uint32_t i = (uint32_t)h & mask;; i = (i + 1) & mask) {
            const uint32_t v = slot[i];
            if (!v) {
                if ((keys.size() + 1) * 2 > slot.size()) { grow(); return get_h(s, tag, h, fresh); }
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
    static int action_of(const SV &a) {
        static const char *names[] = {"makeMap", "makeTable", "makeList", "makeText", "ins", "set", "del", "link", "inc"};
        for (int i = 0; i < 9; i++) if (is(a, names[i])) return i;
        return -1;
    }
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
                            o.action = (int8_t)action_of(a);
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

}  // namespace
}  // namespace hmscan
