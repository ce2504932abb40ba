// docset.cpp — the host engine of the Node drop-in (include/hypermerge_amd.h, hm_docset_*).
//
// What the reference runs on the JS main thread for every arriving block, per document,
// natively and over many documents per call:
//   Actor.parseBlock / Block.unpack / JsonBuffer.parse   (src/Actor.ts:137-141, src/Block.ts:18-29,
//                                                         src/JsonBuffer.ts:1-4)
//   DocBackend.applyRemoteChanges -> Backend.applyChanges (src/DocBackend.ts:169-185)
//   DocBackend.updateClock, the patch of RemotePatchMsg   (src/DocBackend.ts:135-142, :173-183)
// A docset owns the documents of one device: their interners (actor ids ranked in JS string
// order, object UUIDs, (object, key|elemId) registers, string values, content identity of
// changes — columnar.js DocEncoder, kept across rounds), their placement in the resident
// stores (one hm_store per actor-stride class 8/16/32/64/128/256: a document moves to a wider class
// when a new actor outgrows its rows, its log rows re-submitted from the old store), and the
// patch base (the document as the last patch left it).  One call = one applyChanges round
// for every document of the call: decode on host threads, submit per class, wait, commit or
// roll back each document (a throwing applyChanges leaves DocBackend.back unchanged), read
// back only the registers the round's ops hit (every register when changes were queued), and
// render each document's patch, opSet clock / deps and DocBackend.clock as JSON text.
//
// Content identity (Automerge's `Inconsistent reuse of sequence number` check, Immutable
// `equals` of two changes with one (actor, seq)) is a 128-bit hash of each change's
// canonical form (maps order-insensitive, last duplicate key wins, numbers by value), kept
// per (actor, seq): the blocks themselves stay with the caller.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>
#include "../../include/hypermerge_amd.h"
#include "engine_internal.h"
#include "scan.h"

namespace {

using namespace hmscan;

constexpr uint32_t N_CLASS = 6;
constexpr uint32_t STRIDES[N_CLASS] = {8, 16, 32, 64, 128, 256};
// a document's actors: rank 255 stays free for the stores' 0xFF "no rank" entries
constexpr uint32_t MAX_ACTORS = HM_MAX_STRIDE - 1;
constexpr uint8_t NO_CLASS = 0xFF;
constexpr uint8_t NO_TYPE = 0xFF;

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

// (tag, bytes) -> dense id in first-insertion order, owning its bytes
struct Names {
    std::string arena;
    struct K { uint32_t off, len, tag, h; };
    std::vector<K> keys;
    std::vector<uint32_t> slot;                              // id + 1, 0 = empty
    uint32_t mask = 0;
    uint32_t size() const { return (uint32_t)keys.size(); }
    const char *ptr(uint32_t id) const { return arena.data() + keys[id].off; }
    uint32_t len(uint32_t id) const { return keys[id].len; }
    uint32_t tag(uint32_t id) const { return keys[id].tag; }
    void rehash(size_t cap) {
        slot.assign(cap, 0);
        mask = (uint32_t)cap - 1;
        for (uint32_t id = 0; id < keys.size(); id++) {
            uint32_t i = keys[id].h & mask;
            while (slot[i]) i = (i + 1) & mask;
            slot[i] = id + 1;
        }
    }
    uint32_t get(const char *p, uint32_t n, uint32_t tg, bool &fresh) {
        if ((keys.size() + 1) * 2 > slot.size()) rehash(std::max<size_t>(16, slot.size() * 2));
        const uint32_t h = (uint32_t)hash_bytes(p, n, tg);
        for (uint32_t i = h & mask;; i = (i + 1) & mask) {
            const uint32_t v = slot[i];
            if (!v) {
                slot[i] = size() + 1;
                keys.push_back({(uint32_t)arena.size(), n, tg, h});
                arena.append(p, n);
                fresh = true;
                return size() - 1;
            }
            const K &k = keys[v - 1];
            if (k.h == h && k.tag == tg && k.len == n && !memcmp(arena.data() + k.off, p, n)) { fresh = false; return v - 1; }
        }
    }
    void truncate(uint32_t n) {
        if (n >= keys.size()) return;
        arena.resize(keys[n].off);
        keys.resize(n);
        rehash(std::max<size_t>(16, slot.size()));
    }
};

// ---------------- content identity: a 128-bit hash of a change's canonical form ----------------
struct H2 { uint64_t a, b; bool operator==(const H2 &o) const { return a == o.a && b == o.b; } };

H2 leaf(uint64_t tag, const char *p, size_t n) {
    return {mix64(hash_bytes(p, (uint32_t)n, 0x51ED270B27A1F00Dull ^ tag)), mix64(hash_bytes(p, (uint32_t)n, 0x2545F4914F6CDD1Dull + tag))};
}

struct CHash {
    const char *p, *e;
    std::vector<std::pair<H2, H2>> &stk;                     // (key, value) of the open objects' fields
    std::string &tmp;
    void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
    bool str(H2 &h) {
        if (p >= e || *p != '"') return false;
        const char *s = p + 1, *q = s;
        while (q < e && *q != '"' && *q != '\\') q++;
        if (q < e && *q == '"') { h = leaf(5, s, (size_t)(q - s)); p = q + 1; return true; }
        Parser P{p, e};
        if (!P.string(tmp)) return false;
        p = P.p;
        h = leaf(5, tmp.data(), tmp.size());
        return true;
    }
    bool val(H2 &h, int depth) {
        if (depth > 256) return false;
        ws();
        if (p >= e) return false;
        const char c = *p;
        if (c == '"') return str(h);
        if (c == '{') {
            p++;
            const size_t base = stk.size();
            ws();
            if (p < e && *p == '}') p++;
            else for (;;) {
                ws();
                H2 k, v;
                if (!str(k)) return false;
                ws();
                if (p >= e || *p != ':') return false;
                p++;
                if (!val(v, depth + 1)) return false;
                bool dup = false;                             // JSON.parse: the last duplicate key wins
                for (size_t i = base; i < stk.size(); i++) if (stk[i].first == k) { stk[i].second = v; dup = true; }
                if (!dup) stk.push_back({k, v});
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == '}') { p++; break; }
                return false;
            }
            uint64_t A = 0, B = 0;                            // order-insensitive over the fields
            for (size_t i = base; i < stk.size(); i++) {
                A += mix64(stk[i].first.a * 0x9E3779B97F4A7C15ull ^ stk[i].second.a);
                B += mix64(stk[i].first.b + 0xD6E8FEB86659FD93ull * stk[i].second.b);
            }
            const uint64_t n = stk.size() - base;
            stk.resize(base);
            h = {mix64(A ^ (0x7A11ull << 48) ^ n), mix64(B + 0x0B1Eull + n)};
            return true;
        }
        if (c == '[') {
            p++;
            uint64_t A = 0x1234567ull, B = 0x89ABCDEFull, n = 0;
            ws();
            if (p < e && *p == ']') p++;
            else for (;;) {
                H2 v;
                if (!val(v, depth + 1)) return false;
                A = mix64(A * 31 + v.a); B = mix64(B ^ (v.b + n));
                n++;
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == ']') { p++; break; }
                return false;
            }
            h = {A ^ n, B + n};
            return true;
        }
        if (e - p >= 4 && !memcmp(p, "null", 4)) { p += 4; h = leaf(0, "", 0); return true; }
        if (e - p >= 4 && !memcmp(p, "true", 4)) { p += 4; h = leaf(2, "", 0); return true; }
        if (e - p >= 5 && !memcmp(p, "false", 5)) { p += 5; h = leaf(1, "", 0); return true; }
        Parser P{p, e};                                       // a number, compared by value (0 == -0)
        JV j;
        if (!P.value(j, 0) || j.t != J_NUM) return false;
        p = P.p;
        double v = j.num == 0 ? 0.0 : j.num;
        h = leaf(3, (const char *)&v, 8);
        return true;
    }
};

// A list's placed elements in document order, in blocks: a position, an insertion or a visible
// index costs O(blocks + block size) instead of O(elements) (a text document holds thousands of
// elements, and the per-op replay asks for one of these per list op).  Blocks have stable ids;
// `where` (per register, the document's) names each placed element's block; a block keeps its
// count of visible elements (a non-empty survivor set).
struct ListOrder {
    static constexpr uint32_t SPLIT = 256;
    struct Blk { std::vector<uint32_t> el; uint32_t vis = 0; };
    std::vector<Blk> pool;                                   // by block id
    std::vector<uint32_t> seq;                               // block ids in document order
    uint32_t n = 0;
    uint32_t size() const { return n; }
    uint32_t pos_of(uint32_t e, const std::vector<uint32_t> &where) const {
        const uint32_t b = where[e];
        uint32_t at = 0;
        for (uint32_t id : seq) {
            if (id == b) break;
            at += (uint32_t)pool[id].el.size();
        }
        const auto &v = pool[b].el;
        return at + (uint32_t)(std::find(v.begin(), v.end(), e) - v.begin());
    }
    template <typename Vis>
    uint32_t vis_before(uint32_t e, const std::vector<uint32_t> &where, Vis &&vis) const {
        if (e >= where.size() || where[e] == HM_NONE) return 0;
        const uint32_t b = where[e];
        uint32_t c = 0;
        for (uint32_t id : seq) {
            if (id == b) break;
            c += pool[id].vis;
        }
        for (uint32_t x : pool[b].el) {
            if (x == e) break;
            c += vis(x) ? 1u : 0u;
        }
        return c;
    }
    // the elements `sub` (in order) at position pos
    template <typename Vis>
    void insert_at(uint32_t pos, const std::vector<uint32_t> &sub, std::vector<uint32_t> &where, Vis &&vis) {
        if (sub.empty()) return;
        if (seq.empty()) { pool.emplace_back(); seq.push_back(0); }
        uint32_t k = 0, at = 0;
        while (k + 1 < seq.size() && at + pool[seq[k]].el.size() < pos) at += (uint32_t)pool[seq[k++]].el.size();
        const uint32_t b = seq[k];
        Blk &B = pool[b];
        B.el.insert(B.el.begin() + (pos - at), sub.begin(), sub.end());
        for (uint32_t x : sub) { where[x] = b; B.vis += vis(x) ? 1u : 0u; }
        n += (uint32_t)sub.size();
        if (pool[b].el.size() > SPLIT) {                     // split off the second half
            const uint32_t nb = (uint32_t)pool.size();
            pool.emplace_back();
            Blk &L = pool[b], &R = pool[nb];
            const size_t half = L.el.size() / 2;
            R.el.assign(L.el.begin() + half, L.el.end());
            L.el.resize(half);
            R.vis = 0;
            for (uint32_t x : R.el) { where[x] = nb; R.vis += vis(x) ? 1u : 0u; }
            L.vis -= R.vis;
            seq.insert(seq.begin() + k + 1, nb);
        }
    }
    void vis_change(uint32_t e, const std::vector<uint32_t> &where, bool now) {
        if (e < where.size() && where[e] != HM_NONE) { Blk &B = pool[where[e]]; B.vis = now ? B.vis + 1 : B.vis - 1; }
    }
};

// ---------------- one document ----------------
struct DocSt {
    bool ready = false;
    Names actors, objs, regs, strs;                          // actors: ids in first-appearance order
    std::vector<uint16_t> rank_of, by_rank;                  // actor id -> rank (JS string order) and back
    // content identity: (actor id, seq) -> chain of (canonical hash, content id)
    std::vector<uint64_t> ckey;                              // key + 1, 0 = empty slot
    std::vector<uint32_t> chead;
    struct CE { uint64_t key; H2 h; uint32_t cid, next; };
    std::vector<CE> cents;
    uint32_t n_content = 0;
    // the log (what the stores hold), per op: its change's actor id and datatype (rendering)
    std::vector<uint16_t> op_actor;
    std::vector<uint8_t> op_dt;
    uint32_t n_changes = 0, n_ops = 0;
    uint16_t flags = 0;
    uint8_t cls = NO_CLASS;
    uint32_t handle = 0;
    uint32_t hist_len = 0, n_queued = 0;
    // the patch base: the document as the last patch left it
    std::vector<uint8_t> obj_type, obj_emitted;
    std::vector<uint64_t> sig;                               // per register: rendered entry hash, 0 = absent
    std::vector<std::pair<uint32_t, std::vector<uint32_t>>> lists;   // list object -> visible element registers
    // the per-op patch base (op_diffs): the log's op rows, and the document as the last
    // applied op left it — per register its survivors (winner first), per list element its
    // insertion and place in the insertion tree, per list object its reachable elements in
    // document order
    std::vector<hm_op_row> oplog;
    std::vector<uint32_t> op_seq;                            // per op: its change's seq
    std::vector<uint32_t> ch_op0;                            // per change: its first op
    std::vector<std::vector<hm_surv_result>> rs;             // per register
    std::vector<uint32_t> el_op;                             // per register: its ins op, or HM_NONE
    std::vector<uint8_t> el_in;                              // per register: placed in its list's order
    std::vector<uint32_t> el_blk;                            // per register: its ListOrder block (HM_NONE = not placed)
    std::unordered_map<uint32_t, std::vector<uint32_t>> kids;      // parent key -> children, (elem, actor) descending
    std::vector<std::pair<uint32_t, ListOrder>> ord;         // list object -> placed elements in document order
    void setup() {
        bool f;
        objs.get(ROOT_ID, 36, 0, f);
        obj_type.assign(1, HM_MAKE_MAP);
        obj_emitted.assign(1, 1);
        ready = true;
    }
    void crehash(size_t cap) {
        ckey.assign(cap, 0);
        chead.assign(cap, 0);
        const uint64_t m = cap - 1;
        for (uint32_t i = 0; i < cents.size(); i++) {
            uint64_t s = mix64(cents[i].key) & m;
            while (ckey[s] && ckey[s] != cents[i].key + 1) s = (s + 1) & m;
            cents[i].next = ckey[s] ? chead[s] : HM_NONE;
            ckey[s] = cents[i].key + 1;
            chead[s] = i;
        }
    }
    uint32_t content_id(uint64_t key, const H2 &h) {
        if ((cents.size() + 1) * 2 > ckey.size()) crehash(std::max<size_t>(64, ckey.size() * 2));
        const uint64_t m = ckey.size() - 1;
        uint64_t s = mix64(key) & m;
        while (ckey[s] && ckey[s] != key + 1) s = (s + 1) & m;
        uint32_t nx = HM_NONE;
        if (ckey[s]) {
            for (uint32_t i = chead[s]; i != HM_NONE; i = cents[i].next)
                if (cents[i].h == h) return cents[i].cid;
            nx = chead[s];
        }
        cents.push_back({key, h, n_content, nx});
        ckey[s] = key + 1;
        chead[s] = (uint32_t)cents.size() - 1;
        return n_content++;
    }
    std::vector<uint32_t> *list_of(uint32_t obj, bool make) {
        for (auto &l : lists) if (l.first == obj) return &l.second;
        if (!make) return nullptr;
        lists.emplace_back(obj, std::vector<uint32_t>());
        return &lists.back().second;
    }
    ListOrder &order_of(uint32_t obj) {
        for (auto &x : ord) if (x.first == obj) return x.second;
        ord.emplace_back(obj, ListOrder());
        return ord.back().second;
    }
};

// JS string order (UTF-16 code units) of two UTF-8 names
bool js_less(const char *a, uint32_t na, const char *b, uint32_t nb) {
    bool ascii = true;
    for (uint32_t i = 0; i < na && ascii; i++) ascii = (unsigned char)a[i] < 0x80;
    for (uint32_t i = 0; i < nb && ascii; i++) ascii = (unsigned char)b[i] < 0x80;
    if (ascii) {
        const int r = memcmp(a, b, std::min(na, nb));
        return r ? r < 0 : na < nb;
    }
    return u16(std::string(a, na)) < u16(std::string(b, nb));
}

// One document's binary patch: u32 words, f64 numbers, and the strings it names (pointers into
// the document's name tables, local indices).  Words:
//   clock, deps, DocBackend.clock of the log, of this call: each n, then n x (actor string, seq)
//   n_diffs, then per diff a head word (action 0 create | 1 set | 2 remove | 3 insert, type << 3)
//   and: create: obj | set (map): obj key entry | remove (map): obj key | remove (list): obj index
//        insert: obj index elemId entry | set (list): obj index entry
//   entry: n_surv, the winner's value word, then per conflict: actor string, value word
//   value word: vtag | datatype << 3 | payload << 5 (payload: string index for STR / OBJ, number
//   index for INT / FLOAT)
struct BinDoc {
    std::vector<uint32_t> w;
    std::vector<double> nums;
    std::vector<std::pair<const char *, uint32_t>> strs;
    bool exotic = false;                                      // a lone surrogate: the call falls back to JSON
};

// One document's part of a call.
struct Round {
    uint32_t doc = 0, b0 = 0, b1 = 0;
    int32_t status = HM_OK;
    uint32_t err_block = HM_NONE;
    std::vector<hm_change_row> ch;
    std::vector<hm_dep_row> dp;
    std::vector<hm_op_row> op;
    uint16_t n_actors = 0, flags = 0;
    uint32_t n_regs = 0, n_objs = 0;
    std::vector<uint8_t> remap;                              // old rank -> new rank (empty = identity)
    // snapshot for the rollback
    uint32_t s_actors = 0, s_objs = 0, s_regs = 0, s_strs = 0, s_cents = 0, s_content = 0, s_ops = 0;
    std::vector<uint16_t> s_rank_of, s_by_rank;
    bool started = false;                                    // its decode took the snapshot above
    // placement in this call
    uint8_t cls = NO_CLASS;
    uint32_t handle = 0, row = 0;
    bool moved = false, placed = false, fresh = false;       // fresh: handle taken for it in this call
    hm_doc_result res = {};
    const uint32_t *clock = nullptr, *back = nullptr, *heads = nullptr;
    bool full = false;                                       // patch from every register (else the hit ones)
    uint32_t q0 = 0, q1 = 0;                                 // its register requests
    std::string patch, bclock, cclock;
    BinDoc bin;
    uint32_t h0 = 0, h1 = 0, prev_hist = 0;                  // op diffs: its rows of the class's history slices
    std::vector<uint32_t> touched;                           // op diffs: the registers its applied ops hit
};

struct Scratch {
    Ctx cx;
    std::vector<H2> hs;
    std::vector<std::pair<H2, H2>> stk;
    std::string tmp;
    std::vector<uint32_t> t2n;
};

// f(lo, hi, t) over T ranges of [0, n) on host threads.  A worker's exception (out of memory: block
// data comes from peers, brotli output is unbounded) is caught in the worker, every started
// thread is joined, a range whose thread cannot be created runs on this one, and the failure is
// rethrown here as std::bad_alloc (the call returns HM_ERR_NOMEM instead of terminating the process).
template <typename F> void par_for(uint32_t n, uint32_t T, F &&f) {
    T = std::max(1u, std::min(T, n));
    if (T <= 1) { f(0u, n, 0u); return; }
    std::atomic<bool> failed{false};
    auto run = [&f, &failed, n, T](uint32_t t) {
        try { f((uint32_t)((uint64_t)n * t / T), (uint32_t)((uint64_t)n * (t + 1) / T), t); } catch (...) { failed = true; }
    };
    std::vector<std::thread> th;
    try { th.reserve(T); } catch (...) {}
    for (uint32_t t = 0; t < T; t++) {
        try { th.emplace_back(run, t); } catch (...) { run(t); }
    }
    for (auto &x : th) x.join();
    if (failed) throw std::bad_alloc();
}

void rollback(DocSt &d, Round &R) {
    d.actors.truncate(R.s_actors);
    if (!R.s_rank_of.empty() || R.s_actors == 0) { d.rank_of = R.s_rank_of; d.by_rank = R.s_by_rank; }
    d.objs.truncate(R.s_objs);
    d.regs.truncate(R.s_regs);
    d.strs.truncate(R.s_strs);
    if (d.cents.size() > R.s_cents) {
        d.cents.resize(R.s_cents);
        d.crehash(std::max<size_t>(64, d.ckey.size()));
    }
    d.n_content = R.s_content;
    d.op_actor.resize(R.s_ops);
    d.op_dt.resize(R.s_ops);
}

bool unpack(const uint8_t *data, const uint64_t *bo, uint32_t b, Ctx &cx, const char *&s, size_t &len) {
    s = (const char *)data + bo[b];
    len = (size_t)(bo[b + 1] - bo[b]);
    if (len >= 2 && s[0] == 'B' && s[1] == 'R') {
        cx.arena.emplace_back();
        if (!brotli_decompress((const uint8_t *)s + 2, len - 2, cx.arena.back())) return false;
        s = cx.arena.back().data(); len = cx.arena.back().size();
        return true;
    }
    return len >= 2 && s[0] == '{' && s[1] == '"';            // else 'fail to unpack blocks - head is ...'
}

// decode one document's blocks of the call into rows against its interners
void decode_round(DocSt &d, Round &R, const uint8_t *data, const uint64_t *bo, Scratch &X) {
    if (!d.ready) d.setup();
    R.s_actors = d.actors.size(); R.s_objs = d.objs.size(); R.s_regs = d.regs.size(); R.s_strs = d.strs.size();
    R.s_cents = (uint32_t)d.cents.size(); R.s_content = d.n_content; R.s_ops = (uint32_t)d.op_actor.size();
    R.started = true;
    Ctx &cx = X.cx;
    const uint32_t n = R.b1 - R.b0;
    cx.arena.clear();
    cx.cs.assign(n, ScanChange());
    cx.ops.clear();
    cx.deps.clear();
    cx.actors.reset(16);
    X.hs.resize(n);
    auto fail = [&](int32_t st, uint32_t b) { R.status = st; R.err_block = b; };
    for (uint32_t i = 0; i < n; i++) {
        const char *s; size_t len;
        if (!unpack(data, bo, R.b0 + i, cx, s, len)) return fail(HM_ERR_INVALID, i);
        Scan S{s, s + len, &cx};
        cx.cs[i].text = s; cx.cs[i].len = (uint32_t)len;
        if (!S.change(cx.cs[i])) return fail(HM_ERR_INVALID, i);
        CHash C{s, s + len, X.stk, X.tmp};
        if (!C.val(X.hs[i], 0)) return fail(HM_ERR_INVALID, i);
    }
    // actors: the call's names -> the document's actor ids; a new actor re-ranks (JS string order)
    const auto &tk = cx.actors.keys;
    X.t2n.resize(tk.size());
    bool fresh_any = false;
    for (size_t k = 0; k < tk.size(); k++) {
        bool f;
        X.t2n[k] = d.actors.get(tk[k].s.p, tk[k].s.n, 0, f);
        fresh_any |= f;
    }
    const uint32_t na = d.actors.size();
    if (na > MAX_ACTORS) return fail(HM_ERR_UNSUPPORTED, HM_NONE);
    if (fresh_any) {
        R.s_rank_of = d.rank_of; R.s_by_rank = d.by_rank;
        std::vector<uint16_t> order(na);
        for (uint32_t i = 0; i < na; i++) order[i] = (uint16_t)i;
        std::sort(order.begin(), order.end(), [&](uint16_t x, uint16_t y) {
            return js_less(d.actors.ptr(x), d.actors.len(x), d.actors.ptr(y), d.actors.len(y)); });
        std::vector<uint16_t> rank_of(na);
        for (uint32_t r = 0; r < na; r++) rank_of[order[r]] = (uint16_t)r;
        bool ident = true;
        std::vector<uint8_t> remap(R.s_actors);
        for (uint32_t r = 0; r < R.s_actors; r++) {
            remap[r] = (uint8_t)rank_of[d.by_rank[r]];
            ident &= remap[r] == r;
        }
        if (!ident) R.remap = std::move(remap);
        d.rank_of = std::move(rank_of);
        d.by_rank = std::move(order);
    }
    R.n_actors = (uint16_t)na;
    bool f;
    uint32_t last_obj_id = 0;
    SV last_obj{ROOT_ID, 36};
    auto obj = [&](const SV &u) {
        if (u == last_obj) return last_obj_id;
        last_obj_id = d.objs.get(u.p, u.n, 0, f);
        last_obj = u;
        return last_obj_id;
    };
    R.ch.reserve(n); R.dp.reserve(cx.deps.size()); R.op.reserve(cx.ops.size());
    std::string el;
    for (uint32_t i = 0; i < n; i++) {
        const ScanChange &c = cx.cs[i];
        const uint32_t aid = X.t2n[c.actor];
        hm_change_row row = {};
        row.actor = d.rank_of[aid];
        row.seq = (uint32_t)(int64_t)c.seq;
        row.content_id = d.content_id(((uint64_t)aid << 32) | row.seq, X.hs[i]);
        row.dep_off = (uint32_t)R.dp.size();
        for (uint32_t k = 0; k < c.ndeps; k++) {
            const ScanDep &dd = cx.deps[c.dep0 + k];
            hm_dep_row r = {};
            r.actor = d.rank_of[X.t2n[dd.actor]];
            r.seq = (uint32_t)(int64_t)dd.seq;
            R.dp.push_back(r);
        }
        row.n_deps = (uint16_t)c.ndeps;
        row.op_first = (uint32_t)R.op.size();
        for (uint32_t k = 0; k < c.nops; k++) {
            const ScanOp &o = cx.ops[c.op0 + k];
            const int a = o.action;
            if (a < 0 || !o.obj.p) return fail(HM_ERR_INVALID, i);
            hm_op_row r = {};
            r.obj = obj(o.obj);
            r.reg = HM_NONE; r.parent = HM_NONE;
            if (a == HM_INS) {
                if (!o.has_key || !o.has_elem) return fail(HM_ERR_INVALID, i);
                r.elem = (uint32_t)(int64_t)o.elem;
                el.assign(d.actors.ptr(aid), d.actors.len(aid));
                el += ':';
                char nb[40];
                el.append(nb, js_num_text(o.elem, nb));
                r.reg = d.regs.get(el.data(), (uint32_t)el.size(), r.obj, f);
                r.parent = Scan::is(o.key, "_head") ? HM_HEAD : d.regs.get(o.key.p, o.key.n, r.obj, f);
            } else if (a >= HM_SET) {
                if (!o.has_key) return fail(HM_ERR_INVALID, i);
                r.reg = d.regs.get(o.key.p, o.key.n, r.obj, f);
                r.key = d.strs.get(o.key.p, o.key.n, 0, f);
                if (a == HM_LINK) {
                    if (o.vt != J_STR) return fail(HM_ERR_INVALID, i);
                    r.vtag = HM_V_OBJ; r.value = obj(o.sval);
                } else if (a != HM_DEL) {
                    if (!o.has_value || o.vt == J_NULL) r.vtag = HM_V_NULL;
                    else if (o.vt == J_TRUE) r.vtag = HM_V_TRUE;
                    else if (o.vt == J_FALSE) r.vtag = HM_V_FALSE;
                    else if (o.vt == J_NUM) {
                        if (js_int(o.num)) { r.vtag = HM_V_INT; r.value = (uint64_t)(int64_t)o.num; }
                        else { r.vtag = HM_V_FLOAT; memcpy(&r.value, &o.num, 8); }
                    } else if (o.vt == J_STR) { r.vtag = HM_V_STR; r.value = d.strs.get(o.sval.p, o.sval.n, 0, f); }
                    else return fail(HM_ERR_INVALID, i);            // 'unsupported op value'
                }
            }
            r.datatype = o.datatype;
            r.action = (uint8_t)a;
            if (a == HM_MAKE_LIST || a == HM_MAKE_TEXT) R.flags |= HM_DOC_HAS_LISTS;
            if (a == HM_INC || r.datatype == HM_DT_COUNTER) R.flags |= HM_DOC_HAS_COUNTERS;
            R.op.push_back(r);
            d.op_actor.push_back((uint16_t)aid);
            d.op_dt.push_back(r.datatype);
        }
        row.n_ops = c.nops;
        R.ch.push_back(row);
    }
    R.n_regs = d.regs.size();
    R.n_objs = d.objs.size();
}

// ---------------- JSON rendering (what JSON.parse turns back into the JS values) ----------------
void jstr(std::string &o, const char *p, size_t n) {
    static const char *hex = "0123456789abcdef";
    o += '"';
    for (size_t i = 0; i < n; i++) {
        const unsigned char c = (unsigned char)p[i];
        if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
        else if (c < 0x20) {
            switch (c) {
            case '\b': o += "\\b"; break; case '\f': o += "\\f"; break; case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break; case '\t': o += "\\t"; break;
            default: o += "\\u00"; o += hex[c >> 4]; o += hex[c & 15];
            }
        } else if (c == 0xED && i + 2 < n && ((unsigned char)p[i + 1] & 0xE0) == 0xA0) {
            // a lone surrogate (kept as its 3-byte form by the decoder): back to \uD8xx / \uDCxx
            const uint32_t u = 0xD000 | (((unsigned char)p[i + 1] & 0x3F) << 6) | ((unsigned char)p[i + 2] & 0x3F);
            o += "\\u";
            for (int s = 12; s >= 0; s -= 4) o += hex[(u >> s) & 15];
            i += 2;
        } else o += (char)c;
    }
    o += '"';
}

void jnum(std::string &o, uint32_t vtag, uint64_t value) {
    char b[48];
    if (vtag == HM_V_INT) { snprintf(b, sizeof b, "%lld", (long long)(int64_t)value); o += b; return; }
    double v;
    memcpy(&v, &value, 8);
    if (v != v) { o += "null"; return; }                       // JSON.stringify(NaN)
    if (v == 1.0 / 0.0) { o += "1e999"; return; }              // JSON.parse -> Infinity
    if (v == -1.0 / 0.0) { o += "-1e999"; return; }
    snprintf(b, sizeof b, "%.17g", v);                         // round-trips to the same double
    o += b;
}

void jvalue(std::string &o, const DocSt &d, const hm_surv_result &s) {
    o += "\"value\":";
    switch (s.vtag) {
    case HM_V_NULL: o += "null"; break;
    case HM_V_FALSE: o += "false"; break;
    case HM_V_TRUE: o += "true"; break;
    case HM_V_INT: case HM_V_FLOAT: jnum(o, s.vtag, s.value); break;
    case HM_V_STR: {
        const uint32_t id = (uint32_t)s.value;
        if (id < d.strs.size()) jstr(o, d.strs.ptr(id), d.strs.len(id)); else o += "null";
        break;
    }
    case HM_V_OBJ: {
        const uint32_t id = (uint32_t)s.value;
        if (id < d.objs.size()) jstr(o, d.objs.ptr(id), d.objs.len(id)); else o += "null";
        o += ",\"link\":true";
        break;
    }
    default: o += "null";
    }
    const uint8_t dt = s.op < d.op_dt.size() ? d.op_dt[s.op] : 0;
    if (dt == HM_DT_COUNTER) o += ",\"datatype\":\"counter\"";
    else if (dt == HM_DT_TIMESTAMP) o += ",\"datatype\":\"timestamp\"";
}

// a register's survivors (winner first) -> the fields of its diff entry:
// value[, link][, datatype][, conflicts: [{actor, value[, link][, datatype]}]]
void jentry(std::string &o, const DocSt &d, const hm_surv_result *sv, uint32_t n) {
    jvalue(o, d, sv[0]);
    if (n <= 1) return;
    o += ",\"conflicts\":[";
    for (uint32_t i = 1; i < n; i++) {
        if (i > 1) o += ',';
        o += "{\"actor\":";
        const uint32_t a = sv[i].op < d.op_actor.size() ? d.op_actor[sv[i].op] : 0;
        jstr(o, d.actors.ptr(a), d.actors.len(a));
        o += ',';
        jvalue(o, d, sv[i]);
        o += '}';
    }
    o += ']';
}

void jclock(std::string &o, const DocSt &d, const uint32_t *row, uint32_t n_actors) {
    o += '{';
    bool first = true;
    for (uint32_t r = 0; r < n_actors; r++) {
        if (!row[r]) continue;
        if (!first) o += ',';
        first = false;
        const uint32_t a = d.by_rank[r];
        jstr(o, d.actors.ptr(a), d.actors.len(a));
        o += ':';
        o += std::to_string(row[r]);
    }
    o += '}';
}

const char *TYPE_NAME[4] = {"map", "table", "list", "text"};

// What the frontend sees of a register's survivors (the winner's value / link / datatype, each
// conflict's actor, value, link, datatype): equal signatures render equal diff entries.
uint64_t entry_sig(const DocSt &d, const hm_surv_result *sv, uint32_t n) {
    if (!n) return 0;
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t op = sv[i].op;
        const uint64_t dt = op < d.op_dt.size() ? d.op_dt[op] : 0;
        const uint64_t act = i && op < d.op_actor.size() ? (uint64_t)d.op_actor[op] + 1 : 0;
        h = mix64(h ^ ((uint64_t)sv[i].vtag | dt << 8 | act << 16));
        h = mix64(h + sv[i].value);
    }
    return h | 1;
}

// Patch writers: JSON text (what JSON.parse turns back into the patch) and a compact binary
// form the Node host turns into the same objects without a JSON parse (HM_DOCSET_BINARY).
struct JsonW {
    std::string &o;
    const DocSt &d;
    bool any = false;
    void sep() { if (any) o += ','; any = true; }
    void clock(const uint32_t *row, uint32_t n_actors) { jclock(o, d, row, n_actors); }
    void head(const char *action, uint8_t t, uint32_t obj) {
        sep();
        o += "{\"action\":\""; o += action; o += "\",\"type\":\""; o += TYPE_NAME[t & 3]; o += "\",\"obj\":";
        jstr(o, d.objs.ptr(obj), d.objs.len(obj));
    }
    void create(uint32_t obj, uint8_t t) {
        sep();
        o += "{\"action\":\"create\",\"obj\":";
        jstr(o, d.objs.ptr(obj), d.objs.len(obj));
        o += ",\"type\":\""; o += TYPE_NAME[t & 3]; o += "\"}";
    }
    void map_set(uint8_t t, uint32_t obj, uint32_t g, const hm_surv_result *sv, uint32_t n) {
        head("set", t, obj);
        o += ",\"key\":"; jstr(o, d.regs.ptr(g), d.regs.len(g)); o += ','; jentry(o, d, sv, n); o += '}';
    }
    void map_remove(uint8_t t, uint32_t obj, uint32_t g) {
        head("remove", t, obj);
        o += ",\"key\":"; jstr(o, d.regs.ptr(g), d.regs.len(g)); o += '}';
    }
    void list_remove(uint8_t t, uint32_t obj, uint32_t i) { head("remove", t, obj); o += ",\"index\":" + std::to_string(i) + '}'; }
    void list_insert(uint8_t t, uint32_t obj, uint32_t i, uint32_t g, const hm_surv_result *sv, uint32_t n) {
        head("insert", t, obj);
        o += ",\"index\":" + std::to_string(i) + ",\"elemId\":";
        jstr(o, d.regs.ptr(g), d.regs.len(g));
        o += ','; jentry(o, d, sv, n); o += '}';
    }
    void list_set(uint8_t t, uint32_t obj, uint32_t i, const hm_surv_result *sv, uint32_t n) {
        head("set", t, obj);
        o += ",\"index\":" + std::to_string(i) + ','; jentry(o, d, sv, n); o += '}';
    }
};

struct StrMap {                                              // (kind, id) -> local string index, per document
    std::vector<uint64_t> key;
    std::vector<uint32_t> val, gen;
    uint32_t g = 0, mask = 0;
    void reset() {
        if (key.empty()) { key.assign(256, 0); val.assign(256, 0); gen.assign(256, 0); mask = 255; }
        if (++g == 0) { std::fill(gen.begin(), gen.end(), 0u); g = 1; }
    }
    void grow() {
        std::vector<uint64_t> k2 = key; std::vector<uint32_t> v2 = val, g2 = gen;
        const size_t cap = key.size() * 2;
        key.assign(cap, 0); val.assign(cap, 0); gen.assign(cap, 0); mask = (uint32_t)cap - 1;
        for (size_t i = 0; i < k2.size(); i++) if (g2[i] == g) {
            uint32_t s = (uint32_t)mix64(k2[i]) & mask;
            while (gen[s] == g) s = (s + 1) & mask;
            key[s] = k2[i]; val[s] = v2[i]; gen[s] = g;
        }
    }
};

struct BinW {
    BinDoc &b;
    const DocSt &d;
    StrMap &m;
    uint32_t n_diffs = 0;
    size_t diffs_at = 0;
    uint32_t str(uint32_t kind, uint32_t id) {
        const uint64_t k = ((uint64_t)kind << 32) | id;
        if ((b.strs.size() + 1) * 2 > m.key.size()) m.grow();
        uint32_t s = (uint32_t)mix64(k) & m.mask;
        while (m.gen[s] == m.g) { if (m.key[s] == k) return m.val[s]; s = (s + 1) & m.mask; }
        const Names &nm = kind == 0 ? d.actors : kind == 1 ? d.objs : kind == 2 ? d.regs : d.strs;
        const char *p = nm.ptr(id);
        const uint32_t n = nm.len(id);
        for (uint32_t i = 0; i + 2 < n; i++) if ((unsigned char)p[i] == 0xED && ((unsigned char)p[i + 1] & 0xE0) == 0xA0) b.exotic = true;
        m.key[s] = k; m.val[s] = (uint32_t)b.strs.size(); m.gen[s] = m.g;
        b.strs.emplace_back(p, n);
        return (uint32_t)b.strs.size() - 1;
    }
    void clock(const uint32_t *row, uint32_t n_actors) {
        const size_t at = b.w.size();
        b.w.push_back(0);
        for (uint32_t r = 0; r < n_actors; r++) {
            if (!row[r]) continue;
            b.w.push_back(str(0, d.by_rank[r]));
            b.w.push_back(row[r]);
            b.w[at]++;
        }
    }
    void begin() { diffs_at = b.w.size(); b.w.push_back(0); }
    void end() { b.w[diffs_at] = n_diffs; }
    void head(uint32_t action, uint8_t t, uint32_t obj) { n_diffs++; b.w.push_back(action | (uint32_t)(t & 3) << 3); b.w.push_back(str(1, obj)); }
    void value(const hm_surv_result &s) {
        const uint8_t dt = s.op < d.op_dt.size() ? d.op_dt[s.op] : 0;
        uint32_t payload = 0;
        switch (s.vtag) {
        case HM_V_INT: payload = (uint32_t)b.nums.size(); b.nums.push_back((double)(int64_t)s.value); break;
        case HM_V_FLOAT: { double v; memcpy(&v, &s.value, 8); payload = (uint32_t)b.nums.size(); b.nums.push_back(v); break; }
        case HM_V_STR: payload = str(3, (uint32_t)s.value); break;
        case HM_V_OBJ: payload = str(1, (uint32_t)s.value); break;
        default: break;
        }
        b.w.push_back((s.vtag & 7) | (uint32_t)(dt & 3) << 3 | payload << 5);
    }
    void entry(const hm_surv_result *sv, uint32_t n) {
        b.w.push_back(n);
        value(sv[0]);
        for (uint32_t i = 1; i < n; i++) {
            b.w.push_back(str(0, sv[i].op < d.op_actor.size() ? d.op_actor[sv[i].op] : 0));
            value(sv[i]);
        }
    }
    void create(uint32_t obj, uint8_t t) { head(0, t, obj); }
    void map_set(uint8_t t, uint32_t obj, uint32_t g, const hm_surv_result *sv, uint32_t n) { head(1, t, obj); b.w.push_back(str(2, g)); entry(sv, n); }
    void map_remove(uint8_t t, uint32_t obj, uint32_t g) { head(2, t, obj); b.w.push_back(str(2, g)); }
    void list_remove(uint8_t t, uint32_t obj, uint32_t i) { head(2, t, obj); b.w.push_back(i); }
    void list_insert(uint8_t t, uint32_t obj, uint32_t i, uint32_t g, const hm_surv_result *sv, uint32_t n) {
        head(3, t, obj); b.w.push_back(i); b.w.push_back(str(2, g)); entry(sv, n);
    }
    void list_set(uint8_t t, uint32_t obj, uint32_t i, const hm_surv_result *sv, uint32_t n) { head(1, t, obj); b.w.push_back(i); entry(sv, n); }
};

// A document's binary patch as the JSON form (the exotic-string fallback: JSON escapes lone
// surrogates, the binary blob cannot carry them through Buffer.toString)
void bin_to_json(const BinDoc &b, std::string &patch, std::string &bclock, std::string &cclock) {
    size_t p = 0;
    const auto &w = b.w;
    auto S = [&](uint32_t i, std::string &o) { jstr(o, b.strs[i].first, b.strs[i].second); };
    auto clock = [&](std::string &o) {
        const uint32_t n = w[p++];
        o += '{';
        for (uint32_t i = 0; i < n; i++) {
            if (i) o += ',';
            S(w[p], o);
            o += ':' + std::to_string(w[p + 1]);
            p += 2;
        }
        o += '}';
    };
    auto value = [&](std::string &o) {
        const uint32_t v = w[p++], tag = v & 7, dt = (v >> 3) & 3, pay = v >> 5;
        o += "\"value\":";
        switch (tag) {
        case HM_V_NULL: o += "null"; break;
        case HM_V_FALSE: o += "false"; break;
        case HM_V_TRUE: o += "true"; break;
        case HM_V_INT: case HM_V_FLOAT: { uint64_t bits; memcpy(&bits, &b.nums[pay], 8); jnum(o, HM_V_FLOAT, bits); break; }
        case HM_V_STR: S(pay, o); break;
        case HM_V_OBJ: S(pay, o); o += ",\"link\":true"; break;
        default: o += "null";
        }
        if (dt == HM_DT_COUNTER) o += ",\"datatype\":\"counter\"";
        else if (dt == HM_DT_TIMESTAMP) o += ",\"datatype\":\"timestamp\"";
    };
    auto entry = [&](std::string &o) {
        const uint32_t n = w[p++];
        value(o);
        if (n <= 1) return;
        o += ",\"conflicts\":[";
        for (uint32_t i = 1; i < n; i++) {
            if (i > 1) o += ',';
            o += "{\"actor\":";
            S(w[p++], o);
            o += ',';
            value(o);
            o += '}';
        }
        o += ']';
    };
    std::string &o = patch;
    o += "{\"clock\":"; clock(o);
    o += ",\"deps\":"; clock(o);
    clock(bclock);
    clock(cclock);
    o += ",\"canUndo\":false,\"canRedo\":false,\"diffs\":[";
    const uint32_t nd = w[p++];
    for (uint32_t k = 0; k < nd; k++) {
        if (k) o += ',';
        const uint32_t hd = w[p++], action = hd & 7, t = (hd >> 3) & 3;
        const bool list = t >= 2;
        static const char *ACT[4] = {"create", "set", "remove", "insert"};
        if (action == 0) {
            o += "{\"action\":\"create\",\"obj\":"; S(w[p++], o);
            o += ",\"type\":\""; o += TYPE_NAME[t]; o += "\"}";
            continue;
        }
        o += "{\"action\":\""; o += ACT[action]; o += "\",\"type\":\""; o += TYPE_NAME[t]; o += "\",\"obj\":";
        S(w[p++], o);
        if (!list) {
            o += ",\"key\":"; S(w[p++], o);
            if (action == 1) { o += ','; entry(o); }
        } else {
            o += ",\"index\":" + std::to_string(w[p++]);
            if (action == 3) { o += ",\"elemId\":"; S(w[p++], o); }
            if (action != 2) { o += ','; entry(o); }
        }
        o += '}';
    }
    o += "]}";
}

// The diffs that take the patch base to the registers' new state (hm_reg_result rows of the
// requested registers, survivors at `surv`): objects created first, then map keys in
// request order, then per list removals (descending old index), insertions (ascending new
// index) and value changes.  The base is advanced to the new state.
template <typename W>
void render_diffs(W &w, DocSt &d, const uint32_t *req, const hm_reg_result *rows, const hm_surv_result *surv, uint32_t n) {
    for (uint32_t ob = 1; ob < d.obj_type.size(); ob++) {
        if (d.obj_type[ob] == NO_TYPE || d.obj_emitted[ob]) continue;
        d.obj_emitted[ob] = 1;
        w.create(ob, d.obj_type[ob]);
    }
    struct LOp { uint32_t g, idx, q; };
    struct LD { uint32_t obj; std::vector<uint32_t> rem; std::vector<LOp> ins, set; };
    std::vector<LD> lds;
    for (uint32_t q = 0; q < n; q++) {
        const uint32_t g = req[q];
        const hm_reg_result &r = rows[q];
        if (r.obj == HM_NONE || r.obj >= d.obj_type.size()) continue;
        const uint8_t t = d.obj_type[r.obj] == NO_TYPE ? HM_MAKE_MAP : d.obj_type[r.obj];
        const bool list = t == HM_MAKE_LIST || t == HM_MAKE_TEXT;
        const uint64_t sg = entry_sig(d, surv + r.surv_off, r.n_surv);
        const uint64_t old = d.sig[g];
        if (!list) {
            if (sg == old) continue;
            d.sig[g] = sg;
            if (sg) w.map_set(t, r.obj, g, surv + r.surv_off, r.n_surv);
            else w.map_remove(t, r.obj, g);
            continue;
        }
        const bool vis = r.n_surv > 0 && r.list_index >= 0;
        const uint64_t ns = vis ? sg : 0;
        if (ns == old) continue;
        LD *L = nullptr;
        for (auto &x : lds) if (x.obj == r.obj) L = &x;
        if (!L) { lds.push_back(LD{r.obj, {}, {}, {}}); L = &lds.back(); }
        std::vector<uint32_t> &el = *d.list_of(r.obj, true);
        if (old && !vis) L->rem.push_back((uint32_t)(std::find(el.begin(), el.end(), g) - el.begin()));
        else (old ? L->set : L->ins).push_back(LOp{g, (uint32_t)r.list_index, q});
        d.sig[g] = ns;
    }
    for (auto &L : lds) {
        std::vector<uint32_t> &el = *d.list_of(L.obj, true);
        const uint8_t t = d.obj_type[L.obj];
        std::sort(L.rem.begin(), L.rem.end(), std::greater<uint32_t>());
        for (uint32_t i : L.rem) {
            if (i >= el.size()) continue;
            el.erase(el.begin() + i);
            w.list_remove(t, L.obj, i);
        }
        std::stable_sort(L.ins.begin(), L.ins.end(), [](const LOp &a, const LOp &b) { return a.idx < b.idx; });
        for (auto &x : L.ins) {
            const uint32_t i = std::min<uint32_t>(x.idx, (uint32_t)el.size());
            el.insert(el.begin() + i, x.g);
            w.list_insert(t, L.obj, i, x.g, surv + rows[x.q].surv_off, rows[x.q].n_surv);
        }
        for (auto &x : L.set) {
            const uint32_t i = (uint32_t)(std::find(el.begin(), el.end(), x.g) - el.begin());
            w.list_set(t, L.obj, i, surv + rows[x.q].surv_off, rows[x.q].n_surv);
        }
    }
}

// ---------------- per-op diffs (Automerge makePatch) ----------------
// Automerge collects one diff per applied op, in application order: `create` per make op,
// per map assign the key's state after it (`set` with the winner and its conflicts, or
// `remove`), per list-element assign `insert` / `set` / `remove` at the element's index at
// that moment, nothing for `ins` (oracle/js/backend.js:92-170 restates the same sequence).
// The GPU fixes what was applied and in which order (the round's history slice, with every
// applied change's allDeps row: hm_store_read_history); the renderer walks those changes' ops
// over the patch base — per register the survivors the previous op left, per list the
// insertion tree and document order of the placed elements — applying exactly
// applyAssign's filter (isConcurrent reduces to allDeps(new)[x.actor] < x.seq: nothing
// resident depends on the new op), inc's counter sums and the sortBy(actor).reverse(), and
// RGA placement ((elem, actor) descending siblings, pre-order), to know each op's diff.  The
// registers it ends on are compared with the device's merged registers afterwards.
struct Replay {
    DocSt &d;
    uint32_t S;
    static uint32_t pkey(const hm_op_row &o) { return o.parent == HM_HEAD ? (0x80000000u | o.obj) : o.parent; }
    static uint32_t find(const std::vector<uint32_t> &v, uint32_t x) {
        return (uint32_t)(std::find(v.begin(), v.end(), x) - v.begin());
    }
    uint32_t rank(uint32_t op) const { return d.rank_of[d.op_actor[op]]; }
    // lamportCompare (elem, actor) of two element registers: a after b in sibling order?
    bool sib_before(uint32_t a, uint32_t b) const {
        const uint32_t oa = d.el_op[a], ob = d.el_op[b];
        if (d.oplog[oa].elem != d.oplog[ob].elem) return d.oplog[oa].elem > d.oplog[ob].elem;
        return rank(oa) > rank(ob);
    }
    // applyInsert: the element joins its parent's children; once its chain reaches _head it
    // (and any subtree inserted under it earlier) takes its pre-order place
    void insert(uint32_t k) {
        const hm_op_row &o = d.oplog[k];
        const uint32_t e = o.reg;
        d.el_op[e] = k;
        std::vector<uint32_t> &sib = d.kids[pkey(o)];
        uint32_t i = 0;
        while (i < sib.size() && sib_before(sib[i], e)) i++;
        sib.insert(sib.begin() + i, e);
        if (o.parent != HM_HEAD && !(o.parent < d.el_in.size() && d.el_in[o.parent])) return;
        ListOrder &ov = d.order_of(o.obj);
        uint32_t pos;
        if (i == 0) pos = o.parent == HM_HEAD ? 0u : ov.pos_of(o.parent, d.el_blk) + 1;
        else if (i + 1 < sib.size()) pos = ov.pos_of(sib[i + 1], d.el_blk);
        else {                                               // after the parent's subtree
            pos = ov.size();
            for (uint32_t x = o.parent; x != HM_HEAD;) {
                const hm_op_row &xo = d.oplog[d.el_op[x]];
                const std::vector<uint32_t> &xs = d.kids[pkey(xo)];
                const uint32_t j = find(xs, x);
                if (j + 1 < xs.size()) { pos = ov.pos_of(xs[j + 1], d.el_blk); break; }
                x = xo.parent;
            }
        }
        std::vector<uint32_t> sub, stk{e};
        while (!stk.empty()) {
            const uint32_t x = stk.back();
            stk.pop_back();
            sub.push_back(x);
            d.el_in[x] = 1;
            auto it = d.kids.find(x);
            if (it != d.kids.end())
                for (size_t c = it->second.size(); c-- > 0;) stk.push_back(it->second[c]);
        }
        ov.insert_at(pos, sub, d.el_blk, [&](uint32_t x) { return !d.rs[x].empty(); });
    }
    uint32_t visible_before(uint32_t obj, uint32_t e) {
        return d.order_of(obj).vis_before(e, d.el_blk, [&](uint32_t x) { return !d.rs[x].empty(); });
    }
    static bool numeric(uint32_t vt) { return vt == HM_V_INT || vt == HM_V_FLOAT; }
    static double num(uint32_t vt, uint64_t v) {
        if (vt == HM_V_INT) return (double)(int64_t)v;
        double x;
        memcpy(&x, &v, 8);
        return x;
    }
    // applyAssign (A.2) of op k of a change whose allDeps row is ad
    template <typename W>
    void assign(W &w, uint32_t k, const uint32_t *ad) {
        const hm_op_row &o = d.oplog[k];
        std::vector<hm_surv_result> &sv = d.rs[o.reg];
        const bool was = !sv.empty();
        auto concurrent = [&](const hm_surv_result &x) {
            const uint32_t r = rank(x.op);
            return (r < S ? ad[r] : 0u) < d.op_seq[x.op];
        };
        if (o.action == HM_INC) {
            for (hm_surv_result &x : sv) {
                if (d.oplog[x.op].datatype != HM_DT_COUNTER || !numeric(x.vtag) || concurrent(x)) continue;
                if (x.vtag == HM_V_INT && o.vtag == HM_V_INT) x.value = (uint64_t)((int64_t)x.value + (int64_t)o.value);
                else {
                    const double r = num(x.vtag, x.value) + num(o.vtag, o.value);
                    memcpy(&x.value, &r, 8);
                    x.vtag = HM_V_FLOAT;
                }
            }
        } else {
            sv.erase(std::remove_if(sv.begin(), sv.end(), [&](const hm_surv_result &x) { return !concurrent(x); }), sv.end());
        }
        if (o.action == HM_SET || o.action == HM_LINK) {
            hm_surv_result y;
            y.op = k; y.vtag = o.vtag; y.value = o.value;
            sv.push_back(y);
        }
        // sortBy(actor).reverse() = reversed, then a stable sort by actor descending (insertion
        // sort: a register holds a handful of survivors)
        std::reverse(sv.begin(), sv.end());
        for (size_t i = 1; i < sv.size(); i++) {
            const hm_surv_result x = sv[i];
            const uint32_t rx = rank(x.op);
            size_t j = i;
            for (; j > 0 && rank(sv[j - 1].op) < rx; j--) sv[j] = sv[j - 1];
            sv[j] = x;
        }
        const uint8_t t = o.obj < d.obj_type.size() && d.obj_type[o.obj] != NO_TYPE ? d.obj_type[o.obj] : (uint8_t)HM_MAKE_MAP;
        if (was != !sv.empty() && o.reg < d.el_in.size() && d.el_in[o.reg])   // a placed element's visibility
            d.order_of(o.obj).vis_change(o.reg, d.el_blk, !sv.empty());
        if (t != HM_MAKE_LIST && t != HM_MAKE_TEXT) {
            if (sv.empty()) w.map_remove(t, o.obj, o.reg);
            else w.map_set(t, o.obj, o.reg, sv.data(), (uint32_t)sv.size());
            return;
        }
        // updateListElement
        if (was) {
            const uint32_t i = visible_before(o.obj, o.reg);
            if (sv.empty()) w.list_remove(t, o.obj, i);
            else w.list_set(t, o.obj, i, sv.data(), (uint32_t)sv.size());
        } else if (!sv.empty() && o.reg < d.el_in.size() && d.el_in[o.reg]) {
            w.list_insert(t, o.obj, visible_before(o.obj, o.reg), o.reg, sv.data(), (uint32_t)sv.size());
        }
    }
    // the round: n applied changes (log indices, application order) with their allDeps rows
    template <typename W>
    void round(W &w, const uint32_t *log, const uint32_t *ads, uint32_t n, std::vector<uint32_t> &touched) {
        for (uint32_t r = 0; r < n; r++) {
            const uint32_t ci = log[r];
            const uint32_t k0 = d.ch_op0[ci], k1 = ci + 1 < d.ch_op0.size() ? d.ch_op0[ci + 1] : (uint32_t)d.oplog.size();
            for (uint32_t k = k0; k < k1; k++) {
                const hm_op_row &o = d.oplog[k];
                if (o.action <= HM_MAKE_TEXT) { w.create(o.obj, o.action); continue; }
                if (o.action == HM_INS) { insert(k); continue; }
                if (o.reg == HM_NONE || o.reg >= d.rs.size()) continue;
                assign(w, k, ads + (size_t)r * S);
                touched.push_back(o.reg);
            }
        }
        std::sort(touched.begin(), touched.end());
        touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
    }
};

// a replayed register against the device's merged register (numbers compared by value)
bool same_register(const DocSt &d, uint32_t g, const hm_reg_result &r, const hm_surv_result *sv) {
    const std::vector<hm_surv_result> &h = d.rs[g];
    if (h.size() != r.n_surv) return false;
    for (uint32_t i = 0; i < r.n_surv; i++) {
        const hm_surv_result &a = h[i], &b = sv[r.surv_off + i];
        if (a.op != b.op) return false;
        if (Replay::numeric(a.vtag) && Replay::numeric(b.vtag)) {
            if (Replay::num(a.vtag, a.value) != Replay::num(b.vtag, b.value)) return false;
        } else if (a.vtag != b.vtag || a.value != b.value) return false;
    }
    return true;
}

// the document as the patch base holds it: {uuid: {type, keys: [[key, entry]], elems: [[elemId, entry]]}}
void render_view(std::string &o, const DocSt &d, const hm_reg_result *rows, const hm_surv_result *surv, uint32_t n_regs) {
    std::vector<std::string> keys(d.obj_type.size()), elems(d.obj_type.size());
    std::vector<std::vector<std::pair<int32_t, uint32_t>>> order(d.obj_type.size());
    std::string tmp;
    for (uint32_t g = 0; g < n_regs; g++) {
        const hm_reg_result &r = rows[g];
        if (!r.n_surv || r.obj == HM_NONE || r.obj >= d.obj_type.size()) continue;
        const uint8_t t = d.obj_type[r.obj] == NO_TYPE ? HM_MAKE_MAP : d.obj_type[r.obj];
        if (t == HM_MAKE_LIST || t == HM_MAKE_TEXT) { if (r.list_index >= 0) order[r.obj].push_back({r.list_index, g}); continue; }
        std::string &k = keys[r.obj];
        if (!k.empty()) k += ',';
        k += '[';
        jstr(k, d.regs.ptr(g), d.regs.len(g));
        k += ",{";
        jentry(k, d, surv + r.surv_off, r.n_surv);
        k += "}]";
    }
    o += '{';
    for (uint32_t ob = 0; ob < d.obj_type.size(); ob++) {
        if (d.obj_type[ob] == NO_TYPE && keys[ob].empty() && order[ob].empty()) continue;
        if (o.size() > 1) o += ',';
        jstr(o, d.objs.ptr(ob), d.objs.len(ob));
        const uint8_t t = d.obj_type[ob] == NO_TYPE ? HM_MAKE_MAP : d.obj_type[ob];
        o += ":{\"type\":\""; o += TYPE_NAME[t & 3]; o += "\",\"keys\":[";
        o += keys[ob];
        o += "],\"elems\":[";
        std::sort(order[ob].begin(), order[ob].end());
        for (size_t i = 0; i < order[ob].size(); i++) {
            const uint32_t g = order[ob][i].second;
            if (i) o += ',';
            o += '[';
            jstr(o, d.regs.ptr(g), d.regs.len(g));
            o += ",{";
            jentry(o, d, surv + rows[g].surv_off, rows[g].n_surv);
            o += "}]";
        }
        o += "]}";
    }
    o += '}';
}

}  // namespace

struct hm_docset {
    hm_engine *e = nullptr;
    uint32_t threads = 16;
    bool patches = true;
    bool binary = false;                                     // HM_DOCSET_BINARY results
    bool op_diffs = true;                                    // Automerge's per-op diff sequence (else HM_DOCSET_NET_DIFFS)
    hm_store *stores[N_CLASS] = {};
    std::vector<uint32_t> free_h[N_CLASS];                   // released handles (empty documents), reused first
    uint32_t opened[N_CLASS] = {};                           // handles opened per store
    // documents: fixed chunks, so hm_docset_open may run while a call works on earlier documents
    static constexpr uint32_t CHUNK = 4096;
    std::vector<std::unique_ptr<DocSt[]>> chunks;
    std::atomic<uint32_t> n_docs{0};
    std::mutex open_mu;
    std::atomic<bool> busy{false};
    bool broken = false;                                     // a failed call could not be undone on a store
    uint64_t routing[3] = {0, 0, 0};                         // document rounds: incremental, re-merged, handed back
    uint64_t stat[8] = {0, 0, 0, 0, 0, 0, 0, 0};           // rounds, docs, restrides, hit-register patches, full patches,
                                                             // per-op patches, replay mismatches, replay checks skipped
    DocSt &doc(uint32_t i) { return chunks[i / CHUNK][i % CHUNK]; }
};

struct hm_text {
    std::string s;
    std::vector<hm_doc_result> res;
};

namespace {

int store_of(hm_docset *ds, uint32_t c, hm_store **out) {
    if (!ds->stores[c]) {
        hm_store_config sc = {STRIDES[c], 0};
        const int r = hm_store_create(ds->e, &sc, &ds->stores[c]);
        if (r) return r;
    }
    *out = ds->stores[c];
    return HM_OK;
}

uint8_t class_for(uint32_t n_actors) {
    for (uint32_t c = 0; c < N_CLASS; c++) if (n_actors <= STRIDES[c]) return (uint8_t)c;
    return NO_CLASS;
}

struct Busy {
    hm_docset *ds;
    bool ok;
    explicit Busy(hm_docset *d) : ds(d) { bool f = false; ok = ds->busy.compare_exchange_strong(f, true); }
    ~Busy() { if (ok) ds->busy.store(false); }
};

int apply(hm_docset *ds, const uint8_t *data, const uint64_t *bo, const uint32_t *doc_block, const uint32_t *docs, uint32_t n,
          hm_text *out) {
    const uint32_t nd = ds->n_docs.load();
    {
        std::vector<uint8_t> seen(nd, 0);
        for (uint32_t i = 0; i < n; i++) {
            if (docs[i] >= nd || seen[docs[i]]) return hm_engine_fail(ds->e, HM_ERR_INVALID, "bad or repeated docset document");
            seen[docs[i]] = 1;
            if (doc_block[i] > doc_block[i + 1]) return hm_engine_fail(ds->e, HM_ERR_INVALID, "doc_block not ascending");
        }
    }
    const bool prof = getenv("HM_DOCSET_PROFILE") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (!prof) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[hm_docset] %-14s %9.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    };
    std::vector<Round> R(n);
    for (uint32_t i = 0; i < n; i++) { R[i].doc = docs[i]; R[i].b0 = doc_block[i]; R[i].b1 = doc_block[i + 1]; }
    const uint32_t T = std::min<uint32_t>(ds->threads, std::max<uint32_t>(1, n / 64));
    try {
        par_for(n, T, [&](uint32_t lo, uint32_t hi, uint32_t) {
            Scratch X;
            for (uint32_t i = lo; i < hi; i++) {
                DocSt &d = ds->doc(R[i].doc);
                decode_round(d, R[i], data, bo, X);
                if (R[i].status != HM_OK) { rollback(d, R[i]); R[i].started = false; }
            }
        });
    } catch (...) {
        // a decode ran out of memory: every document whose decode started goes back
        for (uint32_t i = 0; i < n; i++) if (R[i].started) rollback(ds->doc(R[i].doc), R[i]);
        throw;
    }
    mark("decode");
    // placement: a document lives in the narrowest class that holds its actors
    std::vector<std::vector<uint32_t>> by_cls(N_CLASS);
    for (uint32_t i = 0; i < n; i++) {
        Round &x = R[i];
        if (x.status != HM_OK) continue;
        DocSt &d = ds->doc(x.doc);
        uint8_t c = class_for(x.n_actors);
        if (d.cls != NO_CLASS && d.cls > c) c = d.cls;
        x.cls = c;
        x.placed = d.cls == NO_CLASS;
        x.moved = !x.placed && c != d.cls;
        x.handle = d.handle;
        by_cls[c].push_back(i);
    }
    struct ClsOut {
        std::vector<hm_doc_result> res;
        std::vector<uint32_t> clock, back, heads;
        uint64_t id = 0;
        bool sub = false, done = false;                      // submitted / waited (applied on the device)
    };
    std::vector<ClsOut> co(N_CLASS);
    uint64_t call_routing[3] = {0, 0, 0};                      // this call's routing (ds->routing once it commits)
    int rc = HM_OK;
    // fault injection for the tests (HM_DOCSET_INJECT_FAIL=wait:<k> fails the call after the k-th
    // class's batch is applied, =read after every class's; the call must then be undone everywhere)
    const char *inj = getenv("HM_DOCSET_INJECT_FAIL");
    const int inj_wait = inj && !strncmp(inj, "wait:", 5) ? atoi(inj + 5) : -1;
    const bool inj_read = inj && !strcmp(inj, "read");
    int n_waited = 0;
    for (uint32_t c = 0; c < N_CLASS && rc == HM_OK; c++) {
        auto &rows = by_cls[c];
        if (rows.empty()) continue;
        hm_store *st;
        if ((rc = store_of(ds, c, &st))) break;
        const uint32_t S = STRIDES[c];
        // fresh handles for placed and moved documents: released ones first, then new ones
        uint32_t fresh = 0;
        for (uint32_t i : rows) fresh += R[i].placed || R[i].moved;
        std::vector<uint32_t> fh;
        size_t next_fh = 0;
        {
            std::vector<uint32_t> &fl = ds->free_h[c];
            const size_t k = std::min<size_t>(fresh, fl.size());
            fh.assign(fl.end() - k, fl.end());
            fl.resize(fl.size() - k);
            uint32_t h0 = 0;
            if (fresh > k && (rc = hm_doc_open_n(st, fresh - (uint32_t)k, &h0))) { fl.insert(fl.end(), fh.begin(), fh.end()); break; }
            ds->opened[c] += fresh - (uint32_t)k;
            for (uint32_t j = 0; j < fresh - k; j++) fh.push_back(h0 + j);
        }
        std::vector<hm_doc_row> drows(rows.size());
        std::vector<hm_change_row> ch;
        std::vector<hm_dep_row> dp;
        std::vector<hm_op_row> op;
        std::vector<uint32_t> hand(rows.size());
        std::vector<uint8_t> remap;
        bool any_remap = false;
        for (uint32_t k = 0; k < rows.size(); k++) if (!R[rows[k]].moved && !R[rows[k]].placed && !R[rows[k]].remap.empty()) any_remap = true;
        if (any_remap) {
            remap.resize(rows.size() * (size_t)S);
            for (uint32_t k = 0; k < rows.size(); k++) for (uint32_t a = 0; a < S; a++) remap[(size_t)k * S + a] = (uint8_t)a;
        }
        size_t tc = 0, td = 0, to = 0;
        for (uint32_t i : rows) { tc += R[i].ch.size(); td += R[i].dp.size(); to += R[i].op.size(); }
        ch.reserve(tc); dp.reserve(td); op.reserve(to);
        for (uint32_t k = 0; k < rows.size(); k++) {
            Round &x = R[rows[k]];
            DocSt &d = ds->doc(x.doc);
            x.row = k;
            hm_doc_row &r = drows[k];
            r = hm_doc_row{};
            r.change_off = (uint32_t)ch.size(); r.dep_off = (uint32_t)dp.size(); r.op_off = (uint32_t)op.size();
            const uint32_t c0 = (uint32_t)ch.size(), d0 = (uint32_t)dp.size(), o0 = (uint32_t)op.size();
            if (x.placed || x.moved) { x.handle = fh[next_fh++]; x.fresh = true; }
            hand[k] = x.handle;
            if (x.moved) {
                // the whole log moves: its rows from the old store, ranks re-mapped to this round's
                ds->stat[2]++;
                hm_doc_info_t inf;
                hm_store *old = ds->stores[d.cls];
                if ((rc = hm_doc_info(old, d.handle, &inf))) break;
                std::vector<hm_change_row> lc(inf.n_changes);
                std::vector<hm_dep_row> ld(inf.n_deps);
                std::vector<hm_op_row> lo(inf.n_ops);
                if ((rc = hm_doc_log(old, d.handle, lc.data(), ld.data(), lo.data()))) break;
                for (auto &cr : lc) {
                    if (!x.remap.empty() && cr.actor < x.remap.size()) cr.actor = x.remap[cr.actor];
                    cr.dep_off += d0; cr.op_first += o0;
                    ch.push_back(cr);
                }
                for (auto &dr : ld) { if (!x.remap.empty() && dr.actor < x.remap.size()) dr.actor = x.remap[dr.actor]; dp.push_back(dr); }
                op.insert(op.end(), lo.begin(), lo.end());
            } else if (!x.placed && !x.remap.empty()) {
                for (size_t a = 0; a < x.remap.size(); a++) remap[(size_t)k * S + a] = x.remap[a];
            }
            const uint32_t d1 = (uint32_t)dp.size(), o1 = (uint32_t)op.size();
            for (auto cr : x.ch) { cr.dep_off += d1; cr.op_first += o1; ch.push_back(cr); }
            dp.insert(dp.end(), x.dp.begin(), x.dp.end());
            op.insert(op.end(), x.op.begin(), x.op.end());
            r.n_changes = (uint32_t)ch.size() - c0; r.n_deps = (uint32_t)dp.size() - d0; r.n_ops = (uint32_t)op.size() - o0;
            r.n_regs = x.n_regs; r.n_objs = x.n_objs; r.n_actors = x.n_actors;
            r.flags = (uint16_t)(x.flags | (x.moved ? d.flags : 0));
        }
        // handles taken but not handed to a document (a failed log read) are still empty
        ds->free_h[c].insert(ds->free_h[c].end(), fh.begin() + next_fh, fh.end());
        if (rc) break;
        hm_batch b = {};
        b.n_docs = (uint32_t)rows.size(); b.n_changes = (uint32_t)ch.size(); b.n_deps = (uint32_t)dp.size(); b.n_ops = (uint32_t)op.size();
        b.a_stride = S;
        b.docs = drows.data(); b.changes = ch.data(); b.deps = dp.data(); b.ops = op.data();
        if ((rc = hm_batch_submit(st, &b, hand.data(), any_remap ? remap.data() : nullptr, &co[c].id))) break;
        co[c].sub = true;
        ClsOut &O = co[c];
        O.res.resize(rows.size()); O.clock.resize(rows.size() * (size_t)S); O.back.resize(rows.size() * (size_t)S);
        O.heads.resize(rows.size() * (size_t)S);
        if ((rc = hm_batch_wait(st, O.id, O.res.data(), O.clock.data(), O.back.data(), O.heads.data()))) break;
        O.sub = false;
        O.done = true;
        {
            uint32_t r3[3] = {0, 0, 0};
            if (hm_store_last_routing(st, r3) == HM_OK)
                for (int k = 0; k < 3; k++) call_routing[k] += r3[k];     // (counted once the call commits)
        }
        if (n_waited++ == inj_wait) { rc = hm_engine_fail(ds->e, HM_ERR_DEVICE, "injected failure (HM_DOCSET_INJECT_FAIL)"); break; }
        for (uint32_t k = 0; k < rows.size(); k++) {
            Round &x = R[rows[k]];
            x.res = O.res[k];
            x.clock = O.clock.data() + (size_t)k * S; x.back = O.back.data() + (size_t)k * S; x.heads = O.heads.data() + (size_t)k * S;
        }
    }
    // released handles (a moved document's old one, a fresh one its document does not keep) go
    // back to their store as empty documents (hm_doc_reset) and are reused by later calls; their
    // rows are reclaimed when the store compacts
    std::vector<std::vector<uint32_t>> rel(N_CLASS);
    auto release = [&]() {
        for (uint32_t c = 0; c < N_CLASS; c++) {
            if (rel[c].empty()) continue;
            if (hm_doc_reset(ds->stores[c], rel[c].data(), (uint32_t)rel[c].size()) == HM_OK)
                ds->free_h[c].insert(ds->free_h[c].end(), rel[c].begin(), rel[c].end());
            rel[c].clear();
        }
    };
    // a call-level failure: the call is applied to no store — a store whose batch is in flight is
    // waited for, the batches already applied are undone (hm_batch_undo) — and every document of
    // the call rolls back on the host
    auto fail_call = [&](int why) {
        for (auto &v : rel) v.clear();                       // (every fresh handle is listed below)
        // a store whose batch cannot be waited for or undone keeps rows the host no longer
        // describes: the docset refuses every later call rather than diverge silently
        bool lost = false;
        for (uint32_t c = 0; c < N_CLASS; c++) {
            if (co[c].sub) {
                std::vector<hm_doc_result> tmp(by_cls[c].size());
                if (hm_batch_wait(ds->stores[c], co[c].id, tmp.data(), nullptr, nullptr, nullptr) == HM_OK) co[c].done = true;
                else lost = true;                              // submitted, neither waited for nor undoable
                co[c].sub = false;
            }
            if (co[c].done) {
                if (hm_batch_undo(ds->stores[c], co[c].id) != HM_OK) lost = true;
                co[c].done = false;
            }
        }
        for (uint32_t i = 0; i < n; i++) {
            Round &x = R[i];
            DocSt &d = ds->doc(x.doc);
            if (x.status == HM_OK) rollback(d, x);
            if (!x.fresh) continue;
            // a new document whose own merge failed was given its fresh handle above (an empty
            // document in its store); the handle goes back to the free list, so the document
            // must not keep it
            if (x.placed && d.cls == x.cls && d.handle == x.handle) { d.cls = NO_CLASS; d.handle = 0; }
            rel[x.cls].push_back(x.handle);
        }
        release();
        if (lost) ds->broken = true;
        return why;
    };
    if (rc) return fail_call(rc);
    mark("merge");
    // failed documents roll back; the registers and history slices each patch reads are requested
    // before any document's host state advances (a failed read then fails the call on every store)
    std::vector<std::vector<uint32_t>> qdocs(N_CLASS), qregs(N_CLASS), hreq(N_CLASS);
    std::vector<uint32_t> cap(N_CLASS, 0);
    for (uint32_t i = 0; i < n; i++) {
        Round &x = R[i];
        DocSt &d = ds->doc(x.doc);
        if (x.status == HM_OK && x.res.status != HM_OK) x.status = x.res.status;
        if (x.status != HM_OK) {
            if (x.cls != NO_CLASS) rollback(d, x);
            if (x.placed) { d.cls = x.cls; d.handle = x.handle; }          // an empty document in its store
            else if (x.moved) rel[x.cls].push_back(x.handle);               // it stays where it was
            continue;
        }
        x.prev_hist = d.hist_len;
        if (!ds->patches) continue;
        if (ds->op_diffs) { hreq[x.cls].push_back(i); continue; }
        x.full = !(d.n_queued == 0 && x.res.n_queued == 0 && x.res.hist_len - d.hist_len == x.ch.size());
        x.q0 = (uint32_t)qregs[x.cls].size();
        if (x.full) {
            for (uint32_t g = 0; g < x.n_regs; g++) { qdocs[x.cls].push_back(x.handle); qregs[x.cls].push_back(g); }
            ds->stat[4]++;
        } else {
            // the registers the round's set/del/link/inc ops hit, first hit first
            std::vector<uint32_t> &q = qregs[x.cls];
            for (const hm_op_row &o : x.op) {
                if (o.action < HM_SET || o.reg == HM_NONE) continue;
                bool dup = false;
                for (uint32_t j = x.q0; j < q.size() && !dup; j++) dup = q[j] == o.reg;
                if (dup) continue;
                q.push_back(o.reg);
                qdocs[x.cls].push_back(x.handle);
            }
            ds->stat[3]++;
        }
        x.q1 = (uint32_t)qregs[x.cls].size();
        cap[x.cls] += x.res.n_surv;
    }
    std::vector<std::vector<hm_reg_result>> rrows(N_CLASS);
    std::vector<std::vector<hm_surv_result>> rsurv(N_CLASS);
    if (inj_read) return fail_call(hm_engine_fail(ds->e, HM_ERR_DEVICE, "injected failure (HM_DOCSET_INJECT_FAIL)"));
    for (uint32_t c = 0; c < N_CLASS; c++) {
        if (qregs[c].empty()) continue;
        rrows[c].resize(qregs[c].size());
        rsurv[c].resize(std::max<uint32_t>(cap[c], 1));
        uint32_t got = 0;
        rc = hm_store_read_regs(ds->stores[c], (uint32_t)qregs[c].size(), qdocs[c].data(), qregs[c].data(), rrows[c].data(),
                                rsurv[c].data(), (uint32_t)rsurv[c].size(), &got);
        if (rc) return fail_call(rc);
    }
    // op diffs: each document's history slice of this round (the changes the GPU applied, in
    // application order) with their allDeps rows
    std::vector<std::vector<uint32_t>> hlog(N_CLASS), had(N_CLASS);
    for (uint32_t c = 0; c < N_CLASS; c++) {
        if (hreq[c].empty()) continue;
        const uint32_t m = (uint32_t)hreq[c].size();
        std::vector<uint32_t> hh(m), from(m), to(m), off(m + 1, 0);
        for (uint32_t k = 0; k < m; k++) {
            Round &x = R[hreq[c][k]];
            hh[k] = x.handle;
            to[k] = x.res.hist_len;
            from[k] = x.prev_hist;
            off[k + 1] = off[k] + (to[k] - from[k]);
            x.h0 = off[k]; x.h1 = off[k + 1];
        }
        hlog[c].resize(std::max(1u, off[m]));                 // (rounds that applied nothing: no rows)
        had[c].resize(std::max<size_t>(1, (size_t)off[m] * STRIDES[c]));
        rc = hm_store_read_history(ds->stores[c], m, hh.data(), from.data(), to.data(), off.data(), hlog[c].data(), had[c].data());
        if (rc) return fail_call(rc);
    }
    mark("read history");
    // commit: every successful document's host state advances with the device's (a call lists a
    // document once, so the documents advance in parallel; the released handles of moved documents
    // go to the shared lists first)
    for (uint32_t i = 0; i < n; i++)
        if (R[i].status == HM_OK && R[i].moved) { const DocSt &d = ds->doc(R[i].doc); rel[d.cls].push_back(d.handle); }
    par_for(n, T, [&](uint32_t lo, uint32_t hi, uint32_t) {
    for (uint32_t i = lo; i < hi; i++) {
        Round &x = R[i];
        if (x.status != HM_OK) continue;
        DocSt &d = ds->doc(x.doc);
        const uint32_t old_n_ops = d.n_ops;
        d.cls = x.cls; d.handle = x.handle;
        d.flags |= x.flags;
        d.n_changes += (uint32_t)x.ch.size();
        d.n_ops += (uint32_t)x.op.size();
        d.hist_len = x.res.hist_len; d.n_queued = x.res.n_queued;
        d.obj_type.resize(x.n_objs, NO_TYPE);
        d.obj_emitted.resize(x.n_objs, 0);
        d.sig.resize(x.n_regs, 0);
        for (const hm_op_row &o : x.op)
            if (o.action <= HM_MAKE_TEXT && o.obj < d.obj_type.size() && d.obj_type[o.obj] == NO_TYPE) d.obj_type[o.obj] = o.action;
        if (ds->patches && ds->op_diffs) {
            // the replay's view of the log (op indices are the store's: appended in order)
            for (const hm_change_row &c : x.ch) {
                d.ch_op0.push_back(old_n_ops + c.op_first);
                d.op_seq.insert(d.op_seq.end(), c.n_ops, c.seq);
            }
            d.oplog.insert(d.oplog.end(), x.op.begin(), x.op.end());
            d.rs.resize(x.n_regs);
            d.el_op.resize(x.n_regs, HM_NONE);
            d.el_in.resize(x.n_regs, 0);
            d.el_blk.resize(x.n_regs, HM_NONE);
        }
    }
    });
    for (int k = 0; k < 3; k++) ds->routing[k] += call_routing[k];
    mark("commit");
    release();
    mark("read regs");
    // render every document's patch and DocBackend.clock
    auto round_clock = [](const Round &x, uint32_t *rc) {      // this call's changes alone (updateClock(changes))
        for (uint32_t a = 0; a < HM_MAX_STRIDE; a++) rc[a] = 0;
        for (const hm_change_row &c : x.ch) if (c.actor < HM_MAX_STRIDE && c.seq > rc[c.actor]) rc[c.actor] = c.seq;
    };
    bool exotic = false;
    if (ds->binary) {
        par_for(n, std::min<uint32_t>(ds->threads, std::max<uint32_t>(1, n / 128)), [&](uint32_t lo, uint32_t hi, uint32_t) {
            StrMap m;
            for (uint32_t i = lo; i < hi; i++) {
                Round &x = R[i];
                if (x.status != HM_OK) continue;
                DocSt &d = ds->doc(x.doc);
                m.reset();
                BinW w{x.bin, d, m};
                x.bin.w.reserve(64);
                w.clock(x.clock, x.n_actors);
                w.clock(x.heads, x.n_actors);
                w.clock(x.back, x.n_actors);
                uint32_t rc[HM_MAX_STRIDE];
                round_clock(x, rc);
                w.clock(rc, x.n_actors);
                w.begin();
                if (ds->patches && ds->op_diffs) {
                    Replay rp{d, STRIDES[x.cls]};
                    rp.round(w, hlog[x.cls].data() + x.h0, had[x.cls].data() + (size_t)x.h0 * STRIDES[x.cls], x.h1 - x.h0, x.touched);
                } else if (ds->patches) {
                    if (x.q1 > x.q0) render_diffs(w, d, qregs[x.cls].data() + x.q0, rrows[x.cls].data() + x.q0, rsurv[x.cls].data(), x.q1 - x.q0);
                    else render_diffs(w, d, nullptr, nullptr, nullptr, 0);
                }
                w.end();
            }
        });
        for (auto &x : R) exotic |= x.bin.exotic;
    }
    if (!ds->binary || exotic) {
        par_for(n, std::min<uint32_t>(ds->threads, std::max<uint32_t>(1, n / 128)), [&](uint32_t lo, uint32_t hi, uint32_t) {
            for (uint32_t i = lo; i < hi; i++) {
                Round &x = R[i];
                if (x.status != HM_OK) continue;
                DocSt &d = ds->doc(x.doc);
                if (exotic) {                                  // the binary pass already advanced the patch base
                    // re-render from the words is not possible in JSON form without the base: rebuild
                    // the JSON from the binary document (same diffs, same order)
                    bin_to_json(x.bin, x.patch, x.bclock, x.cclock);
                    continue;
                }
                std::string &o = x.patch;
                o.reserve(256);
                JsonW w{o, d};
                o += "{\"clock\":";
                jclock(o, d, x.clock, x.n_actors);
                o += ",\"deps\":";
                jclock(o, d, x.heads, x.n_actors);
                o += ",\"canUndo\":false,\"canRedo\":false,\"diffs\":[";
                if (ds->patches && ds->op_diffs) {
                    Replay rp{d, STRIDES[x.cls]};
                    rp.round(w, hlog[x.cls].data() + x.h0, had[x.cls].data() + (size_t)x.h0 * STRIDES[x.cls], x.h1 - x.h0, x.touched);
                } else if (ds->patches) {
                    if (x.q1 > x.q0) render_diffs(w, d, qregs[x.cls].data() + x.q0, rrows[x.cls].data() + x.q0, rsurv[x.cls].data(), x.q1 - x.q0);
                    else render_diffs(w, d, nullptr, nullptr, nullptr, 0);
                }
                o += "]}";
                jclock(x.bclock, d, x.back, x.n_actors);
                uint32_t rc[HM_MAX_STRIDE];
                round_clock(x, rc);
                jclock(x.cclock, d, rc, x.n_actors);
            }
        });
    }
    mark("diffs");
    if (ds->patches && ds->op_diffs) {
        // the replay's registers against the device's merged registers
        for (uint32_t c = 0; c < N_CLASS; c++) {
            std::vector<uint32_t> vd, vr, vx;
            uint32_t vcap = 0;
            for (uint32_t i : hreq[c]) {
                Round &x = R[i];
                for (uint32_t g : x.touched) { vd.push_back(x.handle); vr.push_back(g); vx.push_back(i); }
                vcap += x.res.n_surv;
            }
            if (vr.empty()) continue;
            std::vector<hm_reg_result> gr(vr.size());
            std::vector<hm_surv_result> gs(std::max<uint32_t>(vcap, 1));
            uint32_t got = 0;
            // (a self-check of the committed round: a read that fails skips it, stat[7])
            if (hm_store_read_regs(ds->stores[c], (uint32_t)vr.size(), vd.data(), vr.data(), gr.data(), gs.data(),
                                   (uint32_t)gs.size(), &got) != HM_OK) { ds->stat[7]++; continue; }
            std::atomic<uint64_t> bad{0};
            const uint32_t nq = (uint32_t)vr.size();
            par_for(nq, std::min<uint32_t>(ds->threads, std::max<uint32_t>(1, nq / 4096)), [&](uint32_t lo, uint32_t hi, uint32_t) {
                uint32_t bad_doc = HM_NONE;
                uint64_t nb = 0;
                for (uint32_t q = lo; q < hi; q++) {
                    DocSt &d = ds->doc(R[vx[q]].doc);
                    bool ok = same_register(d, vr[q], gr[q], gs.data());
                    const uint32_t ob = gr[q].obj;
                    if (ok && !d.rs[vr[q]].empty() && ob < d.obj_type.size() &&
                        (d.obj_type[ob] == HM_MAKE_LIST || d.obj_type[ob] == HM_MAKE_TEXT)) {
                        Replay rp{d, STRIDES[c]};
                        ok = gr[q].list_index == (int32_t)rp.visible_before(ob, vr[q]);
                    }
                    if (!ok && bad_doc != vx[q]) { nb++; bad_doc = vx[q]; }
                }
                bad += nb;
            });
            ds->stat[6] += bad.load();
        }
        for (uint32_t c = 0; c < N_CLASS; c++) ds->stat[5] += hreq[c].size();
        mark("verify");
    }
    std::string &s = out->s;
    s.clear();
    if (ds->binary && !exotic) {
        // HMP1 layout: header u32[8] {magic, n_docs, n_strings, n_words, n_nums, blob_bytes, ascii, 0},
        // doc_word_off / doc_str_base / doc_num_base u32[n_docs + 1] each, str_off u32[n_strings + 1]
        // (byte offsets into the blob), words u32[n_words], (8-aligned) nums f64[n_nums], blob
        std::vector<uint32_t> wo(n + 1, 0), sb(n + 1, 0), nb(n + 1, 0);
        std::vector<uint64_t> bo(n + 1, 0);                  // each document's first blob byte
        for (uint32_t i = 0; i < n; i++) {
            const BinDoc &x = R[i].bin;
            wo[i + 1] = wo[i] + (uint32_t)x.w.size(); sb[i + 1] = sb[i] + (uint32_t)x.strs.size(); nb[i + 1] = nb[i] + (uint32_t)x.nums.size();
            uint64_t b = 0;
            for (auto &t : x.strs) b += t.second;
            bo[i + 1] = bo[i] + b;
        }
        const uint64_t blob = bo[n];
        const uint32_t ns = sb[n], nw = wo[n], nn = nb[n];
        size_t head = 4 * (8 + 3 * ((size_t)n + 1) + (size_t)ns + 1 + nw);
        const size_t pad = (8 - head % 8) % 8;
        s.resize(head + pad + 8 * (size_t)nn + blob);
        uint32_t *h = (uint32_t *)&s[0];
        h[0] = 0x31504D48u; h[1] = n; h[2] = ns; h[3] = nw; h[4] = nn; h[5] = (uint32_t)blob; h[6] = 1; h[7] = 0;
        uint32_t *p = h + 8;
        memcpy(p, wo.data(), 4 * ((size_t)n + 1)); p += n + 1;
        memcpy(p, sb.data(), 4 * ((size_t)n + 1)); p += n + 1;
        memcpy(p, nb.data(), 4 * ((size_t)n + 1)); p += n + 1;
        uint32_t *so = p;
        p += ns + 1;
        uint32_t *words = p;
        double *nums = (double *)(&s[0] + head + pad);
        char *bl = &s[0] + head + pad + 8 * (size_t)nn;
        so[0] = 0;
        // documents copied in parallel: every one has its own word / number / string ranges
        std::atomic<bool> ascii{true};
        par_for(n, std::min<uint32_t>(ds->threads, std::max<uint32_t>(1, n / 256)), [&](uint32_t lo, uint32_t hi, uint32_t) {
            bool asc = true;
            for (uint32_t i = lo; i < hi; i++) {
                const BinDoc &x = R[i].bin;
                if (!x.w.empty()) memcpy(words + wo[i], x.w.data(), 4 * x.w.size());
                if (!x.nums.empty()) memcpy(nums + nb[i], x.nums.data(), 8 * x.nums.size());
                uint64_t at = bo[i];
                uint32_t k = sb[i];
                for (auto &t : x.strs) {
                    memcpy(bl + at, t.first, t.second);
                    if (asc)
                        for (uint32_t c = 0; c < t.second; c++) asc &= (unsigned char)t.first[c] < 0x80;
                    at += t.second;
                    so[++k] = (uint32_t)at;
                }
            }
            if (!asc) ascii = false;
        });
        h[6] = ascii ? 1 : 0;
    } else {
        // {"p": [patch | null per document], "b": [max over the whole log | null], "c": [max over this call's changes | null]}
        size_t tot = 16;
        for (auto &x : R) tot += x.patch.size() + x.bclock.size() + x.cclock.size() + 18;
        s.reserve(tot);
        s += "{\"p\":[";
        for (uint32_t i = 0; i < n; i++) { if (i) s += ','; if (R[i].status == HM_OK) s += R[i].patch; else s += "null"; }
        s += "],\"b\":[";
        for (uint32_t i = 0; i < n; i++) { if (i) s += ','; if (R[i].status == HM_OK) s += R[i].bclock; else s += "null"; }
        s += "],\"c\":[";
        for (uint32_t i = 0; i < n; i++) { if (i) s += ','; if (R[i].status == HM_OK) s += R[i].cclock; else s += "null"; }
        s += "]}";
    }
    out->res.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        Round &x = R[i];
        hm_doc_result &r = out->res[i];
        if (x.cls == NO_CLASS && x.status != HM_OK) {                    // the call's blocks did not decode
            r = hm_doc_result{};
            r.status = x.status; r.err_change = x.err_block; r.err_op = HM_NONE;
            DocSt &d = ds->doc(x.doc);
            r.hist_len = d.hist_len; r.n_queued = d.n_queued;
        } else r = x.res;
    }
    ds->stat[0]++;
    ds->stat[1] += n;
    mark("render");
    return HM_OK;
}

}  // namespace

extern "C" {

int hm_docset_create(hm_engine *e, const hm_docset_config *cfg, hm_docset **out) {
    if (!e || !out) return HM_ERR_INVALID;
    *out = nullptr;
    hm_docset *ds = new (std::nothrow) hm_docset();
    if (!ds) return HM_ERR_NOMEM;
    ds->e = e;
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    ds->threads = cfg && cfg->threads ? cfg->threads : std::min<uint32_t>(16, hw);
    ds->patches = !(cfg && (cfg->flags & HM_DOCSET_NO_PATCHES));
    ds->binary = cfg && (cfg->flags & HM_DOCSET_BINARY);
    ds->op_diffs = !(cfg && (cfg->flags & HM_DOCSET_NET_DIFFS));
    ds->chunks.reserve(1u << 16);
    *out = ds;
    return HM_OK;
}

void hm_docset_destroy(hm_docset *ds) {
    if (!ds) return;
    for (auto *s : ds->stores) if (s) hm_store_destroy(s);
    delete ds;
}

hm_engine *hm_docset_engine(hm_docset *ds) { return ds ? ds->e : nullptr; }

int hm_docset_open(hm_docset *ds, uint32_t n, uint32_t *out_first) {
    if (!ds || !out_first) return HM_ERR_INVALID;
    try {
        std::lock_guard<std::mutex> g(ds->open_mu);
        const uint32_t first = ds->n_docs.load();
        const uint64_t need = (uint64_t)first + n;
        if (need > (uint64_t)hm_docset::CHUNK * (1u << 16)) return HM_ERR_NOMEM;
        while ((uint64_t)ds->chunks.size() * hm_docset::CHUNK < need) ds->chunks.emplace_back(new DocSt[hm_docset::CHUNK]);
        ds->n_docs.store((uint32_t)need);
        *out_first = first;
        return HM_OK;
    } catch (...) {
        return HM_ERR_NOMEM;
    }
}

int hm_docset_apply(hm_docset *ds, const uint8_t *data, const uint64_t *block_off, const uint32_t *doc_block,
                    const uint32_t *docs, uint32_t n_docs, hm_text **out) {
    if (!ds || !out || (n_docs && (!block_off || !doc_block || !docs))) return HM_ERR_INVALID;
    *out = nullptr;
    Busy b(ds);
    if (!b.ok) return hm_engine_fail(ds->e, HM_ERR_INVALID, "hm_docset_apply: another call on this docset is running");
    if (ds->broken)
        return hm_engine_fail(ds->e, HM_ERR_DEVICE, "hm_docset_apply: an earlier failed call could not be undone on its store");
    try {
        std::unique_ptr<hm_text> t(new hm_text());
        const int rc = apply(ds, data, block_off, doc_block, docs, n_docs, t.get());
        if (rc) return rc;
        *out = t.release();
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(ds->e, HM_ERR_NOMEM, "exception in hm_docset_apply");
    }
}

const char *hm_text_data(const hm_text *t, size_t *len) {
    if (!t) return nullptr;
    if (len) *len = t->s.size();
    return t->s.data();
}

const hm_doc_result *hm_text_results(const hm_text *t, uint32_t *n) {
    if (!t) return nullptr;
    if (n) *n = (uint32_t)t->res.size();
    return t->res.data();
}

void hm_text_free(hm_text *t) { delete t; }

int hm_docset_doc_info(hm_docset *ds, uint32_t doc, hm_docset_doc_info_t *out) {
    if (!ds || !out || doc >= ds->n_docs.load()) return HM_ERR_INVALID;
    Busy b(ds);
    if (!b.ok) return hm_engine_fail(ds->e, HM_ERR_INVALID, "docset busy");
    DocSt &d = ds->doc(doc);
    memset(out, 0, sizeof *out);
    out->a_stride = d.cls == NO_CLASS ? 0 : STRIDES[d.cls];
    out->n_changes = d.n_changes; out->n_ops = d.n_ops; out->n_actors = d.actors.size();
    out->n_objs = std::max<uint32_t>(1, d.objs.size()); out->n_regs = d.regs.size();
    out->hist_len = d.hist_len; out->n_queued = d.n_queued;
    return HM_OK;
}

int hm_docset_history_prefix(hm_docset *ds, uint32_t doc, uint32_t n, uint32_t *out) {
    if (!ds || doc >= ds->n_docs.load() || (n && !out)) return HM_ERR_INVALID;
    Busy b(ds);
    if (!b.ok) return hm_engine_fail(ds->e, HM_ERR_INVALID, "docset busy");
    DocSt &d = ds->doc(doc);
    if (d.cls == NO_CLASS) return 0;
    return hm_doc_history_prefix(ds->stores[d.cls], d.handle, n, out);
}

int hm_docset_clock_update(hm_docset *ds, uint32_t n, const uint32_t *docs, uint8_t *out_written, uint8_t *out_differs,
                           hm_text **out_stored) {
    if (!ds || (n && !docs)) return HM_ERR_INVALID;
    Busy b(ds);
    if (!b.ok) return hm_engine_fail(ds->e, HM_ERR_INVALID, "docset busy");
    try {
        const uint32_t nd = ds->n_docs.load();
        for (uint32_t i = 0; i < n; i++) if (docs[i] >= nd) return hm_engine_fail(ds->e, HM_ERR_INVALID, "bad docset document");
        std::vector<std::string> js(n, "{}");
        for (uint32_t c = 0; c < N_CLASS; c++) {
            std::vector<uint32_t> idx, hs;
            for (uint32_t i = 0; i < n; i++) if (ds->doc(docs[i]).cls == c) { idx.push_back(i); hs.push_back(ds->doc(docs[i]).handle); }
            if (idx.empty()) continue;
            const uint32_t S = STRIDES[c], k = (uint32_t)idx.size();
            std::vector<uint8_t> w(k), df(k);
            std::vector<uint32_t> stv((size_t)k * S);
            const int rc = hm_store_clock_update(ds->stores[c], k, hs.data(), w.data(), df.data(), stv.data());
            if (rc) return rc;
            for (uint32_t j = 0; j < k; j++) {
                const uint32_t i = idx[j];
                if (out_written) out_written[i] = w[j];
                if (out_differs) out_differs[i] = df[j];
                js[i].clear();
                const DocSt &d = ds->doc(docs[i]);
                jclock(js[i], d, stv.data() + (size_t)j * S, d.actors.size());
            }
        }
        for (uint32_t i = 0; i < n; i++) if (ds->doc(docs[i]).cls == NO_CLASS) {
            if (out_written) out_written[i] = 0;
            if (out_differs) out_differs[i] = 0;
        }
        if (out_stored) {
            std::unique_ptr<hm_text> t(new hm_text());
            t->s = "[";
            for (uint32_t i = 0; i < n; i++) { if (i) t->s += ','; t->s += js[i]; }
            t->s += ']';
            *out_stored = t.release();
        }
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(ds->e, HM_ERR_NOMEM, "exception in hm_docset_clock_update");
    }
}

int hm_docset_view(hm_docset *ds, uint32_t doc, hm_text **out) {
    if (!ds || !out || doc >= ds->n_docs.load()) return HM_ERR_INVALID;
    *out = nullptr;
    Busy b(ds);
    if (!b.ok) return hm_engine_fail(ds->e, HM_ERR_INVALID, "docset busy");
    try {
        DocSt &d = ds->doc(doc);
        if (!d.ready) d.setup();
        std::unique_ptr<hm_text> t(new hm_text());
        if (d.cls == NO_CLASS) {
            render_view(t->s, d, nullptr, nullptr, 0);
        } else {
            hm_doc_info_t inf;
            int rc = hm_doc_info(ds->stores[d.cls], d.handle, &inf);
            if (rc) return rc;
            std::vector<hm_reg_result> regs(inf.n_regs + 1);
            std::vector<hm_surv_result> surv(inf.n_ops + 1);
            rc = hm_doc_read(ds->stores[d.cls], d.handle, nullptr, nullptr, regs.data(), surv.data(), nullptr, nullptr, nullptr);
            if (rc) return rc;
            render_view(t->s, d, regs.data(), surv.data(), inf.n_regs);
        }
        *out = t.release();
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(ds->e, HM_ERR_NOMEM, "exception in hm_docset_view");
    }
}

int hm_docset_handles(const hm_docset *ds, uint32_t a_stride, uint32_t *out_opened, uint32_t *out_free) {
    if (!ds || !out_opened || !out_free) return HM_ERR_INVALID;
    for (uint32_t c = 0; c < N_CLASS; c++)
        if (STRIDES[c] == a_stride) { *out_opened = ds->opened[c]; *out_free = (uint32_t)ds->free_h[c].size(); return HM_OK; }
    return HM_ERR_INVALID;
}

int hm_docset_routing(const hm_docset *ds, uint64_t *out3) {
    if (!ds || !out3) return HM_ERR_INVALID;
    for (int k = 0; k < 3; k++) out3[k] = ds->routing[k];
    return HM_OK;
}

int hm_docset_stats(const hm_docset *ds, uint64_t *out8) {
    if (!ds || !out8) return HM_ERR_INVALID;
    for (int i = 0; i < 8; i++) out8[i] = ds->stat[i];
    return HM_OK;
}

}  // extern "C"
