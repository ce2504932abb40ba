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
// Documents decode in parallel (one thread per contiguous document range, each appending to its
// own tables, no per-name allocation); the string pool is merged afterwards in document order
// and the parts are laid end to end, so the rows are identical whatever the thread count.
// Brotli blocks use the system libbrotlidec (loaded on first use); without it a 'BR' block is
// an undecodable block.  An undecodable block (the reference's Block.unpack / JSON.parse
// throw) marks its document HM_ERR_INVALID with no rows; other documents are unaffected.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <type_traits>
#include <sys/mman.h>
#include <vector>
#include "../../include/hypermerge_amd.h"
#include "scan.h"

namespace {

using namespace hmscan;


// A growable table of POD rows in its own anonymous mapping: growth moves the pages
// (mremap) instead of copying them, and the mapping asks for transparent huge pages, so a
// table of hundreds of MB is not first-touched 4 KB at a time (page faults were the single
// largest cost of a cold batch).  Untouched capacity costs no memory.
template <typename T> struct Buf {
    static_assert(std::is_trivially_copyable<T>::value, "rows are POD");
    T *p = nullptr;
    size_t n = 0, cap = 0;
    Buf() = default;
    Buf(const Buf &) = delete;
    Buf &operator=(const Buf &) = delete;
    Buf(Buf &&o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
    Buf &operator=(Buf &&o) noexcept { if (this != &o) { release(); std::swap(p, o.p); std::swap(n, o.n); std::swap(cap, o.cap); } return *this; }
    ~Buf() { release(); }
    static size_t map_bytes(size_t k) {                     // 64 KB granules, 2 MB ones from 4 MB up
        const size_t b = std::max<size_t>(k * sizeof(T), 1), a = b >= ((size_t)4 << 20) ? (size_t)2 << 20 : (size_t)64 << 10;
        return (b + a - 1) / a * a;
    }
    void release() { if (p) munmap(p, map_bytes(cap)); p = nullptr; n = cap = 0; }
    void reserve(size_t k) {
        if (k <= cap) return;
        const size_t nb = map_bytes(std::max(k, cap * 2));
        void *q = p ? mremap(p, map_bytes(cap), nb, MREMAP_MAYMOVE)
                    : mmap(nullptr, nb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (q == MAP_FAILED) throw std::bad_alloc();
        if (nb >= ((size_t)4 << 20)) madvise(q, nb, MADV_HUGEPAGE);
        p = (T *)q;
        cap = nb / sizeof(T);
    }
    // capacity hint: a mapping the system refuses is left to growth on demand
    void try_reserve(size_t k) { try { reserve(k); } catch (const std::bad_alloc &) {} }
    void push_back(const T &v) { if (n == cap) reserve(n + 1); p[n++] = v; }
    void append(const T *v, size_t k) { reserve(n + k); if (k) memcpy(p + n, v, k * sizeof(T)); n += k; }
    void resize(size_t k) { reserve(k); n = k; }           // new rows are not initialised
    size_t size() const { return n; }
    bool empty() const { return !n; }
    T *data() { return p; }
    const T *data() const { return p; }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
};

// A list of byte strings in one buffer: entry i is blob[end[i - 1], end[i]).
struct StrTab {
    Buf<char> blob;
    Buf<uint64_t> end;
    void push(const char *p, size_t n) { blob.append(p, n); end.push_back(blob.size()); }
    size_t size() const { return end.size(); }
    const char *at(size_t i, size_t *len) const {
        const uint64_t b = i ? end[i - 1] : 0;
        if (len) *len = (size_t)(end[i] - b);
        return blob.data() + b;
    }
    void truncate(size_t k) { blob.resize(k ? end[k - 1] : 0); end.resize(k); }
};

// Per-thread bump allocator for the elemId names a document interns: stable addresses while
// the document's tables hold views of them, reused from document to document.
struct Bump {
    std::vector<std::pair<std::unique_ptr<char[]>, size_t>> chunks;
    size_t k = 0, used = 0;
    void reset() { k = 0; used = 0; }
    char *alloc(size_t n) {
        if (k >= chunks.size() || used + n > chunks[k].second) {
            if (k < chunks.size()) k++;
            used = 0;
            const size_t c = std::max<size_t>(n, 1 << 16);
            if (k == chunks.size()) chunks.emplace_back(std::unique_ptr<char[]>(new char[c]), c);
            else if (chunks[k].second < n) chunks[k] = {std::unique_ptr<char[]>(new char[c]), c};
        }
        char *r = chunks[k].first.get() + used;
        used += n;
        return r;
    }
    void give_back(size_t n) { used -= n; }                  // the tail of the last alloc
};

// One thread's output for its contiguous range of documents, in document order: the batch
// tables are the parts laid end to end.  Change dep / op offsets are relative to the part's
// tables; op string ids index the part's `strings` (remapped to the batch pool at the merge).
struct Part {
    struct Doc { int32_t status; uint32_t n_ch, n_dp, n_op, n_str, n_act, n_obj, n_reg; uint16_t flags; };
    std::vector<Doc> docs;
    Buf<hm_change_row> ch;
    Buf<hm_dep_row> dp;
    Buf<hm_op_row> op;
    Buf<uint8_t> op_str;                                     // per op: bit 0 key, bit 1 value is a string id
    StrTab strings;                                          // each document's, in first-appearance order
    Buf<uint64_t> str_h;                                     // their hash_bytes(., 0)
    StrTab actors, objs, regs;                               // rank -> actor id, object id -> uuid, register -> key | elemId
    Buf<uint32_t> reg_obj;                                   // register -> object
    struct Mark { size_t ch, dp, op, str, act, obj, reg; };
    Mark mark() const { return {ch.size(), dp.size(), op.size(), strings.size(), actors.size(), objs.size(), regs.size()}; }
    void rollback(const Mark &m) {
        ch.resize(m.ch); dp.resize(m.dp); op.resize(m.op); op_str.resize(m.op);
        strings.truncate(m.str); str_h.resize(m.str);
        actors.truncate(m.act); objs.truncate(m.obj); regs.truncate(m.reg); reg_obj.resize(m.reg);
    }
};


bool decode_doc(const uint8_t *data, const uint64_t *block_off, uint32_t b0, uint32_t b1, Part &D, Part::Doc &doc,
                Ctx &cx, Bump &bump) {
    const uint32_t n = b1 - b0;
    const Part::Mark m0 = D.mark();
    cx.arena.clear();
    bump.reset();
    cx.cs.assign(n, ScanChange());
    cx.ops.clear();
    cx.deps.clear();
    cx.actors.reset(16);
    for (uint32_t i = 0; i < n; i++) {
        const char *s = (const char *)data + block_off[b0 + i];
        size_t len = (size_t)(block_off[b0 + i + 1] - block_off[b0 + i]);
        if (len >= 2 && s[0] == 'B' && s[1] == 'R') {
            cx.arena.emplace_back();
            if (!brotli_decompress((const uint8_t *)s + 2, len - 2, cx.arena.back())) return false;
            s = cx.arena.back().data(); len = cx.arena.back().size();
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
    for (uint32_t r = 0; r < na; r++) { cx.rank[order[r]] = r; D.actors.push(an[order[r]].s.p, an[order[r]].s.n); }

    const size_t nops = cx.ops.size();
    cx.objs.reset(8); cx.strs.reset(nops); cx.regs.reset(nops);
    bool fresh;
    cx.objs.get(SV{ROOT_ID, 36}, 0, fresh);
    D.objs.push(ROOT_ID, 36);
    SV last_obj{ROOT_ID, 36};
    uint32_t last_obj_id = 0;
    auto obj = [&](const SV &u) {
        if (u == last_obj) return last_obj_id;
        const uint32_t id = cx.objs.get(u, 0, fresh);
        last_obj = u; last_obj_id = id;
        if (fresh) D.objs.push(u.p, u.n);
        return id;
    };
    auto reg = [&](uint32_t o, const SV &k) {
        const uint32_t id = cx.regs.get(k, o, fresh);
        if (fresh) { D.regs.push(k.p, k.n); D.reg_obj.push_back(o); }
        return id;
    };
    const uint32_t str0 = (uint32_t)m0.str;                  // string ids are part-relative
    auto str = [&](const SV &v) {
        const uint32_t id = cx.strs.get(v, 0, fresh);
        if (fresh) { D.strings.push(v.p, v.n); D.str_h.push_back(cx.strs.keys[id].h); }
        return str0 + id;
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
    uint16_t flags = 0;
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
        const SV &author = an[order[row.actor]].s;
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
                // elemId `${actor}:${elem}`
                const size_t cap = (size_t)author.n + 41;
                char *el = bump.alloc(cap);
                memcpy(el, author.p, author.n);
                el[author.n] = ':';
                const uint32_t len = author.n + 1 + js_num_text(o.elem, el + author.n + 1);
                bump.give_back(cap - len);
                r.reg = reg(r.obj, SV{el, len});
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
                    } else if (o.vt == J_STR) { r.vtag = HM_V_STR; r.value = str(o.sval); sv = 2; }
                    else return false;                                        // 'unsupported op value'
                }
            }
            r.datatype = o.datatype;
            r.action = (uint8_t)a;
            if (a == HM_MAKE_LIST || a == HM_MAKE_TEXT) flags |= HM_DOC_HAS_LISTS;
            if (a == HM_INC || r.datatype == HM_DT_COUNTER) flags |= HM_DOC_HAS_COUNTERS;
            D.op.push_back(r);
            D.op_str.push_back(sk | sv);
        }
        row.n_ops = c.nops;
        D.ch.push_back(row);
    }
    doc.status = HM_OK;
    doc.n_ch = n;
    doc.n_dp = (uint32_t)(D.dp.size() - m0.dp);
    doc.n_op = (uint32_t)(D.op.size() - m0.op);
    doc.n_str = (uint32_t)(D.strings.size() - m0.str);
    doc.n_act = na;
    doc.n_obj = (uint32_t)(D.objs.size() - m0.obj);
    doc.n_reg = (uint32_t)(D.regs.size() - m0.reg);
    doc.flags = flags;
    return true;
}

}  // namespace

// a table of POD rows written once by the decoder threads (no zero fill before they write it)
template <typename T> struct Rows : Buf<T> {
    void alloc(size_t k) { this->resize(k); }
};

// the batch's name tables (every document's entries, laid end to end)
struct NameTab {
    Rows<char> blob;
    Rows<uint64_t> end;
    const char *at(size_t i, size_t *len) const {
        const uint64_t b = i ? end.data()[i - 1] : 0;
        if (len) *len = (size_t)(end.data()[i] - b);
        return blob.data() + b;
    }
};

struct hm_decoded {
    std::vector<hm_doc_row> docs;
    Rows<hm_change_row> ch;
    Rows<hm_dep_row> dp;
    Rows<hm_op_row> op;
    std::vector<int32_t> status;
    StrTab strings;
    NameTab actors, objs, regs;
    Rows<uint32_t> reg_obj;
    std::vector<uint64_t> act_first, obj_first;              // per document: its first actor / object entry
    uint32_t a_stride = 1, max_changes = 0, max_ops = 0, max_regs = 0, max_objs = 0, max_deps = 0, doc_flags = 0;
};

extern "C" {

int hm_decode_blocks(const uint8_t *data, const uint64_t *block_off, const uint32_t *doc_block, uint32_t n_docs,
                     uint32_t a_stride, int threads, hm_decoded **out) {
    if (!out || (n_docs && (!block_off || !doc_block))) return HM_ERR_INVALID;
    *out = nullptr;
    try {
        const auto t_start = std::chrono::steady_clock::now();
        const int T = (n_docs < 2) ? 1 : std::max(1, std::min({threads, 256, (int)n_docs}));
        std::vector<Part> parts(T);
        std::vector<uint32_t> lo(T + 1);
        for (int t = 0; t <= T; t++) lo[t] = (uint32_t)((uint64_t)n_docs * t / T);
        // an exception inside a worker (out of memory) fails the call, not the process
        auto par = [&](auto &&f) {
            if (T == 1) { f(0); return; }
            std::atomic<bool> failed{false};
            std::vector<std::thread> th;
            auto run = [&](int t) { try { f(t); } catch (...) { failed = true; } };
            for (int t = 0; t < T; t++) {
                try { th.emplace_back(run, t); } catch (...) { run(t); }   // no thread to be had: this one
            }
            for (auto &x : th) x.join();
            if (failed) throw std::bad_alloc();
        };
        par([&](int t) {
            Ctx cx;
            Bump bump;
            Part &P = parts[t];
            P.docs.resize(lo[t + 1] - lo[t]);
            // capacity for the range up front (untouched capacity is free): one change per block,
            // and no op or name row takes fewer than 16 bytes of JSON
            const uint64_t nb = block_off[doc_block[lo[t + 1]]] - block_off[doc_block[lo[t]]];
            P.ch.try_reserve(doc_block[lo[t + 1]] - doc_block[lo[t]]);
            P.op.try_reserve(nb / 16 + 16); P.op_str.try_reserve(nb / 16 + 16);
            for (uint32_t d = lo[t]; d < lo[t + 1]; d++) {
                Part::Doc &doc = P.docs[d - lo[t]];
                const Part::Mark m = P.mark();
                if (!decode_doc(data, block_off, doc_block[d], doc_block[d + 1], P, doc, cx, bump)) {
                    P.rollback(m);
                    P.objs.push(ROOT_ID, 36);
                    doc = Part::Doc{HM_ERR_INVALID, 0, 0, 0, 0, 0, 1, 0, 0};
                }
            }
        });
        const auto t_par = std::chrono::steady_clock::now();
        hm_decoded *D = new hm_decoded();
        std::unique_ptr<hm_decoded> own(D);
        // the batch's string pool, in document order (columnar.js StringPool over documents):
        // the one serial step, over hashes the documents' tables already computed
        std::vector<std::vector<uint32_t>> remap(T);
        {
            Intern pool;
            pool.reset(1024);
            for (int t = 0; t < T; t++) {
                const Part &P = parts[t];
                remap[t].resize(P.strings.size());
                for (size_t i = 0; i < P.strings.size(); i++) {
                    bool fresh;
                    size_t len;
                    const char *p = P.strings.at(i, &len);
                    remap[t][i] = pool.get_h(SV{p, (uint32_t)len}, 0, P.str_h[i], fresh);
                    if (fresh) D->strings.push(p, len);
                }
            }
        }
        // document rows and table offsets (prefix over documents; each part's tables start at
        // its first document's offsets), then the rows are copied by the threads, part by part
        D->docs.resize(n_docs);
        D->status.resize(n_docs); D->act_first.resize(n_docs); D->obj_first.resize(n_docs);
        struct Base { uint64_t ch, dp, op, act, obj, reg, ab, ob, rb; };
        std::vector<Base> base(T + 1);
        Base run = {};
        uint32_t maxa = 1;
        for (int t = 0; t < T; t++) {
            const Part &P = parts[t];
            base[t] = run;
            uint64_t act = run.act, obj = run.obj;
            for (uint32_t j = 0; j < P.docs.size(); j++) {
                const Part::Doc &x = P.docs[j];
                const uint32_t d = lo[t] + j;
                hm_doc_row &r = D->docs[d];
                r = hm_doc_row{};
                r.change_off = (uint32_t)run.ch; r.n_changes = x.n_ch;
                r.dep_off = (uint32_t)run.dp; r.n_deps = x.n_dp;
                r.op_off = (uint32_t)run.op; r.n_ops = x.n_op;
                r.reg_off = (uint32_t)run.reg; r.n_regs = x.n_reg; r.n_objs = x.n_obj;
                r.n_actors = (uint16_t)x.n_act; r.flags = x.flags;
                run.ch += x.n_ch; run.dp += x.n_dp; run.op += x.n_op; run.reg += x.n_reg;
                D->act_first[d] = act; D->obj_first[d] = obj;
                act += x.n_act; obj += x.n_obj;
                D->status[d] = x.status;
                maxa = std::max<uint32_t>(maxa, r.n_actors);
                D->max_changes = std::max(D->max_changes, r.n_changes); D->max_ops = std::max(D->max_ops, r.n_ops);
                D->max_regs = std::max(D->max_regs, r.n_regs); D->max_objs = std::max(D->max_objs, r.n_objs);
                D->max_deps = std::max(D->max_deps, r.n_deps); D->doc_flags |= r.flags;
            }
            run.act = act; run.obj = obj;
            run.ab += P.actors.blob.size(); run.ob += P.objs.blob.size(); run.rb += P.regs.blob.size();
        }
        base[T] = run;
        if (run.ch > UINT32_MAX || run.dp > UINT32_MAX || run.op > UINT32_MAX || run.reg > UINT32_MAX) return HM_ERR_INVALID;
        D->ch.alloc(run.ch); D->dp.alloc(run.dp); D->op.alloc(run.op);
        D->actors.blob.alloc(std::max<uint64_t>(run.ab, 1)); D->actors.end.alloc(run.act);
        D->objs.blob.alloc(std::max<uint64_t>(run.ob, 1)); D->objs.end.alloc(run.obj);
        D->regs.blob.alloc(std::max<uint64_t>(run.rb, 1)); D->regs.end.alloc(run.reg);
        D->reg_obj.alloc(run.reg);
        par([&](int t) {
            Part &P = parts[t];
            const Base &B = base[t];
            hm_change_row *ch = D->ch.data() + B.ch;
            for (size_t i = 0; i < P.ch.size(); i++) {
                hm_change_row c = P.ch[i];
                c.dep_off += (uint32_t)B.dp; c.op_first += (uint32_t)B.op;
                ch[i] = c;
            }
            if (!P.dp.empty()) memcpy(D->dp.data() + B.dp, P.dp.data(), P.dp.size() * sizeof(hm_dep_row));
            hm_op_row *op = D->op.data() + B.op;
            const uint32_t *rm = remap[t].data();
            for (size_t i = 0; i < P.op.size(); i++) {
                hm_op_row o = P.op[i];
                const uint8_t f = P.op_str[i];
                if (f & 1) o.key = rm[o.key];
                if (f & 2) o.value = rm[(size_t)o.value];
                op[i] = o;
            }
            auto names = [](NameTab &dst, const StrTab &src, uint64_t e0, uint64_t b0) {
                if (!src.blob.empty()) memcpy(dst.blob.data() + b0, src.blob.data(), src.blob.size());
                uint64_t *end = dst.end.data() + e0;
                for (size_t i = 0; i < src.end.size(); i++) end[i] = src.end[i] + b0;
            };
            names(D->actors, P.actors, B.act, B.ab);
            names(D->objs, P.objs, B.obj, B.ob);
            names(D->regs, P.regs, B.reg, B.rb);
            if (!P.reg_obj.empty()) memcpy(D->reg_obj.data() + B.reg, P.reg_obj.data(), P.reg_obj.size() * 4);
            P = Part();
        });
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
    return d->strings.at(i, len);
}

const char *hm_decoded_actor(const hm_decoded *d, uint32_t doc, uint32_t rank, size_t *len) {
    if (!d || doc >= d->docs.size() || rank >= d->docs[doc].n_actors) return nullptr;
    return d->actors.at(d->act_first[doc] + rank, len);
}

const char *hm_decoded_obj(const hm_decoded *d, uint32_t doc, uint32_t obj, size_t *len) {
    if (!d || doc >= d->docs.size() || obj >= d->docs[doc].n_objs) return nullptr;
    return d->objs.at(d->obj_first[doc] + obj, len);
}

const char *hm_decoded_reg(const hm_decoded *d, uint32_t doc, uint32_t reg, uint32_t *obj, size_t *len) {
    if (!d || doc >= d->docs.size() || reg >= d->docs[doc].n_regs) return nullptr;
    const uint64_t g = (uint64_t)d->docs[doc].reg_off + reg;
    if (obj) *obj = d->reg_obj.data()[g];
    return d->regs.at(g, len);
}

void hm_decoded_free(hm_decoded *d) { delete d; }

}  // extern "C"
