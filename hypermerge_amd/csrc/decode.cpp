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
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>
#include "../../include/hypermerge_amd.h"
#include "scan.h"

namespace {

using namespace hmscan;


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
