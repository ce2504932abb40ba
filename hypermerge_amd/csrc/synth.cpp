// synth.cpp — deterministic synthetic multi-actor change feeds in the
// columnar layout of include/hypermerge_amd.h (SURVEY.md §8(d) inputs).
//
// Not part of the merge path: it produces the *input* a hypermerge repo
// would have decoded from hypercore blocks (src/Actor.ts:137-141).
//
// Causality model ("gossip with delay"): every actor keeps a vector clock of
// what it has incorporated.  Before each of its changes, an actor merges the
// state another actor had `delay` steps ago (delay ~ Geometric(1/2)), so what
// it knows is always causally closed.  A new change's deps are the heads of
// its known set minus its own actor — what Automerge 0.12's frontend puts in
// a request (state.deps without the own actor) — so the merge sees genuine
// concurrency.  Documents are independent; each is generated from
// splitmix64(seed ^ global_doc_index), so a doc is identical whatever the
// shard/batch it lands in.
#include <cstdint>
#include <cstring>
#include <vector>
#include <thread>
#include <algorithm>
#include <string>
#include "../../include/hypermerge_amd.h"

namespace {

struct Rng {
    uint64_t s[4];
    static uint64_t splitmix(uint64_t &x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    explicit Rng(uint64_t seed) { for (auto &v : s) v = splitmix(seed); }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    uint32_t below(uint32_t n) { return n ? (uint32_t)((next() >> 32) * (uint64_t)n >> 32) : 0; }
    bool pct(uint32_t p) { return below(100) < p; }
    uint32_t geom() { uint32_t k = 1; while (k < 16 && (next() & 1)) k++; return k; }
};

// base58 of a 32-byte key, as hypermerge encodes public keys (src/Keys.ts)
std::string base58(const uint8_t *in, int n) {
    static const char *ALPHA = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
    uint8_t buf[64]; memcpy(buf, in, n);
    char out[96]; int o = 0, start = 0;
    while (start < n && buf[start] == 0) { out[o++] = '1'; start++; }
    std::string digits;
    while (start < n) {
        int rem = 0;
        for (int i = start; i < n; i++) {
            int acc = rem * 256 + buf[i];
            buf[i] = (uint8_t)(acc / 58); rem = acc % 58;
        }
        digits.push_back(ALPHA[rem]);
        while (start < n && buf[start] == 0) start++;
    }
    std::string s(out, o);
    s.append(digits.rbegin(), digits.rend());
    return s;
}

uint64_t fnv1a64(const std::string &s) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (unsigned char c : s) { h ^= c; h *= 0x100000001b3ull; }
    return h;
}

}  // namespace

extern "C" {

typedef struct {
    uint64_t seed;
    uint64_t doc_base;          // global index of the first candidate document
    uint32_t n_docs;            // documents to emit (after shard filtering)
    uint32_t shard, n_shards;   // keep docs with FNV-1a64(docId) % n_shards == shard
    uint32_t kind;              // 0 flat map, 1 text, 2 nested maps/lists
    uint32_t actors;
    uint32_t changes_per_actor; // kind 0/2: changes per actor; kind 1: typing ops per doc
    uint32_t ops_min, ops_max;  // ops per change (kind 0/2)
    uint32_t n_keys;            // keys per map object
    uint32_t counter_pct;       // kind 0: % of keys that are counters
    uint32_t del_pct;           // % of assignments that are deletes
    uint32_t arrival;           // 0 generation order, 1 actor-major (loadDocument), 2 shuffled
    uint32_t shuffle_pct;       // arrival 2: % of changes pulled ahead of their position
    uint32_t dup_pct;           // % of changes delivered twice
    uint32_t alternate;         // kind 0: actors strictly alternate, key = i mod n_keys (C1)
    uint32_t threads;
} hm_synth_config;

}  // extern "C"

namespace {

struct DocOut {
    std::vector<hm_change_row> ch;
    std::vector<hm_dep_row> dp;
    std::vector<hm_op_row> op;
    uint32_t n_regs = 0, n_objs = 1, n_actors = 0, flags = 0;
};

struct Gen {
    const hm_synth_config &c;
    Rng r;
    uint32_t A;
    std::vector<uint32_t> V;        // V[a*A+b] known count
    std::vector<std::vector<uint32_t>> FC;   // FC[a][(s-1)*A + b] full clock of (a,s)
    std::vector<std::vector<uint32_t>> snaps; // ring of 17 snapshots of V
    uint32_t t = 0;
    std::vector<uint32_t> rank;     // creation index -> rank (random permutation)
    uint32_t content = 0;
    struct Pending { hm_change_row row; std::vector<hm_dep_row> deps; std::vector<hm_op_row> ops; };
    std::vector<Pending> gen;       // in generation order

    Gen(const hm_synth_config &cfg, uint64_t seed) : c(cfg), r(seed), A(cfg.actors) {
        V.assign(A * A, 0); FC.assign(A, {}); snaps.assign(17, std::vector<uint32_t>(A * A, 0));
        rank.resize(A);
        for (uint32_t i = 0; i < A; i++) rank[i] = i;
        for (uint32_t i = A; i > 1; i--) std::swap(rank[i - 1], rank[r.below(i)]);
    }
    const uint32_t *fc(uint32_t a, uint32_t s) { return &FC[a][(size_t)(s - 1) * A]; }
    bool knows(uint32_t a, uint32_t b, uint32_t s) { return V[a * A + b] >= s; }

    void gossip(uint32_t a) {
        uint32_t rounds = 1 + (r.next() & 1);
        for (uint32_t k = 0; k < rounds && A > 1; k++) {
            uint32_t b = r.below(A - 1); if (b >= a) b++;
            uint32_t d = r.geom();
            const std::vector<uint32_t> &sn = snaps[(t + 17 - std::min(d, t)) % 17];
            for (uint32_t x = 0; x < A; x++) V[a * A + x] = std::max(V[a * A + x], sn[b * A + x]);
        }
    }
    // deps = heads(V[a]) minus a
    void heads(uint32_t a, std::vector<hm_dep_row> &out) {
        for (uint32_t b = 0; b < A; b++) {
            if (b == a) continue;
            uint32_t vb = V[a * A + b];
            if (!vb) continue;
            bool head = true;
            for (uint32_t x = 0; x < A && head; x++) {
                if (x == b) continue;
                uint32_t vx = V[a * A + x];
                if (vx && fc(x, vx)[b] >= vb) head = false;
            }
            if (head) out.push_back(hm_dep_row{(uint16_t)rank[b], 0, vb});
        }
    }
    uint32_t produce(uint32_t a, std::vector<hm_op_row> &&ops, uint32_t nops_hint = 0) {
        (void)nops_hint;
        Pending p;
        heads(a, p.deps);
        uint32_t seq = V[a * A + a] + 1;
        FC[a].resize((size_t)seq * A);
        uint32_t *f = &FC[a][(size_t)(seq - 1) * A];
        for (uint32_t x = 0; x < A; x++) f[x] = V[a * A + x];
        f[a] = seq;
        V[a * A + a] = seq;
        p.row = hm_change_row{(uint16_t)rank[a], (uint16_t)p.deps.size(), seq, 0,
                              (uint32_t)ops.size(), 0, content++};
        p.ops = std::move(ops);
        gen.push_back(std::move(p));
        t++;
        snaps[t % 17].assign(V.begin(), V.end());
        return seq;
    }

    hm_op_row mk(uint32_t action, uint32_t obj, uint32_t reg, uint32_t key = 0) {
        hm_op_row o; memset(&o, 0, sizeof(o));
        o.action = (uint8_t)action; o.obj = obj; o.reg = reg; o.parent = HM_NONE; o.key = key;
        return o;
    }
    void scalar(hm_op_row &o) {
        uint32_t k = r.below(100);
        if (k < 60) { o.vtag = HM_V_INT; o.value = (uint64_t)(int64_t)(int32_t)(uint32_t)r.next(); }
        else if (k < 85) { o.vtag = HM_V_STR; o.value = r.below(4096); }
        else { o.vtag = (r.next() & 1) ? HM_V_TRUE : HM_V_FALSE; }
    }

    // ---------------- kind 0: flat map (C1, C2, C4) ----------------
    void flat_map(DocOut &d) {
        uint32_t m = c.changes_per_actor, K = c.n_keys ? c.n_keys : 16;
        uint32_t ncounter = K * c.counter_pct / 100;
        // counter-set registry: the first (actor, seq) that set each counter key
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> csets(K);
        std::vector<uint32_t> left(A, m);
        uint32_t total = A * m;
        for (uint32_t i = 0; i < total; i++) {
            uint32_t a;
            if (c.alternate) a = i % A;
            else { do a = r.below(A); while (!left[a]); }
            left[a]--;
            gossip(a);
            uint32_t nops = c.alternate ? 1 : c.ops_min + r.below(c.ops_max - c.ops_min + 1);
            std::vector<hm_op_row> ops;
            uint32_t seq_next = V[a * A + a] + 1;
            for (uint32_t j = 0; j < nops; j++) {
                uint32_t key = c.alternate ? (i % K) : r.below(K);
                hm_op_row o = mk(HM_SET, 0, key, key);
                if (key < ncounter) {
                    bool known = false;
                    for (auto &cs : csets[key]) if (cs.first == a ? cs.second < seq_next : knows(a, cs.first, cs.second)) known = true;
                    if (known) { o.action = HM_INC; o.vtag = HM_V_INT; o.value = (uint64_t)(int64_t)((int)r.below(100) + 1) * ((r.next() & 1) ? 1 : -1); }
                    else { o.datatype = HM_DT_COUNTER; o.vtag = HM_V_INT; o.value = 0; csets[key].push_back({a, seq_next}); }
                } else if (c.del_pct && r.pct(c.del_pct)) {
                    o.action = HM_DEL;
                } else if (c.alternate) {
                    o.vtag = HM_V_INT; o.value = (uint64_t)(int64_t)(int32_t)(uint32_t)r.next();
                } else scalar(o);
                ops.push_back(o);
            }
            produce(a, std::move(ops));
        }
        d.n_regs = K; d.n_objs = 1; d.flags = ncounter ? HM_DOC_HAS_COUNTERS : 0;
    }

    // ---------------- kind 1: text (C3) ----------------
    struct Elem { uint32_t actor, seq, elem, reg; };
    void text(DocOut &d) {
        // change 0 by actor 0: makeText + link; everyone depends on it via gossip
        uint32_t regs = 1;   // reg 0 = root key "text"
        std::vector<Elem> elems;            // in creation order
        std::vector<std::vector<uint32_t>> maxel(A);   // per actor chain: prefix max elem per seq
        {
            std::vector<hm_op_row> ops;
            ops.push_back(mk(HM_MAKE_TEXT, 1, HM_NONE));
            hm_op_row l = mk(HM_LINK, 0, 0, 0); l.vtag = HM_V_OBJ; l.value = 1; ops.push_back(l);
            produce(0, std::move(ops));
            maxel[0].push_back(0);
        }
        // everyone learns the text object before typing
        for (uint32_t a = 1; a < A; a++) V[a * A + 0] = std::max(V[a * A + 0], 1u);
        snaps[t % 17].assign(V.begin(), V.end());
        std::vector<uint32_t> cursor(A, HM_HEAD);
        uint32_t typed = 0, target = c.changes_per_actor ? c.changes_per_actor : 2000;
        while (typed < target) {
            uint32_t a = r.below(A);
            gossip(a);
            uint32_t seq_next = V[a * A + a] + 1;
            // maxElem known to a
            uint32_t mx = 0;
            for (uint32_t b = 0; b < A; b++) { uint32_t vb = V[a * A + b]; if (vb && vb <= maxel[b].size()) mx = std::max(mx, maxel[b][vb - 1]); }
            // cursor: keep the own last insert, or jump to a random known element
            if (cursor[a] == HM_HEAD || r.pct(15)) {
                cursor[a] = HM_HEAD;
                if (!elems.empty()) for (int tries = 0; tries < 4; tries++) {
                    const Elem &e = elems[r.below((uint32_t)elems.size())];
                    if (knows(a, e.actor, e.seq)) { cursor[a] = e.reg; break; }
                }
            }
            uint32_t run = 1 + r.below(16);
            std::vector<hm_op_row> ops;
            uint32_t cmax = 0;
            for (uint32_t j = 0; j < run && typed < target; j++, typed++) {
                if (!elems.empty() && r.pct(20)) {
                    const Elem &e = elems[r.below((uint32_t)elems.size())];
                    if (e.actor == a ? e.seq < seq_next || e.seq == seq_next : knows(a, e.actor, e.seq)) {
                        ops.push_back(mk(HM_DEL, 1, e.reg));
                        continue;
                    }
                }
                uint32_t el = ++mx;
                hm_op_row ins = mk(HM_INS, 1, regs++);
                ins.parent = cursor[a]; ins.elem = el;
                ops.push_back(ins);
                hm_op_row s = mk(HM_SET, 1, ins.reg);
                s.vtag = HM_V_STR; s.value = 'a' + r.below(26);
                ops.push_back(s);
                elems.push_back(Elem{a, seq_next, el, ins.reg});
                cursor[a] = ins.reg;
                cmax = std::max(cmax, el);
            }
            if (ops.empty()) continue;
            uint32_t prev = maxel[a].empty() ? 0 : maxel[a].back();
            maxel[a].push_back(std::max(prev, cmax));
            produce(a, std::move(ops));
        }
        d.n_regs = regs; d.n_objs = 2; d.flags = HM_DOC_HAS_LISTS;
    }

    // ---------------- kind 2: nested maps + lists (C5) ----------------
    void nested(DocOut &d) {
        uint32_t K = c.n_keys ? c.n_keys : 4;
        // schema change by actor 0: root -> m1 -> m2 -> m3 (3 deep) and two lists
        uint32_t nobj = 1, regs = 0;
        std::vector<uint32_t> maps, lists, mapreg0;     // first reg of each map
        auto new_map = [&](std::vector<hm_op_row> &ops, uint32_t parent_map, uint32_t key) {
            uint32_t o = nobj++;
            ops.push_back(mk(HM_MAKE_MAP, o, HM_NONE));
            hm_op_row l = mk(HM_LINK, parent_map, mapreg0[parent_map] + key, key); l.vtag = HM_V_OBJ; l.value = o;
            ops.push_back(l);
            return o;
        };
        std::vector<uint32_t> objkind;   // per obj: 0 map 1 list
        std::vector<std::pair<uint32_t, uint32_t>> map_by;   // per maps[] entry: creating (actor, seq)
        mapreg0.push_back(0); regs = K; objkind.push_back(0);
        std::vector<hm_op_row> ops;
        maps.push_back(0); map_by.push_back({0, 0});
        uint32_t parent = 0;
        for (int depth = 0; depth < 3; depth++) {
            uint32_t o = new_map(ops, parent, depth % K);
            mapreg0.push_back(regs); regs += K; objkind.push_back(0); maps.push_back(o);
            map_by.push_back({0, 1});
            parent = o;
        }
        for (int li = 0; li < 2; li++) {
            uint32_t o = nobj++;
            ops.push_back(mk(HM_MAKE_LIST, o, HM_NONE));
            uint32_t host = maps[1 + li];
            hm_op_row l = mk(HM_LINK, host, mapreg0[host] + (K - 1), K - 1); l.vtag = HM_V_OBJ; l.value = o;
            ops.push_back(l);
            mapreg0.push_back(HM_NONE); objkind.push_back(1); lists.push_back(o);
        }
        produce(0, std::move(ops));
        for (uint32_t a = 1; a < A; a++) V[a * A + 0] = std::max(V[a * A + 0], 1u);
        snaps[t % 17].assign(V.begin(), V.end());
        struct LE { uint32_t obj, actor, seq, reg; };
        std::vector<LE> les;
        std::vector<std::vector<uint32_t>> maxel(A);
        maxel[0].push_back(0);
        uint32_t total = A * c.changes_per_actor;
        for (uint32_t i = 0; i < total; i++) {
            uint32_t a = r.below(A);
            gossip(a);
            uint32_t seq_next = V[a * A + a] + 1;
            uint32_t mx = 0;
            for (uint32_t b = 0; b < A; b++) { uint32_t vb = V[a * A + b]; if (vb && vb <= maxel[b].size()) mx = std::max(mx, maxel[b][vb - 1]); }
            uint32_t nops = c.ops_min + r.below(c.ops_max - c.ops_min + 1);
            std::vector<hm_op_row> o2;
            uint32_t cmax = 0;
            auto pick_map = [&]() {
                for (;;) {
                    uint32_t i = r.below((uint32_t)maps.size());
                    auto by = map_by[i];
                    if (by.second == 0 || (by.first == a ? by.second <= seq_next : knows(a, by.first, by.second))) return maps[i];
                }
            };
            for (uint32_t j = 0; j < nops; j++) {
                uint32_t kind = r.below(100);
                if (kind < 55) {                         // map assignment (hot keys -> conflicts)
                    uint32_t mo = pick_map();
                    uint32_t key = r.below(K - 1);
                    hm_op_row o = mk(HM_SET, mo, mapreg0[mo] + key, key);
                    if (r.pct(c.del_pct)) o.action = HM_DEL; else scalar(o);
                    o2.push_back(o);
                    if (r.pct(8)) o2.push_back(o);       // same key twice in one change (tie case)
                } else if (kind < 60 && nobj < 60) {     // fresh nested map linked over a key
                    uint32_t mo = pick_map();
                    uint32_t no = nobj++;
                    o2.push_back(mk(HM_MAKE_MAP, no, HM_NONE));
                    uint32_t key = r.below(K - 1);
                    hm_op_row l = mk(HM_LINK, mo, mapreg0[mo] + key, key); l.vtag = HM_V_OBJ; l.value = no;
                    o2.push_back(l);
                    mapreg0.push_back(regs); regs += K; objkind.push_back(0);
                    maps.push_back(no); map_by.push_back({a, seq_next});
                } else {                                  // list edit
                    uint32_t lo = lists[r.below((uint32_t)lists.size())];
                    uint32_t p = HM_HEAD;
                    if (!les.empty() && r.pct(70)) {
                        const LE &e = les[r.below((uint32_t)les.size())];
                        bool kn = e.actor == a ? true : knows(a, e.actor, e.seq);
                        if (kn && e.obj == lo) p = e.reg;
                        if (kn && r.pct(c.del_pct * 2)) { o2.push_back(mk(HM_DEL, e.obj, e.reg)); continue; }
                        if (kn && r.pct(10)) { hm_op_row s = mk(HM_SET, e.obj, e.reg); scalar(s); o2.push_back(s); continue; }
                    }
                    uint32_t el = ++mx;
                    hm_op_row ins = mk(HM_INS, lo, regs++);
                    ins.parent = p; ins.elem = el;
                    o2.push_back(ins);
                    hm_op_row s = mk(HM_SET, lo, ins.reg); scalar(s);
                    o2.push_back(s);
                    les.push_back(LE{lo, a, seq_next, ins.reg});
                    cmax = std::max(cmax, el);
                }
            }
            uint32_t prev = maxel[a].empty() ? 0 : maxel[a].back();
            maxel[a].push_back(std::max(prev, cmax));
            produce(a, std::move(o2));
        }
        d.n_regs = regs; d.n_objs = nobj; d.flags = HM_DOC_HAS_LISTS;
    }

    void run(DocOut &d) {
        if (c.kind == 1) text(d); else if (c.kind == 2) nested(d); else flat_map(d);
        d.n_actors = A;
        // arrival order
        std::vector<uint32_t> order(gen.size());
        for (uint32_t i = 0; i < order.size(); i++) order[i] = i;
        if (c.arrival == 1) {
            std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return gen[x].row.actor < gen[y].row.actor; });
        } else if (c.arrival == 2) {
            for (uint32_t i = 1; i < order.size(); i++)
                if (r.pct(c.shuffle_pct)) {
                    uint32_t back = 1 + r.below(std::min<uint32_t>(i, 8));
                    uint32_t x = order[i];
                    memmove(&order[i - back + 1], &order[i - back], back * sizeof(uint32_t));
                    order[i - back] = x;
                }
        }
        std::vector<uint32_t> final_order;
        for (uint32_t i = 0; i < order.size(); i++) {
            final_order.push_back(order[i]);
            if (c.dup_pct && r.pct(c.dup_pct)) {
                uint32_t j = r.below(i + 1);
                final_order.push_back(order[j]);
            }
        }
        for (uint32_t gi : final_order) {
            Pending &p = gen[gi];
            hm_change_row row = p.row;
            row.dep_off = (uint32_t)d.dp.size();
            row.op_first = (uint32_t)d.op.size();
            d.dp.insert(d.dp.end(), p.deps.begin(), p.deps.end());
            d.op.insert(d.op.end(), p.ops.begin(), p.ops.end());
            d.ch.push_back(row);
        }
    }
};

struct Output {
    std::vector<hm_doc_row> docs;
    std::vector<hm_change_row> ch;
    std::vector<hm_dep_row> dp;
    std::vector<hm_op_row> op;
    uint32_t a_stride = 1;
    uint64_t n_regs = 0;
};

std::string doc_id(uint64_t seed, uint64_t g) {
    uint64_t x = seed ^ (g * 0xD1B54A32D192ED03ull), k[4];
    for (auto &v : k) v = Rng::splitmix(x);
    return base58(reinterpret_cast<const uint8_t *>(k), 32);
}

}  // namespace

extern "C" {

void *hm_synth_generate(const hm_synth_config *cfg) {
    const hm_synth_config c = *cfg;
    // choose the global doc indices of this shard
    std::vector<uint64_t> gidx;
    gidx.reserve(c.n_docs);
    if (c.n_shards <= 1) {
        for (uint64_t i = 0; i < c.n_docs; i++) gidx.push_back(c.doc_base + i);
    } else {
        uint32_t T = std::max(1u, c.threads);
        uint64_t g = c.doc_base, chunk = (uint64_t)c.n_docs * c.n_shards / 4 + 1024;
        while (gidx.size() < c.n_docs) {
            std::vector<std::vector<uint64_t>> part(T);
            std::vector<std::thread> th;
            for (uint32_t t = 0; t < T; t++)
                th.emplace_back([&, t] {
                    uint64_t lo = g + chunk * t / T, hi = g + chunk * (t + 1) / T;
                    for (uint64_t i = lo; i < hi; i++)
                        if (fnv1a64(doc_id(c.seed, i)) % c.n_shards == c.shard) part[t].push_back(i);
                });
            for (auto &x : th) x.join();
            for (auto &p : part) for (uint64_t i : p) if (gidx.size() < c.n_docs) gidx.push_back(i);
            g += chunk;
        }
    }
    uint32_t T = std::max(1u, std::min<uint32_t>(c.threads, c.n_docs ? c.n_docs : 1));
    std::vector<std::vector<DocOut>> parts(T);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; t++)
        th.emplace_back([&, t] {
            size_t lo = gidx.size() * t / T, hi = gidx.size() * (t + 1) / T;
            parts[t].resize(hi - lo);
            for (size_t i = lo; i < hi; i++) {
                uint64_t x = c.seed ^ (gidx[i] * 0x9E3779B97F4A7C15ull);
                Gen gen(c, Rng::splitmix(x));
                gen.run(parts[t][i - lo]);
            }
        });
    for (auto &x : th) x.join();
    Output *o = new Output();
    size_t nc = 0, nd = 0, no = 0;
    for (auto &p : parts) for (auto &d : p) { nc += d.ch.size(); nd += d.dp.size(); no += d.op.size(); }
    o->ch.reserve(nc); o->dp.reserve(nd); o->op.reserve(no); o->docs.reserve(gidx.size());
    size_t k = 0;                        // docs come out in gidx order
    for (auto &p : parts)
        for (auto &d : p) {
            hm_doc_row row;
            memset(&row, 0, sizeof(row));
            // the document's global index in the doc-id stream (its key across shards)
            row.reserved[0] = (uint32_t)gidx[k]; row.reserved[1] = (uint32_t)(gidx[k] >> 32);
            k++;
            row.change_off = (uint32_t)o->ch.size(); row.n_changes = (uint32_t)d.ch.size();
            row.dep_off = (uint32_t)o->dp.size(); row.n_deps = (uint32_t)d.dp.size();
            row.op_off = (uint32_t)o->op.size(); row.n_ops = (uint32_t)d.op.size();
            row.reg_off = (uint32_t)o->n_regs; row.n_regs = d.n_regs; row.n_objs = d.n_objs;
            row.n_actors = (uint16_t)d.n_actors; row.flags = (uint16_t)d.flags;
            uint32_t dbase = (uint32_t)o->dp.size(), obase = row.op_off;
            for (auto ch : d.ch) { ch.dep_off += dbase; ch.op_first += obase; o->ch.push_back(ch); }
            o->dp.insert(o->dp.end(), d.dp.begin(), d.dp.end());
            o->op.insert(o->op.end(), d.op.begin(), d.op.end());
            o->n_regs += d.n_regs;
            o->a_stride = std::max<uint32_t>(o->a_stride, d.n_actors);
            o->docs.push_back(row);
            std::vector<hm_change_row>().swap(d.ch);
            std::vector<hm_dep_row>().swap(d.dp);
            std::vector<hm_op_row>().swap(d.op);
        }
    return o;
}

void hm_synth_sizes(void *h, uint64_t *out6) {
    Output *o = (Output *)h;
    out6[0] = o->docs.size(); out6[1] = o->ch.size(); out6[2] = o->dp.size();
    out6[3] = o->op.size(); out6[4] = o->n_regs; out6[5] = o->a_stride;
}

void hm_synth_copy(void *h, hm_doc_row *docs, hm_change_row *ch, hm_dep_row *dp, hm_op_row *op) {
    Output *o = (Output *)h;
    if (docs) memcpy(docs, o->docs.data(), o->docs.size() * sizeof(hm_doc_row));
    if (ch) memcpy(ch, o->ch.data(), o->ch.size() * sizeof(hm_change_row));
    if (dp) memcpy(dp, o->dp.data(), o->dp.size() * sizeof(hm_dep_row));
    if (op) memcpy(op, o->op.data(), o->op.size() * sizeof(hm_op_row));
}

void hm_synth_free(void *h) { delete (Output *)h; }

uint64_t hm_synth_fnv1a64_docid(uint64_t seed, uint64_t g) { return fnv1a64(doc_id(seed, g)); }

// Hypercore blocks of a synthetic batch, as Actor.writeChange / Block.pack store changes
// (src/Actor.ts:73-80, src/Block.ts:6-16), uncompressed JSON form: one block per change, the
// documents' changes in their arrival order.  Actor ids are "<docId>.<rank>" (their string
// order is the rank order), map keys "k<register>", object ids ROOT or "o<id>-<docId>".
// Sizes first (blocks == NULL): returns the total bytes; then fills data / block_off
// [n_changes + 1] / doc_block [n_docs + 1].
uint64_t hm_synth_blocks(uint64_t seed, const hm_doc_row *docs, uint32_t n_docs, const hm_change_row *ch,
                         const hm_dep_row *dp, const hm_op_row *op, char *data, uint64_t *block_off,
                         uint32_t *doc_block) {
    static const char *names[] = {"makeMap", "makeTable", "makeList", "makeText", "ins", "set", "del", "link", "inc"};
    const char *ROOT = "00000000-0000-0000-0000-000000000000";
    uint64_t total = 0;
    uint32_t nb = 0;
    std::string js;
    for (uint32_t d = 0; d < n_docs; d++) {
        const hm_doc_row &D = docs[d];
        const uint64_t g = (uint64_t)D.reserved[0] | ((uint64_t)D.reserved[1] << 32);
        const std::string id = doc_id(seed, g);
        auto actor = [&](uint32_t r) { char b[8]; snprintf(b, sizeof b, ".%02u", r); return id + b; };
        auto objn = [&](uint32_t o) { return o == 0 ? std::string(ROOT) : "o" + std::to_string(o) + "-" + id; };
        if (doc_block) doc_block[d] = nb;
        for (uint32_t c = D.change_off; c < D.change_off + D.n_changes; c++) {
            const hm_change_row &C = ch[c];
            js = "{\"actor\":\"" + actor(C.actor) + "\",\"seq\":" + std::to_string(C.seq) + ",\"deps\":{";
            for (uint32_t k = 0; k < C.n_deps; k++) {
                const hm_dep_row &P = dp[C.dep_off + k];
                js += (k ? ",\"" : "\"") + actor(P.actor) + "\":" + std::to_string(P.seq);
            }
            js += "},\"ops\":[";
            for (uint32_t k = 0; k < C.n_ops; k++) {
                const hm_op_row &O = op[C.op_first + k];
                js += k ? ",{" : "{";
                js += "\"action\":\"" + std::string(names[O.action < 9 ? O.action : 5]) + "\",\"obj\":\"" + objn(O.obj) + "\"";
                if (O.action >= 5) {
                    js += ",\"key\":\"k" + std::to_string(O.reg) + "\"";
                    if (O.action == 7) js += ",\"value\":\"" + objn((uint32_t)O.value) + "\"";
                    else if (O.action != 6) {
                        if (O.vtag == HM_V_INT) js += ",\"value\":" + std::to_string((long long)O.value);
                        else if (O.vtag == HM_V_TRUE) js += ",\"value\":true";
                        else if (O.vtag == HM_V_FALSE) js += ",\"value\":false";
                        else if (O.vtag == HM_V_STR) js += ",\"value\":\"s" + std::to_string((long long)O.value) + "\"";
                        else js += ",\"value\":null";
                    }
                    if (O.datatype == HM_DT_COUNTER) js += ",\"datatype\":\"counter\"";
                }
                js += "}";
            }
            js += "]}";
            if (block_off) block_off[nb] = total;
            if (data) memcpy(data + total, js.data(), js.size());
            total += js.size();
            nb++;
        }
    }
    if (block_off) block_off[nb] = total;
    if (doc_block) doc_block[n_docs] = nb;
    return total;
}

// Repo-global record keys of a synthetic shard (the clock exchange, exchange.hip): per document
// FNV-1a64 of its base58 doc id, per (document, actor rank < n_actors) FNV-1a64 of the actor's
// synthetic id "<docId>/<rank>" (0 past n_actors).
void hm_synth_keys(uint64_t seed, const hm_doc_row *docs, uint32_t n, uint32_t S, uint64_t *doc_keys,
                   uint64_t *actor_keys) {
    for (uint32_t d = 0; d < n; d++) {
        const uint64_t g = (uint64_t)docs[d].reserved[0] | ((uint64_t)docs[d].reserved[1] << 32);
        const std::string id = doc_id(seed, g);
        doc_keys[d] = fnv1a64(id);
        for (uint32_t a = 0; a < S; a++)
            actor_keys[(size_t)d * S + a] = a < docs[d].n_actors ? fnv1a64(id + "/" + std::to_string(a)) : 0;
    }
}

}  // extern "C"
