// store.cpp — the resident document store of include/hypermerge_amd.h (hm_store_*,
// hm_doc_*, hm_batch_submit/wait, hm_store_clock_update, hm_sync_ranges_device).
//
// Replaces the per-document Automerge BackendState that DocBackend keeps in
// `this.back` (src/DocBackend.ts:50) for every open document of a repo, plus the
// DocBackend / ClockStore bookkeeping around it.  Layout in HBM:
//
//   change space  changes[]  hist[]  all_deps[][S]      (one segment per document)
//   dep space     deps[]
//   op space      ops[]      surv[]
//   reg space     regs[]
//   per handle    res_docs[] clock[][S] back_clock[][S] heads[][S] min_clock[][S] stored_clock[][S]
//
// A document's segments have power-of-two capacities; an append that overflows one
// moves the document to a fresh segment at the arena's end (append_kernel copies and
// rebases the old rows once).  When an arena is full every document is compacted into
// a new, larger arena and re-merged.  A submit appends the new rows; a document whose new
// changes apply in arrival order on its resident state (nothing queued, map ops) is
// advanced in place by inc_apply_kernel, touching only the registers the new ops hit;
// any other document re-merges its whole log with the batch merge kernels (applyChanges
// is a left fold of addChange, so the state after A then B is the state after A ++ B).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>
#include "../../include/hypermerge_amd.h"
#include "engine_internal.h"
#include "store_kernels.h"

namespace {

struct Seg { uint32_t off = 0, cap = 0; };

struct DocMeta {
    Seg c, d, o, r;                     // change, dep, op, register segments
    uint32_t n_c = 0, n_d = 0, n_o = 0, n_r = 0, n_objs = 1, n_actors = 0;
    uint16_t flags = 0;
    hm_doc_result last = {};            // result of the last successful merge
};

template <typename T>
struct DBuf {                            // device buffer of T with capacity
    T *p = nullptr;
    size_t cap = 0;
};

uint32_t pow2ceil(uint32_t x) {
    uint32_t c = 1;
    while (c < x) c <<= 1;
    return c;
}

}  // namespace

struct hm_store {
    hm_engine *e = nullptr;
    uint32_t S = 8;
    std::vector<DocMeta> docs;
    // arenas (capacity in rows) and bump pointers
    size_t cap_c = 0, cap_d = 0, cap_o = 0, cap_r = 0;
    size_t used_c = 0, used_d = 0, used_o = 0, used_r = 0;
    hm_change_row *changes = nullptr; int32_t *hist = nullptr; uint32_t *all_deps = nullptr;
    hm_dep_row *deps = nullptr;
    hm_op_row *ops = nullptr; hm_surv_result *surv = nullptr;
    hm_reg_result *regs = nullptr;
    // per handle
    size_t cap_h = 0;
    hm_doc_result *res_docs = nullptr;
    uint32_t *clock = nullptr, *back_clock = nullptr, *heads = nullptr, *min_clock = nullptr, *stored = nullptr;
    // staging (device)
    DBuf<uint8_t> stage;
    // in-flight batch
    std::atomic<bool> pending{false};             // a submitted batch not yet waited for (other threads may read it)
    uint64_t next_id = 1, pending_id = 0;
    std::vector<uint32_t> p_handles;              // batch rows -> handles
    struct OldMeta { uint32_t n_c, n_d, n_o, n_r, n_objs; uint16_t n_actors, flags; };
    std::vector<OldMeta> p_old;                   // log sizes before the append (rollback)
    std::vector<int32_t> p_inv_row;               // batch row -> offset of its inverse remap in p_inv (-1 = none)
    std::vector<uint8_t> p_inv;                   // inverse remap rows [S]
    uint8_t *p_gather_dev = nullptr;
    // per-submit host scratch kept between submits (a 1M-document submit would otherwise
    // allocate and first-touch ~130 MB every round)
    std::vector<AppendDesc> descs;
    std::vector<uint32_t> grow;
    // incremental applyRemoteChanges (inc_apply_kernel) and the last submit's routing
    bool incremental = true;
    uint32_t st_inc = 0, st_cold = 0, st_bail = 0;
};

namespace {

#define SCHK(s, call)                                                              \
    do {                                                                           \
        hipError_t _r = (call);                                                    \
        if (_r != hipSuccess)                                                      \
            return hm_engine_fail((s)->e, HM_ERR_DEVICE, (std::string(#call) + ": " + hipGetErrorString(_r)).c_str()); \
    } while (0)

template <typename T>
int dev_alloc(hm_store *s, T **p, size_t n) {
    *p = nullptr;
    if (!n) n = 1;
    if (hipMalloc((void **)p, n * sizeof(T)) != hipSuccess) return hm_engine_fail(s->e, HM_ERR_NOMEM, "hipMalloc store arena");
    return HM_OK;
}

int ensure_stage(hm_store *s, size_t bytes) {
    if (bytes <= s->stage.cap) return HM_OK;
    SCHK(s, hipStreamSynchronize(hm_engine_stream(s->e)));
    if (s->stage.p) (void)hipFree(s->stage.p);
    s->stage.p = nullptr; s->stage.cap = 0;
    const size_t cap = std::max(bytes, (size_t)1 << 20) * 2;
    if (hipMalloc((void **)&s->stage.p, cap) != hipSuccess) return hm_engine_fail(s->e, HM_ERR_NOMEM, "hipMalloc store staging");
    s->stage.cap = cap;
    return HM_OK;
}

// grow the per-handle tables to hold `need` documents (contents preserved)
int ensure_handles(hm_store *s, size_t need) {
    if (need <= s->cap_h) return HM_OK;
    const size_t cap = std::max<size_t>(need, std::max<size_t>(1024, s->cap_h * 2));
    hipStream_t st = hm_engine_stream(s->e);
    const uint32_t S = s->S;
    hm_doc_result *rd; int r;
    if ((r = dev_alloc(s, &rd, cap))) return r;
    SCHK(s, hipMemsetAsync(rd, 0, cap * sizeof(hm_doc_result), st));
    if (s->cap_h) SCHK(s, hipMemcpyAsync(rd, s->res_docs, s->cap_h * sizeof(hm_doc_result), hipMemcpyDeviceToDevice, st));
    uint32_t **tabs[5] = {&s->clock, &s->back_clock, &s->heads, &s->min_clock, &s->stored};
    uint32_t *nt[5];
    for (int i = 0; i < 5; i++) {
        if ((r = dev_alloc(s, &nt[i], cap * S))) return r;
        SCHK(s, hipMemsetAsync(nt[i], 0, cap * S * 4, st));
        if (s->cap_h) SCHK(s, hipMemcpyAsync(nt[i], *tabs[i], s->cap_h * S * 4, hipMemcpyDeviceToDevice, st));
    }
    SCHK(s, hipStreamSynchronize(st));
    if (s->res_docs) (void)hipFree(s->res_docs);
    s->res_docs = rd;
    for (int i = 0; i < 5; i++) { if (*tabs[i]) (void)hipFree(*tabs[i]); *tabs[i] = nt[i]; }
    s->cap_h = cap;
    return HM_OK;
}

// HM_STORE_PROFILE=1: per-phase wall times of hm_batch_submit / hm_batch_wait on stderr (the
// stream is synchronised at each mark, so device work is attributed to its phase)
struct PhaseTimer {
    bool on;
    hipStream_t st;
    std::chrono::steady_clock::time_point t;
    explicit PhaseTimer(hipStream_t s) : on(getenv("HM_STORE_PROFILE") != nullptr), st(s), t(std::chrono::steady_clock::now()) {}
    void mark(const char *what) {
        if (!on) return;
        (void)hipStreamSynchronize(st);
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[hm_store] %-18s %9.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// f(lo, hi, t) over [0, n) split in contiguous ranges; host threads for big submits only
// (the box's CPU share is 16 threads)
template <typename F> uint32_t par_for(uint32_t n, F &&f) {
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    const uint32_t T = n >= 65536 ? std::min<uint32_t>(16, hw) : 1;
    if (T == 1) { f(0u, n, 0u); return 1; }
    std::vector<std::thread> th;
    th.reserve(T);
    for (uint32_t t = 0; t < T; t++)
        th.emplace_back([&f, n, t, T] { f((uint32_t)((uint64_t)n * t / T), (uint32_t)((uint64_t)n * (t + 1) / T), t); });
    for (auto &x : th) x.join();
    return T;
}

struct Plan {
    std::vector<AppendDesc> descs;      // documents touched by the append kernel
    std::vector<uint32_t> merge;        // handles to re-merge (batch rows first)
};

// Staged batch layout on the device: [changes][deps][ops][descs][remap][launch docs][handles]
struct StageLayout {
    size_t o_ch, o_dp, o_op, o_desc, o_remap, o_docs, o_hand, o_gather, o_bail, total;
};
StageLayout layout(size_t nc, size_t nd, size_t no, size_t ndesc, size_t nremap, size_t nmerge, size_t ngather, uint32_t S,
                   size_t ninc = 0) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    StageLayout L;
    size_t o = 0;
    L.o_ch = o; o += al(nc * sizeof(hm_change_row) + 1);
    L.o_dp = o; o += al(nd * sizeof(hm_dep_row) + 1);
    L.o_op = o; o += al(no * sizeof(hm_op_row) + 1);
    L.o_desc = o; o += al(ndesc * sizeof(AppendDesc) + 1);
    L.o_remap = o; o += al(nremap + 1);
    L.o_docs = o; o += al(nmerge * sizeof(hm_doc_row) + 1);
    L.o_hand = o; o += al(nmerge * 4 + 1);
    L.o_gather = o; o += al(ngather * (sizeof(hm_doc_result) + 3 * 4 * (size_t)S) + 1);
    L.o_bail = o; o += al(4 * (ninc + 1));
    L.total = o;
    return L;
}

// Launch the merge kernels over `handles` (their current metas) on the engine stream.
int launch_store_merge(hm_store *s, const std::vector<uint32_t> &handles, uint8_t *dev_docs, uint32_t *dev_handles) {
    if (handles.empty()) return HM_OK;
    hipStream_t st = hm_engine_stream(s->e);
    std::vector<hm_doc_row> rows(handles.size());
    hm_batch b = {};
    b.a_stride = s->S;
    size_t tc = 0, td = 0, to = 0, tr = 0;
    for (size_t i = 0; i < handles.size(); i++) {
        const DocMeta &m = s->docs[handles[i]];
        hm_doc_row &r = rows[i];
        r = hm_doc_row{};
        r.change_off = m.c.off; r.n_changes = m.n_c; r.dep_off = m.d.off; r.n_deps = m.n_d;
        r.op_off = m.o.off; r.n_ops = m.n_o; r.reg_off = m.r.off; r.n_regs = m.n_r;
        r.n_objs = m.n_objs; r.n_actors = (uint16_t)m.n_actors; r.flags = m.flags;
        b.max_changes = std::max(b.max_changes, m.n_c); b.max_ops = std::max(b.max_ops, m.n_o);
        b.max_regs = std::max(b.max_regs, m.n_r); b.max_objs = std::max(b.max_objs, m.n_objs);
        b.max_deps = std::max(b.max_deps, m.n_d); b.doc_flags |= m.flags;
        tc += m.n_c; td += m.n_d; to += m.n_o; tr += m.n_r;
    }
    // the large kernel's scratch bound reads the launch totals
    b.n_docs = (uint32_t)handles.size(); b.n_changes = (uint32_t)tc; b.n_deps = (uint32_t)td;
    b.n_ops = (uint32_t)to; b.n_regs = (uint32_t)tr;
    if (!b.max_changes && !b.max_ops && !b.max_regs && !b.max_objs) b.max_objs = 1;   // device hints present
    SCHK(s, hipMemcpyAsync(dev_docs, rows.data(), rows.size() * sizeof(hm_doc_row), hipMemcpyHostToDevice, st));
    SCHK(s, hipMemcpyAsync(dev_handles, handles.data(), handles.size() * 4, hipMemcpyHostToDevice, st));
    b.docs = (const hm_doc_row *)dev_docs;
    b.changes = s->changes; b.deps = s->deps; b.ops = s->ops; b.min_clock = s->min_clock;
    hm_results o;
    o.docs = s->res_docs; o.clock = s->clock; o.back_clock = s->back_clock; o.heads = s->heads;
    o.hist = s->hist; o.all_deps = s->all_deps; o.regs = s->regs; o.surv = s->surv;
    // the launch's host copies must outlive the async H2D copies: synchronise here
    const hm_extents ext = {(uint32_t)s->cap_c, (uint32_t)s->cap_d, (uint32_t)s->cap_o, (uint32_t)s->cap_r};
    int rc = hm_engine_launch_merge(s->e, &b, &o, dev_handles, &ext);
    SCHK(s, hipStreamSynchronize(st));
    return rc;
}

// Allocate a segment of `need` rows from an arena; false if the arena is full.
bool seg_alloc(size_t &used, size_t cap, uint32_t need, Seg &out) {
    const uint32_t c = pow2ceil(std::max<uint32_t>(need, 16));
    if (used + c > cap) return false;
    out.off = (uint32_t)used; out.cap = c;
    used += c;
    return true;
}

// Rebuild every arena larger and compact all documents into it; every document is
// re-merged (its outputs live in the arenas too).  `extra` = rows the caller is about
// to append per space, so the new arenas fit them.
int compact(hm_store *s, size_t extra_c, size_t extra_d, size_t extra_o, size_t extra_r) {
    hipStream_t st = hm_engine_stream(s->e);
    const uint32_t S = s->S;
    size_t live_c = extra_c, live_d = extra_d, live_o = extra_o, live_r = extra_r;
    for (auto &m : s->docs) {
        live_c += pow2ceil(std::max<uint32_t>(m.n_c, 16)); live_d += pow2ceil(std::max<uint32_t>(m.n_d, 16));
        live_o += pow2ceil(std::max<uint32_t>(m.n_o, 16)); live_r += pow2ceil(std::max<uint32_t>(m.n_r, 16));
    }
    const size_t nc = std::max<size_t>(2 * live_c, 1 << 16), nd = std::max<size_t>(2 * live_d, 1 << 16);
    const size_t no = std::max<size_t>(2 * live_o, 1 << 16), nr = std::max<size_t>(2 * live_r, 1 << 16);
    hm_change_row *ch; int32_t *hi; uint32_t *ad; hm_dep_row *dp; hm_op_row *op; hm_surv_result *sv; hm_reg_result *rg;
    int r;
    if ((r = dev_alloc(s, &ch, nc)) || (r = dev_alloc(s, &hi, nc)) || (r = dev_alloc(s, &ad, nc * S)) ||
        (r = dev_alloc(s, &dp, nd)) || (r = dev_alloc(s, &op, no)) || (r = dev_alloc(s, &sv, no)) ||
        (r = dev_alloc(s, &rg, nr)))
        return r;
    // relocate every document (old rows only; no new rows, no remap)
    std::vector<AppendDesc> descs;
    std::vector<uint32_t> all;
    size_t uc = 0, ud = 0, uo = 0, ur = 0;
    std::vector<DocMeta> nm = s->docs;
    for (uint32_t h = 0; h < s->docs.size(); h++) {
        DocMeta &m = nm[h];
        const DocMeta &o = s->docs[h];
        seg_alloc(uc, nc, m.n_c, m.c); seg_alloc(ud, nd, m.n_d, m.d);
        seg_alloc(uo, no, m.n_o, m.o); seg_alloc(ur, nr, m.n_r, m.r);
        AppendDesc D = {};
        D.handle = h;
        D.src_c = o.c.off; D.dst_c = m.c.off; D.n_old_c = o.n_c;
        D.src_d = o.d.off; D.dst_d = m.d.off; D.n_old_d = o.n_d;
        D.src_o = o.o.off; D.dst_o = m.o.off; D.n_old_o = o.n_o;
        D.remap_row = 0xFFFFFFFFu;
        descs.push_back(D);
        all.push_back(h);
    }
    StoreArenas src = {s->changes, s->deps, s->ops, s->min_clock, s->stored};
    StoreArenas dst = {ch, dp, op, s->min_clock, s->stored};
    if (!descs.empty()) {
        const StageLayout L = layout(0, 0, 0, descs.size(), 0, all.size(), 0, S);
        if ((r = ensure_stage(s, L.total))) return r;
        SCHK(s, hipMemcpyAsync(s->stage.p + L.o_desc, descs.data(), descs.size() * sizeof(AppendDesc), hipMemcpyHostToDevice, st));
        SCHK(s, hm_launch_append((const AppendDesc *)(s->stage.p + L.o_desc), (uint32_t)descs.size(), src, dst,
                                 nullptr, nullptr, nullptr, nullptr, S, st));
        SCHK(s, hipStreamSynchronize(st));
    }
    (void)hipFree(s->changes); (void)hipFree(s->hist); (void)hipFree(s->all_deps); (void)hipFree(s->deps);
    (void)hipFree(s->ops); (void)hipFree(s->surv); (void)hipFree(s->regs);
    s->changes = ch; s->hist = hi; s->all_deps = ad; s->deps = dp; s->ops = op; s->surv = sv; s->regs = rg;
    s->cap_c = nc; s->cap_d = nd; s->cap_o = no; s->cap_r = nr;
    s->used_c = uc; s->used_d = ud; s->used_o = uo; s->used_r = ur;
    s->docs = nm;
    if (all.empty()) return HM_OK;
    const StageLayout L = layout(0, 0, 0, 0, 0, all.size(), 0, S);
    if ((r = ensure_stage(s, L.total))) return r;
    return launch_store_merge(s, all, s->stage.p + L.o_docs, (uint32_t *)(s->stage.p + L.o_hand));
}

}  // namespace

extern "C" {

int hm_store_create(hm_engine *e, const hm_store_config *cfg, hm_store **out) {
    if (!e || !out) return HM_ERR_INVALID;
    *out = nullptr;
    const uint32_t S = cfg ? cfg->a_stride : 8;
    if (S == 0 || S > 64) return hm_engine_fail(e, HM_ERR_INVALID, "store a_stride must be in [1,64]");
    hm_store *s = new (std::nothrow) hm_store();
    if (!s) return HM_ERR_NOMEM;
    s->e = e; s->S = S;
    if (hipSetDevice(hm_engine_device(e)) != hipSuccess) { delete s; return HM_ERR_DEVICE; }
    int r = compact(s, 0, 0, 0, 0);
    if (r == HM_OK) r = ensure_handles(s, 1024);
    if (r != HM_OK) { hm_store_destroy(s); return r; }
    *out = s;
    return HM_OK;
}

void hm_store_destroy(hm_store *s) {
    if (!s) return;
    (void)hipStreamSynchronize(hm_engine_stream(s->e));
    void *bufs[] = {s->changes, s->hist, s->all_deps, s->deps, s->ops, s->surv, s->regs, s->res_docs, s->clock,
                    s->back_clock, s->heads, s->min_clock, s->stored, s->stage.p};
    for (void *b : bufs) if (b) (void)hipFree(b);
    delete s;
}

int hm_doc_open(hm_store *s, uint32_t *out_doc) {
    if (!s || !out_doc) return HM_ERR_INVALID;
    try {
        if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "hm_doc_open while a batch is in flight");
        int r = ensure_handles(s, s->docs.size() + 1);
        if (r) return r;
        DocMeta m;
        m.last.err_change = HM_NONE; m.last.err_op = HM_NONE;
        // the new document's merged state is Backend.init(): its result row, written on the
        // engine stream (ordered before any submit; the reads below synchronise the stream)
        const uint32_t h = (uint32_t)s->docs.size();
        s->docs.push_back(m);
        hipStream_t st = hm_engine_stream(s->e);
        SCHK(s, hipMemsetAsync(s->res_docs + h, 0, sizeof(hm_doc_result), st));
        SCHK(s, hipMemsetAsync(&s->res_docs[h].err_change, 0xFF, 2 * sizeof(uint32_t), st));
        *out_doc = h;
        return HM_OK;
    } catch (...) {
        return HM_ERR_NOMEM;
    }
}

int hm_doc_open_n(hm_store *s, uint32_t n, uint32_t *out_first) {
    if (!s || !out_first) return HM_ERR_INVALID;
    try {
        if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "hm_doc_open_n while a batch is in flight");
        const uint32_t h0 = (uint32_t)s->docs.size();
        int r = ensure_handles(s, (size_t)h0 + n);
        if (r) return r;
        DocMeta m;
        m.last.err_change = HM_NONE; m.last.err_op = HM_NONE;
        s->docs.resize((size_t)h0 + n, m);
        std::vector<hm_doc_result> rows(n, m.last);
        if (n) SCHK(s, hipMemcpy(s->res_docs + h0, rows.data(), (size_t)n * sizeof(hm_doc_result), hipMemcpyHostToDevice));
        *out_first = h0;
        return HM_OK;
    } catch (...) {
        return HM_ERR_NOMEM;
    }
}

int hm_batch_submit(hm_store *s, const hm_batch *b, const uint32_t *doc_handles, const uint8_t *actor_remap,
                    uint64_t *out_batch_id) {
    if (!s || !b || (b->n_docs && (!doc_handles || !b->docs))) return HM_ERR_INVALID;
    try {
        if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "a batch is already in flight (call hm_batch_wait)");
        const uint32_t S = s->S, n = b->n_docs;
        if (b->a_stride != S) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch a_stride must equal the store's");
        SCHK(s, hipSetDevice(hm_engine_device(s->e)));
        hipStream_t st = hm_engine_stream(s->e);
        PhaseTimer T(st);
        // validate rows (threads over documents; the first error wins)
        std::vector<uint8_t> seen(s->docs.size(), 0);
        const char *bad = nullptr;
        auto fail_with = [&](const char *m) { const char *expect = nullptr; __atomic_compare_exchange_n(&bad, &expect, m, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED); };
        par_for(n, [&](uint32_t lo, uint32_t hi, uint32_t) {
            for (uint32_t i = lo; i < hi; i++) {
                const uint32_t h = doc_handles[i];
                if (h >= s->docs.size() || __atomic_exchange_n(&seen[h], (uint8_t)1, __ATOMIC_RELAXED)) {
                    fail_with("bad or repeated document handle"); return;
                }
                const hm_doc_row &r = b->docs[i];
                const DocMeta &m = s->docs[h];
                if ((uint64_t)r.change_off + r.n_changes > b->n_changes || (uint64_t)r.dep_off + r.n_deps > b->n_deps ||
                    (uint64_t)r.op_off + r.n_ops > b->n_ops) { fail_with("document rows outside the batch tables"); return; }
                if (r.n_actors > S || r.n_actors < m.n_actors || r.n_regs < m.n_r || r.n_objs < m.n_objs || r.n_objs == 0) {
                    fail_with("document totals must cover the existing log (and n_actors <= a_stride)"); return;
                }
                // every change row must lie inside its document's slice of the batch tables
                for (uint32_t c = r.change_off; c < r.change_off + r.n_changes; c++) {
                    const hm_change_row &cr = b->changes[c];
                    if ((uint64_t)cr.dep_off < r.dep_off || (uint64_t)cr.dep_off + cr.n_deps > (uint64_t)r.dep_off + r.n_deps ||
                        (uint64_t)cr.op_first < r.op_off || (uint64_t)cr.op_first + cr.n_ops > (uint64_t)r.op_off + r.n_ops) {
                        fail_with("change rows outside their document's deps/ops"); return;
                    }
                }
                // the actor re-rank of the existing rows: a permutation into the new ranks.  Checked
                // here, before any document meta or arena pointer moves (a failure leaves the store as it was)
                if (actor_remap) {
                    const uint8_t *mp = actor_remap + (size_t)i * S;
                    uint64_t used = 0;
                    for (uint32_t a = 0; a < m.n_actors; a++) {
                        if (mp[a] >= r.n_actors || ((used >> mp[a]) & 1)) {
                            fail_with("actor remap is not a permutation into the new ranks"); return;
                        }
                        used |= 1ull << mp[a];
                    }
                }
            }
        });
        if (bad) return hm_engine_fail(s->e, HM_ERR_INVALID, bad);
        T.mark("validate");
        // plan segments: a document outgrowing a segment moves to a fresh one at the arena's end;
        // the arenas are compacted first when the worst case would not fit
        {
            std::vector<size_t> part(4 * 16, 0);
            par_for(n, [&](uint32_t lo, uint32_t hi, uint32_t t) {
                size_t c = 0, d = 0, o = 0, g = 0;
                for (uint32_t i = lo; i < hi; i++) {
                    const DocMeta &m = s->docs[doc_handles[i]];
                    c += pow2ceil(std::max<uint32_t>(m.n_c + b->docs[i].n_changes, 16));
                    d += pow2ceil(std::max<uint32_t>(m.n_d + b->docs[i].n_deps, 16));
                    o += pow2ceil(std::max<uint32_t>(m.n_o + b->docs[i].n_ops, 16));
                    g += pow2ceil(std::max<uint32_t>(b->docs[i].n_regs, 16));
                }
                part[4 * t] = c; part[4 * t + 1] = d; part[4 * t + 2] = o; part[4 * t + 3] = g;
            });
            size_t need_c = 0, need_d = 0, need_o = 0, need_r = 0;
            for (uint32_t t = 0; t < 16; t++) { need_c += part[4 * t]; need_d += part[4 * t + 1]; need_o += part[4 * t + 2]; need_r += part[4 * t + 3]; }
            if (s->used_c + need_c > s->cap_c || s->used_d + need_d > s->cap_d || s->used_o + need_o > s->cap_o ||
                s->used_r + need_r > s->cap_r) {
                int r = compact(s, need_c, need_d, need_o, need_r);
                if (r) return r;
            }
        }
        T.mark("plan: sizes");
        s->p_old.resize(n);
        s->p_inv_row.resize(n);
        s->p_inv.clear();
        s->p_handles.assign(doc_handles, doc_handles + n);
        s->descs.resize(n);
        std::vector<AppendDesc> &descs = s->descs;
        uint32_t n_remap = 0;
        std::vector<uint8_t> remap_rows;
        // re-ranked documents (rare): their remap rows, in batch order
        if (actor_remap) {
            for (uint32_t i = 0; i < n; i++) {
                const DocMeta &m = s->docs[doc_handles[i]];
                const uint8_t *mp = actor_remap + (size_t)i * S;
                bool ident = true;
                for (uint32_t a = 0; a < m.n_actors; a++) if (mp[a] != a) ident = false;
                s->p_inv_row[i] = -1;
                if (ident) continue;
                const size_t at = remap_rows.size();
                remap_rows.resize(at + S, 0xFF);
                s->p_inv_row[i] = (int32_t)s->p_inv.size();
                s->p_inv.resize(s->p_inv.size() + S, 0xFF);
                uint8_t *inv = s->p_inv.data() + s->p_inv_row[i];
                for (uint32_t a = 0; a < m.n_actors; a++) { remap_rows[at + a] = mp[a]; inv[mp[a]] = (uint8_t)a; }   // validated above
                descs[i].remap_row = n_remap++;
            }
        }
        // new segments: sizes per document (0 = fits), then arena offsets by a prefix over the
        // batch (threads sum their ranges, one serial pass over the partial sums)
        s->grow.resize(4 * (size_t)n);
        std::vector<uint32_t> &grow = s->grow;
        std::vector<size_t> base(4 * 17, 0);
        const uint32_t TT = par_for(n, [&](uint32_t lo, uint32_t hi, uint32_t t) {
            size_t acc[4] = {0, 0, 0, 0};
            for (uint32_t i = lo; i < hi; i++) {
                const DocMeta &m = s->docs[doc_handles[i]];
                const hm_doc_row &r = b->docs[i];
                uint32_t *g = &grow[4 * (size_t)i];
                g[0] = g[1] = g[2] = g[3] = 0;
                if (m.n_c + r.n_changes > m.c.cap) g[0] = pow2ceil(std::max<uint32_t>(m.n_c + r.n_changes, 16));
                if (m.n_d + r.n_deps > m.d.cap) g[1] = pow2ceil(std::max<uint32_t>(m.n_d + r.n_deps, 16));
                if (m.n_o + r.n_ops > m.o.cap) g[2] = pow2ceil(std::max<uint32_t>(m.n_o + r.n_ops, 16));
                if (r.n_regs > m.r.cap) g[3] = pow2ceil(std::max<uint32_t>(r.n_regs, 16));
                for (int k = 0; k < 4; k++) acc[k] += g[k];
            }
            for (int k = 0; k < 4; k++) base[4 * (t + 1) + k] = acc[k];
        });
        T.mark("plan: grow");
        base[0] = s->used_c; base[1] = s->used_d; base[2] = s->used_o; base[3] = s->used_r;
        for (uint32_t t = 1; t <= TT; t++) for (int k = 0; k < 4; k++) base[4 * t + k] += base[4 * (t - 1) + k];
        s->used_c = base[4 * TT]; s->used_d = base[4 * TT + 1]; s->used_o = base[4 * TT + 2]; s->used_r = base[4 * TT + 3];
        // route: a document whose resident state is clean (last merge ok, nothing queued, no
        // re-rank) and whose new rows fit the incremental tiles is applied by inc_apply_kernel;
        // the rest re-merge their whole log (DocBackend.applyRemoteChanges either way)
        struct Part { std::vector<uint32_t> cold; uint32_t n_inc = 0, mx[6] = {0, 0, 0, 0, 0, 0}; };
        std::vector<Part> parts(16);
        par_for(n, [&](uint32_t lo, uint32_t hi, uint32_t t) {
            size_t at[4] = {base[4 * t], base[4 * t + 1], base[4 * t + 2], base[4 * t + 3]};
            Part P;                                                   // thread-local (no false sharing)
            for (uint32_t i = lo; i < hi; i++) {
                const uint32_t h = doc_handles[i];
                DocMeta &m = s->docs[h];
                const hm_store::OldMeta o = {m.n_c, m.n_d, m.n_o, m.n_r, m.n_objs, (uint16_t)m.n_actors, m.flags};
                s->p_old[i] = o;
                const hm_doc_result last = m.last;
                const hm_doc_row &r = b->docs[i];
                AppendDesc &D = descs[i];
                const uint32_t remap_row = D.remap_row;
                D = AppendDesc{};
                D.handle = h;
                D.src_c = m.c.off; D.n_old_c = m.n_c; D.new_c = r.change_off; D.n_new_c = r.n_changes;
                D.src_d = m.d.off; D.n_old_d = m.n_d; D.new_d = r.dep_off; D.n_new_d = r.n_deps;
                D.src_o = m.o.off; D.n_old_o = m.n_o; D.new_o = r.op_off; D.n_new_o = r.n_ops;
                D.src_r = m.r.off; D.n_old_r = m.n_r;
                const uint32_t *g = &grow[4 * (size_t)i];
                Seg *segs[4] = {&m.c, &m.d, &m.o, &m.r};
                for (int k = 0; k < 4; k++) if (g[k]) { segs[k]->off = (uint32_t)at[k]; segs[k]->cap = g[k]; at[k] += g[k]; }
                D.dst_c = m.c.off; D.dst_d = m.d.off; D.dst_o = m.o.off; D.dst_r = m.r.off;
                if (!actor_remap) s->p_inv_row[i] = -1;
                D.remap_row = actor_remap && s->p_inv_row[i] >= 0 ? remap_row : 0xFFFFFFFFu;
                const bool reranked = D.remap_row != 0xFFFFFFFFu;
                m.n_c += r.n_changes; m.n_d += r.n_deps; m.n_o += r.n_ops;
                m.n_r = r.n_regs; m.n_objs = r.n_objs; m.n_actors = r.n_actors; m.flags |= r.flags;
                D.n_r = m.n_r; D.n_actors = (uint16_t)m.n_actors; D.n_objs = m.n_objs;
                const uint32_t tgt = r.n_deps + r.n_changes;            // fold steps: deps + own predecessor
                const bool inc = s->incremental && last.status == HM_OK && last.n_queued == 0 && !reranked &&
                                 r.n_changes > 0 && r.n_changes <= HM_INC_MAX_NEW_C && r.n_ops <= HM_INC_MAX_NEW_O &&
                                 tgt <= HM_INC_MAX_TGT && m.n_r <= HM_INC_MAX_REGS && last.n_surv <= HM_INC_MAX_SURV &&
                                 o.n_r <= m.n_r && m.n_actors <= S && !((o.flags | r.flags) & HM_DOC_HAS_LISTS);
                if (!inc) { P.cold.push_back(h); continue; }
                D.inc = 1;
                P.n_inc++;
                const uint32_t v[6] = {r.n_changes, tgt, std::min<uint32_t>(o.n_c, HM_INC_MAX_STAGE), m.n_r, last.n_surv,
                                       std::min<uint32_t>(r.n_ops, HM_INC_SLOTS)};
                for (int k = 0; k < 6; k++) P.mx[k] = std::max(P.mx[k], v[k]);
            }
            parts[t] = std::move(P);
        });
        T.mark("plan: route");
        std::vector<uint32_t> cold;
        uint32_t n_inc = 0, mx[6] = {0, 0, 0, 0, 0, 0};
        for (auto &P : parts) {
            cold.insert(cold.end(), P.cold.begin(), P.cold.end());
            n_inc += P.n_inc;
            for (int k = 0; k < 6; k++) mx[k] = std::max(mx[k], P.mx[k]);
        }
        const uint32_t mx_new_c = mx[0], mx_tgt = mx[1], mx_stage = mx[2], mx_regs = mx[3], mx_surv = mx[4], mx_slots = mx[5];
        T.mark("plan+route");
        // stage and launch: append, merge, gather
        const StageLayout L = layout(b->n_changes, b->n_deps, b->n_ops, n, remap_rows.size(), n, n, S, n_inc ? n : 0);
        int rc = ensure_stage(s, L.total);
        if (rc) return rc;
        uint8_t *sp = s->stage.p;
        if (b->n_changes) SCHK(s, hipMemcpyAsync(sp + L.o_ch, b->changes, b->n_changes * sizeof(hm_change_row), hipMemcpyHostToDevice, st));
        if (b->n_deps) SCHK(s, hipMemcpyAsync(sp + L.o_dp, b->deps, b->n_deps * sizeof(hm_dep_row), hipMemcpyHostToDevice, st));
        if (b->n_ops) SCHK(s, hipMemcpyAsync(sp + L.o_op, b->ops, b->n_ops * sizeof(hm_op_row), hipMemcpyHostToDevice, st));
        if (n) SCHK(s, hipMemcpyAsync(sp + L.o_desc, descs.data(), n * sizeof(AppendDesc), hipMemcpyHostToDevice, st));
        T.mark("stage: h2d");
        if (!remap_rows.empty()) SCHK(s, hipMemcpyAsync(sp + L.o_remap, remap_rows.data(), remap_rows.size(), hipMemcpyHostToDevice, st));
        StoreArenas ar = {s->changes, s->deps, s->ops, s->min_clock, s->stored};
        SCHK(s, hm_launch_append((const AppendDesc *)(sp + L.o_desc), n, ar, ar, (const hm_change_row *)(sp + L.o_ch),
                                 (const hm_dep_row *)(sp + L.o_dp), (const hm_op_row *)(sp + L.o_op),
                                 remap_rows.empty() ? nullptr : sp + L.o_remap, S, st));
        T.mark("stage+append");
        if (n_inc) {
            const IncDims M = hm_inc_dims(S, mx_new_c, mx_tgt, mx_stage, mx_regs, mx_surv, mx_slots);
            IncArenas A = {s->changes, s->deps, s->ops, s->hist, s->all_deps, s->regs, s->surv,
                           s->res_docs, s->clock, s->back_clock, s->heads, s->min_clock};
            SCHK(s, hm_launch_inc_apply((const AppendDesc *)(sp + L.o_desc), n, A, M, (uint32_t *)(sp + L.o_bail), st));
        }
        T.mark("incremental");
        rc = launch_store_merge(s, cold, sp + L.o_docs, (uint32_t *)(sp + L.o_hand));
        if (rc) return rc;
        T.mark("remerge");
        s->st_inc = n_inc; s->st_cold = (uint32_t)cold.size(); s->st_bail = 0;
        if (n_inc) {
            // documents the incremental kernel handed back re-merge their whole log
            uint32_t nb = 0;
            SCHK(s, hipMemcpyAsync(&nb, sp + L.o_bail, 4, hipMemcpyDeviceToHost, st));
            SCHK(s, hipStreamSynchronize(st));
            std::vector<uint32_t> again(nb);
            if (nb) {
                SCHK(s, hipMemcpyAsync(again.data(), sp + L.o_bail + 4, (size_t)nb * 4, hipMemcpyDeviceToHost, st));
                SCHK(s, hipStreamSynchronize(st));
                std::sort(again.begin(), again.end());
            }
            s->st_bail = (uint32_t)again.size(); s->st_inc -= s->st_bail;
            rc = launch_store_merge(s, again, sp + L.o_docs, (uint32_t *)(sp + L.o_hand));
            if (rc) return rc;
        }
        T.mark("handed back");
        // the merges above used the handle region for their own document lists
        if (n) SCHK(s, hipMemcpyAsync(sp + L.o_hand, s->p_handles.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hm_launch_gather((const uint32_t *)(sp + L.o_hand), n, S, s->res_docs, s->clock, s->back_clock, s->heads,
                                 sp + L.o_gather, st));
        s->p_gather_dev = sp + L.o_gather;
        T.mark("gather+d2h");
        s->pending = true;
        s->pending_id = s->next_id++;
        if (out_batch_id) *out_batch_id = s->pending_id;
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_batch_submit");
    }
}

int hm_batch_wait(hm_store *s, uint64_t batch_id, hm_doc_result *out_docs, uint32_t *out_clock,
                  uint32_t *out_back_clock, uint32_t *out_heads) {
    if (!s) return HM_ERR_INVALID;
    try {
        if (!s->pending || batch_id != s->pending_id) return hm_engine_fail(s->e, HM_ERR_INVALID, "no such batch in flight");
        SCHK(s, hipSetDevice(hm_engine_device(s->e)));        // the caller may be a host thread of its own
        hipStream_t st = hm_engine_stream(s->e);
        PhaseTimer T(st);
        // the batch stays in flight (pending) until this returns: copy-out and rollback below
        // still read and re-merge the store's documents
        struct Clear { std::atomic<bool> &p; ~Clear() { p.store(false); } } clear_pending{s->pending};
        SCHK(s, hipStreamSynchronize(st));
        T.mark("wait sync");
        const uint32_t n = (uint32_t)s->p_handles.size(), S = s->S;
        // results straight from the gathered device rows into the caller's arrays
        std::vector<hm_doc_result> tmp;
        hm_doc_result *res = out_docs;
        if (!res) { tmp.resize(n); res = tmp.data(); }
        if (n) {
            const uint8_t *g = s->p_gather_dev;
            const size_t rb = (size_t)n * S * 4;
            SCHK(s, hipMemcpyAsync(res, g, (size_t)n * sizeof(hm_doc_result), hipMemcpyDeviceToHost, st));
            g += (size_t)n * sizeof(hm_doc_result);
            if (out_clock) SCHK(s, hipMemcpyAsync(out_clock, g, rb, hipMemcpyDeviceToHost, st));
            if (out_back_clock) SCHK(s, hipMemcpyAsync(out_back_clock, g + rb, rb, hipMemcpyDeviceToHost, st));
            if (out_heads) SCHK(s, hipMemcpyAsync(out_heads, g + 2 * rb, rb, hipMemcpyDeviceToHost, st));
            SCHK(s, hipStreamSynchronize(st));
        }
        T.mark("wait copy-out");
        // roll back documents whose merge threw (or left the envelope): the log returns to
        // its previous length (rows stay where they are), ranks are re-ranked back, and the
        // previous state is re-merged
        std::vector<uint32_t> back;
        std::vector<AppendDesc> descs;
        std::vector<uint8_t> remap_rows;
        uint32_t n_remap = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t h = s->p_handles[i];
            if (res[i].status == HM_OK) { s->docs[h].last = res[i]; continue; }
            DocMeta &m = s->docs[h];
            const hm_store::OldMeta &o = s->p_old[i];
            AppendDesc D = {};
            D.handle = h;
            D.src_c = D.dst_c = m.c.off; D.n_old_c = o.n_c;
            D.src_d = D.dst_d = m.d.off; D.n_old_d = o.n_d;
            D.src_o = D.dst_o = m.o.off; D.n_old_o = o.n_o;
            D.remap_row = 0xFFFFFFFFu;
            if (s->p_inv_row[i] >= 0) {
                D.remap_row = n_remap++;
                const uint8_t *inv = s->p_inv.data() + s->p_inv_row[i];
                remap_rows.insert(remap_rows.end(), inv, inv + S);
            }
            m.n_c = o.n_c; m.n_d = o.n_d; m.n_o = o.n_o; m.n_r = o.n_r; m.n_objs = o.n_objs;
            m.n_actors = o.n_actors; m.flags = o.flags;
            descs.push_back(D);
            back.push_back(h);
        }
        if (!back.empty()) {
            const StageLayout L = layout(0, 0, 0, descs.size(), remap_rows.size(), back.size(), 0, S);
            int rc = ensure_stage(s, L.total);
            if (rc) return rc;
            uint8_t *sp = s->stage.p;
            SCHK(s, hipMemcpyAsync(sp + L.o_desc, descs.data(), descs.size() * sizeof(AppendDesc), hipMemcpyHostToDevice, st));
            if (!remap_rows.empty()) SCHK(s, hipMemcpyAsync(sp + L.o_remap, remap_rows.data(), remap_rows.size(), hipMemcpyHostToDevice, st));
            StoreArenas ar = {s->changes, s->deps, s->ops, s->min_clock, s->stored};
            SCHK(s, hm_launch_append((const AppendDesc *)(sp + L.o_desc), (uint32_t)descs.size(), ar, ar, nullptr, nullptr,
                                     nullptr, remap_rows.empty() ? nullptr : sp + L.o_remap, S, st));
            rc = launch_store_merge(s, back, sp + L.o_docs, (uint32_t *)(sp + L.o_hand));
            if (rc) return rc;
        }
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_batch_wait");
    }
}

int hm_store_set_incremental(hm_store *s, int on) {
    if (!s) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    s->incremental = on != 0;
    return HM_OK;
}

int hm_store_last_routing(const hm_store *s, uint32_t *out3) {
    if (!s || !out3) return HM_ERR_INVALID;
    out3[0] = s->st_inc; out3[1] = s->st_cold; out3[2] = s->st_bail;
    return HM_OK;
}

int hm_doc_info(hm_store *s, uint32_t doc, hm_doc_info_t *out) {
    if (!s || !out || doc >= s->docs.size()) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    SCHK(s, hipStreamSynchronize(hm_engine_stream(s->e)));
    const DocMeta &m = s->docs[doc];
    hm_doc_result r;
    SCHK(s, hipMemcpy(&r, s->res_docs + doc, sizeof(r), hipMemcpyDeviceToHost));
    out->n_changes = m.n_c; out->n_deps = m.n_d; out->n_ops = m.n_o; out->n_regs = m.n_r;
    out->n_objs = m.n_objs; out->n_actors = m.n_actors;
    out->hist_len = r.hist_len; out->n_queued = r.n_queued; out->n_surv = r.n_surv; out->status = r.status;
    return HM_OK;
}

int hm_doc_read(hm_store *s, uint32_t doc, int32_t *hist, uint32_t *all_deps, hm_reg_result *regs,
                hm_surv_result *surv, uint32_t *clock, uint32_t *back_clock, uint32_t *heads) {
    if (!s || doc >= s->docs.size()) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    SCHK(s, hipStreamSynchronize(hm_engine_stream(s->e)));
    const DocMeta &m = s->docs[doc];
    const uint32_t S = s->S;
    if (hist && m.n_c) SCHK(s, hipMemcpy(hist, s->hist + m.c.off, m.n_c * 4, hipMemcpyDeviceToHost));
    if (all_deps && m.n_c) SCHK(s, hipMemcpy(all_deps, s->all_deps + (size_t)m.c.off * S, (size_t)m.n_c * S * 4, hipMemcpyDeviceToHost));
    if (regs && m.n_r) SCHK(s, hipMemcpy(regs, s->regs + m.r.off, m.n_r * sizeof(hm_reg_result), hipMemcpyDeviceToHost));
    if (surv && m.n_o) SCHK(s, hipMemcpy(surv, s->surv + m.o.off, m.n_o * sizeof(hm_surv_result), hipMemcpyDeviceToHost));
    if (clock) SCHK(s, hipMemcpy(clock, s->clock + (size_t)doc * S, S * 4, hipMemcpyDeviceToHost));
    if (back_clock) SCHK(s, hipMemcpy(back_clock, s->back_clock + (size_t)doc * S, S * 4, hipMemcpyDeviceToHost));
    if (heads) SCHK(s, hipMemcpy(heads, s->heads + (size_t)doc * S, S * 4, hipMemcpyDeviceToHost));
    return HM_OK;
}

int hm_doc_log(hm_store *s, uint32_t doc, hm_change_row *changes, hm_dep_row *deps, hm_op_row *ops) {
    if (!s || doc >= s->docs.size()) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    const DocMeta &m = s->docs[doc];
    if (changes && m.n_c) {
        SCHK(s, hipMemcpy(changes, s->changes + m.c.off, m.n_c * sizeof(hm_change_row), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < m.n_c; i++) { changes[i].dep_off -= m.d.off; changes[i].op_first -= m.o.off; }
    }
    if (deps && m.n_d) SCHK(s, hipMemcpy(deps, s->deps + m.d.off, m.n_d * sizeof(hm_dep_row), hipMemcpyDeviceToHost));
    if (ops && m.n_o) SCHK(s, hipMemcpy(ops, s->ops + m.o.off, m.n_o * sizeof(hm_op_row), hipMemcpyDeviceToHost));
    return HM_OK;
}

int hm_store_read_regs(hm_store *s, uint32_t n, const uint32_t *doc_handles, const uint32_t *regs,
                       hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t surv_cap, uint32_t *out_n_surv) {
    if (!s || (n && (!doc_handles || !regs || !out_regs || (surv_cap && !out_surv)))) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    try {
        std::vector<uint32_t> req(2 * (size_t)n);
        for (uint32_t i = 0; i < n; i++) {
            if (doc_handles[i] >= s->docs.size()) return hm_engine_fail(s->e, HM_ERR_INVALID, "bad handle");
            const DocMeta &m = s->docs[doc_handles[i]];
            if (regs[i] >= m.n_r) return hm_engine_fail(s->e, HM_ERR_INVALID, "register outside its document");
            req[i] = m.r.off + regs[i];
            req[n + i] = m.o.off;
        }
        if (out_n_surv) *out_n_surv = 0;
        if (!n) return HM_OK;
        hipStream_t st = hm_engine_stream(s->e);
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t o_req = 0, o_cnt = al(8 * (size_t)n), o_regs = o_cnt + 256,
                     o_surv = o_regs + al((size_t)n * sizeof(hm_reg_result)), total = o_surv + al((size_t)surv_cap * sizeof(hm_surv_result) + 1);
        int rc = ensure_stage(s, total);
        if (rc) return rc;
        uint8_t *sp = s->stage.p;
        SCHK(s, hipMemcpyAsync(sp + o_req, req.data(), req.size() * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hipMemsetAsync(sp + o_cnt, 0, 4, st));
        SCHK(s, hm_launch_read_regs(n, (const uint32_t *)(sp + o_req), (const uint32_t *)(sp + o_req) + n, s->regs, s->surv,
                                    (hm_reg_result *)(sp + o_regs), (hm_surv_result *)(sp + o_surv), surv_cap,
                                    (uint32_t *)(sp + o_cnt), st));
        uint32_t total_surv = 0;
        SCHK(s, hipMemcpyAsync(&total_surv, sp + o_cnt, 4, hipMemcpyDeviceToHost, st));
        SCHK(s, hipMemcpyAsync(out_regs, sp + o_regs, (size_t)n * sizeof(hm_reg_result), hipMemcpyDeviceToHost, st));
        SCHK(s, hipStreamSynchronize(st));
        if (out_n_surv) *out_n_surv = total_surv;
        if (total_surv > surv_cap) return hm_engine_fail(s->e, HM_ERR_NOMEM, "surv_cap below the survivors of the registers");
        if (total_surv) SCHK(s, hipMemcpy(out_surv, sp + o_surv, (size_t)total_surv * sizeof(hm_surv_result), hipMemcpyDeviceToHost));
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_store_read_regs");
    }
}

int hm_doc_history_prefix(hm_store *s, uint32_t doc, uint32_t n, uint32_t *out) {
    if (!s || doc >= s->docs.size() || (n && !out)) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    const DocMeta &m = s->docs[doc];
    std::vector<int32_t> h(m.n_c);
    if (m.n_c) SCHK(s, hipMemcpy(h.data(), s->hist + m.c.off, m.n_c * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> by_pos(m.n_c, HM_NONE);
    uint32_t H = 0;
    for (uint32_t i = 0; i < m.n_c; i++)
        if (h[i] >= 0 && (uint32_t)h[i] < m.n_c) { by_pos[h[i]] = i; H = std::max(H, (uint32_t)h[i] + 1); }
    const uint32_t k = std::min(n, H);
    for (uint32_t i = 0; i < k; i++) out[i] = by_pos[i];
    return (int)k;
}

int hm_doc_set_min_clock(hm_store *s, uint32_t doc, const uint32_t *clock) {
    if (!s || doc >= s->docs.size() || !clock) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    SCHK(s, hipMemcpy(s->min_clock + (size_t)doc * s->S, clock, s->S * 4, hipMemcpyHostToDevice));
    return HM_OK;
}

int hm_store_clock_update(hm_store *s, uint32_t n, const uint32_t *docs, uint8_t *out_written, uint8_t *out_differs,
                          uint32_t *out_stored) {
    if (!s || (n && !docs)) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    try {
        for (uint32_t i = 0; i < n; i++) if (docs[i] >= s->docs.size()) return hm_engine_fail(s->e, HM_ERR_INVALID, "bad handle");
        if (!n) return HM_OK;
        const uint32_t S = s->S;
        hipStream_t st = hm_engine_stream(s->e);
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t o_h = 0, o_w = al(n * 4), o_d = o_w + al(n + 4), o_s = o_d + al(n + 4), total = o_s + al((size_t)n * S * 4);
        int rc = ensure_stage(s, total);
        if (rc) return rc;
        uint8_t *sp = s->stage.p;
        SCHK(s, hipMemcpyAsync(sp + o_h, docs, n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hipMemsetAsync(sp + o_w, 0, o_s - o_w, st));
        SCHK(s, hm_launch_clock_update((const uint32_t *)(sp + o_h), n, S, s->back_clock, s->stored, sp + o_w, sp + o_d,
                                       (uint32_t *)(sp + o_s), st));
        if (out_written) SCHK(s, hipMemcpyAsync(out_written, sp + o_w, n, hipMemcpyDeviceToHost, st));
        if (out_differs) SCHK(s, hipMemcpyAsync(out_differs, sp + o_d, n, hipMemcpyDeviceToHost, st));
        if (out_stored) SCHK(s, hipMemcpyAsync(out_stored, sp + o_s, (size_t)n * S * 4, hipMemcpyDeviceToHost, st));
        SCHK(s, hipStreamSynchronize(st));
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_store_clock_update");
    }
}

int hm_sync_ranges_device(hm_engine *e, const uint64_t *present, const uint64_t *word_off, const uint32_t *lo,
                          const uint32_t *hi, uint32_t *out_end, uint32_t n, void *stream) {
    if (!e) return HM_ERR_INVALID;
    hipError_t r = hm_launch_sync_ranges(present, word_off, lo, hi, out_end, n,
                                         stream ? (hipStream_t)stream : hm_engine_stream(e));
    return r == hipSuccess ? HM_OK : hm_engine_fail(e, HM_ERR_DEVICE, "sync_ranges launch");
}

int hm_sync_ranges_host(hm_engine *e, const uint64_t *present, const uint64_t *word_off, const uint32_t *lo,
                        const uint32_t *hi, uint32_t *out_end, uint32_t n, uint32_t n_words) {
    if (!e || (n && (!present || !word_off || !lo || !hi || !out_end))) return HM_ERR_INVALID;
    if (!n) return HM_OK;
    for (uint32_t i = 0; i < n; i++)
        if (word_off[i] > n_words || hi[i] < lo[i] || word_off[i] + ((uint64_t)hi[i] + 63) / 64 > n_words)
            return hm_engine_fail(e, HM_ERR_INVALID, "sync range outside the present bitmap");
    hipStream_t st = hm_engine_stream(e);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_p = 0, o_w = al(8 * (size_t)n_words + 8), o_lo = o_w + al(8 * (size_t)n), o_hi = o_lo + al(4 * (size_t)n),
                 o_out = o_hi + al(4 * (size_t)n), total = o_out + al(4 * (size_t)n);
    uint8_t *sp = nullptr;
    if (hipMalloc((void **)&sp, total) != hipSuccess) return hm_engine_fail(e, HM_ERR_NOMEM, "hipMalloc sync staging");
    int rc = HM_OK;
    if (hipMemcpyAsync(sp + o_p, present, 8 * (size_t)n_words, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(sp + o_w, word_off, 8 * (size_t)n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(sp + o_lo, lo, 4 * (size_t)n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(sp + o_hi, hi, 4 * (size_t)n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hm_launch_sync_ranges((const uint64_t *)(sp + o_p), (const uint64_t *)(sp + o_w), (const uint32_t *)(sp + o_lo),
                              (const uint32_t *)(sp + o_hi), (uint32_t *)(sp + o_out), n, st) != hipSuccess ||
        hipMemcpyAsync(out_end, sp + o_out, 4 * (size_t)n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        rc = hm_engine_fail(e, HM_ERR_DEVICE, "hm_sync_ranges_host");
    (void)hipFree(sp);
    return rc;
}

}  // extern "C"
