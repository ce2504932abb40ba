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
//
// The documents' segments and totals live on the device (DevDoc, 64 B per handle) and a
// submit is planned there: plan_kernel checks every row and routes it, alloc_kernel takes
// the new segments from device bump pointers and writes the append descriptors, the
// rollback of failed documents is a kernel too.  The host moves only the batch tables, a
// few 64-byte plan summaries, and the per-document results.
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
// a compacted segment: its rows and a quarter as many again, to a power of two (the plan grows
// segments the same way, store_kernels.hip grow_rows)
uint32_t seg_cap(uint32_t n) {
    const uint64_t x = (uint64_t)n + (n >> 2);
    return pow2ceil((uint32_t)std::max<uint64_t>(std::min<uint64_t>(x, 0x80000000ull), 16));
}

}  // namespace

struct hm_store {
    hm_engine *e = nullptr;
    uint32_t S = 8;
    uint32_t n_handles = 0;
    // arenas (capacity in rows); the bump pointers live in the device PlanStats
    size_t cap_c = 0, cap_d = 0, cap_o = 0, cap_r = 0;
    hm_change_row *changes = nullptr; int32_t *hist = nullptr; uint32_t *all_deps = nullptr; uint32_t *ckey = nullptr;
    hm_dep_row *deps = nullptr;
    hm_op_row *ops = nullptr; hm_surv_result *surv = nullptr; uint2 *smeta = nullptr;
    hm_reg_result *regs = nullptr;
    uint32_t *epos = nullptr, *epar = nullptr, *ekey = nullptr, *lorder = nullptr;   // reg space: resident list order
    // per handle
    size_t cap_h = 0;
    DevDoc *dm = nullptr;                         // segments and totals
    IncState *ist = nullptr;                      // survivor slots / metadata state of the incremental path
    uint2 *ldir = nullptr;                        // list directory (HM_INC_LISTS per handle)
    uint32_t *seen = nullptr;                     // submit stamps (repeated-handle check)
    hm_doc_result *res_docs = nullptr;
    uint32_t *clock = nullptr, *back_clock = nullptr, *heads = nullptr, *min_clock = nullptr, *stored = nullptr;
    // per submit (device): plan rows, descriptors, lists, stats
    DBuf<PlanRow> plan;
    DBuf<AppendDesc> descs, bdescs;
    DBuf<uint32_t> list;                          // re-merge list (cold, then handed back)
    DBuf<uint32_t> blist;                         // rollback list
    DBuf<uint32_t> klist;                         // a re-merge's documents that may keep incremental state
    DBuf<int> mpart;                              // inc_meta_kernel's per-workgroup n_valid changes
    DBuf<uint32_t> alist;                         // append list (batch rows with append work)
    DBuf<uint8_t> remap, inv;
    DBuf<hm_doc_row> rows;
    PlanStats *st = nullptr;
    uint32_t stamp = 0;
    // staging (device)
    DBuf<uint8_t> stage;
    // in-flight batch
    std::atomic<bool> pending{false};             // a submitted batch not yet waited for (other threads may read it)
    uint64_t next_id = 1, pending_id = 0;
    uint32_t p_n = 0;                             // batch rows
    uint32_t *p_handles_dev = nullptr;            // batch rows -> handles (staged, or the caller's device array)
    bool p_remap = false;
    uint8_t *p_gather_dev = nullptr;
    uint32_t *p_fail_dev = nullptr;               // rows whose status is not OK (gather_kernel)
    // the last waited batch, for hm_batch_undo (until the next submit)
    uint64_t undo_id = 0;
    uint32_t undo_n = 0;
    DBuf<uint32_t> undo_handles;
    // incremental applyRemoteChanges (inc_apply_kernel) and the last submit's routing
    bool incremental = true;
    // some document holds incremental state a submit can use (PlanStats.n_valid > 0, read back after
    // every re-merge): without one no document can route to the incremental kernels and a submit
    // does not launch them
    bool any_state = false;
    uint32_t inc_mode = 1;                        // 1: small list documents re-merge (cost policy); 2: every one
    uint32_t st_inc = 0, st_cold = 0, st_bail = 0;
    // HIP events around the last submit's incremental kernels and its re-merge (engine stream)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // page-locked host words the submit's small read-backs land in (a pageable destination makes
    // each copy a staged, synchronous one): the plan stats, then the re-merge counts
    PlanStats *h_st = nullptr;
    uint32_t *h_cnt = nullptr;
    bool ev_live = false;                    // ev[] recorded by the pending submit, not read yet
    float last_ms[2] = {0.f, 0.f};
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

// a per-submit device buffer of at least n elements (contents not kept)
template <typename T>
int ensure_buf(hm_store *s, DBuf<T> &b, size_t n) {
    if (n <= b.cap && b.p) return HM_OK;
    SCHK(s, hipStreamSynchronize(hm_engine_stream(s->e)));
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr; b.cap = 0;
    const size_t cap = std::max<size_t>(n, 1024) * 3 / 2;
    if (hipMalloc((void **)&b.p, cap * sizeof(T)) != hipSuccess) return hm_engine_fail(s->e, HM_ERR_NOMEM, "hipMalloc store buffer");
    b.cap = cap;
    return HM_OK;
}

int ensure_stage(hm_store *s, size_t bytes) { return ensure_buf(s, s->stage, bytes); }

PlanStats read_stats(hm_store *s, int *rc) {
    PlanStats st;
    memset(&st, 0, sizeof st);
    hipStream_t q = hm_engine_stream(s->e);
    if (hipMemcpyAsync(s->h_st, s->st, sizeof st, hipMemcpyDeviceToHost, q) != hipSuccess || hipStreamSynchronize(q) != hipSuccess)
        *rc = hm_engine_fail(s->e, HM_ERR_DEVICE, "reading the submit plan");
    else
        st = *s->h_st;
    return st;
}

// zero the per-phase fields of the device stats, keeping the bump pointers
int reset_stats(hm_store *s) {
    SCHK(s, hipMemsetAsync(s->st, 0, offsetof(PlanStats, bump), hm_engine_stream(s->e)));
    return HM_OK;
}

DevDoc read_doc(hm_store *s, uint32_t h, int *rc) {
    DevDoc m;
    memset(&m, 0, sizeof m);
    hipStream_t q = hm_engine_stream(s->e);
    if (hipMemcpyAsync(&m, s->dm + h, sizeof m, hipMemcpyDeviceToHost, q) != hipSuccess || hipStreamSynchronize(q) != hipSuccess)
        *rc = hm_engine_fail(s->e, HM_ERR_DEVICE, "reading a document's meta");
    return m;
}

// grow the per-handle tables to hold `need` documents (contents preserved)
int ensure_handles(hm_store *s, size_t need) {
    if (need <= s->cap_h) return HM_OK;
    const size_t cap = std::max<size_t>(need, std::max<size_t>(1024, s->cap_h * 2));
    hipStream_t st = hm_engine_stream(s->e);
    const uint32_t S = s->S;
    hm_doc_result *rd; DevDoc *dm; uint32_t *seen; IncState *ist; uint2 *ldir; int r;
    if ((r = dev_alloc(s, &rd, cap)) || (r = dev_alloc(s, &dm, cap)) || (r = dev_alloc(s, &seen, cap)) ||
        (r = dev_alloc(s, &ist, cap)) || (r = dev_alloc(s, &ldir, cap * HM_INC_LISTS)))
        return r;
    SCHK(s, hipMemsetAsync(rd, 0, cap * sizeof(hm_doc_result), st));
    SCHK(s, hipMemsetAsync(dm, 0, cap * sizeof(DevDoc), st));
    SCHK(s, hipMemsetAsync(seen, 0, cap * 4, st));
    SCHK(s, hipMemsetAsync(ist, 0, cap * sizeof(IncState), st));
    SCHK(s, hipMemsetAsync(ldir, 0, cap * HM_INC_LISTS * sizeof(uint2), st));
    if (s->cap_h) {
        SCHK(s, hipMemcpyAsync(rd, s->res_docs, s->cap_h * sizeof(hm_doc_result), hipMemcpyDeviceToDevice, st));
        SCHK(s, hipMemcpyAsync(dm, s->dm, s->cap_h * sizeof(DevDoc), hipMemcpyDeviceToDevice, st));
        SCHK(s, hipMemcpyAsync(seen, s->seen, s->cap_h * 4, hipMemcpyDeviceToDevice, st));
        SCHK(s, hipMemcpyAsync(ist, s->ist, s->cap_h * sizeof(IncState), hipMemcpyDeviceToDevice, st));
        SCHK(s, hipMemcpyAsync(ldir, s->ldir, s->cap_h * HM_INC_LISTS * sizeof(uint2), hipMemcpyDeviceToDevice, st));
    }
    uint32_t **tabs[5] = {&s->clock, &s->back_clock, &s->heads, &s->min_clock, &s->stored};
    uint32_t *nt[5];
    for (int i = 0; i < 5; i++) {
        if ((r = dev_alloc(s, &nt[i], cap * S))) return r;
        SCHK(s, hipMemsetAsync(nt[i], 0, cap * S * 4, st));
        if (s->cap_h) SCHK(s, hipMemcpyAsync(nt[i], *tabs[i], s->cap_h * S * 4, hipMemcpyDeviceToDevice, st));
    }
    SCHK(s, hipStreamSynchronize(st));
    if (s->res_docs) (void)hipFree(s->res_docs);
    if (s->dm) (void)hipFree(s->dm);
    if (s->seen) (void)hipFree(s->seen);
    if (s->ist) (void)hipFree(s->ist);
    if (s->ldir) (void)hipFree(s->ldir);
    s->res_docs = rd; s->dm = dm; s->seen = seen; s->ist = ist; s->ldir = ldir;
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

// Staged batch layout on the device: [changes][deps][ops][docs][handles][remap][gather][bail]
struct StageLayout {
    size_t o_ch, o_dp, o_op, o_docs, o_hand, o_remap, o_gather, o_bail, o_defer, o_gdone, o_fail, total;
};
StageLayout layout(size_t nc, size_t nd, size_t no, size_t n, size_t nremap, uint32_t S) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    StageLayout L;
    size_t o = 0;
    L.o_ch = o; o += al(nc * sizeof(hm_change_row) + 1);
    L.o_dp = o; o += al(nd * sizeof(hm_dep_row) + 1);
    L.o_op = o; o += al(no * sizeof(hm_op_row) + 1);
    L.o_docs = o; o += al(n * sizeof(hm_doc_row) + 1);
    L.o_hand = o; o += al(n * 4 + 1);
    L.o_remap = o; o += al(nremap + 1);
    L.o_gather = o; o += al(n * (sizeof(hm_doc_result) + 3 * 4 * (size_t)S) + 1);
    L.o_bail = o; o += al(4 * (n + 1));
    L.o_defer = o; o += al(4 * (n + 1));
    L.o_gdone = o; o += al(n);
    L.o_fail = o; o += 256;
    L.total = o;
    return L;
}

// HM_INC_DEBUG_HANDLE=h (dev diagnostics): the incremental list state of handle h on stderr
void dbg_list_state(hm_store *s, const char *when) {
    const char *e = getenv("HM_INC_DEBUG_HANDLE");
    if (!e) return;
    const uint32_t h = (uint32_t)atoi(e);
    if (h >= s->n_handles) return;
    hipStream_t st = hm_engine_stream(s->e);
    DevDoc m; IncState I; uint2 dir[HM_INC_LISTS];
    (void)hipMemcpyAsync(&m, s->dm + h, sizeof m, hipMemcpyDeviceToHost, st);
    (void)hipMemcpyAsync(&I, s->ist + h, sizeof I, hipMemcpyDeviceToHost, st);
    (void)hipMemcpyAsync(dir, s->ldir + (size_t)h * HM_INC_LISTS, sizeof dir, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    std::vector<uint32_t> lo(m.n_r + 1), ep(m.n_r + 1), pa(m.n_r + 1), ek(m.n_r + 1);
    if (m.n_r) {
        (void)hipMemcpyAsync(lo.data(), s->lorder + m.r_off, m.n_r * 4, hipMemcpyDeviceToHost, st);
        (void)hipMemcpyAsync(ep.data(), s->epos + m.r_off, m.n_r * 4, hipMemcpyDeviceToHost, st);
        (void)hipMemcpyAsync(pa.data(), s->epar + m.r_off, m.n_r * 4, hipMemcpyDeviceToHost, st);
        (void)hipMemcpyAsync(ek.data(), s->ekey + m.r_off, m.n_r * 4, hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
    }
    fprintf(stderr, "[inc dbg %s] h=%u n_r=%u r_off=%u flags=%u n_el=%u nl=%u dir=", when, h, m.n_r, m.r_off, I.flags, I.pad[0], I.pad[1]);
    for (uint32_t k = 0; k < HM_INC_LISTS && k < I.pad[1]; k++) fprintf(stderr, "(%u,%u)", dir[k].x, dir[k].y);
    fprintf(stderr, "\n  lorder:");
    for (uint32_t i = 0; i < I.pad[0] && i < m.n_r; i++) fprintf(stderr, " %u", lo[i]);
    fprintf(stderr, "\n  epos/epar/ekey:");
    for (uint32_t r = 0; r < m.n_r; r++) fprintf(stderr, " %u:%d/%d/%x", r, (int)ep[r], (int)pa[r], ek[r]);
    fprintf(stderr, "\n");
}

// Re-merge the `n` documents listed (handles, device) on the engine stream: their launch rows
// built on the device from their metas, the launch hints read back.
int launch_list_merge(hm_store *s, const uint32_t *dev_list, uint32_t n) {
    if (!n) return HM_OK;
    hipStream_t st = hm_engine_stream(s->e);
    int rc;
    if ((rc = ensure_buf(s, s->rows, n)) || (rc = ensure_buf(s, s->klist, n))) return rc;
    if ((rc = reset_stats(s))) return rc;
    const uint32_t small_lists = hm_small_list_ops(s->S, s->inc_mode);
    // (the states of the documents that keep none are cleared — unless no document holds one)
    SCHK(s, hm_launch_doc_rows(dev_list, n, s->dm, s->rows.p, s->st, small_lists, s->incremental && s->any_state ? s->ist : nullptr,
                               s->klist.p, st));
    rc = HM_OK;
    const PlanStats P = read_stats(s, &rc);
    if (rc) return rc;
    hm_batch b = {};
    b.a_stride = s->S;
    b.n_docs = n;
    b.n_changes = (uint32_t)std::min<unsigned long long>(P.tot_c, 0xFFFFFFFFull);
    b.n_deps = (uint32_t)std::min<unsigned long long>(P.tot_d, 0xFFFFFFFFull);
    b.n_ops = (uint32_t)std::min<unsigned long long>(P.tot_o, 0xFFFFFFFFull);
    b.n_regs = (uint32_t)std::min<unsigned long long>(P.tot_r, 0xFFFFFFFFull);
    b.max_changes = P.max_c; b.max_ops = P.max_o; b.max_regs = P.max_r; b.max_objs = P.max_objs; b.max_deps = P.max_d;
    b.doc_flags = P.flags;
    if (!b.max_changes && !b.max_ops && !b.max_regs && !b.max_objs) b.max_objs = 1;   // device hints present
    b.docs = s->rows.p;
    b.changes = s->changes; b.deps = s->deps; b.ops = s->ops; b.min_clock = s->min_clock;
    hm_results o;
    o.docs = s->res_docs; o.clock = s->clock; o.back_clock = s->back_clock; o.heads = s->heads;
    o.hist = s->hist; o.all_deps = s->all_deps; o.regs = s->regs; o.surv = s->surv;
    const hm_extents ext = {(uint32_t)s->cap_c, (uint32_t)s->cap_d, (uint32_t)s->cap_o, (uint32_t)s->cap_r};
    // the incremental path keeps list documents' element order: positions written by the merge
    // (mode 1: when every listed document holds <= HM_INC_SMALL_LIST_OPS ops, none with lists keeps
    // incremental state — inc_meta skips them — so no positions are needed)
    // (P.mx[3]: listed list documents that may keep incremental state)
    const bool positions = s->incremental && (P.flags & HM_DOC_HAS_LISTS) && P.mx[3] != 0;
    if (positions) SCHK(s, hm_launch_epos_clear(s->klist.p, P.mx[2], s->dm, s->epos, st));     // (the keep list)
    rc = hm_engine_launch_merge(s->e, &b, &o, dev_list, &ext, positions ? s->epos : nullptr);
    // the incremental path's survivor metadata of the re-merged documents that may keep state (the
    // keep list doc_rows_kernel built; it cleared the others' IncState)
    if (rc == HM_OK && s->incremental && P.mx[2]) {
        MetaArgs M;
        M.list = s->klist.p; M.n = P.mx[2]; M.dm = s->dm; M.res_docs = s->res_docs; M.changes = s->changes; M.hist = s->hist;
        M.ckey = s->ckey; M.ops = s->ops; M.surv = s->surv; M.smeta = s->smeta; M.ist = s->ist;
        M.epos = s->epos; M.epar = s->epar; M.ekey = s->ekey; M.lorder = s->lorder; M.ldir = s->ldir;
        M.small_lists = small_lists;
        M.n_valid = &s->st->n_valid;
        if ((rc = ensure_buf(s, s->mpart, HM_META_GRID))) return rc;
        M.part = s->mpart.p;
        SCHK(s, hm_launch_inc_meta(M, st));
    }
    // documents whose state can route them to the incremental kernels, after this re-merge (the
    // only step that adds or drops states): none (e.g. mode 1 with only small list documents, or
    // every document with queued changes) = the next submits launch no incremental kernel
    const bool count = s->incremental && (s->any_state || P.mx[2]);
    if (count) SCHK(s, hipMemcpyAsync(&s->h_cnt[4], &s->st->n_valid, 4, hipMemcpyDeviceToHost, st));
    SCHK(s, hipStreamSynchronize(st));
    if (count) s->any_state = s->h_cnt[4] != 0;
    return rc;
}

// Rebuild every arena larger and compact all documents into it; every document is
// re-merged (its outputs live in the arenas too).  `extra` = rows the caller is about
// to append per space, so the new arenas fit them.  The metas come to the host for it.
int compact(hm_store *s, size_t extra_c, size_t extra_d, size_t extra_o, size_t extra_r) {
    hipStream_t st = hm_engine_stream(s->e);
    const uint32_t S = s->S, n = s->n_handles;
    std::vector<DevDoc> old(n);
    if (n) {
        SCHK(s, hipMemcpyAsync(old.data(), s->dm, (size_t)n * sizeof(DevDoc), hipMemcpyDeviceToHost, st));
        SCHK(s, hipStreamSynchronize(st));
    }
    size_t live_c = extra_c, live_d = extra_d, live_o = extra_o, live_r = extra_r;
    for (auto &m : old) {
        live_c += seg_cap(m.n_c); live_d += seg_cap(m.n_d); live_o += seg_cap(m.n_o); live_r += seg_cap(m.n_r);
    }
    const size_t nc = std::max<size_t>(2 * live_c, 1 << 16), nd = std::max<size_t>(2 * live_d, 1 << 16);
    const size_t no = std::max<size_t>(2 * live_o, 1 << 16), nr = std::max<size_t>(2 * live_r, 1 << 16);
    hm_change_row *ch; int32_t *hi; uint32_t *ad; hm_dep_row *dp; hm_op_row *op; hm_surv_result *sv; hm_reg_result *rg;
    uint2 *sm;
    uint32_t *ck, *ep, *epr, *ek, *lo;
    int r;
    if ((r = dev_alloc(s, &ch, nc)) || (r = dev_alloc(s, &hi, nc)) || (r = dev_alloc(s, &ck, nc)) || (r = dev_alloc(s, &ad, nc * S)) ||
        (r = dev_alloc(s, &dp, nd)) || (r = dev_alloc(s, &op, no)) || (r = dev_alloc(s, &sv, no)) ||
        (r = dev_alloc(s, &sm, no)) || (r = dev_alloc(s, &rg, nr)) || (r = dev_alloc(s, &ep, nr)) ||
        (r = dev_alloc(s, &epr, nr)) || (r = dev_alloc(s, &ek, nr)) || (r = dev_alloc(s, &lo, nr)))
        return r;
    // relocate every document (old rows only; no new rows, no remap)
    std::vector<AppendDesc> descs(n);
    std::vector<DevDoc> nm = old;
    std::vector<uint32_t> all(n);
    uint64_t uc = 0, ud = 0, uo = 0, ur = 0;
    auto seg = [](uint64_t &used, uint32_t need, uint32_t &off, uint32_t &cap) {
        cap = seg_cap(need);
        off = (uint32_t)used;
        used += cap;
    };
    for (uint32_t h = 0; h < n; h++) {
        DevDoc &m = nm[h];
        const DevDoc &o = old[h];
        seg(uc, m.n_c, m.c_off, m.c_cap); seg(ud, m.n_d, m.d_off, m.d_cap);
        seg(uo, m.n_o, m.o_off, m.o_cap); seg(ur, m.n_r, m.r_off, m.r_cap);
        AppendDesc D = {};
        D.handle = h;
        D.src_c = o.c_off; D.dst_c = m.c_off; D.n_old_c = o.n_c;
        D.src_d = o.d_off; D.dst_d = m.d_off; D.n_old_d = o.n_d;
        D.src_o = o.o_off; D.dst_o = m.o_off; D.n_old_o = o.n_o;
        D.remap_row = 0xFFFFFFFFu;
        descs[h] = D;
        all[h] = h;
    }
    StoreArenas src = {s->changes, s->deps, s->ops, s->min_clock, s->stored};
    StoreArenas dst = {ch, dp, op, s->min_clock, s->stored};
    if (n) {
        if ((r = ensure_buf(s, s->descs, n))) return r;
        SCHK(s, hipMemcpyAsync(s->descs.p, descs.data(), (size_t)n * sizeof(AppendDesc), hipMemcpyHostToDevice, st));
        SCHK(s, hm_launch_append(s->descs.p, n, src, dst, nullptr, nullptr, nullptr, nullptr, S, st));
        SCHK(s, hipMemcpyAsync(s->dm, nm.data(), (size_t)n * sizeof(DevDoc), hipMemcpyHostToDevice, st));
        SCHK(s, hipStreamSynchronize(st));
    }
    (void)hipFree(s->changes); (void)hipFree(s->hist); (void)hipFree(s->ckey); (void)hipFree(s->all_deps); (void)hipFree(s->deps);
    (void)hipFree(s->ops); (void)hipFree(s->surv); (void)hipFree(s->smeta); (void)hipFree(s->regs);
    (void)hipFree(s->epos); (void)hipFree(s->epar); (void)hipFree(s->ekey); (void)hipFree(s->lorder);
    s->epos = ep; s->epar = epr; s->ekey = ek; s->lorder = lo;
    s->changes = ch; s->hist = hi; s->ckey = ck; s->all_deps = ad; s->deps = dp; s->ops = op; s->surv = sv; s->smeta = sm; s->regs = rg;
    s->cap_c = nc; s->cap_d = nd; s->cap_o = no; s->cap_r = nr;
    const unsigned long long bump[4] = {uc, ud, uo, ur};
    SCHK(s, hipMemcpyAsync(s->st->bump, bump, sizeof bump, hipMemcpyHostToDevice, st));
    if (!n) { SCHK(s, hipStreamSynchronize(st)); return HM_OK; }
    if ((r = ensure_buf(s, s->list, n))) return r;
    SCHK(s, hipMemcpyAsync(s->list.p, all.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
    return launch_list_merge(s, s->list.p, n);
}

}  // namespace

extern "C" {

int hm_store_create(hm_engine *e, const hm_store_config *cfg, hm_store **out) {
    if (!e || !out) return HM_ERR_INVALID;
    *out = nullptr;
    const uint32_t S = cfg ? cfg->a_stride : 8;
    if (S == 0 || S > HM_MAX_STRIDE) return hm_engine_fail(e, HM_ERR_INVALID, "store a_stride must be in [1,256]");
    hm_store *s = new (std::nothrow) hm_store();
    if (!s) return HM_ERR_NOMEM;
    s->e = e; s->S = S;
    if (hipSetDevice(hm_engine_device(e)) != hipSuccess) { delete s; return HM_ERR_DEVICE; }
    int r = dev_alloc(s, &s->st, 1);
    if (r == HM_OK && hipMemset(s->st, 0, sizeof(PlanStats)) != hipSuccess) r = HM_ERR_DEVICE;
    if (r == HM_OK && (hipHostMalloc((void **)&s->h_st, sizeof(PlanStats), hipHostMallocDefault) != hipSuccess ||
                       hipHostMalloc((void **)&s->h_cnt, 64, hipHostMallocDefault) != hipSuccess))
        r = HM_ERR_NOMEM;
    if (r == HM_OK) r = compact(s, 0, 0, 0, 0);
    if (r == HM_OK) r = ensure_handles(s, 1024);
    if (r != HM_OK) { hm_store_destroy(s); return r; }
    *out = s;
    return HM_OK;
}

void hm_store_destroy(hm_store *s) {
    if (!s) return;
    (void)hipStreamSynchronize(hm_engine_stream(s->e));
    void *bufs[] = {s->changes, s->hist, s->ckey, s->all_deps, s->deps, s->ops, s->surv, s->smeta, s->ist, s->ldir, s->regs, s->epos,
                    s->epar, s->ekey, s->lorder, s->res_docs, s->clock,
                    s->back_clock, s->heads, s->min_clock, s->stored, s->stage.p, s->dm, s->seen, s->plan.p, s->descs.p,
                    s->bdescs.p, s->list.p, s->blist.p, s->alist.p, s->remap.p, s->inv.p, s->rows.p, s->undo_handles.p, s->klist.p, s->mpart.p, s->st};
    for (void *b : bufs) if (b) (void)hipFree(b);
    for (hipEvent_t e : s->ev) if (e) (void)hipEventDestroy(e);
    if (s->h_st) (void)hipHostFree(s->h_st);
    if (s->h_cnt) (void)hipHostFree(s->h_cnt);
    delete s;
}

int hm_doc_open(hm_store *s, uint32_t *out_doc) { return hm_doc_open_n(s, 1, out_doc); }

int hm_doc_open_n(hm_store *s, uint32_t n, uint32_t *out_first) {
    if (!s || !out_first) return HM_ERR_INVALID;
    try {
        if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "hm_doc_open while a batch is in flight");
        const uint32_t h0 = s->n_handles;
        int r = ensure_handles(s, (size_t)h0 + n);
        if (r) return r;
        // Backend.init(): an empty log (ROOT only) and its result row, written on the engine
        // stream (ordered before any submit; the reads below synchronise the stream)
        hipStream_t st = hm_engine_stream(s->e);
        SCHK(s, hm_launch_init_docs(s->dm, h0, n, st));
        if (n) {
            SCHK(s, hipMemsetAsync(s->res_docs + h0, 0, (size_t)n * sizeof(hm_doc_result), st));
            std::vector<hm_doc_result> rows(n);
            for (auto &x : rows) { x = hm_doc_result{}; x.err_change = HM_NONE; x.err_op = HM_NONE; }
            SCHK(s, hipMemcpyAsync(s->res_docs + h0, rows.data(), (size_t)n * sizeof(hm_doc_result), hipMemcpyHostToDevice, st));
            SCHK(s, hipStreamSynchronize(st));
        }
        s->n_handles = h0 + n;
        *out_first = h0;
        return HM_OK;
    } catch (...) {
        return HM_ERR_NOMEM;
    }
}

int hm_doc_reset(hm_store *s, const uint32_t *doc_handles, uint32_t n) {
    if (!s || (n && !doc_handles)) return HM_ERR_INVALID;
    try {
        if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "hm_doc_reset while a batch is in flight");
        if (!n) return HM_OK;
        std::vector<uint32_t> hs(doc_handles, doc_handles + n);
        std::sort(hs.begin(), hs.end());
        if (hs.back() >= s->n_handles) return hm_engine_fail(s->e, HM_ERR_INVALID, "hm_doc_reset: bad handle");
        if (std::adjacent_find(hs.begin(), hs.end()) != hs.end())
            return hm_engine_fail(s->e, HM_ERR_INVALID, "hm_doc_reset: repeated handle");
        int r;
        if ((r = ensure_buf(s, s->blist, n))) return r;
        hipStream_t st = hm_engine_stream(s->e);
        SCHK(s, hipMemcpyAsync(s->blist.p, hs.data(), (size_t)n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hm_launch_reset_docs(s->blist.p, n, s->dm, s->res_docs, s->ist, s->clock, s->back_clock, s->heads, s->min_clock,
                                     s->stored, s->S, &s->st->n_valid, st));
        SCHK(s, hipStreamSynchronize(st));
        s->undo_id = 0;                               // the last batch's undo no longer applies
        return HM_OK;
    } catch (...) {
        return HM_ERR_NOMEM;
    }
}

// hm_batch_submit / hm_batch_submit_device: `dev` = the batch's tables, handles and remap are
// device pointers (no host staging of the rows)
static int submit_impl(hm_store *s, const hm_batch *b, const uint32_t *doc_handles, const uint8_t *actor_remap,
                       uint64_t *out_batch_id, bool dev) {
    if (!s || !b || (b->n_docs && (!doc_handles || !b->docs))) return HM_ERR_INVALID;
    try {
        if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "a batch is already in flight (call hm_batch_wait)");
        const uint32_t S = s->S, n = b->n_docs;
        s->undo_id = 0;                                  // the plan rows hm_batch_undo reads are replaced
        if (b->a_stride != S) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch a_stride must equal the store's");
        SCHK(s, hipSetDevice(hm_engine_device(s->e)));
        hipStream_t st = hm_engine_stream(s->e);
        PhaseTimer T(st);
        int rc;
        // stage the batch (its tables, rows, handles and remap) on the device
        const size_t nremap = actor_remap ? (size_t)n * S : 0;
        const StageLayout L = dev ? layout(0, 0, 0, n, 0, S) : layout(b->n_changes, b->n_deps, b->n_ops, n, nremap, S);
        if ((rc = ensure_stage(s, L.total)) || (rc = ensure_buf(s, s->plan, n)) || (rc = ensure_buf(s, s->descs, n)) ||
            (rc = ensure_buf(s, s->list, n)))
            return rc;
        uint8_t *sp = s->stage.p;
        const hm_doc_row *t_docs = b->docs;
        const hm_change_row *t_ch = b->changes;
        const hm_dep_row *t_dp = b->deps;
        const hm_op_row *t_op = b->ops;
        const uint32_t *t_hand = doc_handles;
        const uint8_t *t_remap = actor_remap;
        if (!dev) {
            if (b->n_changes) SCHK(s, hipMemcpyAsync(sp + L.o_ch, b->changes, b->n_changes * sizeof(hm_change_row), hipMemcpyHostToDevice, st));
            if (b->n_deps) SCHK(s, hipMemcpyAsync(sp + L.o_dp, b->deps, b->n_deps * sizeof(hm_dep_row), hipMemcpyHostToDevice, st));
            if (b->n_ops) SCHK(s, hipMemcpyAsync(sp + L.o_op, b->ops, b->n_ops * sizeof(hm_op_row), hipMemcpyHostToDevice, st));
            if (n) {
                SCHK(s, hipMemcpyAsync(sp + L.o_docs, b->docs, (size_t)n * sizeof(hm_doc_row), hipMemcpyHostToDevice, st));
                SCHK(s, hipMemcpyAsync(sp + L.o_hand, doc_handles, (size_t)n * 4, hipMemcpyHostToDevice, st));
            }
            if (nremap) SCHK(s, hipMemcpyAsync(sp + L.o_remap, actor_remap, nremap, hipMemcpyHostToDevice, st));
            t_docs = (const hm_doc_row *)(sp + L.o_docs); t_ch = (const hm_change_row *)(sp + L.o_ch);
            t_dp = (const hm_dep_row *)(sp + L.o_dp); t_op = (const hm_op_row *)(sp + L.o_op);
            t_hand = (const uint32_t *)(sp + L.o_hand); t_remap = nremap ? sp + L.o_remap : nullptr;
        }
        T.mark("stage: h2d");
        PlanArgs A;
        A.docs = t_docs; A.changes = t_ch;
        A.handles = t_hand; A.remap = nremap ? t_remap : nullptr;
        A.n = n; A.n_changes = b->n_changes; A.n_deps = b->n_deps; A.n_ops = b->n_ops; A.n_handles = s->n_handles;
        A.S = S; A.stamp = ++s->stamp ? s->stamp : ++s->stamp; A.incremental = s->incremental && S <= 64 && s->any_state ? s->inc_mode : 0u;
        // (no document holds a usable state: the plan routes every document to the re-merge and no
        // incremental kernel is launched)
        A.dm = s->dm; A.res_docs = s->res_docs; A.seen = s->seen; A.plan = s->plan.p; A.descs = s->descs.p;
        A.list = s->list.p; A.st = s->st;
        A.ist = A.incremental ? s->ist : nullptr; A.ops = t_op; A.deps = t_dp; A.clock = s->clock;
        A.defer = (uint32_t *)(sp + L.o_defer);
        // the submit's work-list counts and gathered-row flags, zeroed by plan_kernel (no memsets)
        A.bail = (uint32_t *)(sp + L.o_bail); A.fail = (uint32_t *)(sp + L.o_fail); A.gdone = sp + L.o_gdone;
        if ((rc = ensure_buf(s, s->alist, n))) return rc;
        A.alist = s->alist.p;
        A.cap[0] = s->cap_c; A.cap[1] = s->cap_d; A.cap[2] = s->cap_o; A.cap[3] = s->cap_r;
        uint32_t *bail = (uint32_t *)(sp + L.o_bail);            // (count zeroed by the plan)
        if (!s->ev[0])
            for (auto &e : s->ev) SCHK(s, hipEventCreate(&e));
        // plan (checks, growth, routes), alloc, append and the incremental kernels go out back to
        // back: alloc_kernel itself does nothing when the plan failed a check or the arenas cannot
        // take the growth (every later kernel then finds no work), and the host reads the plan's
        // stats once, with the re-merge counts.  A failed check fails the submit with the store
        // as it was; no room compacts the store (every document re-merged) and runs the plan again.
        PlanStats P;
        uint32_t counts[2] = {0, 0};
        for (int attempt = 0;; attempt++) {
            if ((rc = reset_stats(s))) return rc;
            SCHK(s, hm_launch_plan(A, st));
            T.mark("plan");
            SCHK(s, hm_launch_alloc(A, st));
            StoreArenas ar = {s->changes, s->deps, s->ops, s->min_clock, s->stored};
            if (T.on) {
                // what the append has to move: documents whose segments moved, re-ranked ones, old rows
                std::vector<AppendDesc> dd(n);
                SCHK(s, hipMemcpyAsync(dd.data(), s->descs.p, (size_t)n * sizeof(AppendDesc), hipMemcpyDeviceToHost, st));
                SCHK(s, hipStreamSynchronize(st));
                size_t mv = 0, rmp = 0, inc = 0, old_o = 0, new_o = 0;
                for (const AppendDesc &D : dd) {
                    const bool m = D.src_c != D.dst_c || D.src_d != D.dst_d || D.src_o != D.dst_o;
                    mv += m; rmp += D.remap_row != 0xFFFFFFFFu; inc += (D.inc & HM_DINC_ROUTE) != 0; new_o += D.n_new_o;
                    if (m) old_o += D.n_old_o;
                }
                fprintf(stderr, "[hm_store] append: %zu docs, %zu moved (%zu old op rows), %zu re-ranked, %zu incremental, %zu new op rows\n",
                        (size_t)n, mv, old_o, rmp, inc, new_o);
                T.mark("(append census)");
            }
            SCHK(s, hm_launch_append(s->descs.p, n, ar, ar, A.changes, t_dp, t_op, A.remap, S, st, s->alist.p, &s->st->n_app));
            T.mark("alloc+append");
            SCHK(s, hipEventRecord(s->ev[0], st));
            if (A.incremental) {
                IncArgs IA;
                IA.descs = s->descs.p; IA.n = n; IA.list = nullptr; IA.S = S;
                IA.st_changes = A.changes; IA.st_deps = t_dp; IA.st_ops = t_op;
                IA.changes = s->changes; IA.deps = s->deps; IA.ops = s->ops; IA.hist = s->hist; IA.ckey = s->ckey; IA.all_deps = s->all_deps;
                IA.regs = s->regs; IA.surv = s->surv; IA.smeta = s->smeta; IA.res_docs = s->res_docs;
                IA.epos = s->epos; IA.epar = s->epar; IA.ekey = s->ekey; IA.lorder = s->lorder; IA.ldir = s->ldir;
                IA.clock = s->clock; IA.back_clock = s->back_clock; IA.heads = s->heads; IA.min_clock = s->min_clock;
                IA.ist = s->ist; IA.bail = bail; IA.defer = (uint32_t *)(sp + L.o_defer);
                IA.n_lane = S == 8 || S == 16 ? 1u : 0u;                 // (the lane pass reads its count on the device)
                IA.pst = s->st;
                // the documents the incremental kernels finish write their gathered rows themselves
                IA.gout = sp + L.o_gather; IA.gdone = sp + L.o_gdone;      // (gdone zeroed by the plan)
                dbg_list_state(s, "before");
                SCHK(s, hm_launch_inc_apply(IA, st));
                dbg_list_state(s, "after");
            }
            SCHK(s, hipEventRecord(s->ev[1], st));
            T.mark("incremental");
            // the plan's stats and the re-merge counts (cold documents, then those the incremental
            // kernels handed back), one read
            SCHK(s, hipMemcpyAsync(s->h_st, s->st, sizeof(PlanStats), hipMemcpyDeviceToHost, st));
            SCHK(s, hipMemcpyAsync(&s->h_cnt[1], bail, 4, hipMemcpyDeviceToHost, st));
            SCHK(s, hipStreamSynchronize(st));
            P = *s->h_st;
            counts[0] = P.n_cold; counts[1] = s->h_cnt[1];
            if (P.err) {
                const char *why = (P.err & HM_PLAN_BAD_HANDLE) || (P.err & HM_PLAN_REPEATED) ? "bad or repeated document handle"
                                : (P.err & HM_PLAN_ROWS) ? "document rows outside the batch tables"
                                : (P.err & HM_PLAN_TOTALS) ? "document totals must cover the existing log (and n_actors <= a_stride)"
                                : (P.err & HM_PLAN_CHANGE_ROWS) ? "change rows outside their document's deps/ops"
                                : "actor remap is not a permutation into the new ranks";
                if (attempt) return hm_engine_fail(s->e, HM_ERR_INVALID, "submit plan failed after compaction");
                return hm_engine_fail(s->e, HM_ERR_INVALID, why);
            }
            // (P.bump already counts this submit's segments when alloc_kernel ran: its own verdict decides)
            if (!P.mx[1]) break;
            // the arenas cannot take the growth (alloc_kernel did nothing): compact, then plan again
            if (attempt) return hm_engine_fail(s->e, HM_ERR_NOMEM, "the store's arenas cannot take the submit after compaction");
            if ((rc = compact(s, P.need[0], P.need[1], P.need[2], P.need[3]))) return rc;
            A.stamp = ++s->stamp ? s->stamp : ++s->stamp;
            A.dm = s->dm; A.descs = s->descs.p; A.list = s->list.p;     // (compaction may have regrown them)
            A.cap[0] = s->cap_c; A.cap[1] = s->cap_d; A.cap[2] = s->cap_o; A.cap[3] = s->cap_r;
            T.mark("compact");
        }
        if (counts[1]) SCHK(s, hipMemcpyAsync(s->list.p + counts[0], bail + 1, (size_t)counts[1] * 4, hipMemcpyDeviceToDevice, st));
        SCHK(s, hipEventRecord(s->ev[2], st));
        if ((rc = launch_list_merge(s, s->list.p, counts[0] + counts[1]))) return rc;
        SCHK(s, hipEventRecord(s->ev[3], st));
        s->ev_live = true;           // (read by hm_batch_wait after its stream sync: submit stays asynchronous)
        dbg_list_state(s, "after merge");
        T.mark("remerge");
        s->st_inc = P.n_inc - counts[1]; s->st_cold = counts[0]; s->st_bail = counts[1];
        uint32_t *fail = (uint32_t *)(sp + L.o_fail);            // (count zeroed by the plan)
        SCHK(s, hm_launch_gather(A.handles, n, S, s->res_docs, s->clock, s->back_clock, s->heads, sp + L.o_gather, fail, st,
                                 P.n_inc ? sp + L.o_gdone : nullptr));
        s->p_gather_dev = sp + L.o_gather;
        s->p_fail_dev = fail;
        s->p_handles_dev = const_cast<uint32_t *>(A.handles);
        s->p_n = n;
        s->p_remap = nremap != 0;
        if (nremap) {
            // the rollback needs the remap rows after the staging area is reused
            if ((rc = ensure_buf(s, s->remap, nremap))) return rc;
            SCHK(s, hipMemcpyAsync(s->remap.p, A.remap, nremap, hipMemcpyDeviceToDevice, st));
        }
        T.mark("gather");
        s->pending = true;
        s->pending_id = s->next_id++;
        if (out_batch_id) *out_batch_id = s->pending_id;
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_batch_submit");
    }
}

int hm_batch_submit(hm_store *s, const hm_batch *b, const uint32_t *doc_handles, const uint8_t *actor_remap,
                    uint64_t *out_batch_id) {
    return submit_impl(s, b, doc_handles, actor_remap, out_batch_id, false);
}

int hm_batch_submit_device(hm_store *s, const hm_batch *b, const uint32_t *doc_handles, const uint8_t *actor_remap,
                           uint64_t *out_batch_id) {
    return submit_impl(s, b, doc_handles, actor_remap, out_batch_id, true);
}

// Roll documents of the last submit back to their logs before it (every = false: those whose merge
// failed; true: all of them not rolled back yet): totals restored, ranks re-mapped back, the log
// truncated, the previous state re-merged.
static int roll_back(hm_store *s, const uint32_t *handles_dev, uint32_t n, bool every) {
    hipStream_t st = hm_engine_stream(s->e);
    const uint32_t S = s->S;
    int rc;
    if ((rc = ensure_buf(s, s->bdescs, n)) || (rc = ensure_buf(s, s->blist, n)) ||
        (s->p_remap && (rc = ensure_buf(s, s->inv, (size_t)n * S))))
        return rc;
    if ((rc = reset_stats(s))) return rc;
    SCHK(s, hm_launch_rollback(handles_dev, n, s->res_docs, s->plan.p, s->p_remap ? s->remap.p : nullptr, S, s->dm,
                               s->bdescs.p, s->p_remap ? s->inv.p : nullptr, s->blist.p, s->st, every ? 1u : 0u, st));
    uint32_t nb = 0;
    SCHK(s, hipMemcpyAsync(&nb, &s->st->n_back, 4, hipMemcpyDeviceToHost, st));
    SCHK(s, hipStreamSynchronize(st));
    StoreArenas ar = {s->changes, s->deps, s->ops, s->min_clock, s->stored};
    SCHK(s, hm_launch_append(s->bdescs.p, nb, ar, ar, nullptr, nullptr, nullptr, s->p_remap ? s->inv.p : nullptr, S, st));
    return launch_list_merge(s, s->blist.p, nb);
}

// hm_batch_wait / hm_batch_wait_device: the gathered rows to the host arrays, or (out_dev) as one
// device-to-device copy with only the failure count read back
static int wait_impl(hm_store *s, uint64_t batch_id, hm_doc_result *out_docs, uint32_t *out_clock,
                     uint32_t *out_back_clock, uint32_t *out_heads, void *out_dev, uint32_t *out_n_failed) {
    if (!s) return HM_ERR_INVALID;
    try {
        if (!s->pending || batch_id != s->pending_id) return hm_engine_fail(s->e, HM_ERR_INVALID, "no such batch in flight");
        SCHK(s, hipSetDevice(hm_engine_device(s->e)));        // the caller may be a host thread of its own
        hipStream_t st = hm_engine_stream(s->e);
        PhaseTimer T(st);
        // the batch stays in flight (pending) until this returns: copy-out and rollback below
        // still read and re-merge the store's documents
        struct Clear { std::atomic<bool> &p; ~Clear() { p.store(false); } } clear_pending{s->pending};
        const uint32_t n = s->p_n, S = s->S;
        // results straight from the gathered device rows into the caller's arrays
        std::vector<hm_doc_result> tmp;
        hm_doc_result *res = out_docs;
        if (!res && !out_dev) { tmp.resize(n); res = tmp.data(); }
        uint32_t n_fail = 0;
        if (n && out_dev) {
            const size_t bytes = (size_t)n * (sizeof(hm_doc_result) + 3 * 4 * (size_t)S);
            SCHK(s, hipMemcpyAsync(out_dev, s->p_gather_dev, bytes, hipMemcpyDeviceToDevice, st));
            SCHK(s, hipMemcpyAsync(&n_fail, s->p_fail_dev, 4, hipMemcpyDeviceToHost, st));
            SCHK(s, hipStreamSynchronize(st));
        } else if (n) {
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
        if (s->ev_live) {
            // the submit's kernel intervals (hm_store_last_kernel_ms), complete after the sync above
            SCHK(s, hipEventSynchronize(s->ev[3]));
            SCHK(s, hipEventElapsedTime(&s->last_ms[0], s->ev[0], s->ev[1]));
            SCHK(s, hipEventElapsedTime(&s->last_ms[1], s->ev[2], s->ev[3]));
            s->ev_live = false;
        }
        // roll back documents whose merge threw (or left the envelope): the log returns to its
        // previous length (rows stay where they are), ranks are re-ranked back, and the previous
        // state is re-merged
        bool any = n_fail != 0;
        for (uint32_t i = 0; res && i < n && !any; i++) any = res[i].status != HM_OK;
        if (out_n_failed) {
            uint32_t k = n_fail;
            if (!out_dev) for (uint32_t i = 0; i < n; i++) k += res[i].status != HM_OK;
            *out_n_failed = k;
        }
        if (any) {
            const int rc = roll_back(s, s->p_handles_dev, n, false);
            if (rc) return rc;
            T.mark("rollback");
        }
        // hm_batch_undo keeps the batch's handles (the staging area is reused by other calls)
        if (n) {
            int rc = ensure_buf(s, s->undo_handles, n);
            if (rc) return rc;
            SCHK(s, hipMemcpyAsync(s->undo_handles.p, s->p_handles_dev, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
        }
        s->undo_id = batch_id;
        s->undo_n = n;
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_batch_wait");
    }
}

int hm_batch_wait(hm_store *s, uint64_t batch_id, hm_doc_result *out_docs, uint32_t *out_clock,
                  uint32_t *out_back_clock, uint32_t *out_heads) {
    return wait_impl(s, batch_id, out_docs, out_clock, out_back_clock, out_heads, nullptr, nullptr);
}

int hm_batch_wait_device(hm_store *s, uint64_t batch_id, void *out_dev, uint32_t *out_n_failed) {
    if (!out_dev) return HM_ERR_INVALID;
    return wait_impl(s, batch_id, nullptr, nullptr, nullptr, nullptr, out_dev, out_n_failed);
}

int hm_batch_undo(hm_store *s, uint64_t batch_id) {
    if (!s) return HM_ERR_INVALID;
    try {
        if (s->pending || !batch_id || batch_id != s->undo_id)
            return hm_engine_fail(s->e, HM_ERR_INVALID, "hm_batch_undo: not the last waited batch (or a submit since)");
        SCHK(s, hipSetDevice(hm_engine_device(s->e)));
        const int rc = roll_back(s, s->undo_handles.p, s->undo_n, true);
        s->undo_id = 0;
        return rc;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_batch_undo");
    }
}

int hm_store_set_incremental(hm_store *s, int on) {
    if (!s) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    // re-merges while the path was off kept no survivor metadata: every document's next submit
    // re-merges (and rebuilds it)
    if (on && !s->incremental && s->cap_h) {
        SCHK(s, hipMemsetAsync(s->ist, 0, s->cap_h * sizeof(IncState), hm_engine_stream(s->e)));
        SCHK(s, hipMemsetAsync(&s->st->n_valid, 0, 4, hm_engine_stream(s->e)));
        s->any_state = false;
    }
    s->incremental = on != 0;
    s->inc_mode = on == 2 ? 2u : 1u;
    return HM_OK;
}

int hm_store_last_routing(const hm_store *s, uint32_t *out3) {
    if (!s || !out3) return HM_ERR_INVALID;
    out3[0] = s->st_inc; out3[1] = s->st_cold; out3[2] = s->st_bail;
    return HM_OK;
}

int hm_store_inc_states(hm_store *s, uint32_t *out) {
    if (!s || !out) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    hipStream_t st = hm_engine_stream(s->e);
    SCHK(s, hipMemcpyAsync(&s->h_cnt[5], &s->st->n_valid, 4, hipMemcpyDeviceToHost, st));
    SCHK(s, hipStreamSynchronize(st));
    *out = s->h_cnt[5];
    return HM_OK;
}

int hm_store_last_kernel_ms(const hm_store *s, float *out2) {
    if (!s || !out2) return HM_ERR_INVALID;
    out2[0] = s->last_ms[0]; out2[1] = s->last_ms[1];
    return HM_OK;
}

int hm_doc_info(hm_store *s, uint32_t doc, hm_doc_info_t *out) {
    if (!s || !out || doc >= s->n_handles) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    int rc = HM_OK;
    const DevDoc m = read_doc(s, doc, &rc);
    if (rc) return rc;
    hm_doc_result r;
    SCHK(s, hipMemcpy(&r, s->res_docs + doc, sizeof(r), hipMemcpyDeviceToHost));
    out->n_changes = m.n_c; out->n_deps = m.n_d; out->n_ops = m.n_o; out->n_regs = m.n_r;
    out->n_objs = m.n_objs; out->n_actors = m.n_actors;
    out->hist_len = r.hist_len; out->n_queued = r.n_queued; out->n_surv = r.n_surv; out->status = r.status;
    return HM_OK;
}

int hm_doc_read(hm_store *s, uint32_t doc, int32_t *hist, uint32_t *all_deps, hm_reg_result *regs,
                hm_surv_result *surv, uint32_t *clock, uint32_t *back_clock, uint32_t *heads) {
    if (!s || doc >= s->n_handles) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    int rc = HM_OK;
    const DevDoc m = read_doc(s, doc, &rc);
    if (rc) return rc;
    const uint32_t S = s->S;
    if (hist && m.n_c) SCHK(s, hipMemcpy(hist, s->hist + m.c_off, m.n_c * 4, hipMemcpyDeviceToHost));
    if (all_deps && m.n_c) SCHK(s, hipMemcpy(all_deps, s->all_deps + (size_t)m.c_off * S, (size_t)m.n_c * S * 4, hipMemcpyDeviceToHost));
    if ((regs || surv) && m.n_r) {
        // survivor lists may sit anywhere in the op segment's slots (the incremental path moves a
        // list that grows to the end): handed out packed in register order, as a merge writes them
        std::vector<hm_reg_result> rg(m.n_r);
        std::vector<hm_surv_result> sv(m.o_cap ? m.o_cap : 1);
        SCHK(s, hipMemcpy(rg.data(), s->regs + m.r_off, m.n_r * sizeof(hm_reg_result), hipMemcpyDeviceToHost));
        if (m.o_cap) SCHK(s, hipMemcpy(sv.data(), s->surv + m.o_off, m.o_cap * sizeof(hm_surv_result), hipMemcpyDeviceToHost));
        uint32_t off = 0;
        for (uint32_t g = 0; g < m.n_r; g++) {
            hm_reg_result &r = rg[g];
            if ((uint64_t)r.surv_off + r.n_surv > m.o_cap || (uint64_t)off + r.n_surv > m.n_o)
                return hm_engine_fail(s->e, HM_ERR_DEVICE, "register survivors outside the document's slots");
            if (surv) for (uint32_t i = 0; i < r.n_surv; i++) surv[off + i] = sv[r.surv_off + i];
            r.surv_off = off;
            off += r.n_surv;
        }
        if (regs) memcpy(regs, rg.data(), m.n_r * sizeof(hm_reg_result));
    }
    if (clock) SCHK(s, hipMemcpy(clock, s->clock + (size_t)doc * S, S * 4, hipMemcpyDeviceToHost));
    if (back_clock) SCHK(s, hipMemcpy(back_clock, s->back_clock + (size_t)doc * S, S * 4, hipMemcpyDeviceToHost));
    if (heads) SCHK(s, hipMemcpy(heads, s->heads + (size_t)doc * S, S * 4, hipMemcpyDeviceToHost));
    return HM_OK;
}

int hm_doc_log(hm_store *s, uint32_t doc, hm_change_row *changes, hm_dep_row *deps, hm_op_row *ops) {
    if (!s || doc >= s->n_handles) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    int rc = HM_OK;
    const DevDoc m = read_doc(s, doc, &rc);
    if (rc) return rc;
    if (changes && m.n_c) {
        SCHK(s, hipMemcpy(changes, s->changes + m.c_off, m.n_c * sizeof(hm_change_row), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < m.n_c; i++) { changes[i].dep_off -= m.d_off; changes[i].op_first -= m.o_off; }
    }
    if (deps && m.n_d) SCHK(s, hipMemcpy(deps, s->deps + m.d_off, m.n_d * sizeof(hm_dep_row), hipMemcpyDeviceToHost));
    if (ops && m.n_o) SCHK(s, hipMemcpy(ops, s->ops + m.o_off, m.n_o * sizeof(hm_op_row), hipMemcpyDeviceToHost));
    return HM_OK;
}

int hm_store_read_regs(hm_store *s, uint32_t n, const uint32_t *doc_handles, const uint32_t *regs,
                       hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t surv_cap, uint32_t *out_n_surv) {
    if (!s || (n && (!doc_handles || !regs || !out_regs || (surv_cap && !out_surv)))) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    try {
        if (out_n_surv) *out_n_surv = 0;
        if (!n) return HM_OK;
        hipStream_t st = hm_engine_stream(s->e);
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t o_h = 0, o_r = al(4 * (size_t)n), o_cnt = o_r + al(4 * (size_t)n), o_regs = o_cnt + 256,
                     o_surv = o_regs + al((size_t)n * sizeof(hm_reg_result)), total = o_surv + al((size_t)surv_cap * sizeof(hm_surv_result) + 1);
        int rc = ensure_stage(s, total);
        if (rc) return rc;
        uint8_t *sp = s->stage.p;
        SCHK(s, hipMemcpyAsync(sp + o_h, doc_handles, (size_t)n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hipMemcpyAsync(sp + o_r, regs, (size_t)n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hipMemsetAsync(sp + o_cnt, 0, 8, st));
        SCHK(s, hm_launch_read_regs_h(n, (const uint32_t *)(sp + o_h), (const uint32_t *)(sp + o_r), s->dm, s->n_handles, s->regs,
                                      s->surv, (hm_reg_result *)(sp + o_regs), (hm_surv_result *)(sp + o_surv), surv_cap,
                                      (uint32_t *)(sp + o_cnt), (uint32_t *)(sp + o_cnt) + 1, st));
        uint32_t cb[2] = {0, 0};
        SCHK(s, hipMemcpyAsync(cb, sp + o_cnt, 8, hipMemcpyDeviceToHost, st));
        SCHK(s, hipStreamSynchronize(st));
        if (cb[1] & 1) return hm_engine_fail(s->e, HM_ERR_INVALID, "bad handle");
        if (cb[1] & 2) return hm_engine_fail(s->e, HM_ERR_INVALID, "register outside its document");
        SCHK(s, hipMemcpy(out_regs, sp + o_regs, (size_t)n * sizeof(hm_reg_result), hipMemcpyDeviceToHost));
        if (out_n_surv) *out_n_surv = cb[0];
        if (cb[0] > surv_cap) return hm_engine_fail(s->e, HM_ERR_NOMEM, "surv_cap below the survivors of the registers");
        if (cb[0]) SCHK(s, hipMemcpy(out_surv, sp + o_surv, (size_t)cb[0] * sizeof(hm_surv_result), hipMemcpyDeviceToHost));
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_store_read_regs");
    }
}

int hm_store_read_history(hm_store *s, uint32_t n, const uint32_t *doc_handles, const uint32_t *from, const uint32_t *to,
                          const uint32_t *out_off, uint32_t *out_log_index, uint32_t *out_all_deps) {
    if (!s || (n && (!doc_handles || !from || !to || !out_off || !out_log_index))) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    try {
        if (!n) return HM_OK;
        for (uint32_t i = 0; i < n; i++)
            if (to[i] < from[i] || out_off[i + 1] - out_off[i] != to[i] - from[i] || out_off[i + 1] < out_off[i])
                return hm_engine_fail(s->e, HM_ERR_INVALID, "history slice rows do not match out_off");
        const uint32_t rows = out_off[n], S = s->S;
        hipStream_t st = hm_engine_stream(s->e);
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t o_h = 0, o_f = al(4 * (size_t)n), o_t = o_f + al(4 * (size_t)n), o_o = o_t + al(4 * (size_t)n),
                     o_bad = o_o + al(4 * ((size_t)n + 1)), o_log = o_bad + 256, o_ad = o_log + al(4 * (size_t)rows + 4),
                     total = o_ad + (out_all_deps ? al(4 * (size_t)rows * S + 4) : 0);
        int rc = ensure_stage(s, total);
        if (rc) return rc;
        uint8_t *sp = s->stage.p;
        SCHK(s, hipMemcpyAsync(sp + o_h, doc_handles, (size_t)n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hipMemcpyAsync(sp + o_f, from, (size_t)n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hipMemcpyAsync(sp + o_t, to, (size_t)n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hipMemcpyAsync(sp + o_o, out_off, (size_t)n * 4, hipMemcpyHostToDevice, st));
        SCHK(s, hipMemsetAsync(sp + o_bad, 0, 4, st));
        SCHK(s, hipMemsetAsync(sp + o_log, 0xFF, 4 * (size_t)rows + 4, st));
        SCHK(s, hm_launch_read_hist(n, (const uint32_t *)(sp + o_h), (const uint32_t *)(sp + o_f), (const uint32_t *)(sp + o_t),
                                    (const uint32_t *)(sp + o_o), s->dm, s->n_handles, s->hist, s->all_deps, S,
                                    (uint32_t *)(sp + o_log), out_all_deps ? (uint32_t *)(sp + o_ad) : nullptr,
                                    (uint32_t *)(sp + o_bad), st));
        uint32_t bad = 0;
        SCHK(s, hipMemcpyAsync(&bad, sp + o_bad, 4, hipMemcpyDeviceToHost, st));
        if (rows) SCHK(s, hipMemcpyAsync(out_log_index, sp + o_log, 4 * (size_t)rows, hipMemcpyDeviceToHost, st));
        if (rows && out_all_deps) SCHK(s, hipMemcpyAsync(out_all_deps, sp + o_ad, 4 * (size_t)rows * S, hipMemcpyDeviceToHost, st));
        SCHK(s, hipStreamSynchronize(st));
        if (bad) return hm_engine_fail(s->e, HM_ERR_INVALID, "bad handle");
        for (uint32_t r = 0; r < rows; r++)
            if (out_log_index[r] == HM_NONE) return hm_engine_fail(s->e, HM_ERR_INVALID, "history slice past the history");
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(s->e, HM_ERR_NOMEM, "exception in hm_store_read_history");
    }
}

int hm_doc_history_prefix(hm_store *s, uint32_t doc, uint32_t n, uint32_t *out) {
    if (!s || doc >= s->n_handles || (n && !out)) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    int rc = HM_OK;
    const DevDoc m = read_doc(s, doc, &rc);
    if (rc) return -rc;
    std::vector<int32_t> h(m.n_c);
    if (m.n_c) SCHK(s, hipMemcpy(h.data(), s->hist + m.c_off, m.n_c * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> by_pos(m.n_c, HM_NONE);
    uint32_t H = 0;
    for (uint32_t i = 0; i < m.n_c; i++)
        if (h[i] >= 0 && (uint32_t)h[i] < m.n_c) { by_pos[h[i]] = i; H = std::max(H, (uint32_t)h[i] + 1); }
    const uint32_t k = std::min(n, H);
    for (uint32_t i = 0; i < k; i++) out[i] = by_pos[i];
    return (int)k;
}

int hm_doc_set_min_clock(hm_store *s, uint32_t doc, const uint32_t *clock) {
    if (!s || doc >= s->n_handles || !clock) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    SCHK(s, hipMemcpy(s->min_clock + (size_t)doc * s->S, clock, s->S * 4, hipMemcpyHostToDevice));
    // the incremental kernels read the row only for documents that have one
    DevDoc m;
    SCHK(s, hipMemcpy(&m, s->dm + doc, sizeof m, hipMemcpyDeviceToHost));
    m.pad[0] |= HM_DDOC_MINC;
    SCHK(s, hipMemcpy(s->dm + doc, &m, sizeof m, hipMemcpyHostToDevice));
    return HM_OK;
}

int hm_store_clock_update(hm_store *s, uint32_t n, const uint32_t *docs, uint8_t *out_written, uint8_t *out_differs,
                          uint32_t *out_stored) {
    if (!s || (n && !docs)) return HM_ERR_INVALID;
    if (s->pending) return hm_engine_fail(s->e, HM_ERR_INVALID, "batch in flight");
    try {
        for (uint32_t i = 0; i < n; i++) if (docs[i] >= s->n_handles) return hm_engine_fail(s->e, HM_ERR_INVALID, "bad handle");
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
