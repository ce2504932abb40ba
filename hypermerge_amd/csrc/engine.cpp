// engine.cpp — the C-ABI of include/hypermerge_amd.h (host side of the engine).
//
// Owns the HIP device, stream, events and staging buffers; sizes and launches
// the merge kernels.  No C++ exception crosses the ABI: every entry point
// catches and returns an hm_status.  There is no CPU fallback: if the HIP
// library cannot run, calls fail with HM_ERR_DEVICE.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>
#include <algorithm>
#include <new>
#include "../../include/hypermerge_amd.h"
#include "merge_kernels.h"
#include "engine_internal.h"

struct hm_engine {
    int device = 0;
    int flags = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {};
    float last_ms[2] = {0, 0};
    int n_last = 0;
    int num_cus = 256;
    std::string err;
    void *dbuf = nullptr;
    size_t dbuf_size = 0;
    void *pool = nullptr;        // merge_large_kernel cursor + scratch pool
    size_t pool_size = 0;
    hipStream_t h2d = nullptr, d2h = nullptr;   // copy streams of the chunked hm_merge_host pipeline
    const char *last_scratch = nullptr;         // scratch of the last launch (hm_last_deferred)
};

namespace {

int fail(hm_engine *e, int status, const std::string &msg) {
    if (e) e->err = msg;
    return status;
}

int hip_fail(hm_engine *e, hipError_t r, const char *what) {
    return fail(e, HM_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(r));
}

#define HIPCHK(e, call)                                   \
    do {                                                  \
        hipError_t _r = (call);                           \
        if (_r != hipSuccess) return hip_fail(e, _r, #call); \
    } while (0)

struct Caps { uint32_t opl, cls; bool lists, counters; };

Caps launch_caps(const hm_batch *b) {
    Caps c;
    uint32_t mo = b->max_ops;
    c.opl = mo <= 64 ? 1 : (mo <= 128 ? 2 : (mo <= 192 ? 3 : 4));
    // 0 = unknown hint -> the larger class (documents outside it are deferred)
    c.cls = (b->max_regs && b->max_objs && b->max_deps) ? hm_small_class(b->max_regs, b->max_objs, b->max_deps) : 1u;
    c.lists = (b->doc_flags & HM_DOC_HAS_LISTS) != 0;
    c.counters = (b->doc_flags & HM_DOC_HAS_COUNTERS) != 0;
    return c;
}

// The launch's scratch: [counters 256 B: large-kernel cursor, pool bump pointer, deferred
// count][deferred document list, n_docs u32][large-kernel pool].  `scratch` = caller memory of
// hm_launch_scratch_bytes(b) bytes, or NULL for the engine's own pool (calls on the engine pool
// must be serialised: one stream at a time, which the engine enforces by synchronising the
// device before the pool is resized).
int launch_merge(hm_engine *e, const hm_batch *b, const hm_results *o, hipStream_t s, const uint32_t *doc_slot,
                 const hm_extents *ext, void *scratch, uint32_t *epos = nullptr) {
    Caps c = launch_caps(b);
    SmallParams p;
    p.res_epos = epos;
    p.docs = b->docs; p.changes = b->changes; p.deps = b->deps; p.ops = b->ops; p.min_clock = b->min_clock;
    p.res_docs = o->docs; p.res_clock = o->clock; p.res_back_clock = o->back_clock; p.res_heads = o->heads;
    p.res_hist = o->hist; p.res_all_deps = o->all_deps; p.res_regs = o->regs; p.res_surv = o->surv;
    p.n_docs = b->n_docs; p.a_stride = b->a_stride; p.cap_regs = 0; p.cap_objs = 0; p.cap_deps = 0;
    p.counters = c.counters ? 1u : 0u;
    p.general_only = (e->flags & HM_CFG_GENERAL_ONLY) ? 1u : 0u;
    {
        static const int remap = [] { const char *v = getenv("HM_XCD_REMAP"); return v ? atoi(v) : 1; }();
        p.xcd_remap = remap ? 1u : 0u;
    }
    p.doc_slot = doc_slot;
    p.lim_changes = ext ? ext->n_changes : b->n_changes; p.lim_deps = ext ? ext->n_deps : b->n_deps;
    p.lim_ops = ext ? ext->n_ops : b->n_ops; p.lim_regs = ext ? ext->n_regs : b->n_regs;
    if (b->n_docs == 0) { e->n_last = 0; return HM_OK; }
    const size_t list_bytes = ((size_t)b->n_docs * 4 + 255) & ~(size_t)255;
    const size_t need = hm_launch_scratch_bytes(b);
    const size_t pool_bytes = need - 256 - list_bytes;
    char *pb = (char *)scratch;
    if (!pb) {
        if (need > e->pool_size) {
            if (e->pool) { HIPCHK(e, hipDeviceSynchronize()); HIPCHK(e, hipFree(e->pool)); }
            e->pool = nullptr; e->pool_size = 0;
            if (hipMalloc(&e->pool, need) != hipSuccess) return fail(e, HM_ERR_NOMEM, "hipMalloc scratch pool");
            e->pool_size = need;
        }
        pb = (char *)e->pool;
    }
    p.large_cursor = (uint32_t *)pb;
    unsigned long long *pool_used = (unsigned long long *)(pb + 8);
    p.n_deferred = (uint32_t *)(pb + 16);
    p.deferred = (uint32_t *)(pb + 256);
    HIPCHK(e, hipMemsetAsync(pb, 0, 32, s));
    // persistent grid: exactly the resident 1-wave workgroups (VGPR/LDS occupancy of the
    // instantiation), so every wave starts at once and the documents split evenly — a
    // larger grid would leave a partial second round of waves as a tail
    const uint32_t per_cu = hm_small_occupancy(c.opl, c.cls, c.lists, c.counters);
    uint32_t grid = std::min<uint32_t>(b->n_docs, (uint32_t)e->num_cus * per_cu);
    HIPCHK(e, hipEventRecord(e->ev[0], s));
    hipError_t r = hm_launch_small(p, c.opl, c.cls, c.lists, grid, s);
    if (r != hipSuccess) return hip_fail(e, r, "merge_small_kernel launch");
    HIPCHK(e, hipEventRecord(e->ev[1], s));
    HIPCHK(e, hipEventRecord(e->ev[2], s));
    r = hm_launch_large(p, pb + 256 + list_bytes, pool_bytes, pool_used, (uint32_t)e->num_cus * 4, s);
    if (r != hipSuccess) return hip_fail(e, r, "merge_large_kernel launch");
    HIPCHK(e, hipEventRecord(e->ev[3], s));
    e->n_last = 2;
    // the deferred list lives in the scratch: only the engine's own pool outlives this call
    // (caller scratch may be freed or reused before hm_last_deferred)
    e->last_scratch = scratch ? nullptr : pb;
    return HM_OK;
}

}  // namespace

size_t hm_launch_scratch_bytes(const hm_batch *b) {
    const size_t list_bytes = ((size_t)b->n_docs * 4 + 255) & ~(size_t)255;
    return 256 + list_bytes + hm_large_scratch_bound(b);
}

namespace {

// hm_merge_host splits a batch into document ranges when its tables are laid out in document
// order (each doc's changes, deps, ops and registers directly follow the previous doc's, as
// every encoder here writes them); other layouts, and small batches, go in one piece.
uint32_t host_chunks(const hm_batch *b) {
    const uint32_t per = 1u << 16;                 // >= 64k documents per chunk
    if (b->n_docs < 2 * per || !b->docs || !b->changes || !b->ops) return 1;
    uint64_t c = 0, p = 0, o = 0, r = 0;
    for (uint32_t i = 0; i < b->n_docs; i++) {
        const hm_doc_row &d = b->docs[i];
        if (d.change_off != c || d.dep_off != p || d.op_off != o || d.reg_off != r) return 1;
        c += d.n_changes; p += d.n_deps; o += d.n_ops; r += d.n_regs;
    }
    if (c != b->n_changes || p != b->n_deps || o != b->n_ops) return 1;
    return std::min<uint32_t>(16, b->n_docs / per);
}

int check_batch(hm_engine *e, const hm_batch *b) {
    if (!b || b->a_stride == 0 || b->a_stride > HM_MAX_STRIDE) return fail(e, HM_ERR_INVALID, "a_stride must be in [1,256]");
    if (b->n_docs && !b->docs) return fail(e, HM_ERR_INVALID, "docs table missing");
    if ((b->n_changes && !b->changes) || (b->n_deps && !b->deps) || (b->n_ops && !b->ops))
        return fail(e, HM_ERR_INVALID, "row table missing");
    return HM_OK;
}

}  // namespace

// ---- internal interface for store.cpp (engine_internal.h) ----
int hm_engine_launch_merge(hm_engine *e, const hm_batch *b, const hm_results *o, const uint32_t *doc_slot,
                           const hm_extents *ext, uint32_t *epos) {
    return launch_merge(e, b, o, e->stream, doc_slot, ext, nullptr, epos);
}
hipStream_t hm_engine_stream(hm_engine *e) { return e->stream; }
int hm_engine_device(hm_engine *e) { return e->device; }
int hm_engine_fail(hm_engine *e, int status, const char *msg) { return fail(e, status, msg); }

extern "C" {

uint32_t hm_abi_version(void) { return HM_ABI_VERSION; }

const char *hm_status_message(int status) {
    switch (status) {
    case HM_OK: return "ok";
    case HM_ERR_INCONSISTENT_SEQ: return "Inconsistent reuse of sequence number";
    case HM_ERR_UNKNOWN_OBJECT: return "Modification of unknown object";
    case HM_ERR_DUPLICATE_OBJECT: return "Duplicate creation of object";
    case HM_ERR_DUPLICATE_ELEM: return "Duplicate list element ID";
    case HM_ERR_MISSING_ELEM: return "Missing index entry for list element";
    case HM_ERR_UNSUPPORTED: return "document outside the engine envelope";
    case HM_ERR_INVALID: return "invalid batch";
    case HM_ERR_DEVICE: return "HIP device error";
    case HM_ERR_NOMEM: return "out of memory";
    default: return "unknown status";
    }
}

int hm_engine_create(const hm_config *cfg, hm_engine **out) {
    if (!out) return HM_ERR_INVALID;
    *out = nullptr;
    hm_engine *e = new (std::nothrow) hm_engine();
    if (!e) return HM_ERR_NOMEM;
    e->device = cfg ? cfg->device : 0;
    e->flags = cfg ? cfg->flags : 0;
    int n = 0;
    // a failing step is named on stderr (there is no engine to hold the message)
    auto fail = [&](const char *what, hipError_t r) {
        fprintf(stderr, "hm_engine_create: %s failed: %s (device %d, %d devices)\n", what, hipGetErrorString(r), e->device, n);
        delete e;
        return HM_ERR_DEVICE;
    };
    hipError_t r = hipGetDeviceCount(&n);
    if (r != hipSuccess) return fail("hipGetDeviceCount", r);
    if (n <= e->device) return fail("device ordinal", hipErrorInvalidDevice);
    if ((r = hipSetDevice(e->device)) != hipSuccess) return fail("hipSetDevice", r);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, e->device) == hipSuccess) e->num_cus = prop.multiProcessorCount;
    {
        size_t lim = 0, need = hm_large_stack_bytes();
        if (hipDeviceGetLimit(&lim, hipLimitStackSize) == hipSuccess && need > lim &&
            (r = hipDeviceSetLimit(hipLimitStackSize, need)) != hipSuccess) return fail("hipDeviceSetLimit(stack)", r);
    }
    if ((r = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", r);
    for (auto &ev : e->ev)
        if ((r = hipEventCreate(&ev)) != hipSuccess) return fail("hipEventCreate", r);
    *out = e;
    return HM_OK;
}

void hm_engine_destroy(hm_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->dbuf) (void)hipFree(e->dbuf);
    if (e->pool) (void)hipFree(e->pool);
    for (auto &ev : e->ev) if (ev) (void)hipEventDestroy(ev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->h2d) (void)hipStreamDestroy(e->h2d);
    if (e->d2h) (void)hipStreamDestroy(e->d2h);
    delete e;
}

const char *hm_engine_last_error(const hm_engine *e) { return e ? e->err.c_str() : "no engine"; }

size_t hm_scratch_bytes(const hm_batch *b) { return b ? hm_launch_scratch_bytes(b) : 0; }

int hm_merge_device(hm_engine *e, const hm_batch *b, const hm_results *o, void *scratch, void *stream) {
    try {
        if (!e || !o) return HM_ERR_INVALID;
        int st = check_batch(e, b);
        if (st) return st;
        if (b->n_docs && (!b->max_changes && !b->max_ops && !b->max_regs && !b->max_objs))
            return fail(e, HM_ERR_INVALID, "device batches must carry max_* launch hints");
        HIPCHK(e, hipSetDevice(e->device));
        return launch_merge(e, b, o, stream ? (hipStream_t)stream : e->stream, nullptr, nullptr, scratch);
    } catch (...) {
        return fail(e, HM_ERR_DEVICE, "exception in hm_merge_device");
    }
}

int hm_merge_host(hm_engine *e, const hm_batch *hb, const hm_results *ho) {
    try {
        if (!e || !hb || !ho) return HM_ERR_INVALID;
        int st = check_batch(e, hb);
        if (st) return st;
        HIPCHK(e, hipSetDevice(e->device));
        hm_batch b = *hb;
        if (!b.max_changes && !b.max_ops && !b.max_regs && !b.max_objs) {
            for (uint32_t d = 0; d < b.n_docs; d++) {
                b.max_changes = std::max(b.max_changes, hb->docs[d].n_changes);
                b.max_ops = std::max(b.max_ops, hb->docs[d].n_ops);
                b.max_regs = std::max(b.max_regs, hb->docs[d].n_regs);
                b.max_objs = std::max(b.max_objs, hb->docs[d].n_objs);
                b.max_deps = std::max(b.max_deps, hb->docs[d].n_deps);
                b.doc_flags |= hb->docs[d].flags;
            }
        }
        const size_t S = b.a_stride;
        struct Seg { size_t bytes; size_t off; };
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        size_t sz[13] = {
            b.n_docs * sizeof(hm_doc_row), b.n_changes * sizeof(hm_change_row), b.n_deps * sizeof(hm_dep_row),
            b.n_ops * sizeof(hm_op_row), hb->min_clock ? b.n_docs * S * 4 : 0,
            b.n_docs * sizeof(hm_doc_result), b.n_docs * S * 4, b.n_docs * S * 4, b.n_docs * S * 4,
            b.n_changes * 4, b.n_changes * S * 4, b.n_regs * sizeof(hm_reg_result), b.n_ops * sizeof(hm_surv_result)};
        size_t off[13], total = 0;
        for (int i = 0; i < 13; i++) { off[i] = total; total += al(sz[i] ? sz[i] : 1); }
        if (total > e->dbuf_size) {
            if (e->dbuf) (void)hipFree(e->dbuf);
            e->dbuf = nullptr; e->dbuf_size = 0;
            if (hipMalloc(&e->dbuf, total) != hipSuccess) return fail(e, HM_ERR_NOMEM, "hipMalloc staging");
            e->dbuf_size = total;
        }
        char *base = (char *)e->dbuf;
        auto P = [&](int i) { return (void *)(base + off[i]); };
        hipStream_t s = e->stream;
        b.docs = (const hm_doc_row *)P(0); b.changes = (const hm_change_row *)P(1);
        b.deps = (const hm_dep_row *)P(2); b.ops = (const hm_op_row *)P(3);
        b.min_clock = hb->min_clock ? (const uint32_t *)P(4) : nullptr;
        hm_results d;
        d.docs = (hm_doc_result *)P(5); d.clock = (uint32_t *)P(6); d.back_clock = (uint32_t *)P(7);
        d.heads = (uint32_t *)P(8); d.hist = (int32_t *)P(9); d.all_deps = (uint32_t *)P(10);
        d.regs = (hm_reg_result *)P(11); d.surv = (hm_surv_result *)P(12);
        const void *src[5] = {hb->docs, hb->changes, hb->deps, hb->ops, hb->min_clock};
        void *dst[8] = {ho->docs, ho->clock, ho->back_clock, ho->heads, ho->hist, ho->all_deps, ho->regs, ho->surv};
        const uint32_t nchunk = host_chunks(hb);
        if (nchunk <= 1) {
            for (int i = 0; i < 5; i++)
                if (sz[i]) HIPCHK(e, hipMemcpyAsync(P(i), src[i], sz[i], hipMemcpyHostToDevice, s));
            // the survivor table is only defined on [0, n_surv) per doc: zero it for stable host views
            if (sz[12]) HIPCHK(e, hipMemsetAsync(P(12), 0, sz[12], s));
            st = launch_merge(e, &b, &d, s, nullptr, nullptr, nullptr);
            if (st) return st;
            for (int i = 0; i < 8; i++)
                if (sz[5 + i] && dst[i]) HIPCHK(e, hipMemcpyAsync(dst[i], P(5 + i), sz[5 + i], hipMemcpyDeviceToHost, s));
            HIPCHK(e, hipStreamSynchronize(s));
            return HM_OK;
        }
        // Chunked pipeline over document ranges (documents laid out in order, host_chunks):
        // chunk k's upload (h2d stream) overlaps chunk k-1's merge (engine stream) and chunk
        // k-2's download (d2h stream), so both PCIe directions run at once.  Each chunk is a
        // sub-batch whose doc-indexed pointers start at its first document; row offsets inside
        // the doc rows stay absolute into the full-size device tables.
        if (!e->h2d) HIPCHK(e, hipStreamCreateWithFlags(&e->h2d, hipStreamNonBlocking));
        if (!e->d2h) HIPCHK(e, hipStreamCreateWithFlags(&e->d2h, hipStreamNonBlocking));
        std::vector<hipEvent_t> evs(2 * nchunk, nullptr);
        int rc = HM_OK;
        auto cleanup = [&]() {
            (void)hipStreamSynchronize(e->h2d); (void)hipStreamSynchronize(s); (void)hipStreamSynchronize(e->d2h);
            for (auto ev : evs) if (ev) (void)hipEventDestroy(ev);
        };
        for (auto &ev : evs)
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) { cleanup(); return fail(e, HM_ERR_DEVICE, "hipEventCreate"); }
        const hm_doc_row *hd = hb->docs;
        const uint32_t nd = b.n_docs;
        auto H2D = [&](void *dp, const void *hp, size_t bytes) {
            return bytes ? hipMemcpyAsync(dp, hp, bytes, hipMemcpyHostToDevice, e->h2d) : hipSuccess; };
        auto D2H = [&](void *hp, const void *dp, size_t bytes) {
            return (bytes && hp) ? hipMemcpyAsync(hp, dp, bytes, hipMemcpyDeviceToHost, e->d2h) : hipSuccess; };
#define HM_CK(x) do { hipError_t _r = (x); if (_r != hipSuccess) { rc = hip_fail(e, _r, #x); goto done; } } while (0)
        for (uint32_t k = 0; k < nchunk; k++) {
            const uint32_t d0 = (uint32_t)((uint64_t)nd * k / nchunk), d1 = (uint32_t)((uint64_t)nd * (k + 1) / nchunk);
            const uint32_t l = d1 - 1;
            const size_t c0 = hd[d0].change_off, c1 = (size_t)hd[l].change_off + hd[l].n_changes;
            const size_t p0 = hd[d0].dep_off, p1 = (size_t)hd[l].dep_off + hd[l].n_deps;
            const size_t o0 = hd[d0].op_off, o1 = (size_t)hd[l].op_off + hd[l].n_ops;
            const size_t r0 = hd[d0].reg_off, r1 = (size_t)hd[l].reg_off + hd[l].n_regs;
            char *dc = (char *)P(1), *dp = (char *)P(2), *dop = (char *)P(3);
            HM_CK(H2D((char *)P(0) + d0 * sizeof(hm_doc_row), hd + d0, (size_t)(d1 - d0) * sizeof(hm_doc_row)));
            HM_CK(H2D(dc + c0 * sizeof(hm_change_row), hb->changes + c0, (c1 - c0) * sizeof(hm_change_row)));
            HM_CK(H2D(dp + p0 * sizeof(hm_dep_row), hb->deps + p0, (p1 - p0) * sizeof(hm_dep_row)));
            HM_CK(H2D(dop + o0 * sizeof(hm_op_row), hb->ops + o0, (o1 - o0) * sizeof(hm_op_row)));
            if (hb->min_clock) HM_CK(H2D((char *)P(4) + d0 * S * 4, hb->min_clock + d0 * S, (d1 - d0) * S * 4));
            HM_CK(hipEventRecord(evs[2 * k], e->h2d));
            HM_CK(hipStreamWaitEvent(s, evs[2 * k], 0));
            HM_CK(hipMemsetAsync((char *)P(12) + o0 * sizeof(hm_surv_result), 0, (o1 - o0) * sizeof(hm_surv_result), s));
            {
                hm_batch cb = b;
                cb.n_docs = d1 - d0;
                cb.docs = b.docs + d0;
                cb.min_clock = b.min_clock ? b.min_clock + d0 * S : nullptr;
                hm_results co = d;
                co.docs = d.docs + d0; co.clock = d.clock + d0 * S; co.back_clock = d.back_clock + d0 * S;
                co.heads = d.heads + d0 * S;
                rc = launch_merge(e, &cb, &co, s, nullptr, nullptr, nullptr);
                if (rc) goto done;
            }
            HM_CK(hipEventRecord(evs[2 * k + 1], s));
            HM_CK(hipStreamWaitEvent(e->d2h, evs[2 * k + 1], 0));
            HM_CK(D2H(ho->docs ? ho->docs + d0 : nullptr, d.docs + d0, (size_t)(d1 - d0) * sizeof(hm_doc_result)));
            HM_CK(D2H(ho->clock ? ho->clock + d0 * S : nullptr, d.clock + d0 * S, (d1 - d0) * S * 4));
            HM_CK(D2H(ho->back_clock ? ho->back_clock + d0 * S : nullptr, d.back_clock + d0 * S, (d1 - d0) * S * 4));
            HM_CK(D2H(ho->heads ? ho->heads + d0 * S : nullptr, d.heads + d0 * S, (d1 - d0) * S * 4));
            HM_CK(D2H(ho->hist ? ho->hist + c0 : nullptr, d.hist + c0, (c1 - c0) * 4));
            HM_CK(D2H(ho->all_deps ? ho->all_deps + c0 * S : nullptr, d.all_deps + c0 * S, (c1 - c0) * S * 4));
            HM_CK(D2H(ho->regs ? ho->regs + r0 : nullptr, d.regs + r0, (r1 - r0) * sizeof(hm_reg_result)));
            HM_CK(D2H(ho->surv ? ho->surv + o0 : nullptr, d.surv + o0, (o1 - o0) * sizeof(hm_surv_result)));
        }
#undef HM_CK
    done:
        cleanup();
        return rc;
    } catch (...) {
        return fail(e, HM_ERR_DEVICE, "exception in hm_merge_host");
    }
}

int hm_last_kernel_ms(hm_engine *e, float *ms, int max_kernels) {
    if (!e || !ms) return 0;
    int n = std::min(max_kernels, e->n_last);
    for (int i = 0; i < n; i++) {
        if (hipEventSynchronize(e->ev[2 * i + 1]) != hipSuccess) return 0;
        if (hipEventElapsedTime(&ms[i], e->ev[2 * i], e->ev[2 * i + 1]) != hipSuccess) return 0;
    }
    return n;
}

int hm_last_deferred(hm_engine *e, uint32_t *out_docs, uint32_t cap) {
    if (!e) return -HM_ERR_INVALID;
    if (e->n_last < 2) return 0;
    if (!e->last_scratch) return -fail(e, HM_ERR_INVALID, "the last launch used caller scratch: its deferred list is the caller's");
    if (hipEventSynchronize(e->ev[3]) != hipSuccess) return -HM_ERR_DEVICE;
    uint32_t n = 0;
    if (hipMemcpy(&n, e->last_scratch + 16, 4, hipMemcpyDeviceToHost) != hipSuccess) return -HM_ERR_DEVICE;
    const uint32_t k = std::min(n, cap);
    if (k && out_docs && hipMemcpy(out_docs, e->last_scratch + 256, (size_t)k * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return -HM_ERR_DEVICE;
    return (int)n;
}

int hm_clock_cmp_device(hm_engine *e, const uint32_t *a, const uint32_t *b, uint8_t *out, uint32_t n_docs,
                        uint32_t a_stride, void *stream) {
    if (!e) return HM_ERR_INVALID;
    hipError_t r = hm_launch_clock(0, a, b, out, n_docs, a_stride, stream ? (hipStream_t)stream : e->stream);
    return r == hipSuccess ? HM_OK : hip_fail(e, r, "clock_cmp");
}

int hm_clock_union_device(hm_engine *e, const uint32_t *a, const uint32_t *b, uint32_t *c, uint32_t n_docs,
                          uint32_t a_stride, void *stream) {
    if (!e) return HM_ERR_INVALID;
    hipError_t r = hm_launch_clock(1, a, b, c, n_docs, a_stride, stream ? (hipStream_t)stream : e->stream);
    return r == hipSuccess ? HM_OK : hip_fail(e, r, "clock_union");
}

int hm_clock_intersection_device(hm_engine *e, const uint32_t *a, const uint32_t *b, uint32_t *c,
                                 uint32_t n_docs, uint32_t a_stride, void *stream) {
    if (!e) return HM_ERR_INVALID;
    hipError_t r = hm_launch_clock(2, a, b, c, n_docs, a_stride, stream ? (hipStream_t)stream : e->stream);
    return r == hipSuccess ? HM_OK : hip_fail(e, r, "clock_intersection");
}

}  // extern "C"
