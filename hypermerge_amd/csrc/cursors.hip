// cursors.hip — the CursorStore table on the device (include/hypermerge_amd.h, hm_cursors_*).
//
// Replaces the reference's SQLite `Cursors` table for one repo (src/CursorStore.ts:19-79,
// schema src/migrations/0001_initial_schema.sql:15-21): per document, the max seq of every
// actor whose changes belong to it.  It gates RepoBackend.syncChanges (src/RepoBackend.ts:
// 506-531): docsWithActor picks the documents of a synced actor, entry gives each one's upper
// bound.  Here every query is a batch: one launch answers docsWithActor for many actors, entry
// for many (document, actor) pairs, and update upserts many documents' cursors.
//
// Layout in HBM: rows (one per document, dense indices the host assigns) of K entries,
// actor key (u64: FNV-1a64 of the actor id, the repo-global key of the clock exchange) and
// seq (u64, boundedSeq-clamped to [0, INFINITY_SEQ]), plus a per-row entry count.  Entries
// keep their insertion order (SQLite rowid order of `SELECT *`).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>
#include "../../include/hypermerge_amd.h"
#include "engine_internal.h"

namespace {

typedef unsigned long long u64;
constexpr u64 INFINITY_SEQ = 9007199254740991ull;   // Number.MAX_SAFE_INTEGER (src/CursorStore.ts:17)

__device__ __forceinline__ u64 bounded_seq(double s) {        // Math.max(0, Math.min(seq, INFINITY_SEQ))
    if (!(s > 0)) return 0;                                    // NaN and negatives -> 0
    if (s >= (double)INFINITY_SEQ) return INFINITY_SEQ;
    return (u64)s;
}

// update: one 64-lane workgroup per document of the call.  Entries of one document name
// distinct actors (the caller's cursor object), so a lane that appends never races another
// lane for the same actor.  differs[d] = !Clock.equal(input, stored after the update).
__global__ __launch_bounds__(64) void cursor_update_kernel(uint32_t n_docs, const uint32_t *rows, const uint32_t *off,
                                                           const u64 *akey, const double *seq, u64 *tkey, u64 *tseq,
                                                           uint32_t *tcnt, uint32_t K, uint8_t *differs, uint32_t *status) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t d = blockIdx.x; d < n_docs; d += gridDim.x) {
        const uint32_t r = rows[d], e0 = off[d], e1 = off[d + 1];
        u64 *rk = tkey + (size_t)r * K, *rs = tseq + (size_t)r * K;
        const uint32_t c0 = tcnt[r];
        // upsert-max of the existing actors; new actors appended
        for (uint32_t e = e0 + lane; e < e1; e += 64) {
            const u64 k = akey[e], v = bounded_seq(seq[e]);
            uint32_t at = 0xFFFFFFFFu;
            for (uint32_t j = 0; j < c0 && j < K; j++) if (rk[j] == k) { at = j; break; }
            if (at != 0xFFFFFFFFu) {
                atomicMax(&rs[at], v);                         // DO UPDATE SET seq = excluded.seq WHERE excluded.seq > seq
            } else {
                const uint32_t j = atomicAdd(&tcnt[r], 1u);
                if (j < K) { rk[j] = k; rs[j] = v; }
                else atomicOr(status, 1u);                     // row full
            }
        }
        __syncthreads();
        // Clock.equal(input, stored): every stored entry equals the input's value (missing = 0)
        const uint32_t c1 = tcnt[r] < K ? tcnt[r] : K;
        bool ne = false;
        for (uint32_t j = lane; j < c1; j += 64) {
            const u64 k = rk[j];
            double in = 0.0;
            for (uint32_t e = e0; e < e1; e++) if (akey[e] == k) { in = seq[e]; break; }
            ne |= (double)rs[j] != in;
        }
        const bool any = __ballot(ne) != 0;
        if (lane == 0) differs[d] = any ? 1 : 0;
        __syncthreads();
    }
}

// capacity pre-check of an update (all-or-nothing, as the reference's SQLite transaction):
// status |= 1 if a row would outgrow K with the call's new actors; nothing is written
__global__ __launch_bounds__(64) void cursor_capacity_kernel(uint32_t n_docs, const uint32_t *rows, const uint32_t *off,
                                                             const u64 *akey, const u64 *tkey, const uint32_t *tcnt,
                                                             uint32_t K, uint32_t *status) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t d = blockIdx.x; d < n_docs; d += gridDim.x) {
        const uint32_t r = rows[d], e0 = off[d], e1 = off[d + 1];
        const u64 *rk = tkey + (size_t)r * K;
        const uint32_t c0 = tcnt[r] < K ? tcnt[r] : K;
        uint32_t fresh = 0;
        for (uint32_t e = e0 + lane; e < e1; e += 64) {
            const u64 k = akey[e];
            bool have = false;
            for (uint32_t j = 0; j < c0 && !have; j++) have = rk[j] == k;
            fresh += have ? 0u : 1u;
        }
        for (int o = 32; o > 0; o >>= 1) fresh += (uint32_t)__shfl_xor((int)fresh, o);
        if (lane == 0 && c0 + fresh > K) atomicOr(status, 1u);
    }
}

// entry(doc, actor): stored seq or 0 (src/CursorStore.ts:68-70)
__global__ void cursor_entry_kernel(uint32_t n, const uint32_t *rows, const u64 *akey, const u64 *tkey,
                                    const u64 *tseq, const uint32_t *tcnt, uint32_t K, u64 *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = rows[i], c = tcnt[r] < K ? tcnt[r] : K;
    const u64 k = akey[i];
    u64 v = 0;
    for (uint32_t j = 0; j < c; j++) if (tkey[(size_t)r * K + j] == k) { v = tseq[(size_t)r * K + j]; break; }
    out[i] = v;
}

// docsWithActor(actor, seq) for many actors at once: one lane per stored entry, the query
// actors sorted by key (binary search); matches appended through a counter
__global__ void cursor_docs_kernel(uint32_t n_rows, uint32_t K, const u64 *tkey, const u64 *tseq, const uint32_t *tcnt,
                                   uint32_t nq, const u64 *qkey, const u64 *qmin, const uint32_t *qidx, uint32_t cap,
                                   uint32_t *out_row, uint32_t *out_q, u64 *out_seq, uint32_t *counter) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (size_t)n_rows * K) return;
    const uint32_t r = (uint32_t)(g / K), j = (uint32_t)(g % K);
    if (j >= tcnt[r]) return;
    const u64 k = tkey[g], s = tseq[g];
    uint32_t lo = 0, hi = nq;
    while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (qkey[mid] < k) lo = mid + 1; else hi = mid; }
    for (uint32_t q = lo; q < nq && qkey[q] == k; q++) {
        if (s < qmin[q]) continue;                             // WHERE seq >= ?
        const uint32_t at = atomicAdd(counter, 1u);
        if (at < cap) { out_row[at] = r; out_q[at] = qidx[q]; out_seq[at] = s; }
    }
}

}  // namespace

struct hm_cursors {
    hm_engine *e = nullptr;
    uint32_t K = 0, rows = 0, cap_rows = 0;
    u64 *key = nullptr, *seq = nullptr;
    uint32_t *cnt = nullptr;
    uint8_t *stage = nullptr;
    size_t stage_cap = 0;
};

namespace {

#define CCHK(c, call)                                                                \
    do {                                                                             \
        hipError_t _r = (call);                                                      \
        if (_r != hipSuccess)                                                        \
            return hm_engine_fail((c)->e, HM_ERR_DEVICE, (std::string(#call) + ": " + hipGetErrorString(_r)).c_str()); \
    } while (0)

int stage(hm_cursors *c, size_t bytes) {
    if (bytes <= c->stage_cap) return HM_OK;
    if (c->stage) (void)hipFree(c->stage);
    c->stage = nullptr; c->stage_cap = 0;
    const size_t cap = std::max(bytes, (size_t)1 << 16) * 2;
    if (hipMalloc((void **)&c->stage, cap) != hipSuccess) return hm_engine_fail(c->e, HM_ERR_NOMEM, "hipMalloc cursor staging");
    c->stage_cap = cap;
    return HM_OK;
}

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

int hm_cursors_create(hm_engine *e, uint32_t max_actors_per_doc, hm_cursors **out) {
    if (!e || !out || max_actors_per_doc == 0 || max_actors_per_doc > 4096) return HM_ERR_INVALID;
    *out = nullptr;
    hm_cursors *c = new (std::nothrow) hm_cursors();
    if (!c) return HM_ERR_NOMEM;
    c->e = e; c->K = max_actors_per_doc;
    *out = c;
    return HM_OK;
}

void hm_cursors_destroy(hm_cursors *c) {
    if (!c) return;
    (void)hipStreamSynchronize(hm_engine_stream(c->e));
    void *b[] = {c->key, c->seq, c->cnt, c->stage};
    for (void *p : b) if (p) (void)hipFree(p);
    delete c;
}

int hm_cursors_reserve(hm_cursors *c, uint32_t n_rows) {
    if (!c) return HM_ERR_INVALID;
    if (n_rows <= c->rows) return HM_OK;
    CCHK(c, hipSetDevice(hm_engine_device(c->e)));
    hipStream_t st = hm_engine_stream(c->e);
    if (n_rows > c->cap_rows) {
        const uint32_t cap = std::max<uint32_t>(n_rows, std::max<uint32_t>(1024, c->cap_rows * 2));
        u64 *k, *s; uint32_t *n;
        if (hipMalloc((void **)&k, (size_t)cap * c->K * 8) != hipSuccess) return hm_engine_fail(c->e, HM_ERR_NOMEM, "hipMalloc cursors");
        if (hipMalloc((void **)&s, (size_t)cap * c->K * 8) != hipSuccess) { (void)hipFree(k); return hm_engine_fail(c->e, HM_ERR_NOMEM, "hipMalloc cursors"); }
        if (hipMalloc((void **)&n, (size_t)cap * 4) != hipSuccess) { (void)hipFree(k); (void)hipFree(s); return hm_engine_fail(c->e, HM_ERR_NOMEM, "hipMalloc cursors"); }
        CCHK(c, hipMemsetAsync(n, 0, (size_t)cap * 4, st));
        if (c->rows) {
            CCHK(c, hipMemcpyAsync(k, c->key, (size_t)c->rows * c->K * 8, hipMemcpyDeviceToDevice, st));
            CCHK(c, hipMemcpyAsync(s, c->seq, (size_t)c->rows * c->K * 8, hipMemcpyDeviceToDevice, st));
            CCHK(c, hipMemcpyAsync(n, c->cnt, (size_t)c->rows * 4, hipMemcpyDeviceToDevice, st));
        }
        CCHK(c, hipStreamSynchronize(st));
        if (c->key) { (void)hipFree(c->key); (void)hipFree(c->seq); (void)hipFree(c->cnt); }
        c->key = k; c->seq = s; c->cnt = n; c->cap_rows = cap;
    }
    c->rows = n_rows;
    return HM_OK;
}

int hm_cursors_update(hm_cursors *c, uint32_t n_docs, const uint32_t *rows, const uint32_t *entry_off,
                      const uint64_t *actor_keys, const double *seqs, uint8_t *out_differs) {
    if (!c || (n_docs && (!rows || !entry_off))) return HM_ERR_INVALID;
    if (!n_docs) return HM_OK;
    const uint32_t ne = entry_off[n_docs];
    if (ne && (!actor_keys || !seqs)) return HM_ERR_INVALID;
    for (uint32_t d = 0; d < n_docs; d++) {
        if (rows[d] >= c->rows) return hm_engine_fail(c->e, HM_ERR_INVALID, "cursor row not reserved");
        if (entry_off[d] > entry_off[d + 1]) return hm_engine_fail(c->e, HM_ERR_INVALID, "entry offsets not ascending");
    }
    try {
        // one entry per (row, actor) in a call: the kernel upserts rows in parallel, so a repeated
        // row or actor would race (the reference applies one cursor object per document)
        {
            std::vector<uint32_t> rs(rows, rows + n_docs);
            std::sort(rs.begin(), rs.end());
            if (std::adjacent_find(rs.begin(), rs.end()) != rs.end())
                return hm_engine_fail(c->e, HM_ERR_INVALID, "a cursor row appears twice in one update");
            std::vector<u64> ks;
            for (uint32_t d = 0; d < n_docs; d++) {
                ks.assign(actor_keys + entry_off[d], actor_keys + entry_off[d + 1]);
                std::sort(ks.begin(), ks.end());
                if (std::adjacent_find(ks.begin(), ks.end()) != ks.end())
                    return hm_engine_fail(c->e, HM_ERR_INVALID, "an actor appears twice in one document's cursor");
            }
        }
        CCHK(c, hipSetDevice(hm_engine_device(c->e)));
        hipStream_t st = hm_engine_stream(c->e);
        const size_t o_rows = 0, o_off = al(4 * (size_t)n_docs), o_key = o_off + al(4 * ((size_t)n_docs + 1)),
                     o_seq = o_key + al(8 * (size_t)ne + 8), o_dif = o_seq + al(8 * (size_t)ne + 8), o_st = o_dif + al(n_docs),
                     total = o_st + 256;
        int r = stage(c, total);
        if (r) return r;
        uint8_t *sp = c->stage;
        CCHK(c, hipMemcpyAsync(sp + o_rows, rows, 4 * (size_t)n_docs, hipMemcpyHostToDevice, st));
        CCHK(c, hipMemcpyAsync(sp + o_off, entry_off, 4 * ((size_t)n_docs + 1), hipMemcpyHostToDevice, st));
        if (ne) {
            CCHK(c, hipMemcpyAsync(sp + o_key, actor_keys, 8 * (size_t)ne, hipMemcpyHostToDevice, st));
            CCHK(c, hipMemcpyAsync(sp + o_seq, seqs, 8 * (size_t)ne, hipMemcpyHostToDevice, st));
        }
        CCHK(c, hipMemsetAsync(sp + o_st, 0, 4, st));
        const uint32_t grid = std::min<uint32_t>(n_docs, 65535u * 4);
        // all or nothing: a row that would outgrow K fails the call before anything is written
        hipLaunchKernelGGL(cursor_capacity_kernel, dim3(grid), dim3(64), 0, st, n_docs, (const uint32_t *)(sp + o_rows),
                           (const uint32_t *)(sp + o_off), (const u64 *)(sp + o_key), c->key, c->cnt, c->K,
                           (uint32_t *)(sp + o_st));
        CCHK(c, hipGetLastError());
        uint32_t over = 0;
        CCHK(c, hipMemcpyAsync(&over, sp + o_st, 4, hipMemcpyDeviceToHost, st));
        CCHK(c, hipStreamSynchronize(st));
        if (over) return hm_engine_fail(c->e, HM_ERR_INVALID, "a document's cursor would exceed max_actors_per_doc (nothing written)");
        hipLaunchKernelGGL(cursor_update_kernel, dim3(grid), dim3(64), 0, st, n_docs, (const uint32_t *)(sp + o_rows),
                           (const uint32_t *)(sp + o_off), (const u64 *)(sp + o_key), (const double *)(sp + o_seq), c->key,
                           c->seq, c->cnt, c->K, sp + o_dif, (uint32_t *)(sp + o_st));
        CCHK(c, hipGetLastError());
        uint32_t status = 0;
        CCHK(c, hipMemcpyAsync(&status, sp + o_st, 4, hipMemcpyDeviceToHost, st));
        if (out_differs) CCHK(c, hipMemcpyAsync(out_differs, sp + o_dif, n_docs, hipMemcpyDeviceToHost, st));
        CCHK(c, hipStreamSynchronize(st));
        if (status) return hm_engine_fail(c->e, HM_ERR_INVALID, "a document's cursor exceeds max_actors_per_doc");
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(c->e, HM_ERR_NOMEM, "exception in hm_cursors_update");
    }
}

int hm_cursors_get(hm_cursors *c, uint32_t n, const uint32_t *rows, uint32_t *out_count, uint64_t *out_actor,
                   uint64_t *out_seq) {
    if (!c || (n && (!rows || !out_count))) return HM_ERR_INVALID;
    CCHK(c, hipSetDevice(hm_engine_device(c->e)));
    CCHK(c, hipStreamSynchronize(hm_engine_stream(c->e)));
    for (uint32_t i = 0; i < n; i++) {
        if (rows[i] >= c->rows) return hm_engine_fail(c->e, HM_ERR_INVALID, "cursor row not reserved");
        uint32_t k = 0;
        CCHK(c, hipMemcpy(&k, c->cnt + rows[i], 4, hipMemcpyDeviceToHost));
        k = std::min(k, c->K);
        out_count[i] = k;
        if (k && out_actor) CCHK(c, hipMemcpy(out_actor + (size_t)i * c->K, c->key + (size_t)rows[i] * c->K, 8 * (size_t)k, hipMemcpyDeviceToHost));
        if (k && out_seq) CCHK(c, hipMemcpy(out_seq + (size_t)i * c->K, c->seq + (size_t)rows[i] * c->K, 8 * (size_t)k, hipMemcpyDeviceToHost));
    }
    return HM_OK;
}

int hm_cursors_entry(hm_cursors *c, uint32_t n, const uint32_t *rows, const uint64_t *actor_keys, uint64_t *out_seq) {
    if (!c || (n && (!rows || !actor_keys || !out_seq))) return HM_ERR_INVALID;
    if (!n) return HM_OK;
    for (uint32_t i = 0; i < n; i++) if (rows[i] >= c->rows) return hm_engine_fail(c->e, HM_ERR_INVALID, "cursor row not reserved");
    try {
        CCHK(c, hipSetDevice(hm_engine_device(c->e)));
        hipStream_t st = hm_engine_stream(c->e);
        const size_t o_rows = 0, o_key = al(4 * (size_t)n), o_out = o_key + al(8 * (size_t)n), total = o_out + al(8 * (size_t)n);
        int r = stage(c, total);
        if (r) return r;
        uint8_t *sp = c->stage;
        CCHK(c, hipMemcpyAsync(sp + o_rows, rows, 4 * (size_t)n, hipMemcpyHostToDevice, st));
        CCHK(c, hipMemcpyAsync(sp + o_key, actor_keys, 8 * (size_t)n, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(cursor_entry_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, (const uint32_t *)(sp + o_rows),
                           (const u64 *)(sp + o_key), c->key, c->seq, c->cnt, c->K, (u64 *)(sp + o_out));
        CCHK(c, hipGetLastError());
        CCHK(c, hipMemcpyAsync(out_seq, sp + o_out, 8 * (size_t)n, hipMemcpyDeviceToHost, st));
        CCHK(c, hipStreamSynchronize(st));
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(c->e, HM_ERR_NOMEM, "exception in hm_cursors_entry");
    }
}

int hm_cursors_docs_with_actors(hm_cursors *c, uint32_t n_actors, const uint64_t *actor_keys, const double *min_seqs,
                                uint32_t cap, uint32_t *out_row, uint32_t *out_actor, uint64_t *out_seq, uint32_t *out_n) {
    if (!c || !out_n || (n_actors && !actor_keys) || (cap && (!out_row || !out_actor || !out_seq))) return HM_ERR_INVALID;
    *out_n = 0;
    if (!n_actors || !c->rows) return HM_OK;
    try {
        // query actors sorted by key (the kernel binary-searches them), with their min seqs
        std::vector<uint32_t> order(n_actors);
        for (uint32_t i = 0; i < n_actors; i++) order[i] = i;
        std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return actor_keys[a] < actor_keys[b]; });
        std::vector<u64> qk(n_actors), qm(n_actors);
        std::vector<uint32_t> qi(n_actors);
        for (uint32_t i = 0; i < n_actors; i++) {
            const uint32_t o = order[i];
            qk[i] = actor_keys[o]; qi[i] = o;
            const double s = min_seqs ? min_seqs[o] : 0.0;
            qm[i] = !(s > 0) ? 0 : (s >= (double)INFINITY_SEQ ? INFINITY_SEQ : (u64)s);
        }
        CCHK(c, hipSetDevice(hm_engine_device(c->e)));
        hipStream_t st = hm_engine_stream(c->e);
        const size_t o_qk = 0, o_qm = al(8 * (size_t)n_actors), o_qi = o_qm + al(8 * (size_t)n_actors),
                     o_cnt = o_qi + al(4 * (size_t)n_actors), o_row = o_cnt + 256, o_q = o_row + al(4 * (size_t)cap + 4),
                     o_s = o_q + al(4 * (size_t)cap + 4), total = o_s + al(8 * (size_t)cap + 8);
        int r = stage(c, total);
        if (r) return r;
        uint8_t *sp = c->stage;
        CCHK(c, hipMemcpyAsync(sp + o_qk, qk.data(), 8 * (size_t)n_actors, hipMemcpyHostToDevice, st));
        CCHK(c, hipMemcpyAsync(sp + o_qm, qm.data(), 8 * (size_t)n_actors, hipMemcpyHostToDevice, st));
        CCHK(c, hipMemcpyAsync(sp + o_qi, qi.data(), 4 * (size_t)n_actors, hipMemcpyHostToDevice, st));
        CCHK(c, hipMemsetAsync(sp + o_cnt, 0, 4, st));
        const size_t lanes = (size_t)c->rows * c->K;
        hipLaunchKernelGGL(cursor_docs_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, c->rows, c->K, c->key,
                           c->seq, c->cnt, n_actors, (const u64 *)(sp + o_qk), (const u64 *)(sp + o_qm),
                           (const uint32_t *)(sp + o_qi), cap, (uint32_t *)(sp + o_row), (uint32_t *)(sp + o_q),
                           (u64 *)(sp + o_s), (uint32_t *)(sp + o_cnt));
        CCHK(c, hipGetLastError());
        uint32_t got = 0;
        CCHK(c, hipMemcpyAsync(&got, sp + o_cnt, 4, hipMemcpyDeviceToHost, st));
        CCHK(c, hipStreamSynchronize(st));
        *out_n = got;
        if (got > cap) return hm_engine_fail(c->e, HM_ERR_NOMEM, "cap below the matching entries (*out_n holds the count)");
        if (got) {
            CCHK(c, hipMemcpy(out_row, sp + o_row, 4 * (size_t)got, hipMemcpyDeviceToHost));
            CCHK(c, hipMemcpy(out_actor, sp + o_q, 4 * (size_t)got, hipMemcpyDeviceToHost));
            CCHK(c, hipMemcpy(out_seq, sp + o_s, 8 * (size_t)got, hipMemcpyDeviceToHost));
        }
        return HM_OK;
    } catch (...) {
        return hm_engine_fail(c->e, HM_ERR_NOMEM, "exception in hm_cursors_docs_with_actors");
    }
}

}  // extern "C"
