// store_kernels.hip — device side of the resident document store (store.cpp).
//
//  append_kernel<G>     G lanes per document of a submit: moves the document's
//                       log segments when they outgrow their capacity (or on arena
//                       compaction), applies an actor-rank remap to the old rows and to
//                       the rank-indexed per-document rows (minimumClock, stored clock),
//                       and appends the new change/dep/op rows with their offsets rebased
//                       from batch-local to arena positions.
//  (inc_kernels.hip)    incremental applyRemoteChanges on the resident state.
//  gather_kernel        per-document result rows of a batch (by handle) into one
//                       contiguous buffer, so hm_batch_wait is a single D2H copy.
//  clock_update_kernel  ClockStore.update (src/ClockStore.ts:78-91) over many documents:
//                       upsert-max of DocBackend.clock into the stored row, with the
//                       "any row written" and "!Clock.equal(input, stored)" flags.
//  sync_ranges_kernel   syncChanges' contiguous prefix (src/RepoBackend.ts:513-522):
//                       first missing block index at or after lo, below hi.
// All HBM-bound row copies / elementwise work; nothing here is on the merge's
// critical path except the appends, which move each new row exactly once.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/hypermerge_amd.h"
#include "store_kernels.h"

namespace hms {

#define SWG 256

// G lanes per document, 256 / G documents per workgroup.  A submit's appends are a few rows per
// document (C5: 1-2 changes, ~5 ops), so G = 16 keeps four documents' load -> store chains in
// flight per wave instead of one (one wave per document ran 100k documents as ~12 dependent
// chains per wave: 210 us); a compaction or rollback (old rows only, every document moved) takes
// G = 64.  Within a document every copy reads only rows no earlier store of it writes (a moved
// segment is a fresh bump allocation; new rows come from the staging tables), so the pointers
// are restrict-qualified and each loop's loads issue ahead of its stores.
template <int G>
__global__ __launch_bounds__(SWG) void append_kernel(const AppendDesc *descs, uint32_t n_desc, StoreArenas src,
                                                     StoreArenas dst, const hm_change_row *st_changes,
                                                     const hm_dep_row *st_deps, const hm_op_row *st_ops,
                                                     const uint8_t *remap, uint32_t S, const uint32_t *list,
                                                     const uint32_t *count) {
    // with a list, only the listed batch rows (alloc_kernel lists the documents with work here: a
    // round of incremental documents whose segments did not move has none)
    constexpr uint32_t PER = SWG / G;
    const uint32_t t = threadIdx.x & (G - 1);
    const uint32_t nd = list ? *count : n_desc;
    for (uint32_t k = blockIdx.x * PER + threadIdx.x / G; k < nd; k += gridDim.x * PER) {
        const uint32_t di = list ? list[k] : k;
        const AppendDesc D = descs[di];
        const bool moved = D.src_c != D.dst_c || D.src_d != D.dst_d || D.src_o != D.dst_o || src.changes != dst.changes;
        if ((D.inc & HM_DINC_ROUTE) && !moved) continue;   // the incremental kernel appends its rows itself
        const bool rm = D.remap_row != 0xFFFFFFFFu;
        const uint8_t *mp = rm ? remap + (size_t)D.remap_row * S : nullptr;
        // old rows: moved (rebased) and/or re-ranked (in place when not moved: row i -> row i)
        if (moved || rm) {
            const int64_t dd = (int64_t)D.dst_d - (int64_t)D.src_d, dop = (int64_t)D.dst_o - (int64_t)D.src_o;
            for (uint32_t i = t; i < D.n_old_c; i += G) {
                hm_change_row c = src.changes[D.src_c + i];
                c.dep_off = (uint32_t)((int64_t)c.dep_off + dd);
                c.op_first = (uint32_t)((int64_t)c.op_first + dop);
                if (rm && c.actor < S) c.actor = mp[c.actor];
                dst.changes[D.dst_c + i] = c;
            }
            for (uint32_t i = t; i < D.n_old_d; i += G) {
                hm_dep_row r = src.deps[D.src_d + i];
                if (rm && r.actor < S) r.actor = mp[r.actor];
                dst.deps[D.dst_d + i] = r;
            }
        }
        if (moved) {
            // 32-byte op rows as two 16-byte words per lane, four in flight
            const uint4 *__restrict__ so = reinterpret_cast<const uint4 *>(src.ops + D.src_o);
            uint4 *__restrict__ dop = reinterpret_cast<uint4 *>(dst.ops + D.dst_o);
            const uint32_t nw = 2 * D.n_old_o;
            uint32_t i = t;
            for (; i + 3 * G < nw; i += 4 * G) {
                const uint4 x0 = so[i], x1 = so[i + G], x2 = so[i + 2 * G], x3 = so[i + 3 * G];
                dop[i] = x0; dop[i + G] = x1; dop[i + 2 * G] = x2; dop[i + 3 * G] = x3;
            }
            for (; i < nw; i += G) dop[i] = so[i];
        }
        // new rows: batch-local offsets -> arena offsets; every load of the three tables before
        // the stores (the common round: one pass of each loop)
        const uint32_t c_at = D.dst_c + D.n_old_c, d_at = D.dst_d + D.n_old_d, o_at = D.dst_o + D.n_old_o;
        const hm_change_row *__restrict__ nc = st_changes + D.new_c;
        const hm_dep_row *__restrict__ ndp = st_deps + D.new_d;
        const uint4 *__restrict__ no = reinterpret_cast<const uint4 *>(st_ops + D.new_o);
        hm_change_row *__restrict__ oc = dst.changes + c_at;
        hm_dep_row *__restrict__ od = dst.deps + d_at;
        uint4 *__restrict__ oo = reinterpret_cast<uint4 *>(dst.ops + o_at);
        const uint32_t nwo = 2 * D.n_new_o;
        const uint32_t rounds = max(max(D.n_new_c, D.n_new_d), nwo);
        for (uint32_t i = t; i < rounds; i += G) {
            hm_change_row c = {};
            hm_dep_row r = {};
            uint4 o = {};
            if (i < D.n_new_c) c = nc[i];
            if (i < D.n_new_d) r = ndp[i];
            if (i < nwo) o = no[i];
            if (i < D.n_new_c) {
                c.dep_off = d_at + (c.dep_off - D.new_d);
                c.op_first = o_at + (c.op_first - D.new_o);
                oc[i] = c;
            }
            if (i < D.n_new_d) od[i] = r;
            if (i < nwo) oo[i] = o;
        }
        // rank-indexed per-document rows follow the remap: lane t gathers the new ranks t + G j
        // (j < 256 / G: S <= HM_MAX_STRIDE) from every old rank, all loads before any store
        if (rm) {
            constexpr uint32_t NJ = HM_MAX_STRIDE / G;
            uint32_t *rows[2] = {dst.min_clock + (size_t)D.handle * S, dst.stored_clock + (size_t)D.handle * S};
            for (int w = 0; w < 2; w++) {
                uint32_t v[NJ];
#pragma unroll
                for (uint32_t j = 0; j < NJ; j++) v[j] = 0;
                for (uint32_t a = 0; a < S; a++) {
                    const uint32_t na = mp[a];
                    if (na >= S || (na & (G - 1)) != t) continue;
                    const uint32_t x = rows[w][a];
                    const uint32_t jj = na / G;
#pragma unroll
                    for (uint32_t j = 0; j < NJ; j++) v[j] = jj == j ? x : v[j];
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (uint32_t j = 0; j < NJ; j++)
                    if (t + G * j < S) rows[w][t + G * j] = v[j];
            }
        }
    }
}

// out = [n x hm_doc_result][n x S clock][n x S back_clock][n x S heads], one 4-byte word per lane
// (consecutive lanes write consecutive words); n_fail (optional) counts rows whose status is not OK
__global__ void gather_kernel(const uint32_t *handles, uint32_t n, uint32_t S, const hm_doc_result *res_docs,
                              const uint32_t *clock, const uint32_t *back_clock, const uint32_t *heads,
                              uint8_t *out, uint32_t *n_fail) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nr = (size_t)n * 8, ns = (size_t)n * S;
    uint32_t *o = reinterpret_cast<uint32_t *>(out);
    bool fail = false;
    if (t < nr) {
        const uint32_t i = (uint32_t)(t >> 3), w = (uint32_t)(t & 7);
        const uint32_t v = reinterpret_cast<const uint32_t *>(res_docs + handles[i])[w];
        o[t] = v;
        fail = w == 0 && v != (uint32_t)HM_OK;
    } else if (t < nr + 3 * ns) {
        const size_t u = t - nr, k = u / ns, e = u - k * ns;
        const uint32_t i = (uint32_t)(e / S), a = (uint32_t)(e - (size_t)i * S);
        const uint32_t *src = k == 0 ? clock : (k == 1 ? back_clock : heads);
        o[t] = src[(size_t)handles[i] * S + a];
    }
    if (n_fail) {
        const unsigned long long b = __ballot(fail);
        if (b && (threadIdx.x & 63) == 0) atomicAdd(n_fail, (uint32_t)__popcll(b));
    }
}

// The same gather after an incremental round: the documents the incremental kernels finished
// (gdone[i] = 1) wrote their rows already, so one lane per batch row copies the rest — the
// re-merged documents, usually few — row by row.
__global__ void gather_rest_kernel(const uint32_t *handles, uint32_t n, uint32_t S, const hm_doc_result *res_docs,
                                   const uint32_t *clock, const uint32_t *back_clock, const uint32_t *heads,
                                   uint8_t *out, uint32_t *n_fail, const uint8_t *gdone) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool fail = false;
    if (i < n && !gdone[i]) {
        const size_t ns = (size_t)n * S, h = handles[i];
        const hm_doc_result r = res_docs[h];
        reinterpret_cast<hm_doc_result *>(out)[i] = r;
        fail = r.status != HM_OK;
        uint32_t *o = reinterpret_cast<uint32_t *>(out) + (size_t)n * 8 + (size_t)i * S;
        for (uint32_t a = 0; a < S; a++) {
            o[a] = clock[h * S + a];
            o[ns + a] = back_clock[h * S + a];
            o[2 * ns + a] = heads[h * S + a];
        }
    }
    if (n_fail) {
        const unsigned long long b = __ballot(fail);
        if (b && (threadIdx.x & 63) == 0) atomicAdd(n_fail, (uint32_t)__popcll(b));
    }
}

// One lane per (document, entry).  ClockStore.update writes each input entry with
// `ON CONFLICT ... DO UPDATE SET seq=excluded.seq WHERE excluded.seq > seq`, then re-reads
// the stored clock; Clock.equal treats missing and zero entries alike (src/Clock.ts:13-25).
__global__ void clock_update_kernel(const uint32_t *docs, uint32_t n, uint32_t S, const uint32_t *back_clock,
                                    uint32_t *stored, uint8_t *written, uint8_t *differs, uint32_t *out_stored) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = g / S, a = g % S;
    const bool v = i < n;
    uint32_t in = 0, st = 0, ns = 0;
    if (v) {
        const uint32_t h = docs[i];
        in = back_clock[(size_t)h * S + a];
        st = stored[(size_t)h * S + a];
        ns = in > st ? in : st;
        if (ns != st) stored[(size_t)h * S + a] = ns;
        if (out_stored) out_stored[(size_t)i * S + a] = ns;
    }
    // per-document flags: S consecutive lanes (S divides 64 when S is a power of two;
    // otherwise fall back to atomics on the byte's word)
    const bool wr = v && ns != st, df = v && ns != in;
    if (v) {
        if (wr) atomicOr(reinterpret_cast<unsigned int *>(written + (i & ~3u)), 1u << (8 * (i & 3)));
        if (df) atomicOr(reinterpret_cast<unsigned int *>(differs + (i & ~3u)), 1u << (8 * (i & 3)));
    }
}

__global__ void sync_ranges_kernel(const uint64_t *present, const uint64_t *word_off, const uint32_t *lo,
                                   const uint32_t *hi, uint32_t *out_end, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t *bits = present + word_off[i];
    uint32_t j = lo[i];
    const uint32_t h = hi[i];
    while (j < h) {
        const uint64_t w = bits[j >> 6] >> (j & 63);
        const uint64_t miss = ~w;                           // bits at and above j within the word
        const uint32_t run = miss ? (uint32_t)__builtin_ctzll(miss) : 64u - (j & 63);
        if (run < 64u - (j & 63)) { j += run; break; }     // a hole inside this word
        j += 64u - (j & 63);
    }
    // for (i = min; i < max && present(i); i++): i stays at min when min >= max
    out_end[i] = lo[i] >= h ? lo[i] : (j < h ? j : h);
}

// Rows of chosen registers (incremental patches): request i reads register abs_reg[i] and its
// survivors (doc op-segment base surv_base[i] + surv_off) into out_surv at an offset taken
// from a bump counter; its row's surv_off is rewritten to that offset.
__global__ void read_regs_kernel(uint32_t n, const uint32_t *abs_reg, const uint32_t *surv_base, const hm_reg_result *regs,
                                 const hm_surv_result *surv, hm_reg_result *out_regs, hm_surv_result *out_surv,
                                 uint32_t cap, uint32_t *counter) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    hm_reg_result r = regs[abs_reg[i]];
    const uint32_t off = atomicAdd(counter, r.n_surv);
    if (off + r.n_surv <= cap)
        for (uint32_t k = 0; k < r.n_surv; k++) out_surv[off + k] = surv[surv_base[i] + r.surv_off + k];
    r.surv_off = off;
    out_regs[i] = r;
}


// ---------------- the submit plan on the device ----------------
// plan_kernel: one thread per batch row — the checks of hm_batch_submit (handle, repeated handle
// by a per-submit stamp, row ranges, document totals, every change row inside its document's
// deps / ops, the actor remap a permutation into the new ranks), the segments the append
// outgrows and the route (incremental or re-merge).  Nothing in the store changes here: a
// failed check fails the submit with the store as it was.
__device__ __forceinline__ uint32_t grow_rows(uint32_t x) { return x > 0xC0000000u ? x : x + (x >> 2); }
__device__ __forceinline__ uint32_t pow2c(uint32_t x) {
    x = x < 16u ? 16u : x;
    return x <= 1u ? 1u : 1u << (32 - __builtin_clz(x - 1));
}

// the submit's reductions go through LDS to one atomic per workgroup and value: same-address
// atomics from every wave of a million-document submit queue at one L2 channel (~10 ns each:
// ~1.2 ms of a 1M-document incremental plan, the same in doc_rows_kernel)
#define PLAN_WG 256
__global__ __launch_bounds__(PLAN_WG) void plan_kernel(PlanArgs a) {
    __shared__ unsigned long long s_need[4][PLAN_WG / 64];
    __shared__ uint32_t s_inc[PLAN_WG / 64];
    __shared__ uint32_t s_lane[PLAN_WG / 64];
    __shared__ uint32_t s_glst[PLAN_WG / 64];
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    if (ln == 0) {
        for (int k = 0; k < 4; k++) s_need[k][wv] = 0;
        s_inc[wv] = 0;
        s_lane[wv] = 0;
        s_glst[wv] = 0;
    }
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i0 < a.n;
    const uint32_t i = live ? i0 : 0u;
    // the submit's later work lists start empty (in place of a memset launch each)
    if (live && a.gdone) a.gdone[i] = 0;
    if (i0 == 0) {
        if (a.defer) a.defer[0] = 0;
        if (a.bail) a.bail[0] = 0;
        if (a.fail) a.fail[0] = 0;
    }
    uint32_t err = 0;
    const uint32_t h = live ? a.handles[i] : 0u;
    if (live && h >= a.n_handles) err |= HM_PLAN_BAD_HANDLE;
    if (live && !err && atomicExch(&a.seen[h], a.stamp) == a.stamp) err |= HM_PLAN_REPEATED;
    const hm_doc_row r = err ? hm_doc_row{} : a.docs[i];
    const DevDoc m = err ? DevDoc{} : a.dm[live ? h : 0u];
    if ((uint64_t)r.change_off + r.n_changes > a.n_changes || (uint64_t)r.dep_off + r.n_deps > a.n_deps ||
        (uint64_t)r.op_off + r.n_ops > a.n_ops) err |= HM_PLAN_ROWS;
    if (live && (r.n_actors > a.S || r.n_actors < m.n_actors || r.n_regs < m.n_r || r.n_objs < m.n_objs || r.n_objs == 0))
        err |= HM_PLAN_TOTALS;
    if (live && !(err & (HM_PLAN_ROWS | HM_PLAN_BAD_HANDLE)))
        for (uint32_t c = r.change_off; c < r.change_off + r.n_changes; c++) {
            const hm_change_row cr = a.changes[c];
            if ((uint64_t)cr.dep_off < r.dep_off || (uint64_t)cr.dep_off + cr.n_deps > (uint64_t)r.dep_off + r.n_deps ||
                (uint64_t)cr.op_first < r.op_off || (uint64_t)cr.op_first + cr.n_ops > (uint64_t)r.op_off + r.n_ops) {
                err |= HM_PLAN_CHANGE_ROWS;
                break;
            }
        }
    bool remapped = false;
    if (live && !err && a.remap) {
        const uint8_t *mp = a.remap + (size_t)i * a.S;
        unsigned long long u0 = 0, u1 = 0, u2 = 0, u3 = 0;          // ranks taken (S <= 256)
        for (uint32_t x = 0; x < m.n_actors; x++) {
            const uint32_t y = mp[x], k = y >> 6;
            const unsigned long long b = 1ull << (y & 63);
            const unsigned long long u = k == 0 ? u0 : (k == 1 ? u1 : (k == 2 ? u2 : u3));
            if (y >= r.n_actors || (u & b)) { err |= HM_PLAN_REMAP; break; }
            u0 |= k == 0 ? b : 0ull; u1 |= k == 1 ? b : 0ull; u2 |= k == 2 ? b : 0ull; u3 |= k == 3 ? b : 0ull;
            remapped |= y != x;
        }
    }
    const bool wave_ok = __ballot(err != 0) == 0;
    if (err) atomicOr(&a.st->err, err);                            // (rare) one atomic per failing lane
    if (wave_ok) {
    PlanRow p;
    p.n_c = m.n_c; p.n_d = m.n_d; p.n_o = m.n_o; p.n_r = m.n_r; p.n_objs = m.n_objs; p.n_actors = m.n_actors; p.flags = m.flags;
    // a segment that outgrows its capacity moves to one with a quarter of its rows again as headroom
    // (a tight power of two moved a quarter to a half of C5's documents every round: their whole
    // logs copied by append_kernel)
    p.g[0] = live && m.n_c + r.n_changes > m.c_cap ? pow2c(grow_rows(m.n_c + r.n_changes)) : 0u;
    p.g[1] = live && m.n_d + r.n_deps > m.d_cap ? pow2c(grow_rows(m.n_d + r.n_deps)) : 0u;
    p.g[2] = live && m.n_o + r.n_ops > m.o_cap ? pow2c(grow_rows(m.n_o + r.n_ops)) : 0u;
    p.g[3] = live && r.n_regs > m.r_cap ? pow2c(grow_rows(r.n_regs)) : 0u;
    for (int k = 0; k < 4; k++) {
        unsigned long long g = p.g[k];
        for (int o = 32; o > 0; o >>= 1) g += (unsigned long long)__shfl_xor((long long)g, o);
        if (ln == 0) s_need[k][wv] = g;
    }
    // route: a clean resident state (last merge ok, nothing queued, no re-rank) and new rows inside
    // the incremental envelope -> the incremental kernels (which touch only the registers the new
    // ops hit); the rest re-merge their whole log
    const hm_doc_result last = a.res_docs[live ? h : 0u];
    const uint32_t tgt = r.n_deps + r.n_changes;
    // the group / wave passes hold a round in registers (HM_INC_MAX_NEW_C changes, _O ops) and take
    // a longer one in tiles of that size; a longer round of a map document of stride <= 16 takes the
    // one-lane-per-document pass, which applies the changes one after the other (up to
    // HM_INC_LANE_MAX_C / _O, HM_INC_TILED_MAX_C / _O in tiles: longer still keeps one lane / wave
    // busy for longer than the document's re-merge)
    const bool lists = ((r.flags | m.flags) & HM_DOC_HAS_LISTS) != 0;
    const bool small = r.n_changes <= HM_INC_MAX_NEW_C && r.n_ops <= HM_INC_MAX_NEW_O && tgt <= HM_INC_MAX_TGT;
    // (the lane pass is instantiated for row strides 8 and 16 only: its template stride addresses the
    // clock / heads / allDeps rows, so any other stride takes the tiles of the group passes)
    const bool lane = !small && (a.S == 8 || a.S == 16) && !lists && r.n_changes <= HM_INC_LANE_MAX_C &&
                      r.n_ops <= HM_INC_LANE_MAX_O;
    const bool longr = lane || (!small && (lists || (a.S != 8 && a.S != 16)) && r.n_changes <= HM_INC_TILED_MAX_C &&
                                r.n_ops <= HM_INC_TILED_MAX_O);     // (tiles of the group / wave passes)
    bool inc = live && a.incremental && last.status == HM_OK && last.n_queued == 0 && !remapped && r.n_changes > 0 &&
               (small || longr) && m.n_r <= r.n_regs && r.n_actors <= a.S;
    // mode 1: a small list document keeps no incremental state (inc_meta_kernel), so it re-merges
    // before any of the reads below
    const uint32_t small_lists = hm_small_list_ops(a.S, a.incremental);
    if (inc && lists && m.n_o + r.n_ops <= small_lists) inc = false;
    bool wave = false;                                             // list ops: the one-document-per-wave pass
    if (inc && a.ist) {
        // what inc_group_kernel would hand straight back (its state checks, and for documents with
        // lists its op checks): no metadata, or an op it does not take — object creation, an op on
        // an object that is neither a map of the log nor one of the document's resident lists
        const IncState I = a.ist[h];
        if ((I.flags & (HM_IST_VALID | HM_IST_NOCKEY)) != HM_IST_VALID) inc = false;
        else if ((r.flags | m.flags) & HM_DOC_HAS_LISTS)
            // (four op rows in flight per step: the lane's loads are otherwise one round trip each)
            for (uint32_t k0 = r.op_off; k0 < r.op_off + r.n_ops && inc; k0 += 4) {
                uint32_t ob[4], ac[4];
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) {
                    const uint32_t k = k0 + u < r.op_off + r.n_ops ? k0 + u : r.op_off;
                    ob[u] = reinterpret_cast<const uint4 *>(a.ops + k)[0].x;
                    ac[u] = reinterpret_cast<const uint4 *>(a.ops + k)[1].x & 0xFFu;
                }
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) {
                    if (k0 + u >= r.op_off + r.n_ops) break;
                    const uint32_t obj = ob[u];
                    const bool other = obj != 0 && (obj >= 64 || !((I.mapmask >> obj) & 1ull));   // not ROOT / a map
                    if (ac[u] <= HM_MAKE_TEXT || (other && !(I.flags & HM_IST_LIST))) inc = false;
                    wave |= other;
                }
            }
        // causallyReady in arrival order against the resident clock (small strides: the clock in
        // registers): a change the queue would hold, or a duplicate, goes to the re-merge at once.
        // Only for documents with lists, whose failed attempt costs a wave each (the map-only
        // documents' group pass finds it as cheaply as this would)
        if (inc && a.clock && a.S <= 16 && ((r.flags | m.flags) & HM_DOC_HAS_LISTS)) {
            uint32_t ck[16];
#pragma unroll
            for (uint32_t x = 0; x < 16; x++) ck[x] = x < a.S ? a.clock[(size_t)h * a.S + x] : 0u;
            for (uint32_t c = r.change_off; c < r.change_off + r.n_changes && inc; c++) {
                const hm_change_row cr = a.changes[c];
                uint32_t cur = 0;
#pragma unroll
                for (uint32_t x = 0; x < 16; x++) cur = x == cr.actor ? ck[x] : cur;
                if (cr.actor >= a.S || cr.seq != cur + 1u) { inc = false; break; }
                for (uint32_t j = 0; j < cr.n_deps && inc; j++) {
                    const hm_dep_row dr = a.deps[cr.dep_off + j];
                    uint32_t dv = 0;
#pragma unroll
                    for (uint32_t x = 0; x < 16; x++) dv = x == dr.actor ? ck[x] : dv;
                    if (dr.actor != cr.actor && (dr.actor >= a.S || dr.seq > dv)) inc = false;
                }
#pragma unroll
                for (uint32_t x = 0; x < 16; x++) ck[x] = x == cr.actor ? cr.seq : ck[x];
            }
        }
    }
    // cost policy (mode 1): a small list document re-merges in one small-kernel wave; and a round
    // whose new rows are more than 1 / HM_INC_COST of the log after it re-merges — the merge
    // kernels take a log row ~HM_INC_COST times faster than the incremental passes take a new
    // one (C4: 37 ps per change merged vs 0.43-0.53 ns per change applied), so that round is
    // cheaper re-merged (this also sends a first load into a document re-merged empty to the merge)
    if (inc && wave && m.n_o + r.n_ops <= small_lists) inc = false;
    // list documents of strides <= 16 whose round fits a group take the group passes' list
    // instantiation (a longer round goes straight to the wave pass)
    const uint32_t GS = a.S <= 8 ? 8u : 16u;
    if (HM_INC_LIST_GROUPS && a.S <= 16 && r.n_ops <= GS && r.n_deps <= GS && r.n_changes <= HM_INC_MAX_NEW_C)
        wave = false;
    const bool glist = inc && !wave && lists;
    if (inc && a.incremental == 1u &&
        (unsigned long long)HM_INC_COST * (r.n_changes + r.n_ops) > (unsigned long long)m.n_c + m.n_o + r.n_changes + r.n_ops)
        inc = false;
    p.inc = inc ? (wave ? 2u : (lane ? 3u : 1u)) : 0u;
    p.remapped = remapped ? 1u : 0u;
    if (live) a.plan[i] = p;
    const unsigned long long im = __ballot(inc), lm = __ballot(inc && p.inc == 3u), gm = __ballot(glist && p.inc == 1u);
    if (ln == 0) { s_inc[wv] = (uint32_t)__popcll(im); s_lane[wv] = (uint32_t)__popcll(lm); s_glst[wv] = (uint32_t)__popcll(gm); }
    }
    __syncthreads();
    if (threadIdx.x < 7) {                                         // one lane per reduced value
        const uint32_t k = threadIdx.x, nw = PLAN_WG / 64;
        if (k < 4) {
            unsigned long long g = 0;
            for (uint32_t w = 0; w < nw; w++) g += s_need[k][w];
            if (g) atomicAdd(&a.st->need[k], g);
        } else {
            uint32_t c = 0;
            for (uint32_t w = 0; w < nw; w++) c += k == 4 ? s_inc[w] : (k == 5 ? s_lane[w] : s_glst[w]);
            if (c) atomicAdd(k == 4 ? &a.st->n_inc : (k == 5 ? &a.st->mx[0] : &a.st->mx[4]), c);
        }
    }
}

// alloc_kernel: segments for the rows that outgrow theirs (bump allocation at the arenas'
// ends), the append descriptor, the document's new totals, and the three work lists (re-merge,
// wave pass, append).  The list slots are taken one atomic per workgroup and list: the same-
// address atomics of every wave of a submit serialize at one L2 channel (100k documents: ~1.5k
// waves x 3 lists)
#define ALLOC_WG 256
__global__ __launch_bounds__(ALLOC_WG) void alloc_kernel(PlanArgs a) {
    __shared__ uint32_t s_cnt[3][ALLOC_WG / 64];
    __shared__ uint32_t s_base[3];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const bool live = i < a.n;
    // the plan failed a check, or the arenas cannot take the growth: nothing moves (the host finds
    // out from the stats; every later kernel of the submit sees route 0 and empty lists)
    {
        const PlanStats *st = a.st;
        const bool stop = st->err != 0 || st->bump[0] + st->need[0] > a.cap[0] || st->bump[1] + st->need[1] > a.cap[1] ||
                          st->bump[2] + st->need[2] > a.cap[2] || st->bump[3] + st->need[3] > a.cap[3];
        if (stop) {
            if (live) a.descs[i].inc = 0;
            if (i == 0 && st->err == 0) a.st->mx[1] = 1u;         // no room: the host compacts and plans again
            return;
        }
    }
    bool cold = false, wavep = false, app = false;
    uint32_t h = 0;
    if (live) {
        h = a.handles[i];
        const hm_doc_row r = a.docs[i];
        const PlanRow p = a.plan[i];
        DevDoc m = a.dm[h];
        AppendDesc D;
        D.handle = h;
        D.src_c = m.c_off; D.n_old_c = m.n_c; D.new_c = r.change_off; D.n_new_c = r.n_changes;
        D.src_d = m.d_off; D.n_old_d = m.n_d; D.new_d = r.dep_off; D.n_new_d = r.n_deps;
        D.src_o = m.o_off; D.n_old_o = m.n_o; D.new_o = r.op_off; D.n_new_o = r.n_ops;
        D.src_r = m.r_off; D.n_old_r = m.n_r;
        if (p.g[0]) { m.c_off = (uint32_t)atomicAdd(&a.st->bump[0], (unsigned long long)p.g[0]); m.c_cap = p.g[0]; }
        if (p.g[1]) { m.d_off = (uint32_t)atomicAdd(&a.st->bump[1], (unsigned long long)p.g[1]); m.d_cap = p.g[1]; }
        if (p.g[2]) { m.o_off = (uint32_t)atomicAdd(&a.st->bump[2], (unsigned long long)p.g[2]); m.o_cap = p.g[2]; }
        if (p.g[3]) { m.r_off = (uint32_t)atomicAdd(&a.st->bump[3], (unsigned long long)p.g[3]); m.r_cap = p.g[3]; }
        D.dst_c = m.c_off; D.dst_d = m.d_off; D.dst_o = m.o_off; D.dst_r = m.r_off;
        D.remap_row = p.remapped ? i : 0xFFFFFFFFu;
        m.n_c += r.n_changes; m.n_d += r.n_deps; m.n_o += r.n_ops;
        m.n_r = r.n_regs; m.n_objs = r.n_objs; m.n_actors = r.n_actors; m.flags |= r.flags;
        D.n_r = m.n_r; D.n_actors = m.n_actors; D.n_objs = m.n_objs; D.o_cap = m.o_cap;
        D.inc = (uint16_t)(p.inc | (p.inc && (m.pad[0] & HM_DDOC_MINC) ? HM_DINC_MINC : 0u) |
                           (p.inc && (m.flags & HM_DOC_HAS_LISTS) ? HM_DINC_LISTS : 0u));
        a.descs[i] = D;
        a.dm[h] = m;
        cold = !p.inc;                                   // the re-merge list (handles)
        wavep = a.defer && p.inc == 2u;                  // documents with list ops: the one-document-per-wave pass
        app = !p.inc || p.g[0] || p.g[1] || p.g[2] || p.remapped;   // the rows append_kernel must visit
    }
    const unsigned long long mk[3] = {__ballot(cold), __ballot(wavep), __ballot(app)};
    if (ln < 3) s_cnt[ln][wv] = (uint32_t)__popcll(ln == 0 ? mk[0] : ln == 1 ? mk[1] : mk[2]);
    __syncthreads();
    if (threadIdx.x < 3) {
        const uint32_t k = threadIdx.x;
        uint32_t t = 0;
        for (uint32_t w = 0; w < ALLOC_WG / 64; w++) t += s_cnt[k][w];
        uint32_t *ctr = k == 0 ? &a.st->n_cold : k == 1 ? a.defer : &a.st->n_app;
        s_base[k] = t ? atomicAdd(ctr, t) : 0u;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << ln) - 1;
    uint32_t off[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        off[k] = s_base[k] + (uint32_t)__popcll(mk[k] & lt);
        for (uint32_t w = 0; w < wv; w++) off[k] += s_cnt[k][w];
    }
    if (cold) a.list[off[0]] = h;
    if (wavep) a.defer[1 + off[1]] = i;
    if (app) a.alist[off[2]] = i;
}

__global__ __launch_bounds__(PLAN_WG) void doc_rows_kernel(const uint32_t *list, uint32_t n, const DevDoc *dm, hm_doc_row *rows,
                                                          PlanStats *st, uint32_t small_lists, IncState *ist, uint32_t *keep) {
    // per workgroup: 5 maxima, the flags OR, 4 sums, the keep counts -> LDS, then one atomic each
    __shared__ uint32_t s_mx[8];
    __shared__ unsigned long long s_tot[4];
    __shared__ uint32_t s_kw[PLAN_WG / 64], s_kbase;
    if (threadIdx.x < 8) s_mx[threadIdx.x] = 0;
    if (threadIdx.x < 4) s_tot[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    bool kp = false, drop = false;
    uint32_t h = 0;
    if (i < n) {
        h = list[i];
        const DevDoc m = dm[h];
        // documents that may keep incremental state after this re-merge (inc_meta_kernel decides;
        // mode 1's small list documents never do), and those of them with lists; the others'
        // state is cleared here (incremental stores)
        const bool lists = (m.flags & HM_DOC_HAS_LISTS) != 0;
        kp = !(lists && m.n_o <= small_lists);
        if (kp && lists) atomicAdd(&s_mx[7], 1u);
        if (!kp && ist) {
            drop = HM_IST_COUNTS(ist[h].flags);                // (PlanStats.n_valid follows every state cleared)
            IncState z = {};
            ist[h] = z;
        }
        hm_doc_row r;
        r.change_off = m.c_off; r.n_changes = m.n_c; r.dep_off = m.d_off; r.n_deps = m.n_d;
        r.op_off = m.o_off; r.n_ops = m.n_o; r.reg_off = m.r_off; r.n_regs = m.n_r;
        r.n_objs = m.n_objs; r.n_actors = m.n_actors; r.flags = m.flags; r.reserved[0] = r.reserved[1] = 0;
        rows[i] = r;
        atomicMax(&s_mx[0], m.n_c); atomicMax(&s_mx[1], m.n_o); atomicMax(&s_mx[2], m.n_r);
        atomicMax(&s_mx[3], m.n_objs); atomicMax(&s_mx[4], m.n_d); atomicOr(&s_mx[5], (uint32_t)m.flags);
        atomicAdd(&s_tot[0], (unsigned long long)m.n_c); atomicAdd(&s_tot[1], (unsigned long long)m.n_d);
        atomicAdd(&s_tot[2], (unsigned long long)m.n_o); atomicAdd(&s_tot[3], (unsigned long long)m.n_r);
    }
    const uint32_t nd = (uint32_t)__popcll(__ballot(drop));
    if (ln == 0 && nd) atomicSub(&st->n_valid, nd);
    // the keep list (inc_meta's and the position clear's work list): one slot atomic per workgroup
    const unsigned long long km = __ballot(kp);
    if (ln == 0) s_kw[wv] = (uint32_t)__popcll(km);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < PLAN_WG / 64; w++) t += s_kw[w];
        s_kbase = t ? atomicAdd(&st->mx[2], t) : 0u;
    }
    __syncthreads();
    if (kp && keep) {
        uint32_t off = s_kbase + (uint32_t)__popcll(km & ((1ull << ln) - 1));
        for (uint32_t w = 0; w < wv; w++) off += s_kw[w];
        keep[off] = h;
    }
    switch (threadIdx.x) {
    case 0: atomicMax(&st->max_c, s_mx[0]); break;
    case 1: atomicMax(&st->max_o, s_mx[1]); break;
    case 2: atomicMax(&st->max_r, s_mx[2]); break;
    case 3: atomicMax(&st->max_objs, s_mx[3]); break;
    case 4: atomicMax(&st->max_d, s_mx[4]); break;
    case 5: if (s_mx[5]) atomicOr(&st->flags, s_mx[5]); break;
    case 6: atomicAdd(&st->tot_c, s_tot[0]); break;
    case 7: atomicAdd(&st->tot_d, s_tot[1]); break;
    case 8: atomicAdd(&st->tot_o, s_tot[2]); break;
    case 9: atomicAdd(&st->tot_r, s_tot[3]); break;
    case 11: if (s_mx[7]) atomicAdd(&st->mx[3], s_mx[7]); break;
    default: break;
    }
}

// every = 0: the documents whose merge failed (marked in their plan row: rolled back once);
// every = 1: all documents of the batch not rolled back yet (hm_batch_undo)
__global__ void rollback_kernel(const uint32_t *handles, uint32_t n, const hm_doc_result *res_docs, PlanRow *plan,
                                const uint8_t *remap, uint32_t S, DevDoc *dm, AppendDesc *descs, uint8_t *inv,
                                uint32_t *list, PlanStats *st, uint32_t every) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = handles[i];
    if (plan[i].inc == 0xFFFFFFFFu || (!every && res_docs[h].status == HM_OK)) return;
    const PlanRow p = plan[i];
    plan[i].inc = 0xFFFFFFFFu;
    DevDoc m = dm[h];
    const uint32_t k = atomicAdd(&st->n_back, 1u);
    AppendDesc D = {};
    D.handle = h;
    D.src_c = D.dst_c = m.c_off; D.n_old_c = p.n_c;
    D.src_d = D.dst_d = m.d_off; D.n_old_d = p.n_d;
    D.src_o = D.dst_o = m.o_off; D.n_old_o = p.n_o;
    D.remap_row = 0xFFFFFFFFu;
    if (p.remapped && remap) {
        // the old ranks back: the inverse of the submit's remap row
        uint8_t *iv = inv + (size_t)k * S;
        for (uint32_t x = 0; x < S; x++) iv[x] = 0xFF;
        const uint8_t *mp = remap + (size_t)i * S;
        for (uint32_t x = 0; x < p.n_actors; x++) iv[mp[x]] = (uint8_t)x;
        D.remap_row = k;
    }
    m.n_c = p.n_c; m.n_d = p.n_d; m.n_o = p.n_o; m.n_r = p.n_r; m.n_objs = p.n_objs; m.n_actors = p.n_actors; m.flags = p.flags;
    dm[h] = m;
    descs[k] = D;
    list[k] = h;
}

__global__ void init_docs_kernel(DevDoc *dm, uint32_t h0, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    DevDoc m = {};
    m.n_objs = 1;                                            // ROOT
    dm[h0 + i] = m;
}

// hm_doc_reset: the listed handles back to the empty document (init_docs_kernel's row, the
// Backend.init() result row, zero clocks and incremental state); one thread per handle
__global__ void reset_docs_kernel(const uint32_t *handles, uint32_t n, DevDoc *dm, hm_doc_result *res, IncState *ist,
                                  uint32_t *clock, uint32_t *back, uint32_t *heads, uint32_t *minc, uint32_t *stored,
                                  uint32_t S, uint32_t *n_valid) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = handles[i];
    DevDoc m = {};
    m.n_objs = 1;
    dm[h] = m;
    hm_doc_result r = {};
    r.err_change = HM_NONE; r.err_op = HM_NONE;
    res[h] = r;
    if (HM_IST_COUNTS(ist[h].flags)) atomicSub(n_valid, 1u);
    ist[h] = IncState{};
    for (uint32_t a = 0; a < S; a++) {
        const size_t k = (size_t)h * S + a;
        clock[k] = 0; back[k] = 0; heads[k] = 0; minc[k] = 0; stored[k] = 0;
    }
}

__global__ void read_regs_h_kernel(uint32_t n, const uint32_t *handles, const uint32_t *regs, const DevDoc *dm,
                                   uint32_t n_handles, const hm_reg_result *rr, const hm_surv_result *surv,
                                   hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t cap, uint32_t *counter,
                                   uint32_t *bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = handles[i];
    if (h >= n_handles) { atomicOr(bad, 1u); return; }
    const DevDoc m = dm[h];
    if (regs[i] >= m.n_r) { atomicOr(bad, 2u); return; }
    hm_reg_result r = rr[m.r_off + regs[i]];
    const uint32_t off = atomicAdd(counter, r.n_surv);
    if (off + r.n_surv <= cap)
        for (uint32_t k = 0; k < r.n_surv; k++) out_surv[off + k] = surv[m.o_off + r.surv_off + k];
    r.surv_off = off;
    out_regs[i] = r;
}

// history.slice(from, to) of many documents (the changes a round applied, in application order):
// one 64-lane workgroup per request scans the document's history positions; change i with
// from <= hist[i] < to lands at out_off + hist[i] - from (log index, and its allDeps row)
__global__ void read_hist_kernel(uint32_t n, const uint32_t *handles, const uint32_t *from, const uint32_t *to,
                                 const uint32_t *out_off, const DevDoc *dm, uint32_t n_handles, const int32_t *hist,
                                 const uint32_t *all_deps, uint32_t S, uint32_t *out_log, uint32_t *out_ad, uint32_t *bad) {
    for (uint32_t q = blockIdx.x; q < n; q += gridDim.x) {
        const uint32_t h = handles[q];
        if (h >= n_handles) { if (threadIdx.x == 0) atomicOr(bad, 1u); continue; }
        const DevDoc m = dm[h];
        const uint32_t f = from[q], t = to[q], o = out_off[q];
        for (uint32_t i = threadIdx.x; i < m.n_c; i += blockDim.x) {
            const int32_t p = hist[m.c_off + i];
            if (p < 0 || (uint32_t)p < f || (uint32_t)p >= t) continue;
            const uint32_t at = o + (uint32_t)p - f;
            out_log[at] = i;
            if (out_ad)
                for (uint32_t a = 0; a < S; a++) out_ad[(size_t)at * S + a] = all_deps[((size_t)m.c_off + i) * S + a];
        }
    }
}

}  // namespace hms

hipError_t hm_launch_plan(const PlanArgs &a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    hipLaunchKernelGGL(hms::plan_kernel, dim3((a.n + PLAN_WG - 1) / PLAN_WG), dim3(PLAN_WG), 0, s, a);
    return hipGetLastError();
}
hipError_t hm_launch_alloc(const PlanArgs &a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    hipLaunchKernelGGL(hms::alloc_kernel, dim3((a.n + ALLOC_WG - 1) / ALLOC_WG), dim3(ALLOC_WG), 0, s, a);
    return hipGetLastError();
}
hipError_t hm_launch_doc_rows(const uint32_t *list, uint32_t n, const DevDoc *dm, hm_doc_row *rows, PlanStats *st,
                              uint32_t small_lists, IncState *ist, uint32_t *keep, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::doc_rows_kernel, dim3((n + PLAN_WG - 1) / PLAN_WG), dim3(PLAN_WG), 0, s, list, n, dm, rows, st,
                       small_lists, ist, keep);
    return hipGetLastError();
}
hipError_t hm_launch_rollback(const uint32_t *handles, uint32_t n, const hm_doc_result *res_docs, PlanRow *plan,
                              const uint8_t *remap, uint32_t S, DevDoc *dm, AppendDesc *descs, uint8_t *inv,
                              uint32_t *list, PlanStats *st, uint32_t every, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::rollback_kernel, dim3((n + 255) / 256), dim3(256), 0, s, handles, n, res_docs, plan, remap, S, dm,
                       descs, inv, list, st, every);
    return hipGetLastError();
}
hipError_t hm_launch_init_docs(DevDoc *dm, uint32_t h0, uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::init_docs_kernel, dim3((n + 255) / 256), dim3(256), 0, s, dm, h0, n);
    return hipGetLastError();
}
hipError_t hm_launch_reset_docs(const uint32_t *handles, uint32_t n, DevDoc *dm, hm_doc_result *res, IncState *ist,
                                uint32_t *clock, uint32_t *back, uint32_t *heads, uint32_t *minc, uint32_t *stored,
                                uint32_t S, uint32_t *n_valid, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::reset_docs_kernel, dim3((n + 255) / 256), dim3(256), 0, s, handles, n, dm, res, ist, clock, back,
                       heads, minc, stored, S, n_valid);
    return hipGetLastError();
}
hipError_t hm_launch_read_regs_h(uint32_t n, const uint32_t *handles, const uint32_t *regs, const DevDoc *dm,
                                 uint32_t n_handles, const hm_reg_result *rr, const hm_surv_result *surv,
                                 hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t cap, uint32_t *counter,
                                 uint32_t *bad, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::read_regs_h_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, handles, regs, dm, n_handles, rr,
                       surv, out_regs, out_surv, cap, counter, bad);
    return hipGetLastError();
}

hipError_t hm_launch_read_hist(uint32_t n, const uint32_t *handles, const uint32_t *from, const uint32_t *to,
                               const uint32_t *out_off, const DevDoc *dm, uint32_t n_handles, const int32_t *hist,
                               const uint32_t *all_deps, uint32_t S, uint32_t *out_log, uint32_t *out_ad, uint32_t *bad,
                               hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t grid = n < 65535u ? n : 65535u;
    hipLaunchKernelGGL(hms::read_hist_kernel, dim3(grid), dim3(64), 0, s, n, handles, from, to, out_off, dm, n_handles, hist,
                       all_deps, S, out_log, out_ad, bad);
    return hipGetLastError();
}

hipError_t hm_launch_append(const AppendDesc *descs, uint32_t n_desc, const StoreArenas &src, const StoreArenas &dst,
                            const hm_change_row *st_changes, const hm_dep_row *st_deps, const hm_op_row *st_ops,
                            const uint8_t *remap, uint32_t S, hipStream_t s, const uint32_t *list, const uint32_t *count) {
    if (!n_desc) return hipSuccess;
    // new rows: 16 lanes per document; old rows only (compaction, rollback): a wave each
    const bool small = st_changes != nullptr;
    const uint32_t per = small ? SWG / 16 : SWG / 64;
    const uint32_t cap = list ? 4096u : 65535u;                 // (a listed launch: the count is on the device)
    const uint32_t grid = (n_desc + per - 1) / per < cap ? (n_desc + per - 1) / per : cap;
    if (small)
        hipLaunchKernelGGL(hms::append_kernel<16>, dim3(grid), dim3(SWG), 0, s, descs, n_desc, src, dst, st_changes,
                           st_deps, st_ops, remap, S, list, count);
    else
        hipLaunchKernelGGL(hms::append_kernel<64>, dim3(grid), dim3(SWG), 0, s, descs, n_desc, src, dst, st_changes,
                           st_deps, st_ops, remap, S, list, count);
    return hipGetLastError();
}

hipError_t hm_launch_read_regs(uint32_t n, const uint32_t *abs_reg, const uint32_t *surv_base, const hm_reg_result *regs,
                               const hm_surv_result *surv, hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t cap,
                               uint32_t *counter, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::read_regs_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, abs_reg, surv_base, regs, surv,
                       out_regs, out_surv, cap, counter);
    return hipGetLastError();
}

hipError_t hm_launch_gather(const uint32_t *handles, uint32_t n, uint32_t S, const hm_doc_result *res_docs,
                            const uint32_t *clock, const uint32_t *back_clock, const uint32_t *heads, uint8_t *out,
                            uint32_t *n_fail, hipStream_t s, const uint8_t *gdone) {
    if (!n) return hipSuccess;
    if (gdone) {
        hipLaunchKernelGGL(hms::gather_rest_kernel, dim3((n + 255) / 256), dim3(256), 0, s, handles, n, S, res_docs, clock,
                           back_clock, heads, out, n_fail, gdone);
        return hipGetLastError();
    }
    const size_t words = (size_t)n * (8 + 3 * (size_t)S);
    hipLaunchKernelGGL(hms::gather_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, handles, n, S, res_docs,
                       clock, back_clock, heads, out, n_fail);
    return hipGetLastError();
}

hipError_t hm_launch_clock_update(const uint32_t *docs, uint32_t n, uint32_t S, const uint32_t *back_clock,
                                  uint32_t *stored, uint8_t *written, uint8_t *differs, uint32_t *out_stored,
                                  hipStream_t s) {
    if (!n) return hipSuccess;
    const size_t lanes = (size_t)n * S;
    hipLaunchKernelGGL(hms::clock_update_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, docs, n, S,
                       back_clock, stored, written, differs, out_stored);
    return hipGetLastError();
}

hipError_t hm_launch_sync_ranges(const uint64_t *present, const uint64_t *word_off, const uint32_t *lo,
                                 const uint32_t *hi, uint32_t *out_end, uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::sync_ranges_kernel, dim3((n + 255) / 256), dim3(256), 0, s, present, word_off, lo, hi,
                       out_end, n);
    return hipGetLastError();
}
