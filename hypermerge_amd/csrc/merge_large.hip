// merge_large.hip — the general merge kernel: one 256-thread workgroup per document,
// for documents outside merge_small_kernel's envelope (more than 64 changes, more
// than 8 actors, long op lists, big lists/texts).  Per-document working arrays live
// in a device scratch pool (bump-allocated by each workgroup); small tables in LDS.
//
// Same reference semantics as merge_kernels.hip (Automerge
// 0.12.2-beta.0 backend/op_set.js, not vendored — yarn.lock:178-185), computed so
// that long documents parallelise over their changes/ops:
//   L1  first-arrival table per (actor, seq) -> fast path (every change ready on
//       arrival: history = arrival order minus duplicates, one block scan) or the exact
//       queue-pass emulation (wave 0; readiness of 64 queued changes per ballot).
//   L2  allDeps by the LITERAL transitiveDeps fold in history order (lanes = actors):
//       acc = max(acc, allDeps(d) + {d}); acc[actor_d] = seq_d, deps in key order.
//   L3  registers: survivors = set/link ops o with max_{x} allDeps(x)[actor_o] < seq_o
//       over the register's set/del/link ops x (per-register x per-actor atomicMax);
//       order, ties and counters as in the small kernel.
//   L4  RGA order: Euler tour of the insertion tree + pointer jumping (block-wide).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/hypermerge_amd.h"
#include "merge_kernels.h"

#ifndef HML_KARG_RELOAD
#define HML_KARG_RELOAD 1   // merge_large_kernel: launch parameters re-read per document (see the kernel)
#endif
#ifndef HML_WGS_PER_CU
#define HML_WGS_PER_CU 1   // workgroups per CU: 16 waves per CU split into this many documents
#endif
#ifndef HML_LWG
#define HML_LWG (1024 / HML_WGS_PER_CU)   // threads per workgroup
#endif
#define LWG HML_LWG
#define HML_WPE (LWG * HML_WGS_PER_CU / 256)   // waves per SIMD (register budget 512 / HML_WPE)
#define LA_MAX 64    // objects whose tables live in LDS (Shared) rather than the pool
#define LA_ACT 256   // actors per document (HM_MAX_STRIDE): the per-actor tables in Shared
// LDS arena per workgroup (u32 words).  One 1024-thread workgroup per CU owns 150 KB: a
// document's whole L3/L4 working set (op words, assign lists, register / node / parent tables,
// Euler tour) is resident there (l34_res) instead of in the pool, whose per-document tables
// (~300 KB for a C3 text document) cannot stay in an XCD's 4 MB L2 across its workgroups and
// were re-fetched from HBM (7.4x the algorithmic bytes).  Documents whose L2 closure rows
// (2·n·A + T words) or L4 Euler tour (E words, 16-bit links) fit run those phases out of LDS.
#if HML_WGS_PER_CU == 1
#define LARENA 38400
#else
#define LARENA (36864 / HML_WGS_PER_CU)
#endif
#ifndef HML_RES
#define HML_RES 1       // 0: every document takes the pool L3/L4 (dev A/B builds)
#endif
#ifndef HML_STAGE
#define HML_STAGE 1     // 0: L1/L2 read change / dep rows from HBM and keep the L1 table in the pool (dev A/B)
#endif
#ifndef HML_DOC_ATTR
#define HML_DOC_ATTR __noinline__   // the general path: its own register allocation, off merge_doc_res's
#endif
// Explicit address spaces: LDS pointers -> ds_*, pool pointers -> global_* (a generic pointer
// would compile to flat_* ops, which count against lgkmcnt too, so every LDS wait would also
// wait for the outstanding pool loads, stores and atomics).
#if defined(__HIP_DEVICE_COMPILE__)
#define LDS __attribute__((address_space(3)))
#define GLB __attribute__((address_space(1)))
#else
#define LDS
#define GLB
#endif
typedef unsigned long long u64;

#ifndef HM_PAR_HIST
#define HM_PAR_HIST 1   // 0: queued documents always take the serial queue emulation (dev A/B builds)
#endif
#define PH_ATTR __noinline__
#ifndef HM_STAMPS
#define HM_STAMPS 0     // diagnostic builds only: per-phase s_memtime shares (tools/lstamps.py); never timed
#endif
#define HML_NSTAMP 16
// registers with at most this many assigns test survivors against the assign list directly;
// longer lists build per-actor maxima with atomics (SEG_SHORT assign lists cost one LDS row
// read each, where every assign's A atomicMax on shared L2 lines cost ~27 % of C3's kernel)
#define SEG_SHORT 8
#define ORDERED (1ull << 63)     // survabs flag: a counter survivor whose incs are summed in application order

namespace hml {

__device__ __forceinline__ void bsync() { __syncthreads(); }
#if HM_STAMPS
__device__ unsigned long long hml_stamp_acc[HML_NSTAMP];
__shared__ unsigned long long hml_st[HML_NSTAMP + 1];
__device__ __forceinline__ u64 lstamp_now() {
    u64 t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define LSTAMP(i) do { bsync(); const u64 t_ = lstamp_now(); if (threadIdx.x == 0) { hml_st[i] += t_ - hml_st[HML_NSTAMP]; hml_st[HML_NSTAMP] = t_; } } while (0)
#else
#define LSTAMP(i) do { } while (0)
#endif
// order one lane's global writes before the wave's next reads (wave-uniform sections)
__device__ __forceinline__ void wfence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// error key: history position (20 b) | op index + 1 (16 b) | arrival index (20 b) | code (8 b)
__device__ __forceinline__ u64 err_key(uint32_t h, uint32_t op_plus1, uint32_t arr, uint32_t code) {
    return ((u64)(h & 0xFFFFF) << 44) | ((u64)(op_plus1 & 0xFFFF) << 28) | ((u64)(arr & 0xFFFFF) << 8) | code;
}

struct Shared {
    uint32_t base[LA_ACT], maxs[LA_ACT], tabo[LA_ACT + 1], clock[LA_ACT], bclock[LA_ACT], headv[LA_ACT];
    uint32_t maxad[LA_ACT];
    uint32_t oslot[LA_MAX], otype[LA_MAX];   // objslot / objtype of documents with <= LA_MAX objects
    uint32_t listid[LA_MAX], listbase[LA_MAX + 1];   // l34_res: compact list ids, list bases
    uint32_t flags, all_ok, H, nins, nl, total, lists, grew, nmake, nodup, ctrs, nsurv;
    uint32_t late;                      // an insert after an element not yet inserted
    uint32_t gflag[3];
    u64 errkey;
    uint32_t scan[LWG / 64 + 1];
    u64 scratch_base;
    u64 ws_base, ws_size;           // this workgroup's scratch, reused by its next documents
};

enum : uint32_t { LF_UNSUPPORTED = 1u, LF_NOPOOL = 2u };

// device-scope relaxed atomics on pool (global) pointers
template <typename T> __device__ __forceinline__ T g_add(GLB T *p, T v) { return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T> __device__ __forceinline__ T g_or(GLB T *p, T v) { return __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T> __device__ __forceinline__ T g_min(GLB T *p, T v) { return __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T> __device__ __forceinline__ T g_max(GLB T *p, T v) { return __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// The thread index as a value computed where it is used: the per-lane constants of the scans
// (lane, wave, shuffle addresses) were hoisted out of the document loop by the compiler and
// spilled to scratch at 128 VGPRs, so every scan of every document reloaded them through the
// vector memory path (and its s_waitcnt also waited for every older load and store).
__device__ __forceinline__ uint32_t fresh_tid() {
    uint32_t t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((uint32_t)threadIdx.x));
    return t;
}
// DPP lane moves (gfx9 encodings; lanes without a source read 0): inclusive sum / max over the
// wave with row shifts and the row broadcasts — VALU only, no address, no LDS crossbar
#define DPP_ROW_SHR(n) (0x110 + (n))
#define DPP_WAVE_SHR1 0x138
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(1), 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(2), 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(4), 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(8), 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_BCAST15, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_BCAST31, 0xC, 0xF, false);
    return x;
}
__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(1), 0xF, 0xF, false));
    x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(2), 0xF, 0xF, false));
    x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(4), 0xF, 0xF, false));
    x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(8), 0xF, 0xF, false));
    x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_BCAST15, 0xA, 0xF, false));
    x = umax32(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_BCAST31, 0xC, 0xF, false));
    return x;
}

// exclusive scan of v over the block; returns the prefix, *total = block sum
__device__ __forceinline__ uint32_t block_excl_scan(Shared &sh, uint32_t v, uint32_t *total) {
    const uint32_t t = fresh_tid(), lane = t & 63, w = t >> 6;
    const uint32_t x = wave_incl_sum(v);
    if (lane == 63) sh.scan[w] = x;
    bsync();
    uint32_t off = 0, tot = 0;
    for (uint32_t i = 0; i < LWG / 64; i++) { if (i < w) off += sh.scan[i]; tot += sh.scan[i]; }
    bsync();
    *total = tot;
    return off + x - v;
}
// exclusive scan of src[0..N) into dst (dst may be src): each thread owns a contiguous run of
// ceil(N / LWG) entries (its loads are independent, so they overlap), one block scan of the run
// sums.  Two barriers: the one after the wave totals are published, and the trailing one (dst
// complete) — which also orders these reads of sh.scan before the next scan's writes.
// (P, Q: pool or LDS pointers)
template <typename P, typename Q>
__device__ __forceinline__ uint32_t scan_into(Shared &sh, P src, Q dst, uint32_t N) {
    const uint32_t per = (N + LWG - 1) / LWG, tb = fresh_tid();
    const uint32_t b0 = tb * per < N ? tb * per : N;
    const uint32_t b1 = b0 + per < N ? b0 + per : N;
    uint32_t sum = 0;
    for (uint32_t i = b0; i < b1; i++) sum += src[i];
    const uint32_t t = fresh_tid(), lane = t & 63, w = t >> 6;
    const uint32_t x = wave_incl_sum(sum);
    if (lane == 63) sh.scan[w] = x;
    bsync();
    uint32_t off = 0, tot = 0;
    for (uint32_t i = 0; i < LWG / 64; i++) { const uint32_t t = sh.scan[i]; off += i < w ? t : 0u; tot += t; }
    uint32_t ex = off + x - sum;
    for (uint32_t i = b0; i < b1; i++) { const uint32_t v = src[i]; dst[i] = ex; ex += v; }
    bsync();
    return tot;
}
template <typename P>
__device__ __forceinline__ uint32_t scan_array(Shared &sh, P arr, uint32_t N) { return scan_into(sh, arr, arr, N); }
// exclusive scan of f(0..N) into dst, for N <= LWG (one value per thread; the same two barriers)
template <typename F, typename Q>
__device__ __forceinline__ uint32_t scan_fn_small(Shared &sh, F f, Q dst, uint32_t N) {
    const uint32_t i = fresh_tid(), lane = i & 63, w = i >> 6;
    const uint32_t v = i < N ? f(i) : 0u;
    const uint32_t x = wave_incl_sum(v);
    if (lane == 63) sh.scan[w] = x;
    bsync();
    uint32_t off = 0, tot = 0;
    for (uint32_t k = 0; k < LWG / 64; k++) { const uint32_t t = sh.scan[k]; off += k < w ? t : 0u; tot += t; }
    if (i < N) dst[i] = off + x - v;
    bsync();
    return tot;
}

struct Scratch {
    GLB uint32_t *tab, *h2a, *opchg, *segmax, *segcnt, *survcnt, *regoff, *regobj, *segoff, *segfill;
    GLB uint32_t *survtmp, *segk, *survop, *survp, *objtype, *listid, *nodepi, *nreg, *nlist, *regnode, *pcount, *poff;
    GLB uint32_t *pfill, *plist, *fc, *ns, *tour0, *tour1, *tval0, *tval1, *listbase, *vis;
    GLB int32_t *hist;
    GLB uint32_t *insmin, *objslot, *seglist, *nodekey, *kbase, *survk;   // 32-bit op keys (L3)
    GLB u64 *survabs;
    GLB int64_t *survsum;
    GLB uint32_t *vc;                   // [n * A] closure rows (L2 pointer jumping, second buffer)
    GLB uint32_t *hx;                   // parallel history (L1): [ht n][hp n][hnev n][hfill n][hmem n][hoff n+1][pm T]
};

__host__ __device__ inline size_t large_carve(uintptr_t base, uint32_t n, uint32_t m, uint32_t R, uint32_t O,
                                              uint32_t A, uint32_t T, Scratch *S) {
    size_t o = 0;
    const uint32_t NP = R + O, NE = 2 * (m + O);
#define TK(f, T_, cnt) do { S->f = (GLB T_ *)(base + o); o = (o + (size_t)(cnt) * sizeof(T_) + 15) & ~(size_t)15; } while (0)
    TK(survabs, u64, m); TK(survsum, int64_t, m); TK(vc, uint32_t, (size_t)n * A);
    TK(survk, uint32_t, m); TK(insmin, uint32_t, R); TK(objslot, uint32_t, O); TK(seglist, uint32_t, m);
    TK(nodekey, uint32_t, m); TK(kbase, uint32_t, n);
    TK(tab, uint32_t, T); TK(h2a, uint32_t, n); TK(hist, int32_t, n); TK(opchg, uint32_t, m);
    TK(segmax, uint32_t, (size_t)R * A); TK(segcnt, uint32_t, R); TK(survcnt, uint32_t, R);
    TK(regoff, uint32_t, R); TK(regobj, uint32_t, R); TK(segoff, uint32_t, R); TK(segfill, uint32_t, R);
    TK(survtmp, uint32_t, m); TK(segk, uint32_t, m); TK(survop, uint32_t, m); TK(survp, uint32_t, m); TK(objtype, uint32_t, O);
    TK(listid, uint32_t, O); TK(nodepi, uint32_t, m); TK(nreg, uint32_t, m); TK(nlist, uint32_t, m); TK(regnode, uint32_t, R);
    TK(pcount, uint32_t, NP); TK(poff, uint32_t, NP); TK(pfill, uint32_t, NP); TK(plist, uint32_t, m);
    TK(fc, uint32_t, NP); TK(ns, uint32_t, m); TK(tour0, uint32_t, NE); TK(tour1, uint32_t, NE);
    TK(tval0, uint32_t, NE); TK(tval1, uint32_t, NE);
    TK(listbase, uint32_t, O + 1); TK(vis, uint32_t, m);
    TK(hx, uint32_t, 6 * (size_t)n + 1 + T);
#undef TK
    return o;
}

enum Outcome { LOK = 0, LERR = 1, LUNSUP = 2 };

// L3 stages per-change inputs and a 16-bit op -> change map in the LDS arena (merge_doc_large)
__device__ __forceinline__ bool l3_ok(uint32_t n, uint32_t m, uint32_t A) {
    return n < 65536 && n * (A + 5) + (m + 1) / 2 <= LARENA;
}

// allDeps row of the applied change at arrival index ci (global, written in history order)
__device__ __forceinline__ uint32_t *ad_row(const SmallParams &p, const hm_doc_row &doc, uint32_t ci) {
    return p.res_all_deps + ((size_t)doc.change_off + ci) * p.a_stride;
}

// exclusive max-scan of v over the block (identity 0): the max over lower-numbered threads
__device__ __forceinline__ uint32_t block_excl_max(Shared &sh, uint32_t v) {
    const uint32_t t = fresh_tid(), lane = t & 63, w = t >> 6;
    const uint32_t x = wave_incl_max(v);
    const uint32_t ex = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_WAVE_SHR1, 0xF, 0xF, false);
    if (lane == 63) sh.scan[w] = x;
    bsync();
    uint32_t off = 0;
    for (uint32_t i = 0; i < LWG / 64; i++) if (i < w) off = off > sh.scan[i] ? off : sh.scan[i];
    bsync();
    const uint32_t e = lane ? ex : 0u;
    return off > e ? off : e;
}

// ---- L1 parallel: the exact queue-pass history without the serial emulation ----
// (documents without duplicate changes; the rest take the serial emulation)
// The arrival whose processing applies change K is t(K) = the latest arrival among K and its
// ancestors (ancestors = per actor a chain prefix up to the closure clock C(K)[a], so
// t(K) = max(arr(K), max_a PM_a[C(K)[a]]) with PM_a the prefix max of arrival index along
// actor a's seqs; never for a missing ancestor or a dependency cycle).  K applies in pass 1
// of that processing if t(K) = arr(K), else in pass max(2, pass(D) + [arr(D) > arr(K)]) over
// its direct deps D applied in the same processing (a pass walks the queue, which is arrival
// order, applying what is ready).  History = applied changes ordered by (t, pass, arr).
// C(K) comes from pointer jumping over the actor chains (log-depth rounds).  Returns false
// (block-uniform) when the serial emulation must run instead.
// (not inlined: it runs for queued documents only; every argument by value, so the caller's
// parameter block and scratch table stay in registers instead of a stack copy)
__device__ PH_ATTR bool parallel_history(const hm_change_row *CH, const hm_dep_row *deps, Shared &sh,
                                         GLB uint32_t *C, GLB uint32_t *hx, GLB uint32_t *tab, GLB uint32_t *h2a,
                                         GLB int32_t *hist, uint32_t n, uint32_t A, uint32_t T) {
    const uint32_t tid = threadIdx.x;
    const uint32_t INF = 0xFFFFFFFFu;
    // C: [n * A] closure clocks (self excluded); this phase's arrays from one base (hx)
    struct { GLB uint32_t *ht, *hp, *hnev, *hfill, *hmem, *hoff, *pm, *tab, *h2a; GLB int32_t *hist; } Y;
    Y.ht = hx; Y.hp = Y.ht + n; Y.hnev = Y.hp + n; Y.hfill = Y.hnev + n; Y.hmem = Y.hfill + n; Y.hoff = Y.hmem + n;
    Y.pm = Y.hoff + n + 1; Y.tab = tab; Y.h2a = h2a; Y.hist = hist;
    auto arrival = [&](uint32_t a, uint32_t s) -> uint32_t {  // first arrival of (a, s), or INF
        if (a >= A || s < sh.base[a] || s > sh.maxs[a] || sh.maxs[a] == 0) return INF;
        return Y.tab[sh.tabo[a] + (s - sh.base[a])];
    };
    if (tid == 0) sh.nodup = 1;
    bsync();
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = CH[i];
        if (arrival(c.actor, c.seq) != i) sh.nodup = 0;        // a duplicate (actor, seq)
        GLB uint32_t *row = C + (size_t)i * A;
        for (uint32_t a = 0; a < A; a++) row[a] = 0;
        uint32_t nev = c.seq > 1 && arrival(c.actor, c.seq - 1) == INF;
        row[c.actor] = c.seq - 1;
        for (uint32_t j = 0; j < c.n_deps; j++) {
            const hm_dep_row dp = deps[c.dep_off + j];
            if (dp.actor == c.actor || dp.seq == 0) continue;
            if (arrival(dp.actor, dp.seq) == INF) nev = 1;
            if (row[dp.actor] < dp.seq) row[dp.actor] = dp.seq;
        }
        Y.hnev[i] = nev;
    }
    bsync();
    if (!sh.nodup) return false;
    // closure by pointer jumping, in place (entries are valid lower bounds throughout)
    for (uint32_t round = 0;; round++) {
        if (round > 64) return false;
        if (tid == 0) sh.grew = 0;
        bsync();
        bool grew = false;
        for (uint32_t i = tid; i < n; i += LWG) {
            GLB uint32_t *row = C + (size_t)i * A;
            uint32_t nev = Y.hnev[i];
            for (uint32_t a = 0; a < A; a++) {
                const uint32_t s = row[a];
                if (!s) continue;
                const uint32_t j = arrival(a, s);
                if (j >= n) { if (!nev) { nev = 1; grew = true; } continue; }
                if (j == i) continue;
                const GLB uint32_t *r2 = C + (size_t)j * A;
                for (uint32_t b = 0; b < A; b++) { const uint32_t x = r2[b]; if (x > row[b]) { row[b] = x; grew = true; } }
                if (Y.hnev[j] && !nev) { nev = 1; grew = true; }
            }
            Y.hnev[i] = nev;
        }
        if (grew) sh.grew = 1;
        bsync();
        const bool any = sh.grew != 0;
        bsync();
        if (!any) break;
    }
    // PM_a: prefix max of the first-arrival index along each actor's seqs; INF for a missing
    // change and for one that can never apply (a missing ancestor, or on a dependency cycle),
    // so every descendant of those gets t = INF too
    for (uint32_t i = tid; i < T; i += LWG) Y.pm[i] = Y.tab[i];
    bsync();
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = CH[i];
        if (Y.hnev[i] || C[(size_t)i * A + c.actor] >= c.seq) Y.pm[sh.tabo[c.actor] + (c.seq - sh.base[c.actor])] = INF;
    }
    bsync();
    for (uint32_t a = 0; a < A; a++) {
        const uint32_t lo = sh.tabo[a], hi = sh.tabo[a + 1];
        if (hi == lo) continue;
        const uint32_t N = hi - lo, per = (N + LWG - 1) / LWG;
        const uint32_t b0 = lo + (tid * per < N ? tid * per : N), b1 = b0 + per < hi ? b0 + per : hi;
        uint32_t run = sh.base[a] > 1 ? INF : 0u;              // seqs below the batch's first: missing
        for (uint32_t i = b0; i < b1; i++) run = run > Y.pm[i] ? run : Y.pm[i];
        uint32_t cur = block_excl_max(sh, run);
        if (sh.base[a] > 1) cur = INF;
        for (uint32_t i = b0; i < b1; i++) { cur = cur > Y.pm[i] ? cur : Y.pm[i]; Y.pm[i] = cur; }
        bsync();
    }
    // t(K); pass 1 for K applied by its own arrival, else at least 2
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = CH[i];
        const GLB uint32_t *row = C + (size_t)i * A;
        uint32_t t = (Y.hnev[i] || row[c.actor] >= c.seq) ? INF : i;    // missing ancestor / cycle
        for (uint32_t a = 0; a < A && t != INF; a++) {
            const uint32_t s = row[a];
            if (!s) continue;
            const uint32_t v = (s < sh.base[a] || s > sh.maxs[a]) ? INF : Y.pm[sh.tabo[a] + (s - sh.base[a])];
            t = t > v ? t : v;
        }
        Y.ht[i] = t;
        Y.hp[i] = t == INF ? 0u : (t == i ? 1u : 2u);
    }
    bsync();
    for (uint32_t round = 0;; round++) {
        if (round > 256) return false;
        if (tid == 0) sh.grew = 0;
        bsync();
        bool grew = false;
        for (uint32_t i = tid; i < n; i += LWG) {
            const uint32_t t = Y.ht[i];
            if (t == INF || t == i) continue;
            const hm_change_row c = CH[i];
            uint32_t ps = Y.hp[i];
            auto dep = [&](uint32_t j) {
                if (j < n && Y.ht[j] == t) { const uint32_t v = Y.hp[j] + (j > i ? 1u : 0u); ps = ps > v ? ps : v; }
            };
            for (uint32_t j = 0; j < c.n_deps; j++) {
                const hm_dep_row dp = deps[c.dep_off + j];
                if (dp.actor == c.actor || dp.seq == 0) continue;
                dep(arrival(dp.actor, dp.seq));
            }
            if (c.seq > 1) dep(arrival(c.actor, c.seq - 1));
            if (ps > Y.hp[i]) { Y.hp[i] = ps; grew = true; }
        }
        if (grew) sh.grew = 1;
        bsync();
        const bool any = sh.grew != 0;
        bsync();
        if (!any) break;
    }
    // history: bucket by t (counting sort), then (pass, arrival) within a bucket
    for (uint32_t i = tid; i <= n; i += LWG) { Y.hoff[i] = 0; if (i < n) Y.hfill[i] = 0; }
    bsync();
    for (uint32_t i = tid; i < n; i += LWG) if (Y.ht[i] != INF) g_add(&Y.hoff[Y.ht[i]], 1u);
    bsync();
    uint32_t Hn;
    Hn = scan_array(sh, Y.hoff, n + 1);
    for (uint32_t i = tid; i < n; i += LWG) {
        const uint32_t t = Y.ht[i];
        if (t == INF) continue;
        const uint32_t at = g_add(&Y.hfill[t], 1u);
        Y.hmem[Y.hoff[t] + at] = i;
    }
    if (tid == 0) sh.grew = 0;
    bsync();
    for (uint32_t i = tid; i < n; i += LWG) {
        const uint32_t t = Y.ht[i];
        if (t == INF) { Y.hist[i] = -1; continue; }
        const uint32_t lo = Y.hoff[t], sz = Y.hoff[t + 1] - lo, ps = Y.hp[i];
        if (sz > 2048) { sh.grew = 1; continue; }             // a huge batch of queued changes: serial path
        uint32_t rank = 0;
        for (uint32_t k = 0; k < sz; k++) {
            const uint32_t o = Y.hmem[lo + k], po = Y.hp[o];
            rank += (po < ps || (po == ps && o < i)) ? 1u : 0u;
        }
        Y.hist[i] = (int32_t)(lo + rank);
        Y.h2a[lo + rank] = i;
    }
    bsync();
    if (sh.grew) return false;
    if (tid == 0) sh.H = Hn;
    bsync();
    return true;
}

// ---- L3 + L4 with every table resident in the LDS arena (l34_res) ----
// The same rules, in the same order of checks, as the pool L3/L4 in merge_doc_large; only the
// storage differs: 16-bit op / node indices, u8 object ids, assign lists of op indices (keys
// recomputed from the staged per-change key bases), survivors flagged in a bit set and ranked
// within their register's assign list.  Envelope (checked before anything is written; outside
// it the caller runs the pool L3/L4 from its start): A <= 8 (allDeps rows staged), O <= LA_MAX,
// m < 2^16, R + O < 2^15 (16-bit tour links), no counter ops, assign lists <= RES_SEG_MAX per
// register, and the layout below fits the arena.
#define RES_SEG_MAX 64
#define RES_FALLBACK 3
__device__ __forceinline__ int l34_res(const SmallParams &p, Shared &sh, LDS uint32_t *ar, const hm_doc_row &doc,
                                       const LDS hm_change_row *sCH, const LDS int32_t *lh, const LDS uint32_t *lh2a,
                                       uint32_t H, uint32_t ad_off, uint32_t limit, uint32_t AS) {
    const uint32_t tid = fresh_tid();           // (per document: see fresh_tid)
    const uint32_t n = doc.n_changes, A = doc.n_actors, m = doc.n_ops, R = doc.n_regs, O = doc.n_objs;
    const hm_op_row *OP = p.ops + doc.op_off;
    const uint32_t NP = R + O;
    const uint16_t N16 = 0xFFFFu;
    // ---- layout (words); region S and the survivor list die after the ranks (L4 reuses them) ----
    uint32_t off = ad_off;                      // [0, ad_off): L2's first-arrival table (dead)
    auto w32 = [&](uint32_t cnt) -> LDS uint32_t * { LDS uint32_t *q = ar + off; off += cnt; return q; };
    auto w16 = [&](uint32_t cnt) -> LDS uint16_t * { LDS uint16_t *q = (LDS uint16_t *)(ar + off); off += (cnt + 1) / 2; return q; };
    auto w8 = [&](uint32_t cnt) -> LDS uint8_t * { LDS uint8_t *q = (LDS uint8_t *)(ar + off); off += (cnt + 3) / 4; return q; };
    LDS uint32_t *c_ad = w32(n * AS);           // L2's closure rows (= allDeps, row stride AS), already in place
    LDS uint32_t *c_tmp = w32(n), *c_hist = w32(n), *c_act = w32(n), *c_seq = w32(n), *c_op0 = w32(n), *c_kb = w32(n);
    LDS uint32_t *o_w = w32(m);                 // reg (16) | action (4) << 16 | obj (7, 127 unknown) << 20
    LDS uint16_t *o_chg = w16(m);               // op -> arrival index of its change
    LDS uint16_t *a_k = w16(m);                 // assign lists (set/del/link/inc op indices), by register
    LDS uint16_t *s_list = w16(m);              // make ops, then survivors
    LDS uint32_t *s_bits = w32(m / 32 + 1);     // survivor flags by op index
    const uint32_t dead_end = off;              // [0, dead_end) is free once the ranks are done
    LDS uint32_t *r_ins = w32(R), *r_segcnt = w32(R), *r_seg = w32(R), *r_scnt = w32(R), *r_soff = w32(R);
    LDS uint8_t *r_obj = w8(R);                 // 0xFF: HM_NONE
    LDS uint16_t *r_node = w16(R);
    LDS uint16_t *s_op = w16(m);                // survivors in output order
    LDS uint16_t *n_pi = w16(R), *n_reg = w16(R), *n_ns = w16(R), *n_pl = w16(R), *n_op = w16(R);
    LDS uint32_t *n_key = w32(R);
    LDS uint8_t *n_list = w8(R);
    LDS uint32_t *p_cnt = w32(NP), *p_off = w32(NP);
    LDS uint16_t *p_fc = w16(NP);
    const uint32_t tail = off;
    if (A > 8 || O > LA_MAX || m >= 65536 || NP >= 32767 || n >= 65536 || tail > limit) return RES_FALLBACK;
    auto dec_reg = [](uint32_t w) { return w & 0xFFFFu; };
    auto dec_act = [](uint32_t w) { return (w >> 16) & 15u; };
    auto dec_obj = [](uint32_t w) { return (w >> 20) & 127u; };
    auto key_of = [&](uint32_t k, uint32_t ci) -> uint32_t { return c_kb[ci] + (k - c_op0[ci]); };

    // ---- key bases: ops of the changes before each history position ----
    if (H <= LWG) {
        scan_fn_small(sh, [&](uint32_t h) -> uint32_t { return sCH[lh2a[h]].n_ops; }, c_tmp, H);
    } else {
        for (uint32_t h = tid; h < H; h += LWG) c_tmp[h] = sCH[lh2a[h]].n_ops;
        bsync();
        scan_array(sh, c_tmp, H);
    }
    // ---- staging: per-change inputs, op -> change, object / register / parent tables ----
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = sCH[i];
        const int32_t hi = lh[i];
        const uint32_t o0 = c.op_first - doc.op_off;
        c_hist[i] = (uint32_t)hi; c_act[i] = c.actor; c_seq[i] = c.seq; c_op0[i] = o0;
        c_kb[i] = hi >= 0 ? c_tmp[hi] : 0xFFFFFFFFu;
        for (uint32_t j = 0; j < c.n_ops; j++) o_chg[o0 + j] = (uint16_t)i;
    }
    for (uint32_t i = tid; i < O; i += LWG) { sh.oslot[i] = i == 0 ? 0u : 0xFFFFFFFFu; sh.otype[i] = i == 0 ? (uint32_t)HM_MAKE_MAP : 0xFFu; }
    for (uint32_t i = tid; i < R; i += LWG) {
        r_ins[i] = 0xFFFFFFFFu; r_segcnt[i] = 0; r_scnt[i] = 0; r_obj[i] = 0xFFu; r_node[i] = N16;
    }
    for (uint32_t i = tid; i < NP; i += LWG) { p_cnt[i] = 0; p_fc[i] = N16; }
    for (uint32_t i = tid; i <= m / 32; i += LWG) s_bits[i] = 0;
    if (tid == 0) { sh.nmake = 0; sh.nsurv = 0; sh.nins = 0; sh.grew = 0; }
    bsync();
    LSTAMP(11);
    // ---- op scan: rows read once from HBM, four per thread in flight ----
    for (uint32_t k0 = 0; k0 < m; k0 += 4 * LWG) {
        // whole 32-byte rows, loaded unconditionally (a clamped index): a predicated load of only
        // the fields used was compiled as a wait for everything before each of the four loads and
        // a wait for the load itself inside its predicated block (one row in flight, not four)
        uint4 ra[4], rb[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t k = k0 + tid + u * LWG;
            const uint4 *src = reinterpret_cast<const uint4 *>(OP + (k < m ? k : m - 1));
            ra[u] = src[0]; rb[u] = src[1];
        }
        asm volatile("" ::: "memory");          // all four issued here (not sunk into their uses)
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t k = k0 + tid + u * LWG;
            if (k >= m) continue;
            struct { uint4 a, b; } raw = {ra[u], rb[u]};
            hm_op_row o;
            __builtin_memcpy(&o, &raw, sizeof o);
            const uint32_t ci = o_chg[k];
            const int32_t h = (int32_t)c_hist[ci];
            if (o.action == HM_INC || o.datatype == HM_DT_COUNTER) sh.ctrs = 1;
            const bool bad = o.action <= HM_MAKE_TEXT ? o.obj >= O
                           : (o.action <= HM_INC ? (o.reg >= R || (o.action == HM_INS && o.parent != HM_HEAD && o.parent >= R)) : true);
            if (bad) { atomicOr(&sh.flags, LF_UNSUPPORTED); continue; }
            o_w[k] = (o.action <= HM_MAKE_TEXT ? 0u : o.reg) | ((uint32_t)o.action << 16) | ((o.obj < O ? o.obj : 127u) << 20);
            if (h < 0) continue;
            const uint32_t key = key_of(k, ci);
            if (o.action <= HM_MAKE_TEXT) {
                atomicMin(&sh.oslot[o.obj], key + 1);
                s_list[atomicAdd(&sh.nmake, 1u)] = (uint16_t)k;
            } else {
                if (o.obj >= O) continue;                          // an unknown object: the survivor pass throws
                r_obj[o.reg] = (uint8_t)o.obj;
                if (o.action == HM_INS) {
                    atomicMin(&r_ins[o.reg], key + 1);
                    if (o.elem >= (1u << 24)) atomicOr(&sh.flags, LF_UNSUPPORTED);
                    const uint32_t i = atomicAdd(&sh.nins, 1u);
                    if (i < R) {                                   // more inserts than registers: a duplicate throws
                        const uint32_t pi = o.parent == HM_HEAD ? R + o.obj : o.parent;
                        n_pi[i] = (uint16_t)pi; n_reg[i] = (uint16_t)o.reg; n_list[i] = (uint8_t)o.obj; n_op[i] = (uint16_t)k;
                        n_key[i] = (o.elem << 8) | c_act[ci];
                        r_node[o.reg] = (uint16_t)i;
                        atomicAdd(&p_cnt[pi], 1u);
                    }
                } else if (atomicAdd(&r_segcnt[o.reg], 1u) >= RES_SEG_MAX) sh.grew = 1;   // a long assign list
            }
        }
    }
    bsync();
    LSTAMP(12);
    if (sh.flags) return LUNSUP;
    {
        // counters, long assign lists, or a tour that does not fit over the dead region: pool path
        const uint32_t N = sh.nins < R ? sh.nins : R;
        const bool out = sh.ctrs || sh.grew || 2 * (N + O) + N > dead_end;
        if (out) {                                  // (uniform) every thread has read the flags
            bsync();
            if (tid == 0) { sh.nins = 0; sh.ctrs = 0; }
            bsync();
            return RES_FALLBACK;
        }
    }
    // ---- objects: the earliest make op creates, later ones throw ----
    for (uint32_t q = tid; q < sh.nmake; q += LWG) {
        const uint32_t k = s_list[q], w = o_w[k], ci = o_chg[k], obj = dec_obj(w);
        if (sh.oslot[obj] != key_of(k, ci) + 1)
            atomicMin(&sh.errkey, err_key(c_hist[ci], k - c_op0[ci] + 1, ci, HM_ERR_DUPLICATE_OBJECT));
        else sh.otype[obj] = dec_act(w);
    }
    // ---- assign lists: r_seg = exclusive offsets, advanced to the segment ends by the fill ----
    (void)scan_into(sh, r_segcnt, r_seg, R);
    for (uint32_t k = tid; k < m; k += LWG) {
        const uint32_t w = o_w[k], a = dec_act(w);
        if (a < HM_SET || a > HM_INC || dec_obj(w) >= O) continue;     // exactly the ops r_segcnt counted
        if ((int32_t)c_hist[o_chg[k]] < 0) continue;
        a_k[atomicAdd(&r_seg[dec_reg(w)], 1u)] = (uint16_t)k;
    }
    bsync();
    LSTAMP(13);
    // ---- survivors and per-op checks (insert parents loaded from HBM up front, four per thread) ----
    bool any_list = false;
    for (uint32_t k0 = 0; k0 < m; k0 += 4 * LWG) {
    // an insert's parent from its node (the op scan recorded it); only an insert whose register's
    // node is another insert's (a duplicate: it throws) reads its row again
    uint32_t par[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t k = k0 + tid + u * LWG;
        par[u] = HM_HEAD;
        if (k < m && dec_act(o_w[k]) == HM_INS) {
            const uint32_t nd_ = r_node[dec_reg(o_w[k])];
            if (nd_ != N16 && n_op[nd_] == k) { const uint32_t pi = n_pi[nd_]; par[u] = pi >= R ? HM_HEAD : pi; }
            else par[u] = OP[k].parent;
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint32_t k = k0 + tid + u * LWG;
        if (k >= m) continue;
        const uint32_t w = o_w[k], a = dec_act(w), obj = dec_obj(w), reg = dec_reg(w);
        if (a < HM_INS || a > HM_INC) continue;
        const uint32_t ci = o_chg[k];
        const int32_t h = (int32_t)c_hist[ci];
        if (h < 0) continue;
        const uint32_t kx = k - c_op0[ci], key = c_kb[ci] + kx;
        const uint32_t os = obj < O ? sh.oslot[obj] : 0xFFFFFFFFu;
        if (os == 0xFFFFFFFFu || os > key) {
            atomicMin(&sh.errkey, err_key((uint32_t)h, kx + 1, ci, HM_ERR_UNKNOWN_OBJECT));
            continue;
        }
        const uint32_t ot = sh.otype[obj];
        const bool is_list = ot == HM_MAKE_LIST || ot == HM_MAKE_TEXT;
        if (a == HM_INS) {
            any_list = true;
            const uint32_t parent = par[u];
            if (r_ins[reg] != key + 1) atomicMin(&sh.errkey, err_key((uint32_t)h, kx + 1, ci, HM_ERR_DUPLICATE_ELEM));
            if (parent != HM_HEAD && !(r_ins[parent] <= key)) sh.late = 1;   // the general path climbs chains
            continue;
        }
        any_list |= is_list;
        if (a == HM_SET || a == HM_LINK) {
            if (is_list && !(r_ins[reg] <= key)) atomicMin(&sh.errkey, err_key((uint32_t)h, kx + 1, ci, HM_ERR_MISSING_ELEM));
            // survivor: no set/del/link on the register has this op's change among its allDeps
            const uint32_t ao = c_act[ci], so = c_seq[ci], cnt = r_segcnt[reg], e0 = r_seg[reg] - cnt;
            bool surv = true;
            for (uint32_t q = 0; q < cnt; q++) {
                const uint32_t e = a_k[e0 + q];
                if (dec_act(o_w[e]) != HM_INC && c_ad[o_chg[e] * AS + ao] >= so) surv = false;
            }
            if (surv) {
                atomicAdd(&r_scnt[reg], 1u);
                atomicOr(&s_bits[k >> 5], 1u << (k & 31));
                s_list[atomicAdd(&sh.nsurv, 1u)] = (uint16_t)k;
            }
        }
    }
    }
    if (any_list) sh.lists = 1;
    bsync();
    if (sh.late) {                                  // (uniform) every thread has read the flag
        bsync();
        if (tid == 0) { sh.nins = 0; sh.ctrs = 0; }
        bsync();
        return RES_FALLBACK;
    }
    const bool lists_flag = sh.lists != 0;
    const uint32_t nsurv = sh.nsurv;
    if (sh.errkey != ~0ull) return LERR;
    if (sh.flags) return LUNSUP;
    LSTAMP(4);
    // ---- survivor offsets and ranks: actor descending; equal actors (one change) by the
    //      sortBy(actor).reverse() flip, from the assigns applied on the register before each ----
    const uint32_t total = scan_into(sh, r_scnt, r_soff, R);
    for (uint32_t j = tid; j < nsurv; j += LWG) {
        const uint32_t k = s_list[j], reg = dec_reg(o_w[k]), ck = o_chg[k], my_a = c_act[ck];
        const uint32_t cnt = r_scnt[reg];
        uint32_t rank = 0;
        if (cnt > 1) {
            const uint32_t nseg = r_segcnt[reg], sb = r_seg[reg] - nseg;
            const bool odd_n = nseg & 1;
            auto tkey = [&](uint32_t kk) -> uint32_t {
                uint32_t pc = 0;
                const uint32_t key = key_of(kk, o_chg[kk]);
                for (uint32_t q = 0; q < nseg; q++) { const uint32_t e = a_k[sb + q]; pc += key_of(e, o_chg[e]) < key ? 1u : 0u; }
                return (pc & 1) ? (0x80000000u - pc) : (0x80000000u + pc);
            };
            uint32_t my_t = 0;
            bool have_t = false;
            for (uint32_t q = 0; q < nseg; q++) {
                const uint32_t k2 = a_k[sb + q];
                if (k2 == k || !((s_bits[k2 >> 5] >> (k2 & 31)) & 1)) continue;
                const uint32_t a2 = c_act[o_chg[k2]];
                if (a2 > my_a) rank++;
                else if (a2 == my_a) {
                    if (!have_t) { my_t = tkey(k); have_t = true; }
                    const uint32_t t2 = tkey(k2);
                    if (odd_n ? (t2 > my_t) : (t2 < my_t)) rank++;
                }
            }
        }
        s_op[r_soff[reg] + rank] = (uint16_t)k;
    }
    bsync();
    LSTAMP(5);
    // ---- L4: RGA order (Euler tour over the insertion tree, pointer jumping) ----
    if (lists_flag) {
        if (tid < 64) {                                            // compact list ids over <= 64 objects
            const uint32_t t = tid < O ? sh.otype[tid] : 0xFFu;
            const bool isl = t == HM_MAKE_LIST || t == HM_MAKE_TEXT;
            const u64 bm = __ballot(isl);
            sh.listid[tid] = (uint32_t)__popcll(bm & ((1ull << tid) - 1));
            if (tid == 0) sh.total = (uint32_t)__popcll(bm);
        }
        const uint32_t N = sh.nins;
        bsync();
        const uint32_t nl = sh.total;
        (void)scan_into(sh, p_cnt, p_off, NP);
        for (uint32_t i = tid; i < N; i += LWG) {
            const uint32_t pi = n_pi[i];
            if (p_cnt[pi] > 1) n_pl[atomicAdd(&p_off[pi], 1u)] = (uint16_t)i;
            n_list[i] = (uint8_t)sh.listid[n_list[i]];
        }
        bsync();
        // siblings: lamport (elem, actor) descending; an only child needs no list
        for (uint32_t i = tid; i < N; i += LWG) {
            const uint32_t pi = n_pi[i], np = p_cnt[pi];
            if (np == 1) { n_ns[i] = N16; p_fc[pi] = (uint16_t)i; continue; }
            const uint32_t key = n_key[i], b0 = p_off[pi] - np;
            uint32_t best = 0xFFFFFFFFu, bkey = 0;
            bool firstc = true;
            for (uint32_t q = 0; q < np; q++) {
                const uint32_t j = n_pl[b0 + q], kj = n_key[j];
                if (kj > key) firstc = false;
                else if (kj < key && (best == 0xFFFFFFFFu || kj > bkey)) { best = j; bkey = kj; }
            }
            n_ns[i] = best == 0xFFFFFFFFu ? N16 : (uint16_t)best;
            if (firstc) p_fc[pi] = (uint16_t)i;
        }
        bsync();
        LSTAMP(7);
        // tour words (next << 16 | value, END 0xFFFF) over the dead region, then the visibility array
        const uint32_t E = 2 * (N + nl);
        LDS uint32_t *tw = ar, *vis = ar + E;
        for (uint32_t i = tid; i < N; i += LWG) {
            const uint32_t hd = N + n_list[i], f = p_fc[n_reg[i]], pi = n_pi[i], ns = n_ns[i];
            tw[2 * i] = ((f != N16 ? 2 * f : 2 * i + 1) << 16) | 1u;
            tw[2 * i + 1] = (ns != N16 ? 2 * ns : (pi >= R ? 2 * hd + 1 : 2 * (uint32_t)r_node[pi] + 1)) << 16;
        }
        for (uint32_t o = tid; o < O; o += LWG) {
            const uint32_t t = sh.otype[o];
            if (!(t == HM_MAKE_LIST || t == HM_MAKE_TEXT)) continue;
            const uint32_t h = N + sh.listid[o], f = p_fc[R + o];
            tw[2 * h] = (f != N16 ? 2 * f : 2 * h + 1) << 16;
            tw[2 * h + 1] = 0xFFFF0000u;
        }
        bsync();
        // in-place pointer jumping, three hops per round: every word keeps "value = sum from this
        // entry up to its link" at every moment, and if every link spans >= L entries when a round
        // starts it spans >= 4L after it (links only move forward) -> ceil(log4 E) rounds
        const uint32_t rounds = E ? (33 - __builtin_clz(E)) / 2 : 0;
        for (uint32_t rd = 0; rd < rounds; rd++) {
            for (uint32_t e = tid; e < E; e += LWG) {
                const uint32_t w = tw[e];
                uint32_t x = w >> 16, sum = w & 0xFFFFu;
                if (x == 0xFFFFu) continue;
#pragma unroll
                for (int hop = 0; hop < 3; hop++) {
                    if (x == 0xFFFFu) break;
                    const uint32_t w2 = tw[x];
                    sum += w2 & 0xFFFFu;
                    x = w2 >> 16;
                }
                tw[e] = (x << 16) | sum;
            }
            bsync();
        }
        LSTAMP(8);
        auto tsum = [&](uint32_t e) -> uint32_t { return tw[e] & 0xFFFFu; };
        if (tid < 64) {                                            // list bases: exclusive scan over list ids
            const uint32_t t = tid < O ? sh.otype[tid] : 0xFFu;
            const bool isl = t == HM_MAKE_LIST || t == HM_MAKE_TEXT;
            const uint32_t len = isl ? tsum(2 * (N + sh.listid[tid])) : 0u;
            const uint32_t x = wave_incl_sum(len);   // inclusive scan over lanes in object order = list-id order
            if (isl) sh.listbase[sh.listid[tid]] = x - len;
        }
        bsync();
        auto pos_of = [&](uint32_t i, uint32_t l) -> uint32_t { return sh.listbase[l] + tsum(2 * (N + l)) - tsum(2 * i); };
        for (uint32_t i = tid; i < N; i += LWG) vis[pos_of(i, n_list[i])] = r_scnt[n_reg[i]] > 0 ? 1u : 0u;
        bsync();
        (void)scan_array(sh, vis, N);
        for (uint32_t i = tid; i < N; i += LWG) {
            const uint32_t l = n_list[i], rg = n_reg[i];
            r_ins[rg] = r_scnt[rg] > 0 ? vis[pos_of(i, l)] - vis[sh.listbase[l]] : 0xFFFFFFFFu;
            if (p.res_epos) p.res_epos[doc.reg_off + rg] = pos_of(i, l) - sh.listbase[l];
        }
        bsync();
    }
    LSTAMP(9);
    // ---- outputs ----
    for (uint32_t q = tid; q < total; q += LWG) {
        const uint32_t k = s_op[q];
#ifdef HML_DEBUG
        if (k >= m) { printf("RES bad s_op doc %u q %u total %u k %u m %u nsurv %u n %u H %u\n", doc.reserved[0], q, total, k, m, nsurv, n, H); continue; }
#endif
        const hm_op_row o = OP[k];
        hm_surv_result sr; sr.op = k; sr.vtag = o.vtag; sr.value = o.value;
        p.res_surv[doc.op_off + q] = sr;
    }
    for (uint32_t r = tid; r < R; r += LWG) {
        hm_reg_result rr;
        rr.n_surv = r_scnt[r]; rr.surv_off = r_soff[r];
        rr.obj = r_obj[r] == 0xFFu ? HM_NONE : (uint32_t)r_obj[r];
        rr.list_index = (lists_flag && r_node[r] != N16 && r_ins[r] != 0xFFFFFFFFu) ? (int32_t)r_ins[r] : -1;
        p.res_regs[doc.reg_off + r] = rr;
    }
    for (uint32_t i = tid; i < n; i += LWG) p.res_hist[doc.change_off + i] = lh[i];
    if (tid == 0) sh.total = total;
    bsync();
    LSTAMP(10);
    if (sh.flags) return LUNSUP;
    return LOK;
}

// ---- the whole document in LDS (merge_doc_res): setup, L1 fast path, L2 closure, l34_res ----
// For documents whose rows, tables and L3/L4 working set fit the arena and that need none of the
// general path's slow machinery: every change ready on arrival, the closure equal to the literal
// fold, A <= 8.  No pool scratch at all, so nothing here competes for registers with the general
// path (merge_doc_large, not inlined), which takes every document this returns RES_FALLBACK for
// and recomputes it from the start.  Results equal the general path's (same rules, same order).
__device__ __forceinline__ int merge_doc_res(const SmallParams &p, Shared &sh, LDS uint32_t *ar, const hm_doc_row &doc,
                                             int32_t &H_out) {
    const uint32_t tid = fresh_tid();           // (per document: see fresh_tid)
    const uint32_t n = doc.n_changes, A = doc.n_actors, m = doc.n_ops, nd = doc.n_deps;
    const uint32_t S = p.a_stride;
    const hm_change_row *CH = p.changes + doc.change_off;
    if (tid < LA_ACT) { sh.base[tid] = 0xFFFFFFFFu; sh.maxs[tid] = 0; sh.clock[tid] = 0; sh.bclock[tid] = 0;
                        sh.headv[tid] = 0; sh.maxad[tid] = 0; }
    if (tid == 0) { sh.flags = 0; sh.errkey = ~0ull; sh.all_ok = 1; sh.H = 0; sh.nins = 0; sh.total = 0; sh.lists = 0; sh.ctrs = 0; sh.late = 0; }
    // rows at the top of the arena: changes (6n words), deps (2nd), hist (n), h2a (n)
    const uint32_t stage_base = (LARENA - (8 * n + 2 * nd)) & ~1u;
    LDS hm_change_row *sCH = (LDS hm_change_row *)(ar + stage_base);
    LDS hm_dep_row *sDP = (LDS hm_dep_row *)(ar + stage_base + 6 * n);
    LDS int32_t *lh = (LDS int32_t *)(ar + stage_base + 6 * n + 2 * nd);
    LDS uint32_t *lh2a = ar + stage_base + 7 * n + 2 * nd;
    // staging: a thread's dep row and change row loads are issued together (one round trip per
    // 1024 rows, where the deps, then the change rows, then their predecessors were three)
    {
        const uint32_t top = n > nd ? n : nd;
        for (uint32_t j0 = 0; j0 < top; j0 += LWG) {
            const uint32_t j = j0 + tid;
            const bool hd = j < nd, hc = j < n;
            const uint2 dv = hd ? *reinterpret_cast<const uint2 *>(p.deps + doc.dep_off + j) : make_uint2(0, 0);
            const uint2 *cs = reinterpret_cast<const uint2 *>(CH + (hc ? j : 0u));
            const uint2 c0 = hc ? cs[0] : make_uint2(0, 0), c1 = hc ? cs[1] : make_uint2(0, 0), c2 = hc ? cs[2] : make_uint2(0, 0);
            asm volatile("" ::: "memory");
            if (hd) *reinterpret_cast<LDS uint2 *>(sDP + j) = dv;
            if (hc) {
                LDS uint2 *d = reinterpret_cast<LDS uint2 *>(sCH + j);
                d[0] = c0; d[1] = c1; d[2] = c2;
            }
        }
    }
    bsync();
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = sCH[i];
        const uint32_t op0 = i ? sCH[i - 1].op_first + sCH[i - 1].n_ops : doc.op_off;
        const uint32_t dp0 = i ? sCH[i - 1].dep_off + sCH[i - 1].n_deps : doc.dep_off;
        const bool last_bad = i == n - 1 && (c.op_first + c.n_ops != doc.op_off + m || c.dep_off + c.n_deps != doc.dep_off + nd);
        if (c.actor >= A || c.seq == 0 || c.op_first < doc.op_off || c.op_first - doc.op_off + c.n_ops > m ||
            c.dep_off < doc.dep_off || c.dep_off - doc.dep_off + c.n_deps > nd ||
            c.op_first != op0 || c.dep_off != dp0 || last_bad)
            atomicOr(&sh.flags, LF_UNSUPPORTED);
        else { atomicMin(&sh.base[c.actor], c.seq); atomicMax(&sh.maxs[c.actor], c.seq); atomicMax(&sh.bclock[c.actor], c.seq); }
    }
    bsync();
    if (sh.flags) return RES_FALLBACK;
    // table offsets per actor, computed by every thread (A <= 8) and published by thread 0
    uint32_t T = 0;
    for (uint32_t a = 0; a < A; a++) { if (tid == 0) sh.tabo[a] = T; if (sh.maxs[a]) T += sh.maxs[a] - sh.base[a] + 1; }
    if (tid == 0) sh.tabo[A] = T;
    // closure rows at an odd stride: the groups of a wave read rows of different changes, and
    // at stride 8 those rows met in the same banks four apart
    const uint32_t AS = A | 1u;
    if (T > 4 * n + 64 || n * AS + T > stage_base) return RES_FALLBACK;
    LDS uint32_t *lt = ar, *lc = ar + T;            // L1 table, L2 closure rows (stride A)
    for (uint32_t i = tid; i < T; i += LWG) lt[i] = 0xFFFFFFFFu;
    bsync();                                        // (also publishes sh.tabo)
    auto slot_of = [&](uint32_t a, uint32_t s) -> uint32_t {
        if (a >= A || s < sh.base[a] || s > sh.maxs[a] || sh.maxs[a] == 0) return 0xFFFFFFFFu;
        return sh.tabo[a] + (s - sh.base[a]);
    };
    for (uint32_t i = tid; i < n; i += LWG) { const hm_change_row c = sCH[i]; atomicMin(&lt[slot_of(c.actor, c.seq)], i); }
    bsync();
    LSTAMP(0);
    // ---- L1: every dependency arrived earlier (else the general path's queue emulation) ----
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = sCH[i];
        bool ok = true;
        for (uint32_t j = 0; j < c.n_deps; j++) {
            const hm_dep_row dp = sDP[c.dep_off - doc.dep_off + j];
            if (dp.actor >= A) { ok = false; continue; }
            if (dp.actor == c.actor || dp.seq == 0) continue;
            const uint32_t sl = slot_of(dp.actor, dp.seq);
            if (sl == 0xFFFFFFFFu || lt[sl] >= i) ok = false;
        }
        if (c.seq > 1) { const uint32_t sl = slot_of(c.actor, c.seq - 1); if (sl == 0xFFFFFFFFu || lt[sl] >= i) ok = false; }
        const uint32_t f = lt[slot_of(c.actor, c.seq)];
        if (f != i && sCH[f].content_id != c.content_id) ok = false;
        if (!ok) sh.all_ok = 0;
    }
    bsync();
    const bool all_ready = sh.all_ok != 0;          // (next written after the history scan's barriers)
    if (!all_ready) return RES_FALLBACK;
    if (n <= LWG) {
        H_out = 0;
        const uint32_t Hc = scan_fn_small(sh, [&](uint32_t i) -> uint32_t {
            const hm_change_row c = sCH[i];
            return lt[slot_of(c.actor, c.seq)] == i ? 1u : 0u;
        }, lh, n);
        // lh holds exclusive counts: a change is applied iff it is its key's first arrival
        for (uint32_t i = tid; i < n; i += LWG) {
            const hm_change_row c = sCH[i];
            if (lt[slot_of(c.actor, c.seq)] == i) lh2a[lh[i]] = i; else lh[i] = -2;
        }
        if (tid == 0) sh.H = Hc;
    } else {
        uint32_t carry = 0;
        for (uint32_t c0 = 0; c0 < n; c0 += LWG) {
            const uint32_t i = c0 + tid;
            bool app = false;
            if (i < n) { const hm_change_row c = sCH[i]; app = lt[slot_of(c.actor, c.seq)] == i; }
            uint32_t tot;
            const uint32_t ex = block_excl_scan(sh, app ? 1u : 0u, &tot);
            if (i < n) { lh[i] = app ? (int32_t)(carry + ex) : -2; if (app) lh2a[carry + ex] = i; }
            carry += tot;
        }
        if (tid == 0) sh.H = carry;
    }
    bsync();
    const uint32_t H = sh.H;
    LSTAMP(1);
    // ---- L2: closure rows by pointer jumping per (row, actor), then the literal-fold check ----
    for (uint32_t i = tid; i < n; i += LWG) {
        LDS uint32_t *row = lc + i * AS;
        for (uint32_t a = 0; a < A; a++) row[a] = 0;
        if (lh[i] < 0) continue;
        const hm_change_row c = sCH[i];
        for (uint32_t j = 0; j < c.n_deps; j++) {
            const hm_dep_row dp = sDP[c.dep_off - doc.dep_off + j];
            const uint32_t sq = dp.actor == c.actor ? c.seq - 1 : dp.seq;
            if (row[dp.actor] < sq) row[dp.actor] = sq;
        }
        if (row[c.actor] < c.seq - 1) row[c.actor] = c.seq - 1;
    }
    if (tid < 3) sh.gflag[tid] = 0;
    if (tid == 0) sh.all_ok = 1;                    // the literal-fold check's flag (L1 read it two barriers ago)
    bsync();
    auto lslot = [&](uint32_t a, uint32_t sq) -> uint32_t {      // applied change (a, sq) or >= n
        if (sq < sh.base[a] || sq > sh.maxs[a] || sh.maxs[a] == 0) return 0xFFFFFFFFu;
        return lt[sh.tabo[a] + (sq - sh.base[a])];
    };
    // One lane per (row i, actor a) = lane group of 8 per row: lane a reads row[a], finds the
    // applied change (a, row[a]) and loads that change's row; the 8 rows of a group are reduced
    // by DPP (quad xor 1, xor 2, half-row mirror) and lane a keeps entry a — no atomics, one LDS
    // write per grown entry.  Groups read rows other groups are growing: every entry stays a seq
    // the closure contains, and a round in which no entry grows is the fixpoint.
    const uint32_t my_a = tid & 7;
    const bool a_ok = my_a < A;
    const uint32_t a_base = a_ok ? sh.base[my_a] : 1u, a_max = a_ok ? sh.maxs[my_a] : 0u, a_off = a_ok ? sh.tabo[my_a] : 0u;
    auto gmax8 = [](uint32_t x) -> uint32_t {
        uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false); x = x > y ? x : y;   // quad xor 1
        y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false); x = x > y ? x : y;            // quad xor 2
        y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false); return x > y ? x : y;        // half-row mirror
    };
    for (uint32_t round = 0;; round++) {
        bool grew = false;
        for (uint32_t w0 = 0; w0 < n * 8; w0 += LWG) {     // whole lane groups: DPP needs them active
            const uint32_t w = w0 + tid, i = w >> 3;
            const bool live = w < n * 8 && a_ok && lh[i < n ? i : 0] >= 0;
            LDS uint32_t *row = lc + (live ? i : 0u) * AS;
            const uint32_t sq = live ? row[my_a] : 0u;
            const uint32_t ti = (sq && sq >= a_base && sq <= a_max) ? lt[a_off + (sq - a_base)] : 0xFFFFFFFFu;
            const bool src = ti < n;
            const LDS uint32_t *r2 = lc + (src ? ti : 0u) * AS;
            uint32_t v[8];
#pragma unroll
            for (uint32_t b = 0; b < 8; b++) v[b] = (src && b < A) ? r2[b] : 0u;
#pragma unroll
            for (uint32_t b = 0; b < 8; b++) v[b] = gmax8(v[b]);
            uint32_t mine = v[0];
#pragma unroll
            for (uint32_t b = 1; b < 8; b++) mine = my_a == b ? v[b] : mine;
            if (live && mine > sq) { row[my_a] = mine; grew = true; }
        }
        if (tid == 0) sh.gflag[(round + 1) % 3] = 0;
        if (grew) sh.gflag[round % 3] = 1;
        bsync();
        if (!sh.gflag[round % 3]) {
#if HM_STAMPS
            if (tid == 0) hml_st[14] += round + 1;        // closure rounds (diagnostic builds)
#endif
            break;
        }
    }
    LSTAMP(2);
    uint32_t *cur = p.res_all_deps + (size_t)doc.change_off * S;
    for (uint32_t i = tid; i < n; i += LWG) {
        uint32_t *grow_ = cur + (size_t)i * S;
        const LDS uint32_t *row = lc + i * AS;
        for (uint32_t a = 0; a < S; a++) grow_[a] = a < A ? row[a] : 0u;
        if (lh[i] < 0) continue;
        const hm_change_row c = sCH[i];
        bool same = true;
        uint32_t acc[8];
#pragma unroll
        for (uint32_t b = 0; b < 8; b++) acc[b] = 0;
        auto fold = [&](uint32_t a, uint32_t sq) {
            if (sq == 0) return;
            const uint32_t ti = lslot(a, sq);
            if (ti >= n) { same = false; return; }
            const LDS uint32_t *r2 = lc + ti * AS;
#pragma unroll
            for (uint32_t b = 0; b < 8; b++)
                if (b < A) { const uint32_t x = r2[b]; acc[b] = b == a ? sq : (acc[b] > x ? acc[b] : x); }
        };
        bool own = false;
        for (uint32_t j = 0; j < c.n_deps; j++) {
            const hm_dep_row dp = sDP[c.dep_off - doc.dep_off + j];
            if (dp.actor == c.actor) { own = true; fold(c.actor, c.seq - 1); }
            else fold(dp.actor, dp.seq);
        }
        if (!own) fold(c.actor, c.seq - 1);
#pragma unroll
        for (uint32_t b = 0; b < 8; b++) if (b < A) same = same && acc[b] == row[b];
        if (!same) sh.all_ok = 0;
    }
    bsync();
    if (!sh.all_ok) return RES_FALLBACK;       // the literal fold lowers an entry: general path
    LSTAMP(3);
    for (uint32_t h = tid; h < H; h += LWG) {
        const uint32_t ci = lh2a[h];
        const LDS uint32_t *row = lc + ci * AS;
        for (uint32_t a = 0; a < A; a++) atomicMax(&sh.maxad[a], row[a]);
        const hm_change_row c = sCH[ci];
        atomicMax(&sh.clock[c.actor], c.seq);
    }
    bsync();
    if (tid < A && sh.clock[tid] && sh.maxad[tid] < sh.clock[tid]) sh.headv[tid] = sh.clock[tid];
    H_out = (int32_t)H;
    return l34_res(p, sh, ar, doc, sCH, lh, lh2a, H, T, stage_base, AS);
}

__device__ HML_DOC_ATTR Outcome merge_doc_large(const SmallParams &p, Shared &sh, LDS uint32_t *ar, const hm_doc_row &doc, uint32_t d,
                                   uint8_t *pool, u64 pool_bytes, u64 *pool_used, int32_t &H_out) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t n = doc.n_changes, A = doc.n_actors, m = doc.n_ops, R = doc.n_regs, O = doc.n_objs;
    const uint32_t S = p.a_stride;
    const hm_change_row *CH = p.changes + doc.change_off;
    const hm_op_row *OP = p.ops + doc.op_off;
    if (A > LA_ACT || O < 1 || n >= (1u << 20) || m >= (1u << 24)) return LUNSUP;

    // ---- per-actor seq ranges -> first-arrival table size ----
    if (tid < LA_ACT) { sh.base[tid] = 0xFFFFFFFFu; sh.maxs[tid] = 0; sh.clock[tid] = 0; sh.bclock[tid] = 0;
                        sh.headv[tid] = 0; sh.maxad[tid] = 0; }
    if (tid == 0) { sh.flags = 0; sh.errkey = ~0ull; sh.all_ok = 1; sh.H = 0; sh.nins = 0; sh.total = 0; sh.lists = 0; sh.ctrs = 0; sh.late = 0; }
    bsync();
    if (n == 0 && (m || doc.n_deps)) return LUNSUP;
    // Change and dep rows staged at the top of the LDS arena (with LDS copies of hist / h2a) when
    // they take at most a quarter of it: L1 and L2 read them several times each.  The L1 table
    // joins them in LDS when it and L2's closure rows fit below (ltab); otherwise the pool.
    const uint32_t nd = doc.n_deps;
    const bool staged = HML_STAGE && 8 * (size_t)n + 2 * (size_t)nd <= LARENA / 4;
    const uint32_t stage_base = staged ? (LARENA - (8 * n + 2 * nd)) & ~1u : LARENA;
    LDS hm_change_row *sCH = (LDS hm_change_row *)(ar + stage_base);
    LDS hm_dep_row *sDP = (LDS hm_dep_row *)(ar + stage_base + 6 * n);
    LDS int32_t *lh = (LDS int32_t *)(ar + stage_base + 6 * n + 2 * nd);
    LDS uint32_t *lh2a = ar + stage_base + 7 * n + 2 * nd;
    auto chg = [&](uint32_t i) -> hm_change_row { if (staged) return sCH[i]; return CH[i]; };
    auto dep = [&](uint32_t g) -> hm_dep_row { if (staged) return sDP[g - doc.dep_off]; return p.deps[g]; };
    if (staged) for (uint32_t j = tid; j < nd; j += LWG) sDP[j] = p.deps[doc.dep_off + j];
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = CH[i];
        if (staged) sCH[i] = c;
        // layout contract: op and dep rows grouped by change in arrival order, without gaps
        const uint32_t op0 = i ? CH[i - 1].op_first + CH[i - 1].n_ops : doc.op_off;
        const uint32_t dp0 = i ? CH[i - 1].dep_off + CH[i - 1].n_deps : doc.dep_off;
        const bool last_bad = i == n - 1 && (c.op_first + c.n_ops != doc.op_off + m || c.dep_off + c.n_deps != doc.dep_off + doc.n_deps);
        if (c.actor >= A || c.seq == 0 || c.op_first < doc.op_off || c.op_first - doc.op_off + c.n_ops > m ||
            c.dep_off < doc.dep_off || c.dep_off - doc.dep_off + c.n_deps > doc.n_deps ||
            c.op_first != op0 || c.dep_off != dp0 || last_bad)
            atomicOr(&sh.flags, LF_UNSUPPORTED);
        else { atomicMin(&sh.base[c.actor], c.seq); atomicMax(&sh.maxs[c.actor], c.seq); atomicMax(&sh.bclock[c.actor], c.seq); }
    }
    bsync();
    if (sh.flags) return LUNSUP;
    if (tid == 0) {
        uint32_t t = 0;
        for (uint32_t a = 0; a < A; a++) { sh.tabo[a] = t; if (sh.maxs[a]) t += sh.maxs[a] - sh.base[a] + 1; }
        sh.tabo[A] = t;
        if (t > 4 * n + 64) sh.flags |= LF_UNSUPPORTED;    // sparse seqs: leave the envelope
        // scratch for this document
        Scratch tmp;
        const size_t need = large_carve(0, n, m, R, O, A, t, &tmp);
        // reuse the workgroup's previous scratch when it is big enough: its lines are still in
        // L2 / MALL, where fresh pool memory per document cost HBM write-backs and misses
        if (need <= sh.ws_size) sh.scratch_base = sh.ws_base;
        else {
            const u64 at = atomicAdd(pool_used, (u64)need);
            if (at + need > pool_bytes) sh.flags |= LF_NOPOOL;
            else { sh.ws_base = (u64)(uintptr_t)(pool + at); sh.ws_size = need; }
            sh.scratch_base = (u64)(uintptr_t)(pool + at);
        }
    }
    bsync();
    if (sh.flags) return LUNSUP;
    const uint32_t T = sh.tabo[A];
    Scratch X;
    large_carve((uintptr_t)sh.scratch_base, n, m, R, O, A, T, &X);
    const bool regrows = A <= 8;            // L2 rows held in registers: one LDS buffer, updated in place
    const uint32_t l2words = (regrows ? n * A : 2 * n * A) + T;
    const bool ltab = staged && l2words <= stage_base;
    LDS uint32_t *lt = ar;                  // L1 table (ltab) / L2 table
    auto tabv = [&](uint32_t sl) -> uint32_t { if (ltab) return lt[sl]; return X.tab[sl]; };
    for (uint32_t i = tid; i < T; i += LWG) { if (ltab) lt[i] = 0xFFFFFFFFu; else X.tab[i] = 0xFFFFFFFFu; }
    bsync();
    auto slot_of = [&](uint32_t a, uint32_t s) -> uint32_t {     // table index of (a, s) or NONE
        if (a >= A || s < sh.base[a] || s > sh.maxs[a] || sh.maxs[a] == 0) return 0xFFFFFFFFu;
        return sh.tabo[a] + (s - sh.base[a]);
    };
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = chg(i);
        const uint32_t sl = slot_of(c.actor, c.seq);
        if (ltab) atomicMin(&lt[sl], i); else g_min(&X.tab[sl], i);
    }
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = CH[i];
        if (!l3_ok(n, m, A)) for (uint32_t j = 0; j < c.n_ops; j++) X.opchg[c.op_first - doc.op_off + j] = i;
    }
    bsync();
    LSTAMP(0);
    // ---- L1 fast path: every dependency arrived earlier ----
    uint32_t ndup_local = 0;
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = chg(i);
        bool ok = true;
        for (uint32_t j = 0; j < c.n_deps; j++) {
            const hm_dep_row dp = dep(c.dep_off + j);
            if (dp.actor >= A) { atomicOr(&sh.flags, LF_UNSUPPORTED); continue; }
            if (dp.actor == c.actor || dp.seq == 0) continue;
            const uint32_t sl = slot_of(dp.actor, dp.seq);
            if (sl == 0xFFFFFFFFu || tabv(sl) >= i) ok = false;
        }
        if (c.seq > 1) { const uint32_t sl = slot_of(c.actor, c.seq - 1); if (sl == 0xFFFFFFFFu || tabv(sl) >= i) ok = false; }
        const uint32_t f = tabv(slot_of(c.actor, c.seq));
        if (f != i && chg(f).content_id != c.content_id) ok = false;   // mismatched duplicate: exact path
        if (!ok) sh.all_ok = 0;
    }
    bsync();
    if (sh.flags) return LUNSUP;
    // read before the barrier: parallel_history reuses sh.all_ok, and a wave still reading it
    // here must not see that write (every thread takes the same branch)
    const bool all_ready = sh.all_ok != 0;
    bsync();
    if (all_ready) {
        // history = arrival order minus duplicates (block scan of non-duplicate flags)
        uint32_t carry = 0;
        for (uint32_t c0 = 0; c0 < n; c0 += LWG) {
            const uint32_t i = c0 + tid;
            bool app = false;
            if (i < n) { const hm_change_row c = chg(i); app = tabv(slot_of(c.actor, c.seq)) == i; }
            uint32_t tot;
            const uint32_t ex = block_excl_scan(sh, app ? 1u : 0u, &tot);
            if (i < n) {
                const int32_t hv = app ? (int32_t)(carry + ex) : -2;
                X.hist[i] = hv;
                if (app) X.h2a[carry + ex] = i;
                if (staged) { lh[i] = hv; if (app) lh2a[carry + ex] = i; }
            }
            carry += tot;
        }
        if (tid == 0) sh.H = carry;
        (void)ndup_local;
    } else {
    if (ltab) {                             // the slow paths keep their tables in the pool
        for (uint32_t i = tid; i < T; i += LWG) X.tab[i] = lt[i];
        bsync();
    }
    if (HM_PAR_HIST && parallel_history(CH, p.deps, sh, X.vc, X.hx, X.tab, X.h2a, X.hist, n, A, T)) {
        // history from (t, pass, arrival) without the serial queue emulation
    } else if (wave == 0) {
        // ---- exact emulation of addChange / applyQueuedOps; wave 0, wave-uniform control ----
        // hist: -3 not arrived, -1 queued, -2 duplicate (no-op), >= 0 history position
        for (uint32_t i = lane; i < T; i += 64) X.tab[i] = 0xFFFFFFFFu;       // -> applied arrival index
        for (uint32_t i = lane; i < n; i += 64) X.hist[i] = -3;
        wfence();
        uint32_t H = 0;
        bool stop = false;
        // causallyReady: every (a, s) of deps.set(actor, seq-1) has clock[a] >= s
        auto ready = [&](uint32_t i) -> bool {
            const hm_change_row c = CH[i];
            for (uint32_t j = 0; j < c.n_deps; j++) {
                const hm_dep_row dp = p.deps[c.dep_off + j];
                if (dp.actor == c.actor) continue;
                if (sh.clock[dp.actor] < dp.seq) return false;
            }
            return sh.clock[c.actor] >= c.seq - 1;
        };
        auto apply = [&](uint32_t j) {                     // applyChange, wave-uniform j
            const hm_change_row c = CH[j];
            const uint32_t sl = slot_of(c.actor, c.seq);
            if (c.seq <= sh.clock[c.actor]) {              // already applied: must be identical
                const uint32_t k = X.tab[sl];
                if (lane == 0) X.hist[j] = -2;
                if (CH[k].content_id != c.content_id) {
                    if (lane == 0) atomicMin(&sh.errkey, err_key(H, 0, j, HM_ERR_INCONSISTENT_SEQ));
                    stop = true;
                }
            } else {
                if (lane == 0) { sh.clock[c.actor] = c.seq; X.tab[sl] = j; X.hist[j] = (int32_t)H; X.h2a[H] = j; }
                H++;
            }
            wfence();
        };
        // first queued + ready change at index >= cursor (among arrived changes <= i)
        auto find_ready = [&](uint32_t cursor, uint32_t i) -> uint32_t {
            for (uint32_t q0 = cursor; q0 <= i; q0 += 64) {
                const uint32_t q = q0 + lane;
                const bool cand = q <= i && X.hist[q] == -1 && ready(q);
                const u64 bm = __ballot(cand);
                if (bm) return q0 + (uint32_t)__builtin_ctzll(bm);
            }
            return 0xFFFFFFFFu;
        };
        for (uint32_t i = 0; i < n && !stop; i++) {
            if (lane == 0) X.hist[i] = -1;                 // queue.push(change)
            wfence();
            if (!ready(i)) continue;                       // pass 1: only the new change can be ready
            apply(i);
            while (!stop) {                                // further passes until one applies nothing
                bool progress = false;
                uint32_t cursor = 0;
                for (;;) {
                    const uint32_t j = find_ready(cursor, i);
                    if (j == 0xFFFFFFFFu) break;
                    apply(j);
                    progress = true;
                    cursor = j + 1;
                    if (stop) break;
                }
                if (!progress) break;
            }
        }
        for (uint32_t i = lane; i < n; i += 64) if (X.hist[i] == -3) X.hist[i] = -1;
        if (lane == 0) sh.H = H;
    }
    }
    bsync();
    const uint32_t H = sh.H;
    if (!all_ready && staged) {             // tables back into LDS for L2
        if (ltab) for (uint32_t i = tid; i < T; i += LWG) lt[i] = X.tab[i];
        for (uint32_t i = tid; i < n; i += LWG) lh[i] = X.hist[i];
        for (uint32_t h = tid; h < H; h += LWG) lh2a[h] = X.h2a[h];
        bsync();
    }
    auto hist_i = [&](uint32_t i) -> int32_t { if (staged) return lh[i]; return X.hist[i]; };
    auto h2a_i = [&](uint32_t h) -> uint32_t { if (staged) return lh2a[h]; return X.h2a[h]; };
    LSTAMP(1);
    H_out = (int32_t)H;

    // ---- L2: allDeps ----
    // (a) the transitive closure by pointer jumping over the actor chains, every change at once:
    //     v(i) <- max(v(i), v(latest change of actor a known to v(i))) for every actor a, from
    //     v(i) = the change's own deps (deps.set(actor, seq-1)); an actor's changes are a chain, so
    //     the fixpoint is the closure (log-depth rounds instead of a history-length serial walk).
    // (b) every change folds its deps literally (key order, `.set` may lower an entry) over the
    //     closure rows of its deps; if that equals its closure everywhere, the closure is allDeps.
    //     Otherwise (a listed dep dominated by another: never for heads-based deps) the literal
    //     fold runs serially in history order below.
    uint32_t *cur = p.res_all_deps + (size_t)doc.change_off * S, *nxt = X.vc;   // row stride S / A
    LDS uint32_t *lrows = nullptr;          // the closure rows when L2 ran in LDS (stride A)
    if (staged ? ltab : l2words <= LARENA) {
        // the same rounds and check with the first-arrival table and both row buffers in LDS
        LDS uint32_t *lc = ar + T, *ln = ar + T + n * A;        // row stride A
        if (!ltab) for (uint32_t i = tid; i < T; i += LWG) lt[i] = X.tab[i];
        for (uint32_t i = tid; i < n; i += LWG) {
            LDS uint32_t *row = lc + i * A;
            for (uint32_t a = 0; a < A; a++) row[a] = 0;
            if (hist_i(i) < 0) continue;
            const hm_change_row c = chg(i);
            for (uint32_t j = 0; j < c.n_deps; j++) {
                const hm_dep_row dp = dep(c.dep_off + j);
                const uint32_t sq = dp.actor == c.actor ? c.seq - 1 : dp.seq;
                if (row[dp.actor] < sq) row[dp.actor] = sq;
            }
            if (row[c.actor] < c.seq - 1) row[c.actor] = c.seq - 1;
        }
        bsync();
        auto lslot = [&](uint32_t a, uint32_t sq) -> uint32_t {      // applied change (a, sq) or >= n
            if (sq < sh.base[a] || sq > sh.maxs[a] || sh.maxs[a] == 0) return 0xFFFFFFFFu;
            return lt[sh.tabo[a] + (sq - sh.base[a])];
        };
        if (regrows) {
            // in place, one work item per (row, actor a): row |= row of the change (a, row[a]) by LDS
            // atomic max.  Every entry is a seq the closure contains, so reading a row another item
            // is growing mixes valid lower bounds, and a round in which no item sees a larger entry
            // is the fixpoint.  One barrier per round: the grew flag of round r is gflag[r % 3],
            // and thread 0 clears the one of round r + 1 (last read before the barrier of r - 1).
            if (tid < 3) sh.gflag[tid] = 0;
            bsync();
            for (uint32_t round = 0;; round++) {
                bool grew = false;
                for (uint32_t w = tid; w < n * 8; w += LWG) {
                    const uint32_t i = w >> 3, a = w & 7;
                    if (a >= A || hist_i(i) < 0) continue;
                    LDS uint32_t *row = lc + i * A;
                    const uint32_t sq = row[a];
                    if (!sq) continue;
                    const uint32_t ti = lslot(a, sq);
                    if (ti >= n) continue;
                    const LDS uint32_t *r2 = lc + ti * A;
#pragma unroll
                    for (uint32_t b = 0; b < 8; b++)
                        if (b < A && b != a) { const uint32_t x = r2[b]; if (x > row[b]) { atomicMax(&row[b], x); grew = true; } }
                }
                if (tid == 0) sh.gflag[(round + 1) % 3] = 0;
                if (grew) sh.gflag[round % 3] = 1;
                bsync();
                if (!sh.gflag[round % 3]) break;
            }
        } else {
            for (;;) {
                if (tid == 0) sh.grew = 0;
                bsync();
                bool grew = false;
                for (uint32_t i = tid; i < n; i += LWG) {
                    const LDS uint32_t *row = lc + i * A;
                    LDS uint32_t *out = ln + i * A;
                    for (uint32_t a = 0; a < A; a++) out[a] = row[a];
                    if (X.hist[i] < 0) continue;
                    for (uint32_t a = 0; a < A; a++) {
                        const uint32_t sq = row[a];
                        if (!sq) continue;
                        const uint32_t ti = lslot(a, sq);
                        if (ti >= n) continue;
                        const LDS uint32_t *r2 = lc + ti * A;
                        for (uint32_t b = 0; b < A; b++) {
                            const uint32_t v = b == a ? sq : r2[b];
                            if (out[b] < v) { out[b] = v; grew = true; }
                        }
                    }
                }
                if (grew) sh.grew = 1;
                bsync();
                const bool any = sh.grew != 0;
                LDS uint32_t *t = lc; lc = ln; ln = t;          // every row of the new buffer was written
                bsync();
                if (!any) break;
            }
        }
        LSTAMP(2);
        if (tid == 0) sh.all_ok = 1;
        bsync();
        for (uint32_t i = tid; i < n; i += LWG) {
            uint32_t *grow_ = cur + (size_t)i * S;
            const LDS uint32_t *row = lc + i * A;
            for (uint32_t a = 0; a < S; a++) grow_[a] = a < A ? row[a] : 0u;
            if (hist_i(i) < 0) continue;
            const hm_change_row c = chg(i);
            bool same = true;
            if (regrows) {
                uint32_t acc[8];
#pragma unroll
                for (uint32_t b = 0; b < 8; b++) acc[b] = 0;
                auto fold = [&](uint32_t a, uint32_t sq) {
                    if (sq == 0) return;
                    const uint32_t ti = lslot(a, sq);
                    if (ti >= n) { same = false; return; }
                    const LDS uint32_t *r2 = lc + ti * A;
#pragma unroll
                    for (uint32_t b = 0; b < 8; b++)
                        if (b < A) { const uint32_t x = r2[b]; acc[b] = b == a ? sq : (acc[b] > x ? acc[b] : x); }
                };
                bool own = false;
                for (uint32_t j = 0; j < c.n_deps; j++) {
                    const hm_dep_row dp = dep(c.dep_off + j);
                    if (dp.actor == c.actor) { own = true; fold(c.actor, c.seq - 1); }
                    else fold(dp.actor, dp.seq);
                }
                if (!own) fold(c.actor, c.seq - 1);
#pragma unroll
                for (uint32_t b = 0; b < 8; b++) if (b < A) same = same && acc[b] == row[b];
            } else {
                LDS uint32_t *acc = ln + i * A;
                for (uint32_t a = 0; a < A; a++) acc[a] = 0;
                auto fold = [&](uint32_t a, uint32_t sq) {
                    if (sq == 0) return;
                    const uint32_t ti = lslot(a, sq);
                    if (ti >= n) { acc[a] = 0xFFFFFFFFu; return; }
                    const LDS uint32_t *r2 = lc + ti * A;
                    for (uint32_t b = 0; b < A; b++) if (acc[b] < r2[b]) acc[b] = r2[b];
                    acc[a] = sq;
                };
                bool own = false;
                for (uint32_t j = 0; j < c.n_deps; j++) {
                    const hm_dep_row dp = dep(c.dep_off + j);
                    if (dp.actor == c.actor) { own = true; fold(c.actor, c.seq - 1); }
                    else fold(dp.actor, dp.seq);
                }
                if (!own) fold(c.actor, c.seq - 1);
                for (uint32_t a = 0; a < A; a++) same = same && acc[a] == row[a];
            }
            if (!same) sh.all_ok = 0;
        }
        lrows = lc;
        bsync();
    } else {
        for (uint32_t i = tid; i < n; i += LWG) {
            uint32_t *row = cur + (size_t)i * S;
            for (uint32_t a = 0; a < S; a++) row[a] = 0;
            if (X.hist[i] < 0) continue;
            const hm_change_row c = CH[i];
            for (uint32_t j = 0; j < c.n_deps; j++) {
                const hm_dep_row dp = p.deps[c.dep_off + j];
                const uint32_t sq = dp.actor == c.actor ? c.seq - 1 : dp.seq;
                if (row[dp.actor] < sq) row[dp.actor] = sq;
            }
            if (row[c.actor] < c.seq - 1) row[c.actor] = c.seq - 1;
        }
        bsync();
        for (;;) {                                  // monotone and bounded: terminates (rounds ~ log depth)
            if (tid == 0) sh.grew = 0;
            bsync();
            bool grew = false;
            for (uint32_t i = tid; i < n; i += LWG) {
                const uint32_t *row = cur + (size_t)i * S;
                uint32_t *out = nxt + (size_t)i * A;
                for (uint32_t a = 0; a < A; a++) out[a] = row[a];
                if (X.hist[i] < 0) continue;
                for (uint32_t a = 0; a < A; a++) {
                    const uint32_t sq = row[a];
                    if (!sq) continue;
                    const uint32_t sl = slot_of(a, sq), ti = sl == 0xFFFFFFFFu ? 0xFFFFFFFFu : X.tab[sl];
                    if (ti >= n) continue;                           // not applied: cannot occur for deps of applied changes
                    const uint32_t *r2 = cur + (size_t)ti * S;       // the applied change (a, sq)
                    for (uint32_t b = 0; b < A; b++) {
                        const uint32_t v = b == a ? sq : r2[b];
                        if (out[b] < v) { out[b] = v; grew = true; }
                    }
                }
            }
            if (grew) sh.grew = 1;
            bsync();
            const bool any = sh.grew != 0;          // read by every thread before the barrier below,
            for (uint32_t i = tid; i < n; i += LWG) // so thread 0's reset of the next round cannot race it
                for (uint32_t a = 0; a < A; a++) cur[(size_t)i * S + a] = nxt[(size_t)i * A + a];
            bsync();
            if (!any) break;
        }
        LSTAMP(2);
        if (tid == 0) sh.all_ok = 1;
        bsync();
        for (uint32_t i = tid; i < n; i += LWG) {
            if (X.hist[i] < 0) continue;
            const hm_change_row c = CH[i];
            const uint32_t *row = cur + (size_t)i * S;
            uint32_t *acc = nxt + (size_t)i * A;
            for (uint32_t a = 0; a < A; a++) acc[a] = 0;
            auto fold = [&](uint32_t a, uint32_t sq) {
                if (sq == 0) return;
                const uint32_t sl = slot_of(a, sq), ti = sl == 0xFFFFFFFFu ? 0xFFFFFFFFu : X.tab[sl];
                if (ti >= n) { acc[a] = 0xFFFFFFFFu; return; }       // (cannot occur) forces the serial path
                const uint32_t *r2 = cur + (size_t)ti * S;
                for (uint32_t b = 0; b < A; b++) if (acc[b] < r2[b]) acc[b] = r2[b];
                acc[a] = sq;
            };
            bool own = false;
            for (uint32_t j = 0; j < c.n_deps; j++) {
                const hm_dep_row dp = p.deps[c.dep_off + j];
                if (dp.actor == c.actor) { own = true; fold(c.actor, c.seq - 1); }
                else fold(dp.actor, dp.seq);
            }
            if (!own) fold(c.actor, c.seq - 1);
            bool same = true;
            for (uint32_t a = 0; a < A; a++) same = same && acc[a] == row[a];
            if (!same) sh.all_ok = 0;
        }
        bsync();
    }
    const bool closure_ok = sh.all_ok != 0;
    if (closure_ok) {
        for (uint32_t h = tid; h < H; h += LWG) {
            if (lrows) {
                const LDS uint32_t *row = lrows + h2a_i(h) * A;
                for (uint32_t a = 0; a < A; a++) atomicMax(&sh.maxad[a], row[a]);
            } else {
                const uint32_t *row = cur + (size_t)X.h2a[h] * S;
                for (uint32_t a = 0; a < A; a++) atomicMax(&sh.maxad[a], row[a]);
            }
        }
    }
    // literal fold, history order, lanes = actors (wave 0; actors a0 + lane per 64-actor slice)
    if (!closure_ok && wave == 0) {
        for (uint32_t h = 0; h < H; h++) {
            const uint32_t ci = X.h2a[h];
            const hm_change_row c = CH[ci];
            for (uint32_t a0 = 0; a0 < S; a0 += 64) {
                const uint32_t la = a0 + lane;
                uint32_t acc = 0;
                auto fold = [&](uint32_t a, uint32_t s) {
                    if (s == 0) return;
                    const uint32_t dc = tabv(slot_of(a, s));       // the applied change (a, s)
                    const uint32_t t = la < A ? ad_row(p, doc, dc)[la] : 0;
                    acc = acc > t ? acc : t;
                    if (la == a) acc = s;
                };
                bool own = false;
                for (uint32_t j = 0; j < c.n_deps; j++) {
                    const hm_dep_row dp = p.deps[c.dep_off + j];
                    if (dp.actor == c.actor) { own = true; fold(c.actor, c.seq - 1); }
                    else fold(dp.actor, dp.seq);
                }
                if (!own) fold(c.actor, c.seq - 1);
                if (la < S) ad_row(p, doc, ci)[la] = la < A ? acc : 0;
                if (la < A) sh.maxad[la] = sh.maxad[la] > acc ? sh.maxad[la] : acc;
            }
            wfence();                                          // rows are re-read by later changes
        }
        // rows of unapplied changes are zero
        for (uint32_t i = lane; i < n; i += 64)
            if (X.hist[i] < 0) for (uint32_t a = 0; a < S; a++) ad_row(p, doc, i)[a] = 0;
    }
    bsync();
    LSTAMP(3);
    // clock / heads: a head survives unless some applied change's allDeps reaches it
    for (uint32_t h = tid; h < H; h += LWG) {
        const hm_change_row c = chg(h2a_i(h));
        atomicMax(&sh.clock[c.actor], c.seq);
    }
    bsync();
    if (tid < A && sh.clock[tid] && sh.maxad[tid] < sh.clock[tid]) sh.headv[tid] = sh.clock[tid];

    // ---- L3: ops ----
    // Op keys: an applied op's position in application order, i.e. (history position, op index)
    // as one 32-bit number: kbase[change] = the ops of the changes before it in history.
    for (uint32_t h = tid; h < H; h += LWG) X.survp[h] = CH[X.h2a[h]].n_ops;     // survp is free until L3 survivors
    bsync();
    uint32_t m_applied;
    m_applied = scan_array(sh, X.survp, H);
    (void)m_applied;
    // Per-change inputs of the op loops (history position, actor, seq, first op, key base,
    // allDeps row) and the op -> change map (16 bit) are staged in the LDS arena when they fit
    // (L2 is done with it); so is one compact word per op — register (20 b) | action (4 b) |
    // object (8 b) — when the document's ids fit those widths, so the op loops below do not
    // re-read 32-byte op rows from HBM (only INS parents / elems and survivor values are).
    const uint32_t l3_words = n * (A + 5) + (m + 1) / 2;
    const bool l3 = l3_ok(n, m, A);
    const bool lop = l3 && R <= (1u << 20) && O < 255 && l3_words + m <= LARENA;
    LDS uint32_t *l_hist = ar, *l_act = ar + n, *l_seq = ar + 2 * n, *l_op0 = ar + 3 * n, *l_kb = ar + 4 * n,
                 *l_ad = ar + 5 * n, *l_op = ar + l3_words;
    LDS uint16_t *l_opchg = (LDS uint16_t *)(ar + 5 * n + n * A);
    // object tables in LDS when they fit (text / list documents have a handful of objects)
    const bool obj_lds = O <= LA_MAX;
    auto oslot_get = [&](uint32_t o) -> uint32_t { return obj_lds ? sh.oslot[o] : X.objslot[o]; };
    auto otype_get = [&](uint32_t o) -> uint32_t { return obj_lds ? sh.otype[o] : X.objtype[o]; };
    for (uint32_t i = tid; i < O; i += LWG) {
        const uint32_t sl = i == 0 ? 0u : 0xFFFFFFFFu, ty = i == 0 ? (uint32_t)HM_MAKE_MAP : 0xFFu;
        if (obj_lds) { sh.oslot[i] = sl; sh.otype[i] = ty; } else { X.objslot[i] = sl; X.objtype[i] = ty; }
    }
    // RGA nodes are allocated by the op scan when the encoder's hint says the document has
    // lists (HM_DOC_HAS_LISTS), otherwise by a pass of their own in L4 (either way exact)
    const bool early = (doc.flags & HM_DOC_HAS_LISTS) != 0;
    const uint32_t NP = R + O;
    if (early) for (uint32_t i = tid; i < NP; i += LWG) { X.pcount[i] = 0; X.pfill[i] = 0; X.fc[i] = 0xFFFFFFFFu; }
    for (uint32_t i = tid; i < R; i += LWG) {
        X.segcnt[i] = 0; X.survcnt[i] = 0; X.insmin[i] = 0xFFFFFFFFu; X.regobj[i] = HM_NONE; X.segfill[i] = 0;
        if (early) X.regnode[i] = 0xFFFFFFFFu;
    }
    if (tid == 0) { sh.nmake = 0; sh.nsurv = 0; }
    for (uint32_t i = tid; i < n; i += LWG) {
        const hm_change_row c = CH[i];
        const int32_t hi = X.hist[i];
        const uint32_t kb = hi >= 0 ? X.survp[hi] : 0xFFFFFFFFu;
        if (l3) {
            const uint32_t o0 = c.op_first - doc.op_off;
            l_hist[i] = (uint32_t)hi; l_act[i] = c.actor; l_seq[i] = c.seq; l_op0[i] = o0; l_kb[i] = kb;
            const uint32_t *ad = ad_row(p, doc, i);
            for (uint32_t a = 0; a < A; a++) l_ad[i * A + a] = ad[a];
            for (uint32_t j = 0; j < c.n_ops; j++) l_opchg[o0 + j] = (uint16_t)i;
        } else {
            X.kbase[i] = kb;
        }
    }
    bsync();
    LSTAMP(11);
    auto opchg_of = [&](uint32_t k) -> uint32_t { return l3 ? (uint32_t)l_opchg[k] : X.opchg[k]; };
    auto hist_of = [&](uint32_t ci) -> int32_t { return l3 ? (int32_t)l_hist[ci] : X.hist[ci]; };
    auto op0_of = [&](uint32_t ci) -> uint32_t { return l3 ? l_op0[ci] : CH[ci].op_first - doc.op_off; };
    auto act_of = [&](uint32_t ci) -> uint32_t { return l3 ? l_act[ci] : CH[ci].actor; };
    auto seq_of = [&](uint32_t ci) -> uint32_t { return l3 ? l_seq[ci] : CH[ci].seq; };
    auto ad_of = [&](uint32_t ci, uint32_t a) -> uint32_t { return l3 ? l_ad[ci * A + a] : ad_row(p, doc, ci)[a]; };
    auto kb_of = [&](uint32_t ci) -> uint32_t { return l3 ? l_kb[ci] : X.kbase[ci]; };
    // (register, action, object) of op k
    struct OpC { uint32_t reg, action, obj; };
    auto op_c = [&](uint32_t k) -> OpC {
        if (lop) { const uint32_t w = l_op[k]; return OpC{w & 0xFFFFFu, (w >> 20) & 15u, w >> 24}; }
        const hm_op_row &o = OP[k];
        return OpC{o.reg, o.action, o.obj};
    };
    auto key_of = [&](uint32_t k, uint32_t ci) -> uint32_t { return kb_of(ci) + (k - op0_of(ci)); };   // applied ops
    for (uint32_t k = tid; k < m; k += LWG) {
        const hm_op_row o = OP[k];
        const uint32_t ci = opchg_of(k);
        const int32_t h = hist_of(ci);
        if (o.action == HM_INC || o.datatype == HM_DT_COUNTER) sh.ctrs = 1;
        // malformed rows (any op, applied or not) put the whole document outside the envelope
        const bool bad = o.action <= HM_MAKE_TEXT ? o.obj >= O
                       : (o.action <= HM_INC ? (o.reg >= R || (o.action == HM_INS && o.parent != HM_HEAD && o.parent >= R)) : true);
        if (bad) { atomicOr(&sh.flags, LF_UNSUPPORTED); continue; }
        // (object 255: an unknown object id, >= O)
        if (lop) l_op[k] = (o.action <= HM_MAKE_TEXT ? 0u : o.reg) | (o.action << 20) | ((o.obj < O ? o.obj : 255u) << 24);
        if (h < 0) continue;
        const uint32_t key = key_of(k, ci);
        if (o.action <= HM_MAKE_TEXT) {
            if (obj_lds) atomicMin(&sh.oslot[o.obj], key + 1); else g_min(&X.objslot[o.obj], key + 1);
            X.survtmp[atomicAdd(&sh.nmake, 1u)] = k;              // make-op list (survtmp is free until L3 offsets)
        } else {
            if (o.obj >= O) continue;                              // an unknown object: the survivor pass throws
            X.regobj[o.reg] = o.obj;
            if (o.action == HM_INS) {
                g_min(&X.insmin[o.reg], key + 1);
                if (o.elem >= (1u << 24)) atomicOr(&sh.flags, LF_UNSUPPORTED);
                if (early) {
                    const uint32_t i = atomicAdd(&sh.nins, 1u);
                    const uint32_t pi = o.parent == HM_HEAD ? R + o.obj : o.parent;
                    X.nodepi[i] = pi; X.nreg[i] = o.reg; X.nlist[i] = o.obj;     // nlist: object -> list id in L4
                    X.nodekey[i] = (o.elem << 8) | act_of(ci);
                    X.regnode[o.reg] = i;
                    g_add(&X.pcount[pi], 1u);
                }
            } else g_add(&X.segcnt[o.reg], 1u);
        }
    }
    bsync();
    if (sh.flags) return LUNSUP;
    LSTAMP(12);
    const bool ctrs = sh.ctrs != 0;
    for (uint32_t q = tid; q < sh.nmake; q += LWG) {
        const uint32_t k = X.survtmp[q];
        const OpC o = op_c(k);
        const uint32_t ci = opchg_of(k);
        if (oslot_get(o.obj) != key_of(k, ci) + 1)
            atomicMin(&sh.errkey, err_key((uint32_t)hist_of(ci), k - op0_of(ci) + 1, ci, HM_ERR_DUPLICATE_OBJECT));
        else if (obj_lds) sh.otype[o.obj] = o.action;
        else X.objtype[o.obj] = o.action;
    }
    bsync();
    // per-register assign lists (set/del/link/inc; segk = op index | inc << 31), used by the
    // survivor test and by the tie positions; per-actor maxima only for long lists
    for (uint32_t i = tid; i < R; i += LWG) {
        const uint32_t c = X.segcnt[i];
        X.segoff[i] = c;
        if (c > SEG_SHORT) for (uint32_t a = 0; a < A; a++) X.segmax[(size_t)i * A + a] = 0;
    }
    bsync();
    (void)scan_array(sh, X.segoff, R);
    for (uint32_t k = tid; k < m; k += LWG) {
        const OpC o = op_c(k);
        if (o.action < HM_SET || o.action > HM_INC || o.obj >= O) continue;   // exactly the ops segcnt counted
        const uint32_t ci = opchg_of(k);
        if (hist_of(ci) < 0) continue;
        const uint32_t q = X.segoff[o.reg] + g_add(&X.segfill[o.reg], 1u);
        X.seglist[q] = key_of(k, ci);
        X.segk[q] = k | (o.action == HM_INC ? 0x80000000u : 0u);
        if (o.action != HM_INC && X.segcnt[o.reg] > SEG_SHORT)
            for (uint32_t a = 0; a < A; a++) {
                const uint32_t v = ad_of(ci, a);
                if (v) g_max(&X.segmax[(size_t)o.reg * A + a], v);   // 0 is the initial value
            }
    }
    bsync();
    LSTAMP(13);
    // survivors, listed as (op, slot in its register) pairs: survk / survp[0 .. nsurv)
    bool any_list = false;
    for (uint32_t k = tid; k < m; k += LWG) {
        const OpC o = op_c(k);
        if (o.action < HM_INS || o.action > HM_INC) continue;
        const uint32_t ci = opchg_of(k);
        const int32_t h = hist_of(ci);
        if (h < 0) continue;
        const uint32_t kx = k - op0_of(ci), key = kb_of(ci) + kx;
        const uint32_t os = o.obj < O ? oslot_get(o.obj) : 0xFFFFFFFFu;
        if (os == 0xFFFFFFFFu || os > key) {
            atomicMin(&sh.errkey, err_key((uint32_t)h, kx + 1, ci, HM_ERR_UNKNOWN_OBJECT));
            continue;
        }
        const uint32_t ot = otype_get(o.obj);
        const bool is_list = ot == HM_MAKE_LIST || ot == HM_MAKE_TEXT;
        if (o.action == HM_INS) {
            any_list = true;
            const uint32_t parent = OP[k].parent;
            if (X.insmin[o.reg] != key + 1)
                atomicMin(&sh.errkey, err_key((uint32_t)h, kx + 1, ci, HM_ERR_DUPLICATE_ELEM));
            if (parent != HM_HEAD && !(X.insmin[parent] <= key)) sh.late = 1;   // see the chain pass below
            continue;
        }
        any_list |= is_list;
        if (o.action == HM_SET || o.action == HM_LINK) {
            if (is_list && !(X.insmin[o.reg] <= key))
                atomicMin(&sh.errkey, err_key((uint32_t)h, kx + 1, ci, HM_ERR_MISSING_ELEM));
            // survivor: no set/del/link on the register has this op's change among its allDeps
            const uint32_t ao = act_of(ci), so = seq_of(ci), cnt = X.segcnt[o.reg];
            bool surv = true;
            if (cnt > SEG_SHORT) surv = X.segmax[(size_t)o.reg * A + ao] < so;
            else {
                const uint32_t b0 = X.segoff[o.reg];
                for (uint32_t q = 0; q < cnt; q++) {
                    const uint32_t e = X.segk[b0 + q];
                    if (!(e >> 31) && ad_of(opchg_of(e & 0x7FFFFFFFu), ao) >= so) surv = false;
                }
            }
            if (surv) {
                const uint32_t slot = g_add(&X.survcnt[o.reg], 1u);
                const uint32_t j = atomicAdd(&sh.nsurv, 1u);
                X.survk[j] = k; X.survp[j] = slot;
            }
        }
    }
    if (any_list) sh.lists = 1;
    bsync();
    // Inserts after an element not yet inserted (Automerge 0.12 applyInsert accepts them: the op
    // waits in its parent's _following until the parent arrives).  A set
    // or link on a list element runs updateListElement -> getPrevious, which climbs the element's
    // insertion chain and throws 'Missing index entry' at the first element not inserted yet; so
    // the set throws iff attach(e) = max insmin over e's chain exceeds its key.  An element whose
    // chain never reaches '_head' (a missing or cyclic ancestor) is never visible: L4 leaves it
    // out.  attach by pointer jumping over (parent, max) pairs in the (still free) tour arrays.
    const bool late = sh.late != 0;
    uint32_t *cjp = X.tour0, *cmx = X.tval0;       // final chain pointers / maxima (late documents)
    constexpr uint32_t CH_HEAD = 0xFFFFFFFFu;
    if (late) {
        if (R > 2 * (m + O)) return LUNSUP;        // (register ids beyond the tour arrays: no such encoder)
        uint32_t *jp1 = X.tour1, *mx1 = X.tval1;
        for (uint32_t r = tid; r < R; r += LWG) { cjp[r] = CH_HEAD; cmx[r] = X.insmin[r]; }
        bsync();
        for (uint32_t k = tid; k < m; k += LWG) {
            const OpC o = op_c(k);
            if (o.action != HM_INS || o.obj >= O) continue;
            const uint32_t ci = opchg_of(k);
            if (hist_of(ci) < 0 || X.insmin[o.reg] != key_of(k, ci) + 1) continue;   // the applied insertion
            const uint32_t par = OP[k].parent;
            if (par != HM_HEAD) cjp[o.reg] = par;
        }
        bsync();
        const uint32_t rounds = 33 - __builtin_clz(R | 1);
        for (uint32_t rd = 0; rd < rounds; rd++) {
            for (uint32_t r = tid; r < R; r += LWG) {
                const uint32_t j = cjp[r], a = cmx[r];
                if (j == CH_HEAD) { jp1[r] = CH_HEAD; mx1[r] = a; }
                else { jp1[r] = cjp[j]; const uint32_t b = cmx[j]; mx1[r] = a > b ? a : b; }
            }
            bsync();
            uint32_t *t = cjp; cjp = jp1; jp1 = t; t = cmx; cmx = mx1; mx1 = t;
        }
        for (uint32_t k = tid; k < m; k += LWG) {
            const OpC o = op_c(k);
            if ((o.action != HM_SET && o.action != HM_LINK) || o.obj >= O) continue;
            const uint32_t ot = otype_get(o.obj);
            if (!(ot == HM_MAKE_LIST || ot == HM_MAKE_TEXT)) continue;
            const uint32_t ci = opchg_of(k);
            const int32_t h = hist_of(ci);
            if (h < 0) continue;
            const uint32_t kx = k - op0_of(ci), key = kb_of(ci) + kx;
            if (!(cmx[o.reg] <= key)) atomicMin(&sh.errkey, err_key((uint32_t)h, kx + 1, ci, HM_ERR_MISSING_ELEM));
            else if (cjp[o.reg] != CH_HEAD) atomicOr(&sh.flags, LF_UNSUPPORTED);   // a cyclic chain: getPrevious never returns
        }
        bsync();
    }
    const bool lists_flag = sh.lists != 0;
    const uint32_t nsurv = sh.nsurv;
    if (sh.errkey != ~0ull) return LERR;
    if (sh.flags) return LUNSUP;
    LSTAMP(4);
    // survivor offsets
    for (uint32_t i = tid; i < R; i += LWG) X.regoff[i] = X.survcnt[i];
    bsync();
    uint32_t total;
    total = scan_array(sh, X.regoff, R);
    if (tid == 0) sh.total = total;
    for (uint32_t j = tid; j < nsurv; j += LWG) {
        const uint32_t k = X.survk[j];
        X.survtmp[X.regoff[op_c(k).reg] + X.survp[j]] = k;
    }
    bsync();
    // ranks: actor descending; ties (one change) by the sortBy(actor).reverse() flip
    for (uint32_t j = tid; j < nsurv; j += LWG) {
        const uint32_t k = X.survk[j];
        const uint32_t reg = op_c(k).reg;
        const uint32_t my_a = act_of(opchg_of(k));
        const uint32_t b0 = X.regoff[reg], cnt = X.survcnt[reg];
        uint32_t rank = 0;
        if (cnt > 1) {
            const uint32_t nseg = X.segcnt[reg], sb = X.segoff[reg];
            const bool odd_n = nseg & 1;
            auto tkey = [&](uint32_t kk) -> uint32_t {
                uint32_t pc = 0;
                const uint32_t key = key_of(kk, opchg_of(kk));
                for (uint32_t q = 0; q < nseg; q++) pc += X.seglist[sb + q] < key ? 1u : 0u;
                return (pc & 1) ? (0x80000000u - pc) : (0x80000000u + pc);
            };
            uint32_t my_t = 0;
            bool have_t = false;
            for (uint32_t q = 0; q < cnt; q++) {
                const uint32_t k2 = X.survtmp[b0 + q];
                if (k2 == k) continue;
                const uint32_t a2 = act_of(opchg_of(k2));
                if (a2 > my_a) rank++;
                else if (a2 == my_a) {
                    if (!have_t) { my_t = tkey(k); have_t = true; }
                    const uint32_t t2 = tkey(k2);
                    if (odd_n ? (t2 > my_t) : (t2 < my_t)) rank++;
                }
            }
        }
        X.survop[b0 + rank] = k;
        if (ctrs) { X.survsum[b0 + rank] = 0; X.survabs[b0 + rank] = 0; }
    }
    bsync();
    LSTAMP(5);
    // counters
    for (uint32_t k = tid; ctrs && k < m; k += LWG) {
        const hm_op_row o = OP[k];
        if (o.action != HM_INC || o.reg >= R || hist_of(opchg_of(k)) < 0) continue;
        const uint32_t ci = opchg_of(k);
        const uint32_t b0 = X.regoff[o.reg], cnt = X.survcnt[o.reg];
        for (uint32_t q = 0; q < cnt; q++) {
            const uint32_t k2 = X.survop[b0 + q];
            const hm_op_row o2 = OP[k2];
            if (o2.action != HM_SET || o2.datatype != HM_DT_COUNTER || (o2.vtag != HM_V_INT && o2.vtag != HM_V_FLOAT)) continue;
            const uint32_t c2 = opchg_of(k2);
            if (ad_of(ci, act_of(c2)) < seq_of(c2)) continue;                 // concurrent inc: no effect
            // a non-integral base or inc: JS adds doubles, whose sum depends on the order the incs
            // are applied in -> the survivor is folded sequentially below (ORDERED)
            if (o2.vtag != HM_V_INT || o.vtag != HM_V_INT) { g_or(&X.survabs[b0 + q], ORDERED); continue; }
            const int64_t v = (int64_t)o.value;
            g_add((GLB u64 *)&X.survsum[b0 + q], (u64)v);
            g_add(&X.survabs[b0 + q], (u64)(v < 0 ? -v : v));
        }
    }
    bsync();
    // ORDERED survivors (Automerge 0.12 applyAssign): fold the incs of
    // the register that causally follow the counter set, in application order (history
    // position, op index) — one thread per survivor, the next inc found by a min-scan of the
    // register's assign list (seglist keys).  Integer + integer adds stay int64 until the first
    // non-integral operand; from there on the value is an IEEE double, as the JS sum is.
    for (uint32_t q = tid; ctrs && q < total; q += LWG) {
        if (!(X.survabs[q] & ORDERED)) continue;
        const uint32_t k2 = X.survop[q];
        const hm_op_row o2 = OP[k2];
        const uint32_t c2 = opchg_of(k2), a2 = act_of(c2), s2 = seq_of(c2), reg = o2.reg;
        const uint32_t b0 = X.segoff[reg], cnt = X.segcnt[reg];
        bool is_int = o2.vtag == HM_V_INT;
        u64 acc = o2.value;
        uint32_t prev = 0;
        bool first = true;
        for (;;) {
            uint32_t best = 0xFFFFFFFFu;
            uint32_t bk = 0;
            for (uint32_t e = 0; e < cnt; e++) {
                const uint32_t sk = X.segk[b0 + e];
                if (!(sk & 0x80000000u)) continue;                             // incs only
                const uint32_t key = X.seglist[b0 + e];
                if ((!first && key <= prev) || key >= best) continue;
                const uint32_t ki = sk & 0x7FFFFFFFu;
                if (ad_of(opchg_of(ki), a2) < s2) continue;                    // concurrent inc: no effect
                best = key; bk = ki;
            }
            if (best == 0xFFFFFFFFu) break;
            const hm_op_row oi = OP[bk];
            if (is_int && oi.vtag == HM_V_INT) {
                acc = (u64)((int64_t)acc + (int64_t)oi.value);
            } else {
                const double x = is_int ? (double)(int64_t)acc : __longlong_as_double((long long)acc);
                const double y = oi.vtag == HM_V_INT ? (double)(int64_t)oi.value : __longlong_as_double((long long)oi.value);
                acc = (u64)__double_as_longlong(x + y);
                is_int = false;
            }
            prev = best;
            first = false;
        }
        X.survsum[q] = (int64_t)acc;                                            // the folded value's bits
        if (is_int) atomicOr(&sh.flags, LF_UNSUPPORTED);                       // (a float operand was seen: unreachable)
    }
    bsync();
    if (sh.flags) return LUNSUP;

    LSTAMP(6);
    // ---- L4: RGA order ----
    if (lists_flag) {
        // late documents rebuild the nodes without the detached elements
        const bool early_nodes = early && !late;
        if (!early_nodes) {
            for (uint32_t i = tid; i < NP; i += LWG) { X.pcount[i] = 0; X.pfill[i] = 0; X.fc[i] = 0xFFFFFFFFu; }
            for (uint32_t i = tid; i < R; i += LWG) X.regnode[i] = 0xFFFFFFFFu;
            if (tid == 0) sh.nins = 0;
        }
        for (uint32_t i = tid; i < O; i += LWG) { const uint32_t t = otype_get(i); X.listid[i] = (t == HM_MAKE_LIST || t == HM_MAKE_TEXT) ? 1u : 0u; }
        bsync();
        uint32_t nl;
        nl = scan_array(sh, X.listid, O);          // exclusive prefix -> compact list id (valid for list objects)
        // per node i: its register nreg[i], its compact list id nlist[i], parent slot, sibling key
        if (!early_nodes) {
            for (uint32_t k = tid; k < m; k += LWG) {
                const OpC c = op_c(k);
                if (c.action != HM_INS) continue;
                const uint32_t ci = opchg_of(k);
                if (hist_of(ci) < 0) continue;
                if (late && (cjp[c.reg] != CH_HEAD || cmx[c.reg] == 0xFFFFFFFFu)) continue;   // detached: never visible
                const uint32_t parent = OP[k].parent, elem = OP[k].elem;
                const uint32_t i = atomicAdd(&sh.nins, 1u);
                const uint32_t pi = parent == HM_HEAD ? R + c.obj : parent;
                X.nodepi[i] = pi; X.nreg[i] = c.reg; X.nlist[i] = X.listid[c.obj];
                X.nodekey[i] = (elem << 8) | act_of(ci);                    // elem < 2^24 (op scan)
                X.regnode[c.reg] = i;
                g_add(&X.pcount[pi], 1u);
            }
            bsync();
        }
        const uint32_t N = sh.nins;
        for (uint32_t i = tid; i < NP; i += LWG) X.poff[i] = X.pcount[i];
        bsync();
        (void)scan_array(sh, X.poff, NP);
        // sibling lists (an only child needs none: no next sibling, first child of its parent)
        for (uint32_t i = tid; i < N; i += LWG) {
            const uint32_t pi = X.nodepi[i];
            if (X.pcount[pi] > 1) X.plist[X.poff[pi] + g_add(&X.pfill[pi], 1u)] = i;
            if (early_nodes) X.nlist[i] = X.listid[X.nlist[i]];
        }
        bsync();
        for (uint32_t i = tid; i < N; i += LWG) {
            const uint32_t pi = X.nodepi[i], np = X.pcount[pi];
            if (np == 1) { X.ns[i] = 0xFFFFFFFFu; X.fc[pi] = i; continue; }
            const uint32_t key = X.nodekey[i];
            uint32_t best = 0xFFFFFFFFu, bkey = 0; bool firstc = true;
            for (uint32_t q = 0; q < np; q++) {
                const uint32_t j = X.plist[X.poff[pi] + q];
                const uint32_t kj = X.nodekey[j];
                if (kj > key) firstc = false;
                else if (kj < key && (best == 0xFFFFFFFFu || kj > bkey)) { best = j; bkey = kj; }
            }
            X.ns[i] = best;
            if (firstc) X.fc[pi] = i;
        }
        bsync();
        LSTAMP(7);
        const uint32_t E = 2 * (N + nl), END = 0xFFFFFFFFu;
        // tour entries (next, value): two pool arrays, or one LDS word each (next << 16 | value,
        // END = 0xFFFF) when the tour fits the arena and its indices fit 16 bits
        const bool tour_lds = E <= LARENA && E < 0xFFFFu;
        LDS uint32_t *tw = ar;
        uint32_t *nx0 = X.tour0, *nx1 = X.tour1;
        uint32_t *va0 = X.tval0, *va1 = X.tval1;
        auto put = [&](uint32_t e, uint32_t nx, uint32_t va) {
            if (tour_lds) tw[e] = ((nx == END ? 0xFFFFu : nx) << 16) | va;
            else { nx0[e] = nx; va0[e] = va; }
        };
        for (uint32_t i = tid; i < N; i += LWG) {
            const uint32_t hd = N + X.nlist[i];
            const uint32_t f = X.fc[X.nreg[i]];
            const uint32_t pi = X.nodepi[i];
            put(2 * i, f != 0xFFFFFFFFu ? 2 * f : 2 * i + 1, 1);
            put(2 * i + 1, X.ns[i] != 0xFFFFFFFFu ? 2 * X.ns[i] : (pi >= R ? 2 * hd + 1 : 2 * X.regnode[pi] + 1), 0);
        }
        for (uint32_t o = tid; o < O; o += LWG) {
            const uint32_t t = otype_get(o);
            if (!(t == HM_MAKE_LIST || t == HM_MAKE_TEXT)) continue;
            const uint32_t h = N + X.listid[o], f = X.fc[R + o];
            put(2 * h, f != 0xFFFFFFFFu ? 2 * f : 2 * h + 1, 0);
            put(2 * h + 1, END, 0);
        }
        bsync();
        const uint32_t rounds = E ? 32 - __builtin_clz(E) : 0;
        if (tour_lds) {
            // in-place pointer jumping: a word is read and written whole, so every word keeps
            // "value = sum of the values from this entry up to its link" at every moment, and a
            // link at least 2^r entries ahead after round r (links only move forward)
            for (uint32_t rd = 0; rd < rounds; rd++) {
                for (uint32_t e = tid; e < E; e += LWG) {
                    const uint32_t w = tw[e], x = w >> 16;
                    if (x == 0xFFFFu) continue;
                    const uint32_t w2 = tw[x];
                    tw[e] = (w2 & 0xFFFF0000u) | ((w & 0xFFFFu) + (w2 & 0xFFFFu));
                }
                bsync();
            }
        } else {
            for (uint32_t rd = 0; rd < rounds; rd++) {
                for (uint32_t e = tid; e < E; e += LWG) {
                    const uint32_t x = nx0[e];
                    if (x != END) { nx1[e] = nx0[x]; va1[e] = va0[e] + va0[x]; } else { nx1[e] = END; va1[e] = va0[e]; }
                }
                bsync();
                uint32_t *t = nx0; nx0 = nx1; nx1 = t; t = va0; va0 = va1; va1 = t;
            }
        }
        LSTAMP(8);
        // tour sums (entries from here to the end of the list): LDS words or the pool array
        auto tsum = [&](uint32_t e) -> uint32_t { return tour_lds ? (tw[e] & 0xFFFFu) : va0[e]; };
        for (uint32_t o = tid; o < O; o += LWG) {
            const uint32_t t = otype_get(o);
            const bool isl = t == HM_MAKE_LIST || t == HM_MAKE_TEXT;
            if (isl) X.listbase[X.listid[o]] = tsum(2 * (N + X.listid[o]));
        }
        bsync();
        (void)scan_array(sh, X.listbase, nl);
        // pre-order position of node i: its list's base + (entries of its list) - (entries from i on)
        auto pos_of = [&](uint32_t i, uint32_t l) -> uint32_t { return X.listbase[l] + tsum(2 * (N + l)) - tsum(2 * i); };
        for (uint32_t i = tid; i < N; i += LWG) X.vis[pos_of(i, X.nlist[i])] = X.survcnt[X.nreg[i]] > 0 ? 1u : 0u;
        bsync();
        (void)scan_array(sh, X.vis, N);            // exclusive scan of visibility over pre-order positions
        for (uint32_t i = tid; i < N; i += LWG) {
            const uint32_t l = X.nlist[i], rg = X.nreg[i];
            // list elements carry their visible index (or -1) in insmin from here on
            X.insmin[rg] = X.survcnt[rg] > 0 ? X.vis[pos_of(i, l)] - X.vis[X.listbase[l]] : 0xFFFFFFFFu;
            if (p.res_epos) p.res_epos[doc.reg_off + rg] = pos_of(i, l) - X.listbase[l];
        }
        bsync();
    }

    LSTAMP(9);
    // ---- outputs ----
    for (uint32_t q = tid; q < total; q += LWG) {
        const uint32_t k = X.survop[q];
        const hm_op_row o = OP[k];
        hm_surv_result sr; sr.op = k; sr.vtag = o.vtag; sr.value = o.value;
        const u64 sabs = ctrs ? X.survabs[q] : 0ull;
        if (sabs & ORDERED) {
            sr.vtag = HM_V_FLOAT; sr.value = (u64)X.survsum[q];
        } else if (o.action == HM_SET && o.datatype == HM_DT_COUNTER && o.vtag == HM_V_INT) {
            const int64_t b = (int64_t)o.value;
            if (sabs + (u64)(b < 0 ? -b : b) > (1ull << 53)) atomicOr(&sh.flags, LF_UNSUPPORTED);
            sr.value = (u64)(b + X.survsum[q]);
        }
        p.res_surv[doc.op_off + q] = sr;
    }
    for (uint32_t r = tid; r < R; r += LWG) {
        hm_reg_result rr;
        rr.n_surv = X.survcnt[r]; rr.surv_off = X.regoff[r]; rr.obj = X.regobj[r];
        // list elements carry their visible index (or -1) in insmin after L4
        rr.list_index = (lists_flag && X.regnode[r] != 0xFFFFFFFFu && X.insmin[r] != 0xFFFFFFFFu) ? (int32_t)X.insmin[r] : -1;
        p.res_regs[doc.reg_off + r] = rr;
    }
    for (uint32_t i = tid; i < n; i += LWG) p.res_hist[doc.change_off + i] = X.hist[i];
    bsync();
    if (sh.flags) return LUNSUP;
    LSTAMP(10);
    return LOK;
}

__global__ __launch_bounds__(LWG) __attribute__((amdgpu_waves_per_eu(HML_WPE))) void merge_large_kernel(SmallParams p, uint8_t *pool, u64 pool_bytes, u64 *pool_used) {
    __shared__ Shared sh;
    __shared__ __align__(16) uint32_t arena_raw[LARENA];
    LDS uint32_t *arena = (LDS uint32_t *)arena_raw;
    const uint32_t tid = threadIdx.x;
    const uint32_t S = p.a_stride;
    // Deferred documents are listed by merge_small_kernel (p.deferred, p.n_deferred).  Each
    // workgroup claims one document at a time: deferred documents are the long ones, so
    // per-document claiming balances the grid (one atomic per document is noise beside a
    // long document's merge), and an empty list costs one read per workgroup.
    __shared__ uint32_t claim;
    // the general path (not inlined) reads the parameter block from an LDS copy: a reference to
    // the kernel argument itself would copy it to the stack and route every read through scratch
    __shared__ SmallParams psh;
    const uint32_t nd = *p.n_deferred;
    if (tid == 0) { sh.ws_base = 0; sh.ws_size = 0; psh = p; }
#if HM_STAMPS
    if (tid <= HML_NSTAMP) hml_st[tid] = 0;
#endif
#if HML_KARG_RELOAD
    // the loop reads the launch parameters through an opaque pointer to the kernarg segment: a
    // document re-loads the fields it uses (scalar loads) rather than holding them in SGPRs
    // across the loop, where they were spilled to VGPR lanes (readlane / writelane VALU)
    typedef __attribute__((address_space(4))) const SmallParams KParams;
    KParams *kp = (KParams *)__builtin_amdgcn_kernarg_segment_ptr();
#endif
    for (;;) {
#if HML_KARG_RELOAD
        asm volatile("" : "+s"(kp));
        const SmallParams &p = *(const SmallParams *)kp;
#endif
        if (tid == 0) claim = atomicAdd(p.large_cursor, 1u);
        bsync();
        const uint32_t ci = claim;
        if (ci >= nd) break;
        const uint32_t d = p.deferred[ci];
        const hm_doc_row doc = p.docs[d];
        const uint32_t ds = hm_slot(p, d);
        int32_t H = 0;
#if HM_STAMPS
        { const u64 t0 = lstamp_now(); if (tid == 0) hml_st[HML_NSTAMP] = t0; }
#endif
        int rc = RES_FALLBACK;
        const uint32_t dn = doc.n_changes, dd = doc.n_deps;
        if (HML_RES && dn >= 1 && doc.n_actors <= 8 && doc.n_objs >= 1 && doc.n_objs <= LA_MAX && doc.n_ops < 65536 &&
            doc.n_regs + doc.n_objs < 32767 && 8 * (size_t)dn + 2 * (size_t)dd <= LARENA / 4)
            rc = merge_doc_res(p, sh, arena, doc, H);
        const bool via_res = rc != RES_FALLBACK;   // (every change ready on arrival: nothing queued)
        if (!via_res) {
            bsync();
            // the general path (not inlined) takes its row by reference: hand it a copy, so the
            // address that escapes is the copy's and `doc` itself stays in registers (its fields
            // were read from the stack through every phase of the all-LDS path)
            hm_doc_row doc_c;
            __builtin_memcpy(&doc_c, &doc, sizeof doc_c);
            asm volatile("" ::: "memory");
            rc = merge_doc_large(psh, sh, arena, doc_c, d, pool, pool_bytes, pool_used, H);
        }
        const Outcome oc = (Outcome)rc;
        bsync();
        hm_doc_result r = {};
        r.err_change = HM_NONE; r.err_op = HM_NONE;
        if (oc == LERR) {
            const u64 ek = sh.errkey;
            r.status = (int32_t)(ek & 0xFF);
            r.err_change = (uint32_t)((ek >> 8) & 0xFFFFF);
            const uint32_t opp1 = (uint32_t)((ek >> 28) & 0xFFFF);
            r.err_op = opp1 ? opp1 - 1 : HM_NONE;
            if (r.status == HM_ERR_UNSUPPORTED) { r.err_change = HM_NONE; r.err_op = HM_NONE; }
        } else if (oc == LUNSUP) {
            r.status = HM_ERR_UNSUPPORTED;
        } else {
            r.status = HM_OK;
            r.hist_len = (uint32_t)H;
            r.n_surv = sh.total;
            uint32_t q = 0;
            if (!via_res)
                for (uint32_t i = 0; i < doc.n_changes; i++) q += p.res_hist[doc.change_off + i] == -1 ? 1u : 0u;
            r.n_queued = q;
            bool ag = true, bg = true;
            for (uint32_t a = 0; a < S; a++) {
                const uint32_t bc = a < doc.n_actors ? sh.bclock[a] : 0u;
                const uint32_t mc = p.min_clock ? p.min_clock[(size_t)ds * S + a] : 0u;
                if (bc < mc) ag = false;
                if (mc < bc) bg = false;
            }
            r.min_cmp = p.min_clock ? ((ag && bg) ? 0u : (ag ? 1u : (bg ? 2u : 3u))) : 0u;
        }
        if (tid < S) {
            const bool ok = oc == LOK, ar = tid < doc.n_actors;
            p.res_clock[(size_t)ds * S + tid] = ok && ar ? sh.clock[tid] : 0u;
            p.res_heads[(size_t)ds * S + tid] = ok && ar ? sh.headv[tid] : 0u;
            p.res_back_clock[(size_t)ds * S + tid] = ok && ar ? sh.bclock[tid] : 0u;
        }
        if (tid == 0) p.res_docs[ds] = r;
        bsync();
    }
#if HM_STAMPS
    if (tid < HML_NSTAMP) atomicAdd(&hml_stamp_acc[tid], (unsigned long long)hml_st[tid]);
#endif
}

}  // namespace hml

size_t hm_large_scratch_bound(const hm_batch *b) {
    // linear upper bound of large_carve over every document (T <= 4n + 64 per doc)
    // (n_objs <= n_ops + 1 per document: objects are created by make ops)
    hml::Scratch s;
    const uint32_t A = b->a_stride;
    size_t per = hml::large_carve(0, b->n_changes, b->n_ops, b->n_regs, b->n_ops + b->n_docs, A,
                                  4 * b->n_changes + 64 * b->n_docs, &s);
    return per + (size_t)b->n_docs * 48 * 16 + (1u << 20);
}

#if HM_STAMPS
extern "C" int hm_debug_lstamps(unsigned long long *out, int n, int reset) {
    if (n > HML_NSTAMP) n = HML_NSTAMP;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hml::hml_stamp_acc), n * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[HML_NSTAMP] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hml::hml_stamp_acc), z, sizeof z) != hipSuccess) return -1;
    }
    return n;
}
#endif

// per-lane stack (spills) of merge_large_kernel: the engine raises the device stack limit when a
// build needs more than the runtime's default (a dispatch beyond the limit faults)
size_t hm_large_stack_bytes() {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&hml::merge_large_kernel)) != hipSuccess) return 0;
    return fa.localSizeBytes;
}

hipError_t hm_launch_large(const SmallParams &p, void *pool, size_t pool_bytes, unsigned long long *pool_used,
                           uint32_t grid, hipStream_t s) {
#ifndef HML_RESIDENT
#define HML_RESIDENT HML_WGS_PER_CU    // workgroups launched per CU (dev A/B builds launch fewer)
#endif
    hipLaunchKernelGGL(hml::merge_large_kernel, dim3(grid / 4 * HML_RESIDENT), dim3(LWG), 0, s, p, (uint8_t *)pool, (u64)pool_bytes, pool_used);
    return hipGetLastError();
}
