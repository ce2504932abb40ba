// merge_kernels.hip — CDNA4 (gfx950) kernels of the batched CRDT merge.
//
// merge_small_kernel: one wavefront per document ("small" envelope: <= 64
// changes, <= 8 actors, <= 64*OPL ops, registers/objects bounded by the
// launch's LDS carve).  Everything a document needs lives in registers and
// LDS; each input row is read from HBM once (coalesced) and each output row
// written once, so the kernel is HBM-bound.  No MFMA:
// nothing here is a dense contraction.
//
// Stages inside the wave (reference semantics in brackets; restated in
// SURVEY.md Appendix A from Automerge 0.12.2-beta.0 backend/op_set.js, which
// is not vendored — yarn.lock:178-185):
//
//  K1  causal readiness + history order      [addChange / applyQueuedOps / causallyReady]
//      fast path: every change is ready on arrival (first-arrival table in
//      LDS + one ballot) => history = arrival order minus duplicates;
//      slow path: exact emulation of the queue passes with wave-uniform
//      control (per-lane SWAR readiness, ballot, find-first after the cursor).
//  K1b transitive deps                       [transitiveDeps -> allDeps]
//      64-bit ancestor sets over history positions, built by a push in
//      history order (v_readlane of the finished lane, OR into dependents);
//      allDeps[c][a] = popcount(anc(c) & chain(a)) for a cold merge.
//  K1c clocks                                [opSet.clock, opSet.deps; DocBackend.updateClock
//                                             src/DocBackend.ts:135-142; Clock.cmp src/Clock.ts:27-38]
//  K2  map registers                         [applyAssign / updateMapKey]
//      survivors of (obj,key) = set/link ops whose change is not an ancestor
//      of any set/del/link on the register (LDS 64-bit OR per register);
//      order = actor rank descending; equal-actor ties (one change) follow the
//      flip of sortBy(actor).reverse() after every assign; counter `inc`s add
//      to the counter sets that are their ancestors (LDS int64 atomics).
//
// Errors are per document: the earliest (history position, op) error wins —
// the throw that would abort that document's Backend.applyChanges.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/hypermerge_amd.h"
#include "merge_kernels.h"

#ifndef HM_ABLATE
#define HM_ABLATE 0     // dev-only builds: stop (defer the doc) after a phase — 16 validate, 32 deps, 64 push,
                        // 2 K1b, 128 K2 scan, 4 K2 survivors, 256 rank;
                        // 8 stop right after staging
#endif
#ifndef HM_STAMPS
#define HM_STAMPS 0     // diagnostic builds only: per-phase s_memtime shares (tools/stamps.py); never timed
#endif
#define HM_NSTAMP 20
#ifndef HM_PREFETCH_EARLY
#define HM_PREFETCH_EARLY 0 // 1: the next document's rows are loaded before this document's merge
#endif
#ifndef HM_WAVES_PER_EU_OPL4
#define HM_WAVES_PER_EU_OPL4 3  // 256 ops per document: the op arrays need a larger register budget (measured:
                                // C2 0.87 -> 0.65 ms at 3 waves/SIMD; list launches (C5) best at 2: 3.99 -> 3.25 ms)
#endif
#ifndef HM_WAVES_PER_EU_LIST3
#define HM_WAVES_PER_EU_LIST3 3 // list launches of <= 192 ops per document: 168 VGPRs, no spill; K3's tables
                                // overlay the dead K1/K2 tables, so LDS holds 10 such waves per CU
#endif
// Wave priority (s_setprio) for the phases other waves should not hold up: the ancestor push
// (64 dependent readlane steps: a lower-priority wave's VALU issue fills its hazard gaps) and a
// wave's store / next-row staging (its memory requests go out sooner).  C4 A/B over priorities
// 0-3 (profiles/r02 commit log): 2.53 -> 2.43-2.44 ms with (2, 1).
#ifndef HM_PRIO_PUSH
#define HM_PRIO_PUSH 2
#endif
#ifndef HM_PRIO_IO
#define HM_PRIO_IO 1
#endif
#ifndef HM_PRIO_HIST
#define HM_PRIO_HIST 3      // through the queued-change history (K1 slow paths): actor-major C4 4.59 -> 4.34 ms (2), 4.20 ms (3)
#endif
#ifndef HM_PRIO_RANK
#define HM_PRIO_RANK 2      // through the survivor offsets, ranks and ties: C4 2.42 -> 2.39 ms
#endif
#ifndef HM_PRIO_FOLD
#define HM_PRIO_FOLD 0      // dev A/B: the push's priority held through the fold check and table init
#endif
#ifndef HM_PRIO_K3
#define HM_PRIO_K3 0        // dev A/B: priority through K3 (list order)
#endif
#ifndef HM_PRIO_K2
#define HM_PRIO_K2 2        // through the K2 op scan and survivor tests: C4 2.22 -> 2.16 ms, actor-major 3.32 -> 3.28, C5 0.630 -> 0.621 (r05 ab_prio2)
#endif
#ifndef HM_PUSH_BPERM
#define HM_PUSH_BPERM 0     // K1b's ancestor push broadcasts through ds_bpermute instead of v_readlane
#endif
#ifndef HM_KARG_RELOAD
#define HM_KARG_RELOAD 1    // merge_small_kernel: launch parameters re-read per document (see the kernel)
#endif
#ifndef HM_HIST_DP
#define HM_HIST_DP 1        // queued documents: history by the parallel (t, pass, pos) solve before the pass loop
#endif
#ifndef HM_HIST_REGS
#define HM_HIST_REGS 1      // ... iterated in registers (cross-lane reads) when every change has <= 4 dependency lanes
#endif
#ifndef HM_PRIO_K1
#define HM_PRIO_K1 3        // through validation and the dependency pre-pass: C4 2.41 -> 2.37 ms
#endif
#ifndef HM_FENCE_MCMP
#define HM_FENCE_MCMP 1     // pin Clock.cmp(DocBackend.clock, minimumClock) ahead of the next document's row loads
#endif
#ifndef HM_STAGE_FIRST
#define HM_STAGE_FIRST 0    // 1: stage the next document's rows before this document's stores (A/B: C4 2.38 -> 2.44 ms, the
                            // store outputs then waited in write_outputs on reused registers)
#endif
#ifndef HM_ASYNC_NEXT
#define HM_ASYNC_NEXT 1     // the next document's rows by inline-asm loads, waited for by a counted vmcnt that
                            // leaves this document's stores in flight (a compiler-counted load is waited for
                            // with vmcnt(0): the stores' count varies by path, so the staging waited for them)
#endif
#ifndef HM_ASYNC_MAX_OPL
#define HM_ASYNC_MAX_OPL 2  // instantiations (op rows per lane) that load the next document's rows by asm
#endif
#ifndef HM_ASYNC_STORES
#define HM_ASYNC_STORES 10  // store instructions an OK document's write_outputs issues at least (padded)
#endif
#ifndef HM_NT_OUT
#define HM_NT_OUT 0         // dev A/B: the output rows (allDeps, history, registers, survivors) as non-temporal stores
#endif
#ifndef HM_NT_IN
#define HM_NT_IN 0          // dev A/B: the next document's rows as non-temporal loads (read once)
#endif
#ifndef HM_ASYNC_CHECK
#define HM_ASYNC_CHECK 0    // check builds (libhmgpu_check.so): every asynchronously loaded set of rows is re-read
                            // with counted loads and compared (hm_debug_async_check counts the differences)
#endif
#ifndef HM_OPAQUE_LANE
#define HM_OPAQUE_LANE 1    // per-document lane index the compiler cannot hoist out of the document loop
#endif
#ifndef HM_WAVES_PER_EU
#define HM_WAVES_PER_EU 4   // register-allocator target: LDS already caps C4-class launches at ~4.25 waves/SIMD
#endif
#define WAVE 64
#define NA_MAX 8
#define NDEP_MAX 1024                // largest dep table a launch carves
typedef unsigned long long u64;
#if defined(__HIP_DEVICE_COMPILE__)
#define LDS __attribute__((address_space(3)))   // explicit LDS pointers -> ds_* (not flat_*) instructions
#else
#define LDS
#endif

namespace hm {

__device__ __forceinline__ u64 readlane64(u64 v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ u64 shfl64(u64 v, int src) {
    return ((u64)shfl32((uint32_t)(v >> 32), src) << 32) | shfl32((uint32_t)v, src);
}
__device__ __forceinline__ u64 wave_or64(u64 v) {
    for (int o = 1; o < WAVE; o <<= 1) v |= shfl64(v, (int)(threadIdx.x ^ o));
    return v;
}
// DPP lane moves (gfx9 encodings): lanes without a source read 0
#define DPP_ROW_SHR(n) (0x110 + (n))
#define DPP_WAVE_SHR1 0x138
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143
// exclusive prefix sum across the wave; *total = sum over all lanes.  Row-local shifts and
// the gfx9 row broadcasts (VALU only: no LDS round trip as a bpermute ladder would need).
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
    uint32_t x = v;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(1), 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(2), 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(4), 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(8), 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_BCAST15, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_BCAST31, 0xC, 0xF, false);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)x, WAVE - 1);
    return x - v;
}
// wave-wide max of a value (inclusive max-scan, last lane)
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    uint32_t x = v, y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(1), 0xF, 0xF, false); x = x > y ? x : y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(2), 0xF, 0xF, false); x = x > y ? x : y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(4), 0xF, 0xF, false); x = x > y ? x : y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_SHR(8), 0xF, 0xF, false); x = x > y ? x : y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_BCAST15, 0xA, 0xF, false); x = x > y ? x : y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, DPP_ROW_BCAST31, 0xC, 0xF, false); x = x > y ? x : y;
    return (uint32_t)__builtin_amdgcn_readlane((int)x, WAVE - 1);
}
// sum of the 8 bytes of a 64-bit word (v_sad_u8 against 0)
__device__ __forceinline__ uint32_t bytesum64(u64 x) {
    return __builtin_amdgcn_sad_u8((uint32_t)x, 0u, __builtin_amdgcn_sad_u8((uint32_t)(x >> 32), 0u, 0u));
}
// value of the previous lane (lane 0 reads 0)
__device__ __forceinline__ uint32_t prev_lane(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, DPP_WAVE_SHR1, 0xF, 0xF, false);
}
// The lane index as a value computed inside the document loop: lane-based LDS addresses built
// from threadIdx.x are loop-invariant, so the compiler hoists them out of the persistent loop and
// keeps them live across the whole merge — at 128 VGPRs one of them was spilled to scratch, and
// its reload (a global-latency round trip, s_waitcnt vmcnt(0)) sat in the survivor-offset scan
// of every document.  An address built from this value is recomputed where it is used.
__device__ __forceinline__ uint32_t fresh_lane() {
#if HM_OPAQUE_LANE
    uint32_t l;
    asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "v"((uint32_t)threadIdx.x));
    return l;
#else
    return threadIdx.x;
#endif
}
// One-wave workgroups: a wave's LDS instructions execute in issue order, so an exchange
// through LDS between lanes needs only a compiler ordering point — no s_waitcnt, no barrier
// (__syncthreads' workgroup fence would drain lgkmcnt at every exchange).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// error key: (history position, op index + 1, arrival index, code); the first throw is the min
__device__ __forceinline__ u64 err_key(uint32_t h, uint32_t op_plus1, uint32_t arr, uint32_t code) {
    return ((u64)h << 40) | ((u64)(op_plus1 & 0xFFFF) << 24) | ((u64)(arr & 0xFFFF) << 8) | code;
}

struct SmallLds {
    LDS u64 *anc, *chain, *segor, *errkey, *cov;
    LDS u64 *opval;                 // op values (staged with the rows: survivors and counters read them)
    LDS u64 *survpk;                // per register: survivor count per actor rank, one byte each
    LDS int64_t *survsum;           // counter launches only
    LDS uint32_t *first, *base, *bclock, *headv, *objslot, *segcnt, *survcnt, *regoff, *regobj, *insmin;
    LDS uint32_t *flags, *deps, *depinfo;
    LDS uint8_t *seglist;           // K3: visible flag per list position
    LDS uint16_t *survp;            // K3: visible elements before a position
    LDS uint32_t *opmeta;           // action | datatype << 8 | vtag << 16
    LDS uint32_t *opro;             // reg | obj << 16 (clamped to 0xFFFF: >= any carve)
    LDS uint32_t *opelem;           // ins element counter (list launches)
    LDS int32_t *hist_of;
    LDS uint16_t *survop, *opbase, *oppar;
    LDS uint8_t *h2a, *chactor, *objtype;
    LDS uint16_t *opchg;            // op -> arrival index of its change | actor rank << 8
    // K3 (RGA lists); carved only for launches with list documents
    LDS uint32_t *nins, *pcount, *nodekey, *tour0, *listbase;   // tour ranked in place
    LDS uint16_t *poff;
    LDS uint16_t *nodeop, *nodepi, *regnode, *plist, *fc, *ns, *listid;
    LDS u64 *stamps;                // HM_STAMPS builds: [HM_NSTAMP] cycle sums + last stamp
};
#define PAR_HEAD 0xFFFFu             // oppar of an insert after '_head'

// Size classes of the small kernel's carve (registers, objects, dep rows per document).
template <int CLS> struct SizeClass;
template <> struct SizeClass<0> { static constexpr uint32_t NR = 32, NO = 16, ND = 128; };
template <> struct SizeClass<1> { static constexpr uint32_t NR = 256, NO = 64, ND = 512; };
// nested map / list documents of a few dozen changes (C5: <= 108 registers, <= 20 objects): the
// class-1 carve would hold a list launch to 4 waves per CU (35.8 KB), this one to 6 (24.3 KB)
template <> struct SizeClass<2> { static constexpr uint32_t NR = 128, NO = 32, ND = 256; };

// LDS carve, identical for the host size query and the device pointers.  Sized per launch
// (ops, registers, objects, dep rows, lists, counters): LDS is what bounds the number of
// resident waves per CU, so nothing is carved that the launch's documents cannot use.
// The kernel instantiates it with compile-time sizes (a size class), so every LDS address
// folds into a ds_* immediate offset instead of occupying an SGPR.
// Two parts: the tables live until the outputs, then the tables no phase reads after K2
// (validation, readiness, history, ancestors, the op scan, survivor tests, ranks).  K3's
// tables (RGA order, list launches) overlay that second part, so a list launch costs the
// larger of the two, not their sum.
template <typename L_t, typename P>
__host__ __device__ inline size_t small_carve(P base, uint32_t NOp, uint32_t NR, uint32_t NO, uint32_t ND,
                                              bool lists, bool counters, L_t *L) {
    size_t o = 0;
#define TAKE(f, T, cnt) do { L->f = (decltype(L->f))(base + o); o = (o + (size_t)(cnt) * sizeof(T) + 15) & ~(size_t)15; } while (0)
    // ---- live through the outputs (and the counters pass) ----
    TAKE(anc, u64, 64);          TAKE(chain, u64, NA_MAX);     TAKE(opval, u64, NOp);
    TAKE(errkey, u64, 1);        TAKE(base, uint32_t, NA_MAX * 3);
    TAKE(survcnt, uint32_t, NR); TAKE(regoff, uint32_t, NR);   TAKE(regobj, uint32_t, NR);
    TAKE(insmin, uint32_t, NR);  TAKE(flags, uint32_t, 2);
    TAKE(opmeta, uint32_t, NOp); TAKE(opro, uint32_t, NOp);
    TAKE(survop, uint16_t, NOp); TAKE(chactor, uint8_t, 64);   TAKE(objtype, uint8_t, NO);
    if (lists) {
        TAKE(opelem, uint32_t, NOp);
        L->nodekey = L->opelem;                                    // opelem is dead after K2's op scan (K3 runs later)
        TAKE(nins, uint32_t, 1);
    }
    TAKE(stamps, u64, HM_STAMPS ? HM_NSTAMP + 1 : 0);
    // ---- tables no phase reads after K2 (the next document's staging refills deps / oppar only
    //      after this document's outputs).  K1's (first-arrival table, deps, dep lookups: dead
    //      after the fold check) and K2's (survivor tests and ranks: initialised after the fold
    //      check) share one region; K3's tables overlay the whole part ----
    const size_t dead_at = o;
    TAKE(hist_of, int32_t, 64);  TAKE(cov, u64, 1);            TAKE(opbase, uint16_t, 64);
    TAKE(oppar, uint16_t, NOp);  TAKE(h2a, uint8_t, 64);       TAKE(opchg, uint16_t, NOp);
    const size_t k1_at = o;
    TAKE(first, uint32_t, NA_MAX * 64);
    TAKE(deps, uint32_t, ND > NOp ? ND : NOp);                     // flags[1]: max n_deps
    TAKE(depinfo, uint32_t, ND);
    const size_t k1_end = o;
    o = k1_at;
    TAKE(segor, u64, NR);        TAKE(survpk, u64, NR);        TAKE(segcnt, uint32_t, NR);
    TAKE(objslot, uint32_t, NO);
    if (o < k1_end) o = k1_end;
    L->seglist = (decltype(L->seglist))L->first; L->survp = (decltype(L->survp))L->first;   // (K3's: below)
    if (lists) {
        const uint32_t NP = NR + NO, NE = 2 * (NOp + NO);
        size_t q = dead_at;
#define TAKEK(f, T, cnt) do { L->f = (decltype(L->f))(base + q); q = (q + (size_t)(cnt) * sizeof(T) + 15) & ~(size_t)15; } while (0)
        TAKEK(tour0, uint32_t, NE);     TAKEK(pcount, uint32_t, NP);  TAKEK(listbase, uint32_t, NO + 1);
        TAKEK(poff, uint16_t, NP + 1);  TAKEK(survp, uint16_t, NOp);
        TAKEK(nodeop, uint16_t, NOp);   TAKEK(nodepi, uint16_t, NOp); TAKEK(regnode, uint16_t, NR);
        TAKEK(plist, uint16_t, NOp);    TAKEK(fc, uint16_t, NP);      TAKEK(ns, uint16_t, NOp);
        TAKEK(listid, uint16_t, NO);    TAKEK(seglist, uint8_t, NOp);
#undef TAKEK
        if (q > o) o = q;
    }
    // last: the kernel carves with counters on, the host sizes the launch with the batch's flag
    TAKE(survsum, int64_t, counters ? NOp : 0);
#undef TAKE
    L->bclock = L->base + NA_MAX;
    L->headv = L->base + 2 * NA_MAX;
    return o;
}

template <typename T> struct Id { typedef T type; };
template <typename T> __device__ __forceinline__ T lds_or(LDS T *p, typename Id<T>::type v) { return __atomic_fetch_or(p, v, __ATOMIC_RELAXED); }
template <typename T> __device__ __forceinline__ T lds_min(LDS T *p, typename Id<T>::type v) { return __atomic_fetch_min(p, v, __ATOMIC_RELAXED); }
template <typename T> __device__ __forceinline__ T lds_max(LDS T *p, typename Id<T>::type v) { return __atomic_fetch_max(p, v, __ATOMIC_RELAXED); }
template <typename T> __device__ __forceinline__ T lds_add(LDS T *p, typename Id<T>::type v) { return __atomic_fetch_add(p, v, __ATOMIC_RELAXED); }

#if HM_STAMPS
__device__ unsigned long long hm_stamp_acc[HM_NSTAMP];
__device__ __forceinline__ u64 stamp_now() {
    u64 t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define STAMP(L_, i) do { const u64 t_ = stamp_now(); if (threadIdx.x == 0) { (L_).stamps[i] += t_ - (L_).stamps[HM_NSTAMP]; (L_).stamps[HM_NSTAMP] = t_; } } while (0)
#elif defined(HM_MARKS)
#define STAMP(L_, i) asm volatile(";HMMARK " #i)          // static instruction census by phase (dev tool)
#else
#define STAMP(L_, i) do { } while (0)
#endif

enum : uint32_t { FL_UNSUPPORTED = 1u };
enum Outcome { OUT_OK = 0, OUT_ERROR = 1, OUT_UNSUPPORTED = 2, OUT_INVALID = 3 };

// raise byte a of the 8-byte packed requirement (lo: actors 0-3, hi: 4-7) to at least v;
// selects only (a data-dependent reference would push lo/hi to scratch)
__device__ __forceinline__ void need_set(uint32_t &lo, uint32_t &hi, uint32_t a, uint32_t v) {
    const uint32_t sh = (a & 3) * 8;
    const uint32_t w = a < 4 ? lo : hi;
    const uint32_t cur = (w >> sh) & 0xFF;
    const uint32_t nw = v > cur ? ((w & ~(0xFFu << sh)) | (v << sh)) : w;
    lo = a < 4 ? nw : lo;
    hi = a < 4 ? hi : nw;
}


// the (actor, seq) table: NA_MAX x 64 words, slot-major (word s * NA_MAX + a for actor a's
// s-th seq of the batch window): the lanes of a 32-lane half look up (actor, slot) pairs of
// nearby arrivals — every actor at the same few slots — which an actor-major table (stride 64
// words, bank = slot mod 32) put on a handful of banks (4-way conflicts on C4's 8 x 8 logs)
__device__ __forceinline__ uint32_t fidx(uint32_t a, uint32_t s) { return (s & 63) * NA_MAX + (a & (NA_MAX - 1)); }
// all ones, two 16-byte stores per lane
__device__ __forceinline__ void clear_first(LDS uint32_t *first) {
    static_assert(NA_MAX * 64 == 2 * WAVE * 4, "first-table size");
    LDS uint4 *f4 = (LDS uint4 *)first;
    const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
    f4[threadIdx.x] = ones;
    f4[threadIdx.x + WAVE] = ones;
}

// tie order key of an assign at position p on its register: odd p first (p descending),
// then even p ascending ("append, then reverse" after every assign)
__device__ __forceinline__ uint32_t tie_order(uint32_t pc) { return (pc & 1) ? (0x10000u - pc) : (0x20000u + pc); }


// ---------------- K3: RGA document order (applyInsert, updateListElement, getPrevious) ----------------
// The applied `ins` ops of a list form a tree (parent = the elemId inserted after, or
// '_head'); siblings are ordered by lamportCompare (elem, actor) DESCENDING and the list
// is the pre-order of that tree restricted to visible elements (a non-empty survivor
// set).  Pre-order comes from an Euler tour ranked by pointer jumping in LDS.
// Writes the visible index of every element register into L.insmin (as int32, -1 hidden).
template <int OPL>
__device__ __forceinline__ void rga_order(const SmallLds &L, uint32_t R, uint32_t O,
                                          const uint32_t (&oreg)[OPL], const uint32_t (&oobj)[OPL],
                                          const uint32_t (&opar)[OPL], const uint32_t (&oact)[OPL],
                                          const uint32_t (&oelem)[OPL], const uint32_t (&oarr)[OPL],
                                          const int32_t (&oh)[OPL], uint32_t *epos) {
    const uint32_t lane = threadIdx.x;
    const uint32_t NP = R + O;
    constexpr uint32_t END = 0xFFFFu;
    for (uint32_t i = lane; i < NP; i += WAVE) { L.pcount[i] = 0; L.fc[i] = 0xFFFFu; }
    for (uint32_t i = lane; i < R; i += WAVE) L.regnode[i] = 0xFFFFu;
    if (lane == 0) *L.nins = 0;
    // compact ids of the list/text objects
    uint32_t nl = 0;
    for (uint32_t o0 = 0; o0 < O; o0 += WAVE) {
        const uint32_t o = o0 + lane;
        const uint32_t ot = o < O ? L.objtype[o] : 0xFFu;
        const bool isl = ot == HM_MAKE_LIST || ot == HM_MAKE_TEXT;
        const u64 mk = __ballot(isl);
        if (o < O) L.listid[o] = isl ? (uint16_t)(nl + __popcll(mk & ((1ull << lane) - 1))) : (uint16_t)0xFFFFu;
        nl += (uint32_t)__popcll(mk);
    }
    wave_sync();
    // nodes = applied ins ops
#pragma unroll
    for (int t = 0; t < OPL; t++) {
        if (oh[t] < 0 || oact[t] != HM_INS) continue;
        const uint32_t i = lds_add(L.nins, 1u);
        const uint32_t pi = opar[t] == HM_HEAD ? R + oobj[t] : opar[t];
        L.nodeop[i] = (uint16_t)(lane + WAVE * t);
        L.nodepi[i] = (uint16_t)pi;
        L.nodekey[i] = (oelem[t] << 8) | L.chactor[oarr[t]];
        L.regnode[oreg[t]] = (uint16_t)i;
        lds_add(&L.pcount[pi], 1u);
    }
    wave_sync();
    STAMP(L, 16);
    const uint32_t N = *L.nins;
    // children of every parent (CSR over parent slots: element registers, then list heads)
    uint32_t tot = 0;
    for (uint32_t r0 = 0; r0 < NP; r0 += WAVE) {
        const uint32_t r = r0 + lane;
        uint32_t tt;
        const uint32_t ex = wave_excl_scan(r < NP ? L.pcount[r] : 0u, &tt);
        if (r < NP) L.poff[r] = tot + ex;
        tot += tt;
    }
    if (lane == 0) L.poff[NP] = tot;
    wave_sync();
    for (uint32_t i = lane; i < N; i += WAVE) {
        const uint32_t pi = L.nodepi[i];
        L.plist[L.poff[pi] + lds_add(&L.pcount[pi], 0xFFFFFFFFu) - 1u] = (uint16_t)i;   // counts down to 0
    }
    wave_sync();
    // sibling order: next sibling = the largest smaller key; the largest key is the first child
    for (uint32_t i = lane; i < N; i += WAVE) {
        const uint32_t pi = L.nodepi[i], key = L.nodekey[i];
        const uint32_t q0 = L.poff[pi], qn = L.poff[pi + 1] - q0;
        uint32_t best = 0xFFFFu, bkey = 0;
        bool firstc = true;
        for (uint32_t q = 0; q < qn; q++) {
            const uint32_t j = L.plist[q0 + q], kj = L.nodekey[j];
            if (kj > key) firstc = false;
            else if (kj < key && (best == 0xFFFFu || kj > bkey)) { best = j; bkey = kj; }
        }
        L.ns[i] = (uint16_t)best;
        if (firstc) L.fc[pi] = (uint16_t)i;
    }
    wave_sync();
    STAMP(L, 17);
    // Euler tour: down(i) = 2i (value 1), up(i) = 2i+1; list head h = N + listid: 2h, 2h+1 (end)
    const uint32_t E = 2 * (N + nl);
    for (uint32_t i = lane; i < N; i += WAVE) {
        const uint32_t reg = (L.opro[L.nodeop[i]] & 0xFFFFu);
        const uint32_t hd = N + L.listid[L.regobj[reg]];
        const uint32_t f = L.fc[reg];
        const uint32_t sd = f != 0xFFFFu ? 2 * f : 2 * i + 1;
        const uint32_t pi = L.nodepi[i];
        const uint32_t su = L.ns[i] != 0xFFFFu ? 2u * L.ns[i] : (pi >= R ? 2 * hd + 1 : 2u * L.regnode[pi] + 1);
        L.tour0[2 * i] = (sd << 16) | 1u;
        L.tour0[2 * i + 1] = su << 16;
    }
    for (uint32_t o = lane; o < O; o += WAVE) {
        const uint32_t l = L.listid[o];
        if (l == 0xFFFFu) continue;
        const uint32_t h = N + l, f = L.fc[R + o];
        L.tour0[2 * h] = (f != 0xFFFFu ? 2 * f : 2 * h + 1) << 16;
        L.tour0[2 * h + 1] = END << 16;
    }
    wave_sync();
    // in-place pointer jumping, three hops per round: a word (link << 16 | sum up to the link) is
    // read and written whole, so every word is consistent at every moment, and links spanning
    // >= L entries when a round starts span >= 4L after it -> ceil(log4 E) rounds
    LDS uint32_t *cur = L.tour0;
    const uint32_t rounds = E ? (33 - __builtin_clz(E)) / 2 : 0;
    for (uint32_t rd = 0; rd < rounds; rd++) {
        for (uint32_t e = lane; e < E; e += WAVE) {
            const uint32_t x = cur[e];
            uint32_t nx = x >> 16, sum = x & 0xFFFFu;
#pragma unroll
            for (int hop = 0; hop < 3; hop++) {
                if (nx == END) break;
                const uint32_t y = cur[nx];
                sum += y & 0xFFFFu;
                nx = y >> 16;
            }
            cur[e] = (nx << 16) | sum;
        }
        wave_sync();
    }
    STAMP(L, 18);
    // list sizes -> base positions; pre-order position of every node
    uint32_t lb = 0;
    for (uint32_t l0 = 0; l0 < nl; l0 += WAVE) {
        const uint32_t l = l0 + lane;
        uint32_t tt;
        const uint32_t ex = wave_excl_scan(l < nl ? (cur[2 * (N + l)] & 0xFFFFu) : 0u, &tt);
        if (l < nl) L.listbase[l] = lb + ex;
        lb += tt;
    }
    wave_sync();
    for (uint32_t i = lane; i < N; i += WAVE) {
        const uint32_t reg = (L.opro[L.nodeop[i]] & 0xFFFFu);
        const uint32_t l = L.listid[L.regobj[reg]];
        const uint32_t total = cur[2 * (N + l)] & 0xFFFFu;
        const uint32_t pos = L.listbase[l] + total - (cur[2 * i] & 0xFFFFu);
        L.seglist[pos] = L.survcnt[reg] > 0 ? 1u : 0u;       // visible = non-empty survivor set
        L.nodekey[i] = pos;
        if (epos) epos[reg] = pos - L.listbase[l];
        L.insmin[reg] = 0xFFFFFFFFu;                          // -> list index (or -1)
    }
    wave_sync();
    uint32_t vc = 0;
    for (uint32_t q0 = 0; q0 < N; q0 += WAVE) {
        const uint32_t q = q0 + lane;
        uint32_t tt;
        const uint32_t ex = wave_excl_scan(q < N ? L.seglist[q] : 0u, &tt);
        if (q < N) L.survp[q] = vc + ex;
        vc += tt;
    }
    wave_sync();
    for (uint32_t i = lane; i < N; i += WAVE) {
        const uint32_t reg = (L.opro[L.nodeop[i]] & 0xFFFFu);
        const uint32_t pos = L.nodekey[i];
        if (L.seglist[pos]) {
            const uint32_t l = L.listid[L.regobj[reg]];
            const uint32_t first_pos = L.listbase[l];
            L.insmin[reg] = L.survp[pos] - (first_pos < N ? L.survp[first_pos] : vc);
        }
    }
    wave_sync();
    STAMP(L, 19);
}


// The literal-fold check reads only these tables (passed by value: taking the address of
// the whole SmallLds would push every LDS pointer to scratch).
struct FoldView {
    LDS u64 *anc, *chain;
    LDS uint32_t *first, *base, *deps;
    LDS int32_t *hist_of;
};
// FC(h)[x]: latest seq of actor x among change h's ancestors and itself (cold merge)
__device__ __forceinline__ uint32_t fc_of(FoldView L, uint32_t h, uint32_t x) {
    return (uint32_t)__popcll((L.anc[h] | (1ull << h)) & L.chain[x]);
}
// history position of the applied change (a, s) (s >= 1, in this batch)
__device__ __forceinline__ uint32_t hpos_of(FoldView L, uint32_t a, uint32_t s) {
    return (uint32_t)L.hist_of[L.first[fidx(a, (s - L.base[a]))]];
}
// Does the literal transitiveDeps fold differ from the closure for this change?
__device__ __noinline__ bool fold_differs(FoldView L, uint32_t dep0, uint32_t nd, uint32_t actor, uint32_t seq) {
    // entries of deps.set(actor, seq-1) in key order, seq 0 skipped (reduce ignores them)
    uint32_t ex[NA_MAX + 1], es[NA_MAX + 1], eh[NA_MAX + 1], k = 0;
    bool own = false;
    for (uint32_t j = 0; j < nd && k < NA_MAX; j++) {
        const uint32_t pk = L.deps[dep0 + j];
        uint32_t a = pk >> 24, sq = pk & 0xFFFFFF;
        if (a == actor) { sq = seq - 1; own = true; }
        if (sq == 0) continue;
        ex[k] = a; es[k] = sq; eh[k] = hpos_of(L, a, sq); k++;
    }
    if (!own && seq > 1) { ex[k] = actor; es[k] = seq - 1; eh[k] = hpos_of(L, actor, seq - 1); k++; }
    for (uint32_t j = 0; j < k; j++) {
        uint32_t before = 0, after = 0;
        for (uint32_t i = 0; i < k; i++) {
            if (i == j) continue;
            const uint32_t f = fc_of(L, eh[i], ex[j]);
            if (i < j) before = before > f ? before : f; else after = after > f ? after : f;
        }
        if (before > (es[j] > after ? es[j] : after)) return true;
    }
    return false;
}

// One document's input rows in flight.  They are loaded before the previous document's
// output stores (loads and stores share vmcnt on CDNA: loads issued first are not held up
// by the stores) and written to LDS after those stores, so nothing stays live across
// documents.  Named members only (no arrays): the struct is scalarised into VGPRs.
struct Rows {
    uint4 c01;                               // change row (lane < n_changes): words 0-3 ...
    uint2 c2;                                // ... and 4-5, held as the two loads fill them (a
                                             // row split over three 8-byte members needed register
                                             // moves inside the predicated load, i.e. a wait
                                             // for the load right after its issue)
    uint4 a0, b0, a1, b1, a2, b2, a3, b3;    // op rows lane + 64 t (first / second 16 B)
    uint2 d0, d1;                            // dep rows lane, lane + 64
};
// a document row is validated where its rows are first loaded (not where it is read: the
// next document's row is read a whole merge ahead); one whose ranges leave the tables
// becomes an empty row (ok = false)
__device__ __forceinline__ bool check_doc(const SmallParams &p, hm_doc_row &r) {
    const bool ok = hm_doc_row_ok(p, r);
    if (!ok) r = hm_doc_row{};
    return ok;
}
__device__ __forceinline__ void load_op(const SmallParams &p, const hm_doc_row &doc, uint32_t k, uint4 &a, uint4 &b) {
    a = make_uint4(0, 0, 0, 0); b = a;
    if (k < doc.n_ops) {
        const uint4 *src = reinterpret_cast<const uint4 *>(p.ops + doc.op_off + k);
        a = src[0]; b = src[1];
    }
}
template <int OPL>
__device__ __forceinline__ Rows load_rows(const SmallParams &p, const hm_doc_row &doc) {
    const uint32_t lane = threadIdx.x;
    Rows r;
    r.c01 = make_uint4(0, 0, 0, 0);
    r.c2 = r.d0 = r.d1 = make_uint2(0, 0);
    if (lane < doc.n_changes) {
        const uint2 *cs = reinterpret_cast<const uint2 *>(p.changes + doc.change_off + lane);
        const uint2 x0 = cs[0], x1 = cs[1];
        r.c01 = make_uint4(x0.x, x0.y, x1.x, x1.y); r.c2 = cs[2];
    }
    load_op(p, doc, lane, r.a0, r.b0);
    if (OPL > 1) load_op(p, doc, lane + WAVE, r.a1, r.b1);
    if (OPL > 2) load_op(p, doc, lane + 2 * WAVE, r.a2, r.b2);
    if (OPL > 3) load_op(p, doc, lane + 3 * WAVE, r.a3, r.b3);
    const hm_dep_row *dp = p.deps + doc.dep_off;
    if (lane < doc.n_deps) r.d0 = *reinterpret_cast<const uint2 *>(dp + lane);
    if (lane + WAVE < doc.n_deps) r.d1 = *reinterpret_cast<const uint2 *>(dp + lane + WAVE);
    return r;
}
#if HM_ASYNC_CHECK
__device__ unsigned long long hm_async_checked, hm_async_bad;
// the rows the counted loads return against the asynchronously loaded ones (lane-wise, every field)
template <int OPL>
__device__ __forceinline__ void async_check(const SmallParams &p, const hm_doc_row &doc, const Rows &got) {
    const Rows want = load_rows<OPL>(p, doc);
    auto ne4 = [](uint4 a, uint4 b) { return a.x != b.x || a.y != b.y || a.z != b.z || a.w != b.w; };
    auto ne2 = [](uint2 a, uint2 b) { return a.x != b.x || a.y != b.y; };
    bool bad = ne4(want.c01, got.c01) || ne2(want.c2, got.c2) || ne4(want.a0, got.a0) || ne4(want.b0, got.b0) ||
               ne2(want.d0, got.d0) || ne2(want.d1, got.d1);
    if (OPL > 1) bad = bad || ne4(want.a1, got.a1) || ne4(want.b1, got.b1);
    if (OPL > 2) bad = bad || ne4(want.a2, got.a2) || ne4(want.b2, got.b2);
    if (OPL > 3) bad = bad || ne4(want.a3, got.a3) || ne4(want.b3, got.b3);
    const unsigned long long m = __ballot(bad);
    if (threadIdx.x == 0) {
        atomicAdd(&hm_async_checked, 1ull);
        if (m) atomicAdd(&hm_async_bad, 1ull);
    }
}
#endif
#if HM_ASYNC_NEXT
// The next document's rows issued as inline-asm loads: hipcc does not count them, so the staging
// waits with an explicit vmcnt(N) — N the store instructions write_outputs is certain to issue
// after them on the path taken — instead of the vmcnt(0) a counted load gets, which also waited
// for every one of this document's stores.  Lanes past a table's rows re-load its last row (every
// address stays inside the document's range; a uniform branch skips an empty table) and are zeroed
// once the data is in.  The destinations are named "+v" by the wait statement, so no consumer is
// scheduled above it (cdna_hip_programming.md, 'What hipcc does not do' item 1, form ii).
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct AsyncRows { u32x2 c0, c1, c2; u32x4 a0, b0, a1, b1, a2, b2, a3, b3; u32x2 d0, d1; };
#if HM_NT_IN
#define HM_AL_POL " nt"
#else
#define HM_AL_POL ""
#endif
__device__ __forceinline__ u32x2 aload2(const void *p) {
    u32x2 v;
    asm volatile("global_load_dwordx2 %0, %1, off" HM_AL_POL : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ u32x4 aload4(const void *p) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" HM_AL_POL : "=v"(v) : "v"(p) : "memory");
    return v;
}
template <int OPL>
__device__ __forceinline__ AsyncRows load_rows_async(const SmallParams &p, const hm_doc_row &doc) {
    const uint32_t lane = threadIdx.x;
    AsyncRows r;
    r.c0 = r.c1 = r.c2 = r.d0 = r.d1 = u32x2{0u, 0u};
    r.a0 = r.b0 = r.a1 = r.b1 = r.a2 = r.b2 = r.a3 = r.b3 = u32x4{0u, 0u, 0u, 0u};
    if (doc.n_changes) {
        const uint32_t i = lane < doc.n_changes ? lane : doc.n_changes - 1u;
        const uint2 *cs = reinterpret_cast<const uint2 *>(p.changes + doc.change_off + i);
        r.c0 = aload2(cs); r.c1 = aload2(cs + 1); r.c2 = aload2(cs + 2);
    }
    if (doc.n_ops) {
        const uint32_t i0 = lane < doc.n_ops ? lane : doc.n_ops - 1u;
        const uint4 *o0 = reinterpret_cast<const uint4 *>(p.ops + doc.op_off + i0);
        r.a0 = aload4(o0); r.b0 = aload4(o0 + 1);
        if (OPL > 1) {
            const uint32_t i1 = lane + WAVE < doc.n_ops ? lane + WAVE : doc.n_ops - 1u;
            const uint4 *o1 = reinterpret_cast<const uint4 *>(p.ops + doc.op_off + i1);
            r.a1 = aload4(o1); r.b1 = aload4(o1 + 1);
        }
        if (OPL > 2) {
            const uint32_t i2 = lane + 2 * WAVE < doc.n_ops ? lane + 2 * WAVE : doc.n_ops - 1u;
            const uint4 *o2 = reinterpret_cast<const uint4 *>(p.ops + doc.op_off + i2);
            r.a2 = aload4(o2); r.b2 = aload4(o2 + 1);
        }
        if (OPL > 3) {
            const uint32_t i3 = lane + 3 * WAVE < doc.n_ops ? lane + 3 * WAVE : doc.n_ops - 1u;
            const uint4 *o3 = reinterpret_cast<const uint4 *>(p.ops + doc.op_off + i3);
            r.a3 = aload4(o3); r.b3 = aload4(o3 + 1);
        }
    }
    if (doc.n_deps) {
        const uint32_t i0 = lane < doc.n_deps ? lane : doc.n_deps - 1u, i1 = lane + WAVE < doc.n_deps ? lane + WAVE : doc.n_deps - 1u;
        r.d0 = aload2(p.deps + doc.dep_off + i0); r.d1 = aload2(p.deps + doc.dep_off + i1);
    }
    return r;
}
// the wait (see above) and the rows as load_rows returns them: write_outputs padded an OK
// document's stores to at least HM_ASYNC_STORES instructions after the loads (pad_stores), so
// one fixed wait leaves every one of them in flight; other outcomes wait for everything.  (One
// asm statement: a wait chosen at run time would merge register values after it, and the copies
// the compiler may then place ahead of the wait read the destinations before the data lands.)
template <int OPL>
__device__ __forceinline__ Rows take_rows_async(AsyncRows &r, const hm_doc_row &doc, bool padded) {
    // (the statement names only the destinations this instantiation loads: a pinned unused one
    // costs a register across write_outputs)
#define HM_AW2 "+v"(r.c0), "+v"(r.c1), "+v"(r.c2), "+v"(r.a0), "+v"(r.b0), "+v"(r.a1), "+v"(r.b1), "+v"(r.d0), "+v"(r.d1)
#define HM_AW3 HM_AW2, "+v"(r.a2), "+v"(r.b2)
#define HM_AW4 HM_AW3, "+v"(r.a3), "+v"(r.b3)
    if constexpr (OPL <= 2) {
        if (padded) asm volatile("s_waitcnt vmcnt(%9)" : HM_AW2 : "n"(HM_ASYNC_STORES) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" : HM_AW2 :: "memory");
    } else if constexpr (OPL == 3) {
        if (padded) asm volatile("s_waitcnt vmcnt(%11)" : HM_AW3 : "n"(HM_ASYNC_STORES) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" : HM_AW3 :: "memory");
    } else {
        if (padded) asm volatile("s_waitcnt vmcnt(%13)" : HM_AW4 : "n"(HM_ASYNC_STORES) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" : HM_AW4 :: "memory");
    }
#undef HM_AW4
#undef HM_AW3
#undef HM_AW2
    const uint32_t lane = threadIdx.x;
    Rows o;
    const bool c = lane < doc.n_changes, k0 = lane < doc.n_ops, k1 = lane + WAVE < doc.n_ops;
    o.c01 = c ? make_uint4(r.c0.x, r.c0.y, r.c1.x, r.c1.y) : make_uint4(0u, 0u, 0u, 0u);
    o.c2 = c ? make_uint2(r.c2.x, r.c2.y) : make_uint2(0u, 0u);
    o.a0 = k0 ? make_uint4(r.a0.x, r.a0.y, r.a0.z, r.a0.w) : make_uint4(0u, 0u, 0u, 0u);
    o.b0 = k0 ? make_uint4(r.b0.x, r.b0.y, r.b0.z, r.b0.w) : make_uint4(0u, 0u, 0u, 0u);
    o.a1 = k1 ? make_uint4(r.a1.x, r.a1.y, r.a1.z, r.a1.w) : make_uint4(0u, 0u, 0u, 0u);
    o.b1 = k1 ? make_uint4(r.b1.x, r.b1.y, r.b1.z, r.b1.w) : make_uint4(0u, 0u, 0u, 0u);
    const bool k2 = lane + 2 * WAVE < doc.n_ops, k3 = lane + 3 * WAVE < doc.n_ops;
    o.a2 = k2 ? make_uint4(r.a2.x, r.a2.y, r.a2.z, r.a2.w) : make_uint4(0u, 0u, 0u, 0u);
    o.b2 = k2 ? make_uint4(r.b2.x, r.b2.y, r.b2.z, r.b2.w) : make_uint4(0u, 0u, 0u, 0u);
    o.a3 = k3 ? make_uint4(r.a3.x, r.a3.y, r.a3.z, r.a3.w) : make_uint4(0u, 0u, 0u, 0u);
    o.b3 = k3 ? make_uint4(r.b3.x, r.b3.y, r.b3.z, r.b3.w) : make_uint4(0u, 0u, 0u, 0u);
    o.d0 = lane < doc.n_deps ? make_uint2(r.d0.x, r.d0.y) : make_uint2(0u, 0u);
    o.d1 = lane + WAVE < doc.n_deps ? make_uint2(r.d1.x, r.d1.y) : make_uint2(0u, 0u);
    return o;
}
#endif
// an op's 8-byte value, staged in LDS with its row (an L2 re-read would put a global-load
// round trip on the output phase's critical path)
__device__ __forceinline__ u64 op_value(const SmallLds &L, uint32_t k) { return L.opval[k]; }
// dep row -> actor << 24 | seq (all ones: outside the envelope)
__device__ __forceinline__ uint32_t pack_dep(uint2 w) {
    const uint32_t a = w.x & 0xFFFF;
    return (w.y < (1u << 24) && a < 256) ? ((a << 24) | w.y) : 0xFFFFFFFFu;
}
template <bool LISTS>
__device__ __forceinline__ void stage_op(const SmallLds &L, uint32_t k, uint32_t m, uint4 a, uint4 b) {
    if (k >= m) return;
    // a = (obj, reg, parent, elem); b = (action | datatype << 8 | vtag << 16, key, value lo, value hi)
    const uint32_t obj = a.x < 0xFFFFu ? a.x : 0xFFFFu, reg = a.y < 0xFFFFu ? a.y : 0xFFFFu;
    L.opro[k] = reg | (obj << 16);
    L.oppar[k] = (uint16_t)(a.z == HM_HEAD ? PAR_HEAD : (a.z < 0xFFFEu ? a.z : 0xFFFEu));
    L.opmeta[k] = b.x & 0xFFFFFFu;
    L.opval[k] = ((u64)b.w << 32) | b.z;
    if (LISTS) L.opelem[k] = a.w;
}
template <int OPL, bool LISTS>
__device__ __forceinline__ void stage_rows(const SmallParams &p, const SmallLds &L, const hm_doc_row &doc, const Rows &r,
                                           uint32_t cap_deps) {
    const uint32_t lane = threadIdx.x, m = doc.n_ops;
    stage_op<LISTS>(L, lane, m, r.a0, r.b0);
    if (OPL > 1) stage_op<LISTS>(L, lane + WAVE, m, r.a1, r.b1);
    if (OPL > 2) stage_op<LISTS>(L, lane + 2 * WAVE, m, r.a2, r.b2);
    if (OPL > 3) stage_op<LISTS>(L, lane + 3 * WAVE, m, r.a3, r.b3);
    const uint32_t nd = doc.n_deps < cap_deps ? doc.n_deps : cap_deps;
    if (lane < nd) L.deps[lane] = pack_dep(r.d0);
    if (lane + WAVE < nd) L.deps[lane + WAVE] = pack_dep(r.d1);
    for (uint32_t i = lane + 2 * WAVE; i < nd; i += WAVE)     // long dep tables: read on demand
        L.deps[i] = pack_dep(*reinterpret_cast<const uint2 *>(p.deps + doc.dep_off + i));
}
__device__ __forceinline__ hm_change_row change_of(uint2 w0, uint2 w1, uint2 w2) {
    hm_change_row c;
    c.actor = (uint16_t)(w0.x & 0xFFFF); c.n_deps = (uint16_t)(w0.x >> 16); c.seq = w0.y;
    c.dep_off = w1.x; c.n_ops = w1.y; c.op_first = w2.x; c.content_id = w2.y;
    return c;
}
// what the output phase needs besides LDS
struct DocState {
    int32_t hist;             // per arrival lane
    uint32_t H, total;
    bool doc_lists;
};

// Per-op checks of K2 against the document's objects / elements: the first throw kind of the
// op (0 none; ordered as the reference checks them: unknown object, then duplicate or
// missing list element), whether a set/link survives, whether it touches a list, and whether
// it is an insert after an element not inserted yet (Automerge accepts it; whether a later set
// throws depends on the whole insertion chain, which merge_large_kernel climbs: the document
// is deferred).  Reads only LDS (K2's tables), so the rare error-key pass can recompute it
// instead of keeping it live.
struct OpCheck { uint32_t err; bool surv, has_list, late; };
__device__ __forceinline__ OpCheck op_check(const SmallLds &L, int32_t ohv, uint32_t act, uint32_t obj, uint32_t reg,
                                            uint32_t par, uint32_t okey, uint32_t R, uint32_t O) {
    const bool asg = ohv >= 0 && act >= HM_INS && act <= HM_INC && reg < R;
    const uint32_t oi = obj < O ? obj : 0u, ri = reg < R ? reg : 0u;
    const uint32_t pi = par < R ? par : 0u;
    const uint32_t os = obj < O ? L.objslot[oi] : 0xFFFFFFFFu;
    const uint32_t ot = L.objtype[oi], im = L.insmin[ri], ip = L.insmin[pi];
    const u64 so = L.segor[ri];
    const uint32_t h = ohv < 0 ? 0u : (uint32_t)ohv;
    const bool unknown = asg && (os == 0xFFFFFFFFu || os > okey);     // 'Modification of unknown object'
    const bool known = asg && !unknown;
    const bool is_list = ot == HM_MAKE_LIST || ot == HM_MAKE_TEXT;
    const bool ins = known && act == HM_INS;
    const bool sl = known && (act == HM_SET || act == HM_LINK);
    OpCheck r;
    r.has_list = ins || (known && is_list);
    r.surv = sl && !((so >> h) & 1);
    r.late = ins && par != HM_HEAD && !(ip <= okey);
    // (history, op) keys are shared by an op's checks, so the earliest code of one op wins:
    // unknown object < duplicate element < missing element
    uint32_t e = 0;
    if (sl && is_list && !(im <= okey)) e = HM_ERR_MISSING_ELEM;            // 'Missing index entry for list element'
    if (ins && im != okey + 1) e = HM_ERR_DUPLICATE_ELEM;                   // 'Duplicate list element ID'
    if (unknown) e = HM_ERR_UNKNOWN_OBJECT;
    r.err = e;
    return r;
}

// Merge one document with the whole wave (no global stores).  Every return is wave-uniform.
template <int OPL, bool LISTS>
__device__ __forceinline__ Outcome merge_doc_small(const SmallParams &p, const SmallLds &L, const hm_doc_row &doc,
                                                   const uint2 w0, const uint2 w1, const uint2 w2, DocState &st) {
    const uint32_t lane = threadIdx.x;
    const uint32_t n = doc.n_changes, A = doc.n_actors, m = doc.n_ops, R = doc.n_regs, O = doc.n_objs;
    st.hist = -1; st.H = 0; st.total = 0; st.doc_lists = false;

    // ---------------- the staged rows (lane = arrival index) ----------------
    if (HM_ABLATE & 8) return OUT_UNSUPPORTED;
    STAMP(L, 0);
    if (HM_PRIO_K1) __builtin_amdgcn_s_setprio(HM_PRIO_K1);
    const bool act = lane < n;
    const hm_change_row c = change_of(w0, w1, w2);      // zero rows for lanes >= n (load_rows)
    clear_first(L.first);
    if (lane < NA_MAX) { L.base[lane] = 0xFFFFFFFFu; L.bclock[lane] = 0; L.headv[lane] = 0; L.chain[lane] = 0; }
    if (lane == 0) { *L.errkey = ~0ull; L.flags[0] = 0; L.flags[1] = 0; *L.cov = 0; }
    const uint32_t dep_lo = doc.dep_off, ndep = doc.n_deps;
    wave_sync();
    const uint32_t actor = c.actor, seq = c.seq;
    const uint32_t my_dep0 = c.dep_off - dep_lo;
    // layout contract (include/hypermerge_amd.h): op and dep rows are grouped by change in
    // arrival order without gaps; anything else leaves the envelope
    const uint32_t op_end = c.op_first + c.n_ops, dep_end = c.dep_off + c.n_deps;
    const uint32_t prev_op = prev_lane(op_end), prev_dep = prev_lane(dep_end);
    bool bad = (n == 0 && (m || ndep)) ||
               (act && (c.op_first != (lane ? prev_op : doc.op_off) || c.dep_off != (lane ? prev_dep : dep_lo) ||
                        (lane == n - 1 && (op_end != doc.op_off + m || dep_end != dep_lo + ndep))));
    // predicated (no per-lane branches): neutral operands for lanes that must not update
    const bool rowok = act && !(actor >= A || seq == 0 || c.dep_off < dep_lo || my_dep0 + c.n_deps > ndep);
    bad |= act && !rowok;
    bad |= act && (c.op_first < doc.op_off || c.op_first - doc.op_off + c.n_ops > m);
    const uint32_t a8 = actor & (NA_MAX - 1);
    lds_min(&L.base[a8], rowok ? seq : 0xFFFFFFFFu);
    lds_max(&L.bclock[a8], rowok ? seq : 0u);
    L.chactor[lane] = (uint8_t)actor;
    L.opbase[lane] = (uint16_t)(c.op_first - doc.op_off);
    if (__ballot(bad)) return OUT_UNSUPPORTED;
    wave_sync();
    const uint32_t mybase = act ? L.base[a8] : 0;
    const uint32_t slot = seq - mybase;
    if (__ballot(act && slot >= 64)) return OUT_UNSUPPORTED;
    lds_min(&L.first[fidx(a8, (slot & 63))], act ? lane : 0xFFFFFFFFu);
    {
        const uint32_t o0 = c.op_first - doc.op_off;       // ops -> arrival index of their change
        if (act) for (uint32_t j = 0; j < c.n_ops; j++) L.opchg[o0 + j] = (uint16_t)(lane | (a8 << 8));
    }
    wave_sync();

    STAMP(L, 1);
    if (HM_ABLATE & 16) return OUT_UNSUPPORTED;
    // Every dep row at once: its lookups (the actor's base seq, then the first-arrival table)
    // are done per row here, so the per-change loop below reads one LDS word per dep.
    //   depinfo = first-arrival lane (bits 0-6, 0x7F none) | (s - base + 1) << 8 (0x7F outside
    //             the batch's window of that actor, 0 for seq 0) | actor << 16
    {
        bool bad_dep = false;
        for (uint32_t i = lane; i < ndep; i += WAVE) {
            const uint32_t pk = L.deps[i];
            const uint32_t a = pk >> 24, s = pk & 0xFFFFFF;
            bad_dep |= pk == 0xFFFFFFFFu || a >= A;
            const uint32_t ad = a & (NA_MAX - 1);
            const uint32_t b = L.base[ad];
            const bool inwin = b != 0xFFFFFFFFu && s >= b && s - b < 64;
            const uint32_t f = L.first[fidx(ad, ((s - b) & 63))];
            const uint32_t rel = s == 0 ? 0u : (inwin ? s - b + 1 : 0x7Fu);
            L.depinfo[i] = (inwin && f < 64 ? f : 0x7Fu) | (rel << 8) | (ad << 16);
        }
        if (__ballot(bad_dep)) return OUT_UNSUPPORTED;
    }
    const uint32_t first_me = act ? L.first[fidx(actor, slot)] : lane;
    const bool dup = act && first_me != lane;
    const uint32_t cid_first = shfl32(c.content_id, (int)(first_me & 63));
    u64 dmask = 0;                       // direct deps in arrival-index space (fast path)
    uint32_t pred_arr = 0xFFu;
    bool ok = true;                      // ready on arrival
    bool own_row = false;                // the deps map lists the change's own actor
    wave_sync();
    {
        // predicated over the wave's longest deps map, 2 deps per round (reads in flight together)
        const uint32_t maxd = wave_max(act ? (uint32_t)c.n_deps : 0u);
        for (uint32_t j0 = 0; j0 < maxd; j0 += 2) {
            uint32_t inf[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const bool live = act && j0 + u < c.n_deps;
                inf[u] = L.depinfo[live ? my_dep0 + j0 + u : 0u];
            }
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const bool live = act && j0 + u < c.n_deps;
                const uint32_t a = (inf[u] >> 16) & (NA_MAX - 1), rel = (inf[u] >> 8) & 0x7F, f = inf[u] & 0x7F;
                own_row |= live && a == actor;
                const bool use = live && a != actor && rel != 0;                // deps.set(actor, seq-1) overrides
                ok = ok && !(use && (rel == 0x7F || f >= lane));
                dmask |= (use && rel != 0x7F && f < lane) ? (1ull << f) : 0ull;
            }
        }
        const uint32_t ps = seq - 1;
        const bool hp = act && ps != 0, inb = ps >= mybase;
        const uint32_t f = L.first[fidx(a8, ((ps - mybase) & 63))];
        ok = ok && !(hp && (!inb || f >= lane));
        const bool pv = hp && inb && f < lane;
        dmask |= pv ? (1ull << (f & 63)) : 0ull;
        pred_arr = pv ? f : pred_arr;
        ok = ok && !(dup && cid_first != c.content_id);                  // mismatched duplicate: exact path
    }
    wave_sync();

    STAMP(L, 2);
    if (HM_ABLATE & 32) return OUT_UNSUPPORTED;
    int32_t hist = -1;
    uint32_t H = 0;
    bool identity = false;                // history == arrival order (no queueing, no duplicates)
    if (HM_PRIO_K1) __builtin_amdgcn_s_setprio(0);
    const bool queued_doc = __ballot(act && !ok) != 0;
    if (HM_PRIO_HIST && queued_doc) __builtin_amdgcn_s_setprio(HM_PRIO_HIST);
    if (!queued_doc) {
        // every change was ready on arrival: history = arrival order minus duplicates
        const u64 appl = __ballot(act && !dup);
        if (act) hist = dup ? -2 : (int32_t)__popcll(appl & ((1ull << lane) - 1));
        H = (uint32_t)__popcll(appl);
        identity = __ballot(dup) == 0;
    } else if (__ballot(dup && cid_first != c.content_id) == 0) {
        // ---- addChange / applyQueuedOps, a pass at a time (no mismatched duplicates, so every
        // dep is met by its first arrival and a duplicate is ready with its original) ----
        // The queue is arrival order.  After an arrival, pass 1 can only apply it (the queue was
        // at a fixpoint); each further pass applies, in queue order, every queued change whose
        // deps were met before the pass or by an earlier change of the same pass: that set is a
        // fixpoint of one ballot per dependency level.  Duplicates are removed as no-ops.
        // A duplicate copy stands for its (actor, seq) if it is the first copy applied (its
        // original may still wait in the queue): applied-ness is tracked per key = the first
        // arrival's lane.  Documents without duplicates skip the per-copy loops.
        // every dep's first-arrival lane (dall) and whether the batch can satisfy them all
        u64 dall = 0;
        bool never = false;
        uint32_t pred_any = 0xFFu;
        {
            const uint32_t maxd = wave_max(act ? (uint32_t)c.n_deps : 0u);
            for (uint32_t j = 0; j < maxd; j++) {
                const bool live = act && j < c.n_deps;
                const uint32_t inf = L.depinfo[live ? my_dep0 + j : 0u];
                const uint32_t a = (inf >> 16) & (NA_MAX - 1), rel = (inf >> 8) & 0x7F, f = inf & 0x7F;
                const bool use = live && a != actor && rel != 0;
                never |= use && (rel == 0x7F || f == 0x7F);
                dall |= (use && rel != 0x7F && f != 0x7F) ? (1ull << f) : 0ull;
            }
            const uint32_t ps = seq - 1;
            const bool hp = act && ps != 0, inb = ps >= mybase;
            const uint32_t f = L.first[fidx(a8, ((ps - mybase) & 63))];
            never |= hp && (!inb || f >= 64);
            dall |= (hp && inb && f < 64) ? (1ull << f) : 0ull;
            pred_any = (hp && inb && f < 64) ? f : 0xFFu;
        }
        const u64 dupm = __ballot(dup), nodupm = __ballot(act && !dup);
        const u64 below = (1ull << lane) - 1;
        const uint32_t key = first_me & 63;
        u64 applied = 0, queue = 0;                       // applied keys; queued lanes
        bool copy_applied = false;                        // a duplicate copy stands for its key
        bool solved = false;
        if (HM_HIST_DP) {
            // Every change's place in history in parallel, per (actor, seq) key (its first
            // arrival's lane; copies of a key have equal content, hence equal deps).  The arrival
            // whose processing applies key K is t(K) = max(first arrival of K, t(deps)) = the
            // latest first arrival among K and its ancestors (never for a key that cannot apply).
            // Within that processing the arrival itself applies in pass 1 (it is last in the
            // queue); otherwise the queued copy c of K (arrived before t(K)) can apply in pass
            // p(c) = max(2, pass(D) + [D's applied copy after c in the queue]) over the deps D
            // applied by the same arrival, and the copy that applies is the first one a pass
            // reaches: (pass, pos)(K) = min over copies of (p(c), c).  The other copies are
            // duplicate no-ops.  History = applied copies ordered by (t, pass, pos).  The result is
            // checked (every dep ordered before its dependent; a dependency cycle fails the
            // check) and the pass loop below runs otherwise.
            LDS uint32_t *tx = (LDS uint32_t *)L.hist_of;           // free until K1b
            LDS uint32_t *tm = (LDS uint32_t *)L.anc;               // (free until K1b) copy minima
            const uint32_t INF = 0xFFu;
            const bool has_dup = dupm != 0;
            const bool kl = act && !dup;                            // this lane is its key's first arrival
            uint32_t t = (!kl || never) ? INF : lane;
            // Documents whose changes have at most 4 dependency lanes each (C4 / C5: at most 2
            // deps and the predecessor) iterate in registers: the lanes a change reads are fixed,
            // so each round is 4 cross-lane reads (ds_bpermute) and a ballot, with no LDS round
            // trip (the copies of a duplicated key still meet in LDS for their minimum).
            const bool regdp = HM_HIST_REGS && __ballot(act && __popcll(dall) > 4) == 0;
            uint32_t sl0 = lane, sl1 = lane, sl2 = lane, sl3 = lane;
            if (regdp) {
                u64 m = dall;
                sl0 = m ? (uint32_t)__builtin_ctzll(m) : lane; m &= m - 1;
                sl1 = m ? (uint32_t)__builtin_ctzll(m) : lane; m &= m - 1;
                sl2 = m ? (uint32_t)__builtin_ctzll(m) : lane; m &= m - 1;
                sl3 = m ? (uint32_t)__builtin_ctzll(m) : lane;
                for (uint32_t it = 0; it <= n; it++) {
                    const uint32_t x0 = shfl32(t, (int)sl0), x1 = shfl32(t, (int)sl1);
                    const uint32_t x2 = shfl32(t, (int)sl2), x3 = shfl32(t, (int)sl3);
                    uint32_t nt = t;
                    nt = nt > x0 ? nt : x0; nt = nt > x1 ? nt : x1; nt = nt > x2 ? nt : x2; nt = nt > x3 ? nt : x3;
                    nt = (kl && t != INF) ? nt : t;
                    const bool grew = nt != t;
                    t = nt;
                    if (__ballot(grew) == 0) break;
                }
            } else {
                for (uint32_t it = 0; it <= n; it++) {
                    tx[lane] = t;
                    wave_sync();
                    uint32_t nt = t;
                    if (kl && t != INF)
                        for (u64 m = dall; m; m &= m - 1) { const uint32_t x = tx[__builtin_ctzll(m)]; nt = nt > x ? nt : x; }
                    wave_sync();
                    const bool grew = nt != t;
                    t = nt;
                    if (__ballot(grew) == 0) break;
                }
            }
            STAMP(L, 13);
            // every copy learns its key's t; key word = t << 16 | pass << 8 | pos
            tx[lane] = t;
            wave_sync();
            const uint32_t tk = act ? tx[key] : INF;
            wave_sync();
            uint32_t w = (!kl || t == INF) ? 0xFFFFFFFFu : ((t << 16) | ((t == lane ? 1u : 2u) << 8) | lane);
            bool conv = false;
            if (regdp) {
                const bool queued_copy = act && tk != INF && tk != key && lane < tk;
                const uint32_t nsl = (uint32_t)__popcll(dall);
                for (uint32_t it = 0; it <= n + 1; it++) {
                    const uint32_t y0 = shfl32(w, (int)sl0), y1 = shfl32(w, (int)sl1);
                    const uint32_t y2 = shfl32(w, (int)sl2), y3 = shfl32(w, (int)sl3);
                    uint32_t pc = 2;
                    auto fold = [&](uint32_t wd, uint32_t k) {
                        const uint32_t v = ((wd >> 8) & 0xFFu) + ((wd & 0xFFu) > lane ? 1u : 0u);
                        pc = (k < nsl && (wd >> 16) == tk && v > pc) ? v : pc;
                    };
                    fold(y0, 0); fold(y1, 1); fold(y2, 2); fold(y3, 3);
                    const uint32_t cand = queued_copy ? ((tk << 16) | ((pc > 0xFEu ? 0xFEu : pc) << 8) | lane) : 0xFFFFFFFFu;
                    uint32_t nw = w;
                    if (has_dup) {                                  // the first copy a pass reaches applies
                        tm[lane] = 0xFFFFFFFFu;
                        wave_sync();
                        if (cand != 0xFFFFFFFFu) lds_min(&tm[key], cand);
                        wave_sync();
                        if (kl && t != INF && t != lane) nw = tm[lane];
                    } else if (kl && t != INF && t != lane) nw = cand;
                    const bool grew = nw != w;
                    w = nw;
                    if (__ballot(grew) == 0) { conv = true; break; }
                }
            }
            for (uint32_t it = 0; !regdp && it <= n + 1; it++) {
                tx[lane] = w;                                       // meaningful on key lanes
                if (has_dup) tm[lane] = 0xFFFFFFFFu;
                wave_sync();
                uint32_t cand = 0xFFFFFFFFu;
                if (act && tk != INF && tk != key && lane < tk) {   // a queued copy of a queued key
                    uint32_t pc = 2;
                    for (u64 m = dall; m; m &= m - 1) {
                        const uint32_t wd = tx[__builtin_ctzll(m)];
                        if ((wd >> 16) == tk) {
                            const uint32_t v = ((wd >> 8) & 0xFFu) + ((wd & 0xFFu) > lane ? 1u : 0u);
                            pc = pc > v ? pc : v;
                        }
                    }
                    cand = (tk << 16) | ((pc > 0xFEu ? 0xFEu : pc) << 8) | lane;
                }
                wave_sync();
                uint32_t nw = w;
                if (has_dup) {
                    if (cand != 0xFFFFFFFFu) lds_min(&tm[key], cand);
                    wave_sync();
                    if (kl && t != INF && t != lane) nw = tm[lane];
                } else if (kl && t != INF && t != lane) nw = cand;
                const bool grew = nw != w;
                w = nw;
                if (__ballot(grew) == 0) { conv = true; break; }
            }
            STAMP(L, 14);
            tx[lane] = w;
            wave_sync();
            const uint32_t wk = act && tk != INF ? tx[key] : 0xFFFFFFFFu;
            const bool apl = wk != 0xFFFFFFFFu && (wk & 0xFFu) == lane;
            const uint32_t hk = apl ? wk : 0xFFFFFFFFu;
            // check: every dep of an applied copy is applied before it
            bool bad = false;
            if (apl)
                for (u64 m = dall; m; m &= m - 1) bad |= tx[__builtin_ctzll(m)] >= hk;
            wave_sync();
            if (conv && __ballot(bad) == 0) {
                // rank of the key among the applied keys: a radix pass over the bits of t, then of
                // pass, high to low (one ballot each: the lanes whose key agrees so far with a 0
                // there are smaller); the low byte is the applying lane itself, so the lanes still
                // equal after (t, pass) are ordered by lane
                const u64 A = __ballot(apl);
                u64 eq = apl ? A : 0ull;
                uint32_t rank = 0;
                const uint32_t tmax = wave_max(apl ? (hk >> 16) : 0u), pmax = wave_max(apl ? ((hk >> 8) & 0xFFu) : 0u);
                auto rbit = [&](uint32_t b) {
                    const bool one = (hk >> b) & 1u;
                    const u64 B = __ballot(apl && one);
                    rank += one ? (uint32_t)__popcll(eq & ~B) : 0u;
                    eq &= one ? B : ~B;
                };
                for (int b = 16 + (31 - __builtin_clz(tmax | 1u)); b >= 16; b--) rbit((uint32_t)b);
                for (int b = 8 + (31 - __builtin_clz(pmax | 1u)); b >= 8; b--) rbit((uint32_t)b);
                rank += (uint32_t)__popcll(eq & below);
                hist = apl ? (int32_t)rank : (act && tk != INF ? -2 : -1);
                H = (uint32_t)__popcll(__ballot(apl));
                if (apl && dup) L.first[fidx(a8, (slot & 63))] = lane;   // (actor, seq) -> applied copy
                copy_applied = __ballot(apl && dup) != 0;
                solved = true;
            }
            STAMP(L, 15);
        }
        for (uint32_t i = 0; i < n && !solved; i++) {
            queue |= 1ull << i;
            u64 P = __ballot(lane == i && !never && (dall & ~applied) == 0);
            while (P) {
                // which lanes of the pass apply a change (the rest are duplicate no-ops)
                u64 ap = P & nodupm & ~applied, keys = ap;
                for (u64 dm = P & dupm; dm; dm &= dm - 1) {
                    const uint32_t d = (uint32_t)__builtin_ctzll(dm);
                    const uint32_t kd = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)d);
                    if (!((applied | keys) >> kd & 1)) {
                        ap |= 1ull << d; keys |= 1ull << kd; copy_applied = true;
                        if (lane == d) L.first[fidx(a8, (slot & 63))] = lane;   // (actor, seq) -> applied lane
                    }
                }
                if ((P >> lane) & 1) hist = ((ap >> lane) & 1) ? (int32_t)(H + (uint32_t)__popcll(ap & below)) : -2;
                H += (uint32_t)__popcll(ap);
                applied |= keys;
                queue &= ~P;
                // the next pass: queued changes whose deps are met before it or by an earlier
                // change of the same pass
                u64 np = 0;
                for (;;) {
                    u64 kb = np & nodupm & below;                 // keys met earlier in the pass
                    for (u64 dm = np & dupm; dm; dm &= dm - 1) {
                        const uint32_t d = (uint32_t)__builtin_ctzll(dm);
                        const uint32_t kd = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)d);
                        kb |= d < lane ? (1ull << kd) : 0ull;
                    }
                    const u64 nx = __ballot(((queue >> lane) & 1) && !never && ((dall & ~applied) & ~kb) == 0);
                    if (nx == np) break;
                    np = nx;
                }
                P = np;
            }
        }
        // direct deps of the applied changes: their first arrivals, or the applied copies
        const bool ap = act && hist >= 0;
        dmask = ap ? dall : 0ull;
        pred_arr = ap ? pred_any : 0xFFu;
        if (copy_applied) {
            wave_sync();
            dmask = 0; pred_arr = 0xFFu;
            if (ap) {
                for (uint32_t j = 0; j < c.n_deps; j++) {
                    const uint32_t pk = L.deps[my_dep0 + j];
                    const uint32_t a = pk >> 24, s = pk & 0xFFFFFF;
                    if (a == actor || s == 0) continue;
                    dmask |= 1ull << L.first[fidx(a, (s - L.base[a]))];
                }
                if (seq - 1 != 0) { pred_arr = L.first[fidx(actor, (seq - 1 - mybase))]; dmask |= 1ull << pred_arr; }
            }
        }
    } else {
        // ---- exact emulation of addChange / applyQueuedOps (wave-uniform control) ----
        // per-actor clock requirement relative to the batch's first seq of that actor, packed
        // as bytes (0x7F = never satisfiable in this batch)
        uint32_t need_lo = 0, need_hi = 0;
        if (act) {
            for (uint32_t j = 0; j < c.n_deps; j++) {
                const uint32_t inf = L.depinfo[my_dep0 + j];
                const uint32_t a = (inf >> 16) & (NA_MAX - 1), rel = (inf >> 8) & 0x7F;
                need_set(need_lo, need_hi, a, (a != actor && rel != 0) ? rel : 0u);   // deps.set(actor, seq-1) overrides
            }
            const uint32_t ps = seq - 1;
            need_set(need_lo, need_hi, a8, ps != 0 ? (ps >= mybase ? ps - mybase + 1 : 0x7Fu) : 0u);
        }
        clear_first(L.first);                                                           // -> applied lane
        wave_sync();
        uint32_t crel_lo = 0, crel_hi = 0;      // relative applied clock per actor (bytes)
        u64 queued = 0;
        bool stop = false;
        for (uint32_t i = 0; i < n && !stop; i++) {
            queued |= 1ull << i;
            u64 above = 0;
            bool first_pass = true;             // pass 1 can only apply the new change
            for (;;) {                          // passes
                bool progress = false;
                for (;;) {                      // one pass: first ready change after the cursor
                    const uint32_t x0 = ((crel_lo | 0x80808080u) - need_lo) & 0x80808080u;
                    const uint32_t x1 = ((crel_hi | 0x80808080u) - need_hi) & 0x80808080u;
                    u64 r = __ballot(act && x0 == 0x80808080u && x1 == 0x80808080u) & queued;
                    r &= first_pass ? (1ull << i) : above;
                    if (!r) break;
                    const uint32_t j = (uint32_t)__builtin_ctzll(r);
                    const uint32_t aj = (uint32_t)__builtin_amdgcn_readlane((int)actor, (int)j);
                    const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)slot, (int)j);
                    const uint32_t sh = (aj & 3) * 8;
                    const uint32_t cur = (((aj < 4) ? crel_lo : crel_hi) >> sh) & 0xFF;
                    queued &= ~(1ull << j);
                    progress = true;
                    above = (j >= 63) ? 0 : (~0ull << (j + 1));
                    if (sj + 1 <= cur) {                         // seq <= clock: already applied
                        const uint32_t k = L.first[fidx(aj, sj)];
                        const uint32_t ck = (uint32_t)__builtin_amdgcn_readlane((int)c.content_id, (int)k);
                        const uint32_t cj = (uint32_t)__builtin_amdgcn_readlane((int)c.content_id, (int)j);
                        if (lane == j) hist = -2;
                        if (ck != cj) {                          // 'Inconsistent reuse of sequence number'
                            if (lane == 0) lds_min(L.errkey, err_key(H, 0, j, HM_ERR_INCONSISTENT_SEQ));
                            stop = true;
                            break;
                        }
                        if (first_pass) break;
                        continue;
                    }
                    if (aj < 4) crel_lo = (crel_lo & ~(0xFFu << sh)) | ((sj + 1) << sh);
                    else        crel_hi = (crel_hi & ~(0xFFu << sh)) | ((sj + 1) << sh);
                    if (lane == 0) L.first[fidx(aj, sj)] = j;
                    if (lane == j) hist = (int32_t)H;
                    H++;
                    if (first_pass) break;
                }
                if (stop || !progress) break;
                first_pass = false;
                above = ~0ull;
            }
        }
        wave_sync();
        // direct deps over the *applied* lanes
        dmask = 0; pred_arr = 0xFFu;
        if (act && hist >= 0) {
            for (uint32_t j = 0; j < c.n_deps; j++) {
                const uint32_t pk = L.deps[my_dep0 + j];
                const uint32_t a = pk >> 24, s = pk & 0xFFFFFF;
                if (a == actor || s == 0) continue;
                dmask |= 1ull << L.first[fidx(a, (s - L.base[a]))];
            }
            if (seq - 1 != 0) { pred_arr = L.first[fidx(actor, (seq - 1 - mybase))]; dmask |= 1ull << pred_arr; }
        }
    }

    if (HM_PRIO_HIST && queued_doc) __builtin_amdgcn_s_setprio(0);
    STAMP(L, 3);
    if (HM_ABLATE & 512) return OUT_UNSUPPORTED;
    // ---------------- K1b: ancestor sets in history order ----------------
    if (act) L.hist_of[lane] = hist;
    if (act && hist >= 0) L.h2a[hist] = (uint8_t)lane;
    wave_sync();
    const bool hv = lane < H;
    // arrival index at history position `lane` (identity history: the same lane, no gathers)
    uint32_t ai = lane, hactor = actor, hseq = seq, hpred = pred_arr;
    u64 dm_arr = dmask;
    if (!identity) {
        ai = hv ? L.h2a[lane] : 0;
        dm_arr = shfl64(dmask, (int)ai);
        hactor = shfl32(actor, (int)ai); hseq = shfl32(seq, (int)ai); hpred = shfl32(pred_arr, (int)ai);
    }
    u64 D = 0, Dnp = 0;                                   // direct deps (history space); without own pred
    if (identity) {                                       // history position == arrival index
        D = hv ? dm_arr : 0ull;
        Dnp = hv && hpred != 0xFFu ? D & ~(1ull << hpred) : D;
    } else if (hv) {
        u64 x = dm_arr;
        while (x) {
            const uint32_t j = (uint32_t)__builtin_ctzll(x);
            x &= x - 1;
            const u64 bit = 1ull << (uint32_t)L.hist_of[j];
            D |= bit;
            if (j != hpred) Dnp |= bit;
        }
    }
    // covered = union of all ancestor sets = union of the direct deps (every ancestor is
    // some change's direct dep); chains = history positions of each actor
    if (hv) { lds_or(L.cov, D); lds_or(&L.chain[hactor], 1ull << lane); }
    // ancestors-or-self, pushed in history order: lane k is final when the sweep reaches it.
    // Per step: v_readlane of lane k, bit k of D as an all-ones mask (v_bfe_i32), v_and_or.
    // Positions below 32 only have low-word ancestors.
    uint32_t alo = hv && lane < 32 ? 1u << lane : 0u, ahi = hv && lane >= 32 ? 1u << (lane - 32) : 0u;
    if (HM_ABLATE & 1024) return OUT_UNSUPPORTED;
    {
        if (HM_PRIO_PUSH) __builtin_amdgcn_s_setprio(HM_PRIO_PUSH);
        const uint32_t Hs = (uint32_t)__builtin_amdgcn_readfirstlane((int)H);
        const uint32_t Dlo = (uint32_t)D, Dhi = (uint32_t)(D >> 32);
        const uint32_t H1 = Hs < 32 ? Hs : 32;
#if HM_PUSH_BPERM
        // lane k's set broadcast by ds_bpermute (the LDS pipe) instead of v_readlane (a VALU
        // instruction and an SGPR hazard): the kernel is VALU-issue bound, the push a quarter of
        // its VALU instructions
#define PUSH_BC(v, k) ((uint32_t)__builtin_amdgcn_ds_bpermute((k) << 2, (int)(v)))
#else
#define PUSH_BC(v, k) ((uint32_t)__builtin_amdgcn_readlane((int)(v), (int)(k)))
#endif
#define PUSH_LO(k) alo |= PUSH_BC(alo, (k)) & (uint32_t)__builtin_amdgcn_sbfe((int)Dlo, (k), 1)
#define PUSH_HI(k) do { const uint32_t m_ = (uint32_t)__builtin_amdgcn_sbfe((int)Dhi, (k) - 32, 1);          \
                        const uint32_t bl_ = PUSH_BC(alo, (k)), bh_ = PUSH_BC(ahi, (k));                   \
                        alo |= bl_ & m_; ahi |= bh_ & m_; } while (0)
        // Fully unrolled with immediate lane indices (no scalar index arithmetic per step), one
        // wave-uniform check per group of 8.  Steps at positions >= H are no-ops: those lanes
        // hold no ancestors and no lane depends on them.  (A blocked variant — 4 positions per
        // readlane round trip, finished on the scalar unit — measured slower.)
#pragma unroll
        for (int g = 0; g < 32; g += 8) {
            if ((uint32_t)g >= H1) break;
            PUSH_LO(g); PUSH_LO(g + 1); PUSH_LO(g + 2); PUSH_LO(g + 3);
            PUSH_LO(g + 4); PUSH_LO(g + 5); PUSH_LO(g + 6); PUSH_LO(g + 7);
        }
#pragma unroll
        for (int g = 32; g < 64; g += 8) {
            if ((uint32_t)g >= Hs) break;
            PUSH_HI(g); PUSH_HI(g + 1); PUSH_HI(g + 2); PUSH_HI(g + 3);
            PUSH_HI(g + 4); PUSH_HI(g + 5); PUSH_HI(g + 6); PUSH_HI(g + 7);
        }
#undef PUSH_LO
#undef PUSH_HI
#undef PUSH_BC
        if (HM_PRIO_PUSH && !HM_PRIO_FOLD) __builtin_amdgcn_s_setprio(0);
    }
    const u64 anc = hv ? ((((u64)ahi << 32) | alo) & ~(1ull << lane)) : 0ull;   // strict ancestors
    if (hv) L.anc[lane] = anc;
    wave_sync();
    STAMP(L, 4);
    if (HM_ABLATE & 64) return OUT_UNSUPPORTED;
    const u64 covered = *L.cov;
    // transitiveDeps folds deps.set(actor, seq-1) in key order: acc = max(acc, FC(d)); acc[a_d] = s_d.
    // The `.set` can LOWER acc[a_d] when an earlier entry already knows a later change of a_d;
    // compare that literal fold with the closure and leave the envelope only when they differ.
    // Necessary condition (cheap): a listed non-own dep is an ancestor of another listed
    // non-own dep, or the own actor appears as a deps key (then seq-1 is folded in place).
    bool suspect = false;
    if (hv && (Dnp & (Dnp - 1))) {
        u64 x = Dnp;
        while (x) {
            const uint32_t i2 = (uint32_t)__builtin_ctzll(x);
            x &= x - 1;
            if (L.anc[i2] & Dnp) suspect = true;
        }
    }
    uint32_t h_own_row = own_row ? 1u : 0u, h_dep0 = my_dep0, h_nd = c.n_deps;
    if (!identity) {                                                     // all lanes: bpermute sources
        h_own_row = shfl32(h_own_row, (int)ai); h_dep0 = shfl32(my_dep0, (int)ai); h_nd = shfl32(c.n_deps, (int)ai);
    }
    suspect |= hv && h_own_row != 0;
#ifdef HM_DEV_NOFOLD
    suspect = false;                    // dev-only timing build: skips the literal-fold check
#endif
    if (suspect) {
        const FoldView fv = {L.anc, L.chain, L.first, L.base, L.deps, L.hist_of};
        if (fold_differs(fv, h_dep0, h_nd, hactor, hseq)) lds_or(L.flags, FL_UNSUPPORTED);
    }
    if (hv && !((covered >> lane) & 1)) L.headv[hactor] = hseq;     // opSet.deps
    for (uint32_t i = lane; i < O; i += WAVE) { L.objslot[i] = i == 0 ? 0u : 0xFFFFFFFFu; L.objtype[i] = i == 0 ? HM_MAKE_MAP : 0xFF; }
    for (uint32_t i = lane; i < R; i += WAVE) {
        L.segor[i] = 0; L.segcnt[i] = 0; L.survpk[i] = 0; L.insmin[i] = 0xFFFFFFFFu; L.regobj[i] = HM_NONE;
    }
    wave_sync();

    STAMP(L, 5);
    if (HM_PRIO_FOLD && !HM_PRIO_K2) __builtin_amdgcn_s_setprio(0);
    if (HM_PRIO_K2) __builtin_amdgcn_s_setprio(HM_PRIO_K2);
    if (HM_ABLATE & 2) return OUT_UNSUPPORTED;
    // ---------------- K2: ops (lane + 64*t) ----------------
    uint32_t oreg[OPL], oobj[OPL], opar[OPL], oact[OPL], okey[OPL], oarr[OPL], oelem[OPL], oactor[OPL];
    int32_t oh[OPL];
    bool counter_ops = false, malformed = false;
#pragma unroll
    for (int t = 0; t < OPL; t++) {
        const uint32_t k = lane + WAVE * t;
        oh[t] = -1; okey[t] = 0; oarr[t] = 0; oreg[t] = 0; oobj[t] = 0; opar[t] = 0; oact[t] = 0xFF; oelem[t] = 0; oactor[t] = 0;
        if (k < m) {
            const uint32_t meta = L.opmeta[k], ro = L.opro[k], pr = L.oppar[k];
            const uint32_t cw = L.opchg[k], ch = cw & 0xFFu;
            oarr[t] = ch; oactor[t] = cw >> 8; oh[t] = identity ? (int32_t)ch : L.hist_of[ch];
            oreg[t] = ro & 0xFFFFu; oobj[t] = ro >> 16; oact[t] = meta & 0xFF;
            opar[t] = pr == PAR_HEAD ? HM_HEAD : pr;
            if (LISTS) {
                oelem[t] = L.opelem[k];
                if (oact[t] == HM_INS && oelem[t] >= (1u << 24)) lds_or(L.flags, FL_UNSUPPORTED);
            }
            counter_ops |= oact[t] == HM_INC || ((meta >> 8) & 0xFF) == HM_DT_COUNTER;
            okey[t] = ((uint32_t)(oh[t] < 0 ? 0 : oh[t]) << 16) | (k - L.opbase[ch]);
            // malformed rows (any op, applied or not) put the whole document outside the envelope
            const uint32_t a = oact[t];
            const bool bad = a <= HM_MAKE_TEXT ? oobj[t] >= O
                           : (a <= HM_INC ? (oreg[t] >= R || (a == HM_INS && opar[t] != HM_HEAD && opar[t] >= R)) : true);
            malformed |= bad;
            if (oh[t] >= 0 && !bad) {
                if (a <= HM_MAKE_TEXT) lds_min(&L.objslot[oobj[t]], okey[t] + 1);
                else if (oobj[t] < O) {
                    L.regobj[oreg[t]] = oobj[t];
                    if (a == HM_INS) lds_min(&L.insmin[oreg[t]], okey[t] + 1);
                    else {
                        lds_add(&L.segcnt[oreg[t]], 1u);
                        if (a != HM_INC) lds_or(&L.segor[oreg[t]], L.anc[oh[t]]);
                    }
                }
            }
        }
    }
    STAMP(L, 6);
    if (HM_ABLATE & 128) return OUT_UNSUPPORTED;
    if (__ballot(malformed)) return OUT_UNSUPPORTED;
    // counter sums need the carve's survsum table (launches flagged HM_DOC_HAS_COUNTERS)
    if (!p.counters && __ballot(counter_ops)) lds_or(L.flags, FL_UNSUPPORTED);
    wave_sync();
    // objects: the earliest make op creates, later ones throw 'Duplicate creation of object'
#pragma unroll
    for (int t = 0; t < OPL; t++)
        if (oh[t] >= 0 && oact[t] <= HM_MAKE_TEXT && oobj[t] < O) {
            if (L.objslot[oobj[t]] != okey[t] + 1)
                lds_min(L.errkey, err_key((uint32_t)oh[t], (okey[t] & 0xFFFF) + 1, oarr[t], HM_ERR_DUPLICATE_OBJECT));
            else L.objtype[oobj[t]] = (uint8_t)oact[t];
        }
    wave_sync();
    bool surv[OPL];
    bool has_list = false, anyerr = false, late = false;
#pragma unroll
    for (int t = 0; t < OPL; t++) {
        // predicated: every lane reads (clamped) and decides with selects, no per-op branches
        const OpCheck ck = op_check(L, oh[t], oact[t], oobj[t], oreg[t], opar[t], okey[t], R, O);
        has_list |= ck.has_list;
        anyerr |= ck.err != 0;
        late |= ck.late;
        surv[t] = ck.surv;
        // survivors counted per (register, actor rank): the rank below needs no survivor list
        if (surv[t]) lds_add(&L.survpk[oreg[t]], 1ull << (8 * oactor[t]));
    }
    if (__ballot(late)) return OUT_UNSUPPORTED;                  // the general kernel climbs the chains
    if (__ballot(anyerr)) {
        // a throw: its key (history position, op, arrival) orders it against the others
        u64 errk = ~0ull;                // this lane's earliest throw (one wave-wide min below)
#pragma unroll
        for (int t = 0; t < OPL; t++) {
            const OpCheck ck = op_check(L, oh[t], oact[t], oobj[t], oreg[t], opar[t], okey[t], R, O);
            const uint32_t h = oh[t] < 0 ? 0u : (uint32_t)oh[t], kk = (okey[t] & 0xFFFF) + 1;
            const u64 ek = ck.err ? err_key(h, kk, oarr[t], ck.err) : ~0ull;
            errk = errk < ek ? errk : ek;
        }
        lds_min(L.errkey, errk);
    }
    const bool doc_lists = __ballot(has_list) != 0;
    if (!LISTS && doc_lists) lds_or(L.flags, FL_UNSUPPORTED);   // launched without the K3 carve
    wave_sync();
    if (*L.errkey != ~0ull) return OUT_ERROR;                    // the first throw wins
    if (*L.flags & FL_UNSUPPORTED) return OUT_UNSUPPORTED;

    STAMP(L, 7);
    if (HM_PRIO_K2 && !HM_PRIO_RANK) __builtin_amdgcn_s_setprio(0);
    if (HM_PRIO_RANK) __builtin_amdgcn_s_setprio(HM_PRIO_RANK);
    if (HM_ABLATE & 4) return OUT_UNSUPPORTED;
    // survivor offsets: exclusive scan over register ids (a register's count = its byte sum)
    uint32_t total = 0;
    const uint32_t lane_s = LISTS ? lane : fresh_lane();     // (list launches: no spill there; A/B C5 +2 % with it)
    for (uint32_t r0 = 0; r0 < R; r0 += WAVE) {
        const uint32_t r = r0 + lane_s;
        uint32_t tot;
        const uint32_t cnt = r < R ? bytesum64(L.survpk[r]) : 0u;
        const uint32_t ex = wave_excl_scan(cnt, &tot);
        if (r < R) { L.regoff[r] = total + ex; L.survcnt[r] = cnt; }
        total += tot;
    }
    wave_sync();
    // rank: actor rank descending = the survivors of higher actors on the register (bytes above
    // this actor's); equal actors (ties) are ordered below
    uint32_t my_act[OPL], rb0[OPL], rank[OPL];
    bool tie[OPL];
#pragma unroll
    for (int t = 0; t < OPL; t++) {
        const uint32_t ri = surv[t] ? oreg[t] : 0u;
        my_act[t] = surv[t] ? oactor[t] : 0u;
        rb0[t] = L.regoff[ri];
        const u64 pk = L.survpk[ri];
        const uint32_t sh = 8 * (my_act[t] + 1);
        rank[t] = surv[t] ? bytesum64(sh >= 64 ? 0ull : pk >> sh) : 0u;
        tie[t] = surv[t] && ((pk >> (8 * my_act[t])) & 0xFF) > 1;
    }
    bool anytie = false;
#pragma unroll
    for (int t = 0; t < OPL; t++) anytie |= tie[t];
    if (__ballot(anytie)) {
        // ... equal actors = ops of one change on one register (two changes of one actor are
        // causally ordered, so only one change's ops survive together).  p = assigns applied on
        // the register before the op: broadcast each tie op and count the wave's applied assigns
        // on its register with a smaller (history, op) key; then broadcast each tie op's order to
        // the other members of its group.  Registers and ballots only, no LDS round trips.
        uint32_t myt[OPL];
        bool oddn[OPL];
#pragma unroll
        for (int t = 0; t < OPL; t++) {
            myt[t] = 0;
            oddn[t] = tie[t] && (L.segcnt[tie[t] ? oreg[t] : 0u] & 1);   // the group is reversed after an odd count
            u64 tm = __ballot(tie[t]);
            while (tm) {
                const int j = (int)__builtin_ctzll(tm);
                tm &= tm - 1;
                const uint32_t rj = (uint32_t)__builtin_amdgcn_readlane((int)oreg[t], j);
                const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)okey[t], j);
                uint32_t pc = 0;
#pragma unroll
                for (int t2 = 0; t2 < OPL; t2++)
                    pc += (uint32_t)__popcll(__ballot(oh[t2] >= 0 && oact[t2] >= HM_SET && oact[t2] <= HM_INC &&
                                                      oreg[t2] == rj && okey[t2] < kj));
                if ((int)lane == j) myt[t] = tie_order(pc);
            }
        }
#pragma unroll
        for (int t = 0; t < OPL; t++) {
            u64 tm = __ballot(tie[t]);
            while (tm) {
                const int j = (int)__builtin_ctzll(tm);
                tm &= tm - 1;
                const uint32_t rj = (uint32_t)__builtin_amdgcn_readlane((int)oreg[t], j);
                const uint32_t aj = (uint32_t)__builtin_amdgcn_readlane((int)my_act[t], j);
                const uint32_t tj = (uint32_t)__builtin_amdgcn_readlane((int)myt[t], j);
#pragma unroll
                for (int t2 = 0; t2 < OPL; t2++) {
                    const bool peer = tie[t2] && oreg[t2] == rj && my_act[t2] == aj && !(t2 == t && (int)lane == j);
                    rank[t2] += (peer && (oddn[t2] ? (tj > myt[t2]) : (tj < myt[t2]))) ? 1u : 0u;
                }
            }
        }
    }
    // survivor slots: op index (8 bits; < 256 ops per document) and, in counter launches, what
    // the inc pass needs about the survivor without chasing op -> change -> history through LDS:
    // bit 15 a counter set (int or float), bit 14 an integral one, bits 8-13 its change's
    // history position
#pragma unroll
    for (int t = 0; t < OPL; t++) {
        if (!surv[t]) continue;
        const uint32_t pos = rb0[t] + rank[t];
        uint32_t tag = 0;
        if (p.counters) {
            const uint32_t mt = L.opmeta[lane + WAVE * t], vt = (mt >> 16) & 0xFF;
            const bool cset = (mt & 0xFF) == HM_SET && ((mt >> 8) & 0xFF) == HM_DT_COUNTER && (vt == HM_V_INT || vt == HM_V_FLOAT);
            tag = cset ? (0x8000u | (vt == HM_V_INT ? 0x4000u : 0u) | ((uint32_t)oh[t] << 8)) : 0u;
            L.survsum[pos] = 0;
        }
        L.survop[pos] = (uint16_t)((lane + WAVE * t) | tag);
    }
    wave_sync();
    if (HM_PRIO_RANK) __builtin_amdgcn_s_setprio(0);
    STAMP(L, 8);
    if (HM_ABLATE & 256) return OUT_UNSUPPORTED;
    if constexpr (LISTS) {
        if (doc_lists) {
            if (HM_PRIO_K3) __builtin_amdgcn_s_setprio(HM_PRIO_K3);
            rga_order<OPL>(L, R, O, oreg, oobj, opar, oact, oelem, oarr, oh, p.res_epos ? p.res_epos + doc.reg_off : nullptr);
            if (HM_PRIO_K3) __builtin_amdgcn_s_setprio(0);
        }
    }
    // counters: an inc adds to every surviving counter set that is its ancestor.
    // JS numbers: an integer counter is exact only while |base| + sum|inc| <= 2^53; with at
    // most 256 ops per document, |inc| < 2^44 and |base| < 2^52 guarantee it (larger
    // values go to merge_large_kernel, which tracks sum|inc| exactly).
    if (p.counters && __ballot(counter_ops)) {
        bool outside = false;
        // every inc's value load issued before the first is used (they are L2 round trips)
        // and the base values of surviving integer counter sets (the 2^52 envelope check)
        int64_t incv[OPL];
        u64 basev[OPL];
#pragma unroll
        for (int t = 0; t < OPL; t++) {
            incv[t] = (oh[t] >= 0 && oact[t] == HM_INC) ? (int64_t)op_value(L, lane + WAVE * t) : 0;
            const uint32_t q = lane + WAVE * t;
            basev[t] = 0;
            if (q < total) {
                const uint32_t sw = L.survop[q];
                if ((sw & 0xC000u) == 0xC000u) basev[t] = op_value(L, sw & 0xFFu);     // an integral counter set
            }
        }
#pragma unroll
        for (int t = 0; t < OPL; t++) {
            if (oh[t] < 0 || oact[t] != HM_INC) continue;
            const uint32_t k = lane + WAVE * t;
            const uint32_t reg = oreg[t], b0 = L.regoff[reg], cnt = L.survcnt[reg];
            const u64 an = L.anc[oh[t]];
            const uint32_t my_vtag = (L.opmeta[k] >> 16) & 0xFF;
            const int64_t v = incv[t];
            for (uint32_t q = 0; q < cnt; q++) {
                const uint32_t sw = L.survop[b0 + q];
                if (!(sw & 0x8000u)) continue;                                  // not a counter set
                if (!((an >> ((sw >> 8) & 63u)) & 1)) continue;                  // concurrent inc: no effect
                // f64 counters need the ordered sum
                if (!(sw & 0x4000u) || my_vtag != HM_V_INT || (u64)(v < 0 ? -v : v) >= (1ull << 44)) { outside = true; continue; }
                lds_add((LDS u64 *)&L.survsum[b0 + q], (unsigned long long)v);
            }
        }
#pragma unroll
        for (int t = 0; t < OPL; t++) {                   // (total <= WAVE * OPL)
            const int64_t b = (int64_t)basev[t];
            outside |= (u64)(b < 0 ? -b : b) >= (1ull << 52);
        }
        if (__ballot(outside)) return OUT_UNSUPPORTED;
        wave_sync();
    }
    st.hist = hist; st.H = H; st.total = total; st.doc_lists = doc_lists;
    return OUT_OK;
}

// Output phase of one document (all reads from LDS; coalesced stores).
// Clock.cmp(DocBackend.clock, minimumClock) of a merged document, from the min_clock row loaded
// before the merge (mc, lane < S): computed before the next document's rows are requested, so
// no wait for that load sits behind the prefetch and this document's stores
__device__ __forceinline__ uint32_t min_cmp_of(const SmallParams &p, const SmallLds &L, const hm_doc_row &doc, uint32_t mc) {
    const uint32_t lane = threadIdx.x, S = p.a_stride;
    const uint32_t bc = (lane < S && lane < doc.n_actors) ? L.bclock[lane] : 0u;
    const bool aGTE = __ballot(lane < S && bc < mc) == 0;
    const bool bGTE = __ballot(lane < S && mc < bc) == 0;
    return p.min_clock ? ((aGTE && bGTE) ? 0u : (aGTE ? 1u : (bGTE ? 2u : 3u))) : 0u;
}

// A merged document's survivor rows, read out of LDS into registers (lane + WAVE t): the next
// document's rows overwrite the op tables they come from before these are stored.
template <int OPL> struct SurvRows { hm_surv_result r[OPL]; };
template <int OPL>
__device__ __forceinline__ SurvRows<OPL> surv_rows(const SmallParams &p, const SmallLds &L, const DocState &st) {
    const uint32_t lane = threadIdx.x;
    SurvRows<OPL> o;
#pragma unroll
    for (int t = 0; t < OPL; t++) {
        const uint32_t q = lane + WAVE * t;
        const uint32_t k = q < st.total ? (L.survop[q] & 0xFFu) : 0u, mt = L.opmeta[k];
        hm_surv_result sr;
        sr.op = k; sr.vtag = (mt >> 16) & 0xFF; sr.value = op_value(L, k);
        if (p.counters && q < st.total && (mt & 0xFF) == HM_SET && ((mt >> 8) & 0xFF) == HM_DT_COUNTER && sr.vtag == HM_V_INT)
            sr.value = (u64)((int64_t)sr.value + L.survsum[q]);
        o.r[t] = sr;
    }
    return o;
}

// one 16-byte output row (non-temporal under HM_NT_OUT: written once, never read by this kernel)
__device__ __forceinline__ void st16(void *dst, uint4 v) {
#if HM_NT_OUT
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4u *>(dst));
#else
    *reinterpret_cast<uint4 *>(dst) = v;
#endif
}
__device__ __forceinline__ void st4(void *dst, uint32_t v) {
#if HM_NT_OUT
    __builtin_nontemporal_store(v, reinterpret_cast<uint32_t *>(dst));
#else
    *reinterpret_cast<uint32_t *>(dst) = v;
#endif
}
template <int OPL, bool LISTS>
__device__ __forceinline__ void write_outputs(const SmallParams &p, const SmallLds &L, uint32_t d, uint32_t ds,
                                              const hm_doc_row &doc, Outcome oc, const DocState &st, uint32_t mcmp,
                                              const SurvRows<OPL> &sv) {
    const uint32_t lane = threadIdx.x;
    const uint32_t S = p.a_stride;
    const uint32_t n = doc.n_changes, A = doc.n_actors, R = doc.n_regs;
    hm_doc_result *dres = p.res_docs + ds;      // ds: row of the per-document outputs
    if (oc == OUT_ERROR) {
        // an Automerge throw aborted this document's Backend.applyChanges
        const u64 ek = *L.errkey;
        if (lane == 0) {
            hm_doc_result r = {};
            r.status = (int32_t)(ek & 0xFF);
            r.err_change = (uint32_t)((ek >> 8) & 0xFFFF);
            const uint32_t opp1 = (uint32_t)((ek >> 24) & 0xFFFF);
            r.err_op = opp1 ? opp1 - 1 : HM_NONE;
            if (r.status == HM_ERR_UNSUPPORTED) { r.err_change = HM_NONE; r.err_op = HM_NONE; }
            *dres = r;
        }
        return;
    }
    if (oc == OUT_INVALID) {
        // malformed row (ranges outside the batch tables): nothing of it is read or written
        if (lane == 0) {
            hm_doc_result r = {};
            r.status = HM_ERR_INVALID; r.err_change = HM_NONE; r.err_op = HM_NONE;
            *dres = r;
        }
        for (uint32_t a = lane; a < S; a += WAVE) {
            p.res_clock[(size_t)ds * S + a] = 0u; p.res_heads[(size_t)ds * S + a] = 0u;
            p.res_back_clock[(size_t)ds * S + a] = 0u;
        }
        return;
    }
    if (oc == OUT_UNSUPPORTED) {
        // outside this kernel's envelope: merge_large_kernel finds the status and takes the document
        if (lane == 0) {
            hm_doc_result r = {};
            r.status = HM_DEFERRED; r.err_change = HM_NONE; r.err_op = HM_NONE;
            *dres = r;
#if !HM_ABLATE
            p.deferred[atomicAdd(p.n_deferred, 1u)] = d;     // merge_large_kernel's work list
#endif
        }
        return;
    }
    for (uint32_t r = lane; r < R; r += WAVE) {
        const int32_t li = (LISTS && st.doc_lists) ? (int32_t)L.insmin[r] : -1;
        st16(p.res_regs + doc.reg_off + r, make_uint4(L.survcnt[r], L.regoff[r], (uint32_t)li, L.regobj[r]));
    }
    // allDeps rows: lane = arrival index writes its change's row (zeros if not applied;
    // chain[a] is empty for a >= A)
    if (lane < n) {
        const u64 an = st.hist >= 0 ? L.anc[st.hist] : 0ull;
        uint32_t *row = p.res_all_deps + (size_t)(doc.change_off + lane) * S;
        if (S == 8 || S == 4) {
            uint32_t v[NA_MAX];
#pragma unroll
            for (int a = 0; a < NA_MAX; a++) v[a] = (uint32_t)__popcll(an & L.chain[a]);
            st16(row, make_uint4(v[0], v[1], v[2], v[3]));
            if (S == 8) st16(row + 4, make_uint4(v[4], v[5], v[6], v[7]));
        } else {
            for (uint32_t a = 0; a < S; a++) row[a] = a < NA_MAX ? (uint32_t)__popcll(an & L.chain[a]) : 0u;
        }
    }
    if (lane < S) {
        const bool ar = lane < A;
        p.res_clock[(size_t)ds * S + lane] = ar ? (uint32_t)__popcll(L.chain[lane]) : 0u;
        p.res_heads[(size_t)ds * S + lane] = ar ? L.headv[lane] : 0u;
        p.res_back_clock[(size_t)ds * S + lane] = ar ? L.bclock[lane] : 0u;   // DocBackend.clock (queued included)
    }
    for (uint32_t a = WAVE + lane; a < S; a += WAVE) {                   // wide rows: actors >= 64 are absent
        p.res_clock[(size_t)ds * S + a] = 0u; p.res_heads[(size_t)ds * S + a] = 0u; p.res_back_clock[(size_t)ds * S + a] = 0u;
    }
    const bool act = lane < n;
    const u64 q = __ballot(act && st.hist == -1);
    if (act) st4(p.res_hist + doc.change_off + lane, (uint32_t)st.hist);
    if (lane == 0) {
        hm_doc_result r = {};
        r.status = HM_OK; r.err_change = HM_NONE; r.err_op = HM_NONE;
        r.hist_len = st.H; r.n_queued = (uint32_t)__popcll(q); r.n_surv = st.total;
        r.min_cmp = mcmp;
        *dres = r;
    }
#pragma unroll
    for (int t = 0; t < OPL; t++) {
        const uint32_t q = lane + WAVE * t;
        if (q < st.total) st16(p.res_surv + doc.op_off + q, make_uint4(sv.r[t].op, sv.r[t].vtag, (uint32_t)sv.r[t].value,
                                                                       (uint32_t)(sv.r[t].value >> 32)));
    }
}

#if HM_ASYNC_NEXT
// A lower bound on the store instructions write_outputs issues for a document merged OK (each
// term names the stores above it counts): the register rows (one dwordx4 per 64 registers),
// the allDeps rows (two dwordx4 at S = 8, one at S = 4, at least one otherwise, when there are
// changes), the clock / heads / back-clock rows (three), the history positions (one, when there
// are changes), the 32-byte result row (two: no store is wider than 16 bytes), the survivor rows
// (one dwordx4 per 64).  pad_stores tops it up to HM_ASYNC_STORES with stores of the result row's
// pad word (zero, as the row itself wrote it), issued by asm so each is exactly one instruction.
template <int OPL>
__device__ __forceinline__ uint32_t out_stores_min(const SmallParams &p, const hm_doc_row &doc, const DocState &st) {
    const uint32_t S = p.a_stride, n = doc.n_changes;
    uint32_t c = (doc.n_regs + WAVE - 1) / WAVE;
    if (n) c += (S == 8 ? 2u : 1u) + 1u;
    c += 3u + 2u;
    c += (st.total + WAVE - 1) / WAVE < (uint32_t)OPL ? (st.total + WAVE - 1) / WAVE : (uint32_t)OPL;
    return c;
}
template <int OPL>
__device__ __forceinline__ void pad_stores(const SmallParams &p, const hm_doc_row &doc, const DocState &st, uint32_t ds) {
    uint32_t *pad = &p.res_docs[ds].pad;
    const uint32_t zero = 0u;
    for (uint32_t c = out_stores_min<OPL>(p, doc, st); c < HM_ASYNC_STORES; c++)      // (wave-uniform)
        asm volatile("global_store_dword %0, %1, off" :: "v"(pad), "v"(zero) : "memory");
}
#endif

template <int OPL, bool LISTS, int CLS>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(OPL >= 3 ? (LISTS ? (OPL == 3 ? HM_WAVES_PER_EU_LIST3 : HM_WAVES_PER_EU_OPL4 - 1) : HM_WAVES_PER_EU_OPL4) : HM_WAVES_PER_EU)))
void merge_small_kernel(SmallParams p) {
    extern __shared__ __align__(16) uint8_t lds_raw[];
    typedef SizeClass<CLS> C;
    SmallLds L;
    small_carve((LDS uint8_t *)lds_raw, WAVE * OPL, C::NR, C::NO, C::ND, LISTS, true, &L);
    p.cap_regs = C::NR; p.cap_objs = C::NO; p.cap_deps = C::ND;     // (the loop reads the C:: constants)
#if HM_KARG_RELOAD
    // the loop reads the launch parameters through an opaque pointer to the kernarg segment:
    // each document re-loads the fields it uses (scalar loads) instead of holding ~50 SGPRs of
    // them across the loop, where they were spilled to VGPR lanes (readlane / writelane VALU)
    typedef __attribute__((address_space(4))) const SmallParams KParams;
    KParams *kp = (KParams *)__builtin_amdgcn_kernarg_segment_ptr();
#endif
    // workgroups are dealt round-robin over the 8 XCDs (speed only, MI355X_MICROARCH.md): give
    // the workgroups of one XCD consecutive documents, so the 128 B lines a document boundary
    // splits in every table are read and written through one L2 instead of two
    uint32_t d = blockIdx.x;
    if (p.xcd_remap && (gridDim.x & 7) == 0) d = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    if (d >= p.n_docs) return;
#if HM_STAMPS
    if (threadIdx.x == 0) { for (int i = 0; i < HM_NSTAMP; i++) L.stamps[i] = 0; L.stamps[HM_NSTAMP] = stamp_now(); }
#endif
    hm_doc_row doc = p.docs[d];
    bool dok = check_doc(p, doc);
    uint2 w0, w1, w2;                        // this document's change row (lane = arrival index)
    {
        const Rows r = load_rows<OPL>(p, doc);
        stage_rows<OPL, LISTS>(p, L, doc, r, C::ND);
        w0 = make_uint2(r.c01.x, r.c01.y); w1 = make_uint2(r.c01.z, r.c01.w); w2 = r.c2;
    }
    wave_sync();
    for (;;) {
#if HM_KARG_RELOAD
        asm volatile("" : "+s"(kp));
        const SmallParams &p = *(const SmallParams *)kp;
#endif
        // software pipeline over this wave's documents: the next document's rows are
        // loaded before this document's stores and staged to LDS after them
        const uint32_t dn = d + gridDim.x;
        const bool more = dn < p.n_docs;
        bool dokn = true;
        hm_doc_row docn = {};
        // the next document's row, one word per lane (lanes 0-11): nothing waits for it until it
        // is read back after the merge (a uniform load would be moved to scalar registers at once,
        // putting an HBM round trip in front of every document)
        static_assert(sizeof(hm_doc_row) == 12 * sizeof(uint32_t), "doc row words");
        uint32_t docw = 0;
        if (more && threadIdx.x < 12) docw = reinterpret_cast<const uint32_t *>(p.docs + dn)[threadIdx.x];
        auto take_docn = [&]() {
            uint32_t w[12];
#pragma unroll
            for (int j = 0; j < 12; j++) w[j] = (uint32_t)__builtin_amdgcn_readlane((int)docw, j);
            __builtin_memcpy(&docn, w, sizeof docn);
        };
        Rows next;
#if HM_ASYNC_NEXT
        AsyncRows anext;
        constexpr bool ASY = OPL <= HM_ASYNC_MAX_OPL && !HM_PREFETCH_EARLY && !HM_STAGE_FIRST;
#else
        constexpr bool ASY = false;
#endif
#if HM_PREFETCH_EARLY
        if (more) { take_docn(); dokn = check_doc(p, docn); next = load_rows<OPL>(p, docn); }
#endif
        const bool in_env = doc.n_changes <= 64 && doc.n_actors <= NA_MAX && doc.n_ops <= WAVE * OPL && doc.n_ops < 256 &&
                            doc.n_regs <= C::NR && doc.n_objs <= C::NO && doc.n_objs >= 1 &&
                            doc.n_deps <= C::ND && !p.general_only;
        DocState st;
        // output row and minimumClock row requested before the merge: consumed before the next
        // document's rows are requested (min_cmp_of), so neither waits behind that prefetch
        const uint32_t ds = hm_slot(p, d);
        uint32_t mc = 0;
        if (p.min_clock && threadIdx.x < p.a_stride) mc = p.min_clock[(size_t)ds * p.a_stride + threadIdx.x];
        if (p.min_clock && p.a_stride > WAVE) {
            // wide rows (> 64 actors; this kernel merges documents of <= 8): actors >= 64 have
            // DocBackend.clock 0, so they only decide whether any minimumClock entry there is
            // set; lane NA_MAX (clock 0 too) carries that for the comparison
            uint32_t extra = 0;
            for (uint32_t a = WAVE + threadIdx.x; a < p.a_stride; a += WAVE) extra |= p.min_clock[(size_t)ds * p.a_stride + a];
            if (__ballot(extra != 0) && threadIdx.x == NA_MAX) mc |= 1u;
        }
        const Outcome oc = !dok ? OUT_INVALID : in_env ? merge_doc_small<OPL, LISTS>(p, L, doc, w0, w1, w2, st) : OUT_UNSUPPORTED;
        STAMP(L, 9);
        uint32_t mcmp = oc == OUT_OK ? min_cmp_of(p, L, doc, mc) : 0u;
#if HM_FENCE_MCMP
        // computed here, not sunk to its use in write_outputs: there its wait for the minimumClock
        // row (s_waitcnt vmcnt(0)) would also wait for the next document's row loads issued below
        asm volatile("" : "+s"(mcmp) :: "memory");
#endif
#if !HM_PREFETCH_EARLY
        if (more) {
            take_docn();
            dokn = check_doc(p, docn);
#if HM_ASYNC_NEXT
            if constexpr (ASY) anext = load_rows_async<OPL>(p, docn);
            else
#endif
            next = load_rows<OPL>(p, docn);
        }
#endif
        STAMP(L, 12);
        if (HM_PRIO_IO) __builtin_amdgcn_s_setprio(HM_PRIO_IO);
        const SurvRows<OPL> sv = surv_rows<OPL>(p, L, st);
#if HM_STAGE_FIRST
        // the next document's rows go to LDS before this document's stores are issued: a wait
        // for a load also waits for every older store (vmcnt counts both in issue order), so
        // staging after the stores waited for all of them; now nothing waits for the stores
        // until the next document's merge has run
        wave_sync();
        if (more) stage_rows<OPL, LISTS>(p, L, docn, next, C::ND);
        STAMP(L, 11);
        write_outputs<OPL, LISTS>(p, L, d, ds, doc, oc, st, mcmp, sv);
        if (HM_PRIO_IO) __builtin_amdgcn_s_setprio(0);
        wave_sync();
        STAMP(L, 10);
        if (!more) break;
#else
        write_outputs<OPL, LISTS>(p, L, d, ds, doc, oc, st, mcmp, sv);
#if HM_ASYNC_NEXT
        if constexpr (ASY) { if (more && oc == OUT_OK) pad_stores<OPL>(p, doc, st, ds); }
#endif
        wave_sync();
        STAMP(L, 10);
        if (!more) break;
#if HM_ASYNC_NEXT
        if constexpr (ASY) {
            next = take_rows_async<OPL>(anext, docn, oc == OUT_OK);
#if HM_ASYNC_CHECK
            async_check<OPL>(p, docn, next);
#endif
        }
#endif
        stage_rows<OPL, LISTS>(p, L, docn, next, C::ND);
        if (HM_PRIO_IO) __builtin_amdgcn_s_setprio(0);
        wave_sync();
        STAMP(L, 11);
#endif
        w0 = make_uint2(next.c01.x, next.c01.y); w1 = make_uint2(next.c01.z, next.c01.w); w2 = next.c2;
        d = dn;
        doc = docn;
        dok = dokn;
    }
#if HM_STAMPS
    if (threadIdx.x == 0)
        for (int i = 0; i < HM_NSTAMP; i++) atomicAdd(&hm_stamp_acc[i], (unsigned long long)L.stamps[i]);
#endif
}

// ---------------- Clock algebra over dense rows (src/Clock.ts) ----------------
// cmp: 64/S rows per wave, one lane per entry, two ballots (gte(a,b), gte(b,a))
__global__ void clock_cmp_kernel(const uint32_t *a, const uint32_t *b, uint8_t *out, uint32_t n_docs, uint32_t S) {
    const uint32_t lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t rows_per_wave = WAVE / S;
    const uint32_t row = wave * rows_per_wave + lane / S, col = lane % S;
    const bool v = row < n_docs && lane < rows_per_wave * S;
    const uint32_t x = v ? a[(size_t)row * S + col] : 0, y = v ? b[(size_t)row * S + col] : 0;
    const u64 lt = __ballot(v && x < y), gt = __ballot(v && y < x);
    if (v && col == 0) {
        const u64 mask = (S >= 64 ? ~0ull : ((1ull << S) - 1)) << lane;
        const bool aGTE = (lt & mask) == 0, bGTE = (gt & mask) == 0;
        out[row] = (aGTE && bGTE) ? 0 : (aGTE ? 1 : (bGTE ? 2 : 3));
    }
}
__global__ void clock_union_kernel(const uint32_t *a, const uint32_t *b, uint32_t *c, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c[i] = a[i] > b[i] ? a[i] : b[i];
}
__global__ void clock_intersection_kernel(const uint32_t *a, const uint32_t *b, uint32_t *c, size_t n) {
    // Math.min(c1||0, c2||0), kept only when > 0 (zero == absent in a dense row)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c[i] = a[i] < b[i] ? a[i] : b[i];
}

}  // namespace hm

// ---------------- host-side launchers ----------------
// (check builds) documents whose rows were loaded asynchronously and checked, and those whose
// asynchronous rows differed from the counted loads' (both since the last reset)
extern "C" int hm_debug_async_check(unsigned long long *out2, int reset) {
#if HM_ASYNC_CHECK && HM_ASYNC_NEXT
    if (!out2 || hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(&out2[0], HIP_SYMBOL(hm::hm_async_checked), 8) != hipSuccess ||
        hipMemcpyFromSymbol(&out2[1], HIP_SYMBOL(hm::hm_async_bad), 8) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(hm::hm_async_checked), &z, 8) != hipSuccess ||
            hipMemcpyToSymbol(HIP_SYMBOL(hm::hm_async_bad), &z, 8) != hipSuccess) return -1;
    }
    return 1;
#else
    (void)out2; (void)reset;
    return 0;                        // not a check build
#endif
}
#if HM_STAMPS
extern "C" int hm_debug_stamps(unsigned long long *out, int n, int reset) {
    if (n > HM_NSTAMP) n = HM_NSTAMP;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hm::hm_stamp_acc), n * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[HM_NSTAMP] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hm::hm_stamp_acc), z, sizeof z) != hipSuccess) return -1;
    }
    return n;
}
#endif
uint32_t hm_small_class(uint32_t max_regs, uint32_t max_objs, uint32_t max_deps) {
    typedef hm::SizeClass<0> S0;
    typedef hm::SizeClass<2> S2;
    if (max_regs <= S0::NR && max_objs <= S0::NO && max_deps <= S0::ND) return 0u;
    if (max_regs <= S2::NR && max_objs <= S2::NO && max_deps <= S2::ND) return 2u;
    return 1u;
}

template <int CLS> static size_t carve_of(uint32_t opl, bool lists, bool counters) {
    hm::SmallLds L;
    typedef hm::SizeClass<CLS> C;
    return hm::small_carve((uintptr_t)0, 64 * opl, C::NR, C::NO, C::ND, lists, counters, &L);
}

size_t hm_small_lds_bytes(uint32_t opl, uint32_t cls, bool lists, bool counters) {
    return cls == 0 ? carve_of<0>(opl, lists, counters) : cls == 2 ? carve_of<2>(opl, lists, counters) : carve_of<1>(opl, lists, counters);
}

// resident 1-wave workgroups per CU for the instantiation a launch will use (VGPRs and LDS)
uint32_t hm_small_occupancy(uint32_t opl, uint32_t cls, bool lists, bool counters) {
    const size_t lds = hm_small_lds_bytes(opl, cls, lists, counters);
    int n = 0;
    // the persistent grid must be resident at once (a wave that starts after the others drain
    // runs its documents serially at the end): also bound by the LDS with the allocation rounded
    // to 512 bytes (a 13,376-byte carve reported 12 workgroups per CU and ran as if 11 fit)
    const int by_lds = (int)(160u * 1024u / ((lds + 511) & ~(size_t)511));
#define HM_OCC(O_, L_, C_) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, hm::merge_small_kernel<O_, L_, C_>, WAVE, lds)
#define HM_OCC_OPL(L_, C_) switch (opl) { case 1: HM_OCC(1, L_, C_); break; case 2: HM_OCC(2, L_, C_); break; case 3: HM_OCC(3, L_, C_); break; default: HM_OCC(4, L_, C_); }
    if (cls == 0)      { if (lists) { HM_OCC_OPL(true, 0) } else { HM_OCC_OPL(false, 0) } }
    else if (cls == 2) { if (lists) { HM_OCC_OPL(true, 2) } else { HM_OCC_OPL(false, 2) } }
    else               { if (lists) { HM_OCC_OPL(true, 1) } else { HM_OCC_OPL(false, 1) } }
#undef HM_OCC_OPL
#undef HM_OCC
    if (n > by_lds) n = by_lds;
    return n > 0 ? (uint32_t)n : 1u;
}

hipError_t hm_launch_small(const SmallParams &p, uint32_t opl, uint32_t cls, bool lists, uint32_t grid, hipStream_t s) {
    const size_t lds = hm_small_lds_bytes(opl, cls, lists, p.counters != 0);
#define HM_LAUNCH(O_, L_, C_) hipLaunchKernelGGL((hm::merge_small_kernel<O_, L_, C_>), dim3(grid), dim3(WAVE), lds, s, p)
#define HM_OPL(L_, C_) switch (opl) { case 1: HM_LAUNCH(1, L_, C_); break; case 2: HM_LAUNCH(2, L_, C_); break; case 3: HM_LAUNCH(3, L_, C_); break; default: HM_LAUNCH(4, L_, C_); }
    if (cls == 0)      { if (lists) { HM_OPL(true, 0) } else { HM_OPL(false, 0) } }
    else if (cls == 2) { if (lists) { HM_OPL(true, 2) } else { HM_OPL(false, 2) } }
    else               { if (lists) { HM_OPL(true, 1) } else { HM_OPL(false, 1) } }
#undef HM_OPL
#undef HM_LAUNCH
    return hipGetLastError();
}

hipError_t hm_launch_clock(int which, const uint32_t *a, const uint32_t *b, void *out, uint32_t n_docs,
                           uint32_t S, hipStream_t s) {
    if (which == 0) {
        if (S == 0 || S > HM_MAX_STRIDE) return hipErrorInvalidValue;
        const uint32_t rows_per_wave = 64 / S;
        const uint32_t waves = (n_docs + rows_per_wave - 1) / rows_per_wave;
        const uint32_t blocks = (waves + 3) / 4;
        hipLaunchKernelGGL(hm::clock_cmp_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, s, a, b, (uint8_t *)out, n_docs, S);
    } else {
        const size_t n = (size_t)n_docs * S;
        uint32_t blocks = (uint32_t)((n + 255) / 256);
        if (blocks > 8192) blocks = 8192;
        if (which == 1) hipLaunchKernelGGL(hm::clock_union_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, s, a, b, (uint32_t *)out, n);
        else hipLaunchKernelGGL(hm::clock_intersection_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, s, a, b, (uint32_t *)out, n);
    }
    return hipGetLastError();
}
