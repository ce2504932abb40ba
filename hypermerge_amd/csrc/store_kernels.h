// store_kernels.h — launch interface shared by store.cpp and store_kernels.hip
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/hypermerge_amd.h"

// One document of a submit.  src_* / dst_*: the document's segment starts before / after
// the append (equal unless the segment moved); n_old_*: rows already in the log;
// new_* / n_new_*: the new rows' range in the staged batch tables.  The register segment
// (r_*), the document's totals and `inc` (1 = apply incrementally, inc_apply_kernel) are read
// by the incremental path only.
struct AppendDesc {
    uint32_t handle;
    uint32_t src_c, dst_c, n_old_c, new_c, n_new_c;
    uint32_t src_d, dst_d, n_old_d, new_d, n_new_d;
    uint32_t src_o, dst_o, n_old_o, new_o, n_new_o;
    uint32_t remap_row;   // row of the remap table, or 0xFFFFFFFF
    uint32_t src_r, dst_r, n_old_r, n_r;
    uint16_t n_actors, inc;
    uint32_t n_objs;
    uint32_t o_cap;       // the op segment's capacity after the append (survivor slots, incremental path)
};

// A document's log segments and totals, resident on the device (the store plans submits there:
// a million-document round is too much host memory traffic to plan on the host).
struct DevDoc {
    uint32_t c_off, c_cap, d_off, d_cap, o_off, o_cap, r_off, r_cap;
    uint32_t n_c, n_d, n_o, n_r, n_objs;
    uint16_t n_actors, flags;
    uint32_t pad[2];      // pad[0]: HM_DDOC_* bits
};
static_assert(sizeof(DevDoc) == 64, "DevDoc is 64 B");
#define HM_DDOC_MINC 1u   // hm_doc_set_min_clock wrote the document's minimumClock row

// One batch row's plan: the document's totals before the append (the rollback restores them),
// the capacities of the segments it outgrows (0 = fits) and its route.
struct PlanRow {
    uint32_t n_c, n_d, n_o, n_r, n_objs;
    uint16_t n_actors, flags;
    uint32_t g[4];
    uint32_t inc, remapped;
};

// What the host reads back of a submit's device-side plan (one small copy per phase).
struct PlanStats {
    uint32_t err;                              // HM_PLAN_* bits of the failed checks
    uint32_t n_inc, n_cold, n_back, n_app;       // (n_app: batch rows append_kernel has work for)
    uint32_t mx[6];                            // mx[0]: documents routed to the lane pass; mx[1] = 1: alloc_kernel
                                               //   found no room for the growth and moved nothing; mx[2] / mx[3]:
                                               //   doc_rows_kernel's may-keep-state counts (all / with lists);
                                               //   mx[4]: list documents the plan routed to the group passes
    uint32_t max_c, max_o, max_r, max_objs, max_d, flags;   // launch hints of a merge list
    unsigned long long need[4];                // rows the submit's growing segments take, per space
    unsigned long long tot_c, tot_d, tot_o, tot_r;
    unsigned long long bump[4];                // arena bump pointers (device-side segment allocation;
                                               //   last: one memset clears every per-phase field)
    uint32_t n_valid, pad_v;                   // documents whose IncState can route a submit to the incremental
};                                             //   kernels (HM_IST_VALID without NOCKEY): kept by every writer
#define HM_IST_COUNTS(f) (((f) & (HM_IST_VALID | HM_IST_NOCKEY)) == HM_IST_VALID)
#define HM_PLAN_BAD_HANDLE 1u
#define HM_PLAN_REPEATED 2u
#define HM_PLAN_ROWS 4u
#define HM_PLAN_TOTALS 8u
#define HM_PLAN_CHANGE_ROWS 16u
#define HM_PLAN_REMAP 32u

struct StoreArenas {
    hm_change_row *changes;
    hm_dep_row *deps;
    hm_op_row *ops;
    uint32_t *min_clock;      // per handle, rank-indexed
    uint32_t *stored_clock;   // per handle, rank-indexed
};

// Per handle, beside the log: what the incremental path needs to touch only the registers the
// new ops hit (32 B).  Survivor lists of a document live in its op segment's survivor slots
// [0, s_used): a list that shrinks or keeps its length is rewritten in place, a list that grows
// moves to the end (s_used grows); the re-merge repacks.  smeta[slot] = (seq, actor | cset << 8)
// of the survivor's change (cset: a counter set), so isConcurrent and sortBy(actor) need no log
// search.  cabs bounds every integer counter's |base| + sum|inc| (the exact-integer rule of
// the re-merge: an integer counter is exact while that sum is <= 2^53), mapmask marks objects
// created as maps / tables (bit 0 = ROOT).  flags = 0: not built (the next submit re-merges).
struct IncState {
    uint32_t s_used, flags;
    unsigned long long cabs, mapmask;
    uint32_t pad[2];
};
static_assert(sizeof(IncState) == 32, "IncState is 32 B");
#define HM_IST_VALID 1u
// ckey[change slot] = seq | actor << 24 | applied << 31: the log's (actor, seq) keys packed, so the
// incremental path finds a fold source in a few 64-byte lines instead of the 24-byte change rows
// (documents with a seq >= 2^24 are not packed: HM_IST_NOCKEY, they re-merge)
#define HM_IST_NOCKEY 2u
// the document's list / text objects (at most HM_INC_LISTS) have their order resident: the
// lists laid end to end in object-id order, lorder[reg slot k] = the element register at
// position k of that concatenation (every inserted element, visible or not), per element
// register epos (its position), epar (parent element register | HM_HEAD) and ekey (elem << 8 |
// actor: lamportCompare's key); the list directory ldir[handle][k] = (object id, elements) of
// list k; IncState.pad[0] = elements of all lists, pad[1] = lists
#define HM_IST_LIST 4u
#define HM_INC_LISTS 8u
// the cost policy of incremental mode 1: a list document of at most this many ops re-merges (one
// small-kernel wave, all in LDS) rather than taking the one-document-per-wave incremental pass
#define HM_INC_SMALL_LIST_OPS 256u
// dev A/B (round 6, off): the G = 8 / 16 group passes take list / text ops too (list_plan /
// list_insert / list_indices in groups of G lanes, a separate instantiation at 143 VGPRs), list
// documents of strides <= 16 route there and mode 1 stops re-merging small list documents.
// Measured (profiles/r06/ab_list_groups): C5 resident 51 % incremental but 0.84x the re-merge (the
// list instantiation's ~5 ns per document, 10 % handed back, the re-merge of the rest as costly as
// re-merging all), C3 resident 1.56x instead of 2.2x (long lists shifted and re-indexed G
// elements at a time)
#ifndef HM_INC_LIST_GROUPS
#define HM_INC_LIST_GROUPS 0
#endif
// the small-list bound a store of stride S applies in incremental mode `mode`: with the group
// passes taking lists (strides <= 16) a list document's round is as cheap as a map document's, so
// none re-merges for being small; the one-document-per-wave pass (wider strides) costs as much as
// the small kernel's re-merge of such a document, which keeps mode 1's bound
__host__ __device__ inline uint32_t hm_small_list_ops(uint32_t S, uint32_t mode) {
    if (mode != 1u) return 0u;
    return (HM_INC_LIST_GROUPS && S <= 16u) ? 0u : HM_INC_SMALL_LIST_OPS;
}
// ... and a round of more than 1 / HM_INC_COST of the log's rows (changes + ops, the new ones
// included) re-merges: the per-row cost ratio of the incremental passes to the merge kernels,
// measured on C4 (profiles/r05/inc: inc_lane_kernel 25.5 ms for a 60-change first load of 1M
// documents, inc_group_kernel 0.79 ms per 1.5M changes; merge_small_kernel 2.4 ms per 64M)
#define HM_INC_COST 12u
__host__ __device__ inline uint32_t hm_ckey(uint32_t actor, uint32_t seq, bool applied) {
    return (seq & 0xFFFFFFu) | ((actor & 0x7Fu) << 24) | (applied ? 0x80000000u : 0u);
}

struct IncArgs {
    const AppendDesc *descs;
    const hm_change_row *st_changes;           // the submit's staged rows (batch-local offsets): the
    const hm_dep_row *st_deps;                 // kernel appends the new rows of its documents whose
    const hm_op_row *st_ops;                   // segments did not move (append_kernel skips those)
    uint32_t n;                                // batch rows (descs)
    const uint32_t *list;                      // NULL: every desc; else list[0] = count, list[1..] desc indices
    uint32_t S;
    hm_change_row *changes;
    hm_dep_row *deps;
    hm_op_row *ops;
    int32_t *hist;
    uint32_t *ckey;
    uint32_t *all_deps;
    hm_reg_result *regs;
    hm_surv_result *surv;
    uint2 *smeta;
    uint32_t *epos, *epar, *ekey, *lorder;     // list order (reg space), HM_IST_LIST documents
    uint2 *ldir;                               // list directory (HM_INC_LISTS per handle)
    hm_doc_result *res_docs;
    uint32_t *clock, *back_clock, *heads;
    const uint32_t *min_clock;
    IncState *ist;
    uint32_t *bail;                            // [0] count, [1..] handles re-merged
    uint32_t *defer;                           // [0] count, [1..] desc indices for the wave kernel (NULL: bail)
    uint32_t n_lane;                           // documents routed to the lane pass (0: no launch)
    uint8_t *gout;                             // the submit's gather buffer (gather_kernel's layout), or NULL
    uint8_t *gdone;                            // [n] 1: the row was gathered by the incremental kernels
    const PlanStats *pst;                      // the submit's plan stats (n_inc, mx[0]: work for the passes), or NULL
};

// AppendDesc.inc: the route (bits 0-1: 0 re-merge, 1 incremental group pass, 2 wave pass, 3 lane pass) and what
// alloc_kernel adds for the incremental kernels
#define HM_DINC_ROUTE 3u
#define HM_DINC_MINC 4u        // the document has a minimumClock row (else it reads as zeros)
#define HM_DINC_LISTS 8u       // the document has list / text objects

// envelope of the incremental path (larger submits take the full re-merge)
#define HM_INC_MAX_NEW_C 8
#define HM_INC_MAX_NEW_O 64
#define HM_INC_MAX_TGT 128       // transitiveDeps fold steps of a submit's new changes (2 per lane, wave kernel)
#define HM_INC_LANE_MAX_C 64     // the one-lane pass (map documents, strides <= 16)
#define HM_INC_LANE_MAX_O 512
#define HM_INC_TILED_MAX_C 256    // tiles of the group / wave passes (list documents, strides over 16)
#define HM_INC_TILED_MAX_O 4096

struct PlanArgs {
    const hm_doc_row *docs;
    const hm_change_row *changes;
    const uint32_t *handles;
    const uint8_t *remap;                      // [n * S] or NULL
    uint32_t n, n_changes, n_deps, n_ops, n_handles, S, stamp, incremental;
    DevDoc *dm;
    const hm_doc_result *res_docs;
    uint32_t *seen;
    PlanRow *plan;
    AppendDesc *descs;
    uint32_t *list;                            // cold handles
    uint32_t *alist;                           // batch rows to append (cold, moved or re-ranked)
    PlanStats *st;
    const IncState *ist;                       // incremental stores: documents the incremental kernel
    const hm_op_row *ops;                      //   would hand back are routed to the re-merge at once
    const hm_dep_row *deps;                    //   (staged deps, and the resident clocks: changes that
    const uint32_t *clock;                     //   are not causally ready in arrival order)
    uint32_t *defer;                           // the one-document-per-wave pass's list ([0] = count):
                                               //   documents with list ops go there directly
    uint32_t *bail, *fail;                     // counts the plan zeroes for the later kernels (NULL: none)
    unsigned long long cap[4];                 // arena capacities: alloc_kernel does nothing past them
    uint8_t *gdone;                            // [n] the incremental kernels' gathered-row flags (zeroed)
};
hipError_t hm_launch_plan(const PlanArgs &a, hipStream_t s);
hipError_t hm_launch_alloc(const PlanArgs &a, hipStream_t s);
// hm_doc_row of each listed handle from its device meta (+ the launch hints in st)
// (mx[2] / mx[3] of the stats: listed documents that may keep incremental state after their re-merge —
// all but the list documents of at most small_lists ops — and those of them with lists; keep (if
// not NULL) lists the former's handles, ist (if not NULL) has the others' IncState cleared)
hipError_t hm_launch_doc_rows(const uint32_t *list, uint32_t n, const DevDoc *dm, hm_doc_row *rows, PlanStats *st,
                              uint32_t small_lists, IncState *ist, uint32_t *keep, hipStream_t s);
// documents of a batch whose merge failed (every = all of the batch's documents): totals restored,
// rows re-ranked back, listed for re-merge
hipError_t hm_launch_rollback(const uint32_t *handles, uint32_t n, const hm_doc_result *res_docs, PlanRow *plan,
                              const uint8_t *remap, uint32_t S, DevDoc *dm, AppendDesc *descs, uint8_t *inv,
                              uint32_t *list, PlanStats *st, uint32_t every, hipStream_t s);
hipError_t hm_launch_init_docs(DevDoc *dm, uint32_t h0, uint32_t n, hipStream_t s);
hipError_t hm_launch_reset_docs(const uint32_t *handles, uint32_t n, DevDoc *dm, hm_doc_result *res, IncState *ist,
                                uint32_t *clock, uint32_t *back, uint32_t *heads, uint32_t *minc, uint32_t *stored,
                                uint32_t S, uint32_t *n_valid, hipStream_t s);
// chosen registers of resident documents by (handle, register): validated on the device
hipError_t hm_launch_read_hist(uint32_t n, const uint32_t *handles, const uint32_t *from, const uint32_t *to,
                               const uint32_t *out_off, const DevDoc *dm, uint32_t n_handles, const int32_t *hist,
                               const uint32_t *all_deps, uint32_t S, uint32_t *out_log, uint32_t *out_ad, uint32_t *bad,
                               hipStream_t s);
hipError_t hm_launch_read_regs_h(uint32_t n, const uint32_t *handles, const uint32_t *regs, const DevDoc *dm,
                                 uint32_t n_handles, const hm_reg_result *rr, const hm_surv_result *surv,
                                 hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t cap, uint32_t *counter,
                                 uint32_t *bad, hipStream_t s);

// incremental applyRemoteChanges: a group of G = (S <= 8 ? 8 : S <= 16 ? 16 : 64) lanes per document,
// then the documents it handed over (defer list) one per wave; the rest listed in bail
hipError_t hm_launch_inc_apply(const IncArgs &A, hipStream_t s);
// survivor metadata / IncState of re-merged documents (so the next submit can go incremental)
struct MetaArgs {
    const uint32_t *list;
    uint32_t n;
    const DevDoc *dm;
    const hm_doc_result *res_docs;
    const hm_change_row *changes;
    const int32_t *hist;
    uint32_t *ckey;
    const hm_op_row *ops;
    const hm_surv_result *surv;
    uint2 *smeta;
    IncState *ist;
    uint32_t *epos, *epar, *ekey, *lorder;
    uint2 *ldir;
    uint32_t small_lists;                      // list documents of at most this many ops keep no list state
    uint32_t *n_valid;                         // PlanStats.n_valid (the documents' states that count)
    int *part;                                 // [HM_META_GRID] per-workgroup changes of n_valid (scratch)
};
#define HM_META_GRID 65535u                    // inc_meta_kernel's largest grid
hipError_t hm_launch_inc_meta(const MetaArgs &a, hipStream_t s);
// element positions of the listed list documents reset (HM_NONE) before their re-merge writes them
hipError_t hm_launch_epos_clear(const uint32_t *list, uint32_t n, const DevDoc *dm, uint32_t *epos, hipStream_t s);
hipError_t hm_launch_append(const AppendDesc *descs, uint32_t n_desc, const StoreArenas &src, const StoreArenas &dst,
                            const hm_change_row *st_changes, const hm_dep_row *st_deps, const hm_op_row *st_ops,
                            const uint8_t *remap, uint32_t S, hipStream_t s,
                            const uint32_t *list = nullptr, const uint32_t *count = nullptr);
hipError_t hm_launch_read_regs(uint32_t n, const uint32_t *abs_reg, const uint32_t *surv_base, const hm_reg_result *regs,
                               const hm_surv_result *surv, hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t cap,
                               uint32_t *counter, hipStream_t s);
hipError_t hm_launch_gather(const uint32_t *handles, uint32_t n, uint32_t S, const hm_doc_result *res_docs,
                            const uint32_t *clock, const uint32_t *back_clock, const uint32_t *heads, uint8_t *out,
                            uint32_t *n_fail, hipStream_t s, const uint8_t *gdone = nullptr);
hipError_t hm_launch_clock_update(const uint32_t *docs, uint32_t n, uint32_t S, const uint32_t *back_clock,
                                  uint32_t *stored, uint8_t *written, uint8_t *differs, uint32_t *out_stored,
                                  hipStream_t s);
hipError_t hm_launch_sync_ranges(const uint64_t *present, const uint64_t *word_off, const uint32_t *lo,
                                 const uint32_t *hi, uint32_t *out_end, uint32_t n, hipStream_t s);
