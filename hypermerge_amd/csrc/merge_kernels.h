// merge_kernels.h — launch parameters shared by engine.cpp and merge_kernels.hip
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/hypermerge_amd.h"

struct SmallParams {
    const hm_doc_row *docs;
    const hm_change_row *changes;
    const hm_dep_row *deps;
    const hm_op_row *ops;
    const uint32_t *min_clock;
    hm_doc_result *res_docs;
    uint32_t *res_clock, *res_back_clock, *res_heads;
    int32_t *res_hist;
    uint32_t *res_all_deps;
    hm_reg_result *res_regs;
    hm_surv_result *res_surv;
    uint32_t n_docs, a_stride;
    uint32_t cap_regs, cap_objs;     // LDS carve of this launch (set by the kernel's size class)
    uint32_t cap_deps;               // dep rows per document the carve holds
    uint32_t counters;               // the carve has the counter sums (HM_DOC_HAS_COUNTERS)
    uint32_t *large_cursor;          // merge_large_kernel's document cursor (zeroed before the launch)
    uint32_t *n_deferred;            // documents merge_small_kernel handed over (zeroed before the launch)
    uint32_t *deferred;              // [n_docs] their launch rows, in hand-over order
    uint32_t general_only;           // HM_CFG_GENERAL_ONLY: defer every document
    uint32_t xcd_remap;              // 1: neighbouring documents go to workgroups on one XCD
    const uint32_t *doc_slot;        // optional: launch row d -> row of the per-document outputs
                                     // (res_docs, clocks, heads, min_clock); NULL = identity
    // extents of the row tables: a document row whose ranges leave them (or whose n_actors
    // exceeds a_stride) is reported HM_ERR_INVALID and never read through
    uint32_t lim_changes, lim_deps, lim_ops, lim_regs;
    // optional (the resident store): per list element register, its position in its list's
    // document order (every inserted element, visible or not) — the order the incremental path
    // keeps resident; rows of other registers are not written
    uint32_t *res_epos;
};
#ifdef __HIPCC__
__device__ __forceinline__ bool hm_doc_row_ok(const SmallParams &p, const hm_doc_row &d) {
    return (unsigned long long)d.change_off + d.n_changes <= p.lim_changes &&
           (unsigned long long)d.dep_off + d.n_deps <= p.lim_deps &&
           (unsigned long long)d.op_off + d.n_ops <= p.lim_ops &&
           (unsigned long long)d.reg_off + d.n_regs <= p.lim_regs && d.n_actors <= p.a_stride;
}
#endif
#ifdef __HIPCC__
__device__ __forceinline__ uint32_t hm_slot(const SmallParams &p, uint32_t d) { return p.doc_slot ? p.doc_slot[d] : d; }
#endif

// internal: the small kernel hands a document to merge_large_kernel (never returned to callers)
#define HM_DEFERRED 0x7FFFFFFF

// bytes of device scratch a launch over `b` uses: [256 B counters][deferred list][large-kernel pool]
size_t hm_launch_scratch_bytes(const hm_batch *b);

size_t hm_large_scratch_bound(const hm_batch *b);
size_t hm_large_stack_bytes();
hipError_t hm_launch_large(const SmallParams &p, void *pool, size_t pool_bytes, unsigned long long *pool_used,
                           uint32_t grid, hipStream_t s);
// small-kernel size class (LDS carve) for a batch's per-document maxima
uint32_t hm_small_class(uint32_t max_regs, uint32_t max_objs, uint32_t max_deps);
size_t hm_small_lds_bytes(uint32_t opl, uint32_t cls, bool lists, bool counters);
uint32_t hm_small_occupancy(uint32_t opl, uint32_t cls, bool lists, bool counters);
hipError_t hm_launch_small(const SmallParams &p, uint32_t opl, uint32_t cls, bool lists, uint32_t grid, hipStream_t s);
// which: 0 cmp (out uint8_t*), 1 union, 2 intersection (out uint32_t*)
hipError_t hm_launch_clock(int which, const uint32_t *a, const uint32_t *b, void *out, uint32_t n_docs,
                           uint32_t S, hipStream_t s);
