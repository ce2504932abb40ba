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
    uint32_t cap_regs, cap_objs;     // LDS carve of this launch
};

size_t hm_small_lds_bytes(uint32_t opl, uint32_t cap_regs, uint32_t cap_objs, bool lists);
hipError_t hm_launch_small(const SmallParams &p, uint32_t opl, bool lists, uint32_t grid, hipStream_t s);
// which: 0 cmp (out uint8_t*), 1 union, 2 intersection (out uint32_t*)
hipError_t hm_launch_clock(int which, const uint32_t *a, const uint32_t *b, void *out, uint32_t n_docs,
                           uint32_t S, hipStream_t s);
