// store_kernels.h — launch interface shared by store.cpp and store_kernels.hip
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/hypermerge_amd.h"

// One document of a submit.  src_* / dst_*: the document's segment starts before / after
// the append (equal unless the segment moved); n_old_*: rows already in the log;
// new_* / n_new_*: the new rows' range in the staged batch tables.
struct AppendDesc {
    uint32_t handle;
    uint32_t src_c, dst_c, n_old_c, new_c, n_new_c;
    uint32_t src_d, dst_d, n_old_d, new_d, n_new_d;
    uint32_t src_o, dst_o, n_old_o, new_o, n_new_o;
    uint32_t remap_row;   // row of the remap table, or 0xFFFFFFFF
};

struct StoreArenas {
    hm_change_row *changes;
    hm_dep_row *deps;
    hm_op_row *ops;
    uint32_t *min_clock;      // per handle, rank-indexed
    uint32_t *stored_clock;   // per handle, rank-indexed
};

hipError_t hm_launch_append(const AppendDesc *descs, uint32_t n_desc, const StoreArenas &src, const StoreArenas &dst,
                            const hm_change_row *st_changes, const hm_dep_row *st_deps, const hm_op_row *st_ops,
                            const uint8_t *remap, uint32_t S, hipStream_t s);
hipError_t hm_launch_gather(const uint32_t *handles, uint32_t n, uint32_t S, const hm_doc_result *res_docs,
                            const uint32_t *clock, const uint32_t *back_clock, const uint32_t *heads, uint8_t *out,
                            hipStream_t s);
hipError_t hm_launch_clock_update(const uint32_t *docs, uint32_t n, uint32_t S, const uint32_t *back_clock,
                                  uint32_t *stored, uint8_t *written, uint8_t *differs, uint32_t *out_stored,
                                  hipStream_t s);
hipError_t hm_launch_sync_ranges(const uint64_t *present, const uint64_t *word_off, const uint32_t *lo,
                                 const uint32_t *hi, uint32_t *out_end, uint32_t n, hipStream_t s);
