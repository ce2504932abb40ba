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
};

struct StoreArenas {
    hm_change_row *changes;
    hm_dep_row *deps;
    hm_op_row *ops;
    uint32_t *min_clock;      // per handle, rank-indexed
    uint32_t *stored_clock;   // per handle, rank-indexed
};

struct IncArenas {
    const hm_change_row *changes;
    const hm_dep_row *deps;
    const hm_op_row *ops;
    int32_t *hist;
    uint32_t *all_deps;
    hm_reg_result *regs;
    hm_surv_result *surv;
    hm_doc_result *res_docs;
    uint32_t *clock, *back_clock, *heads;
    const uint32_t *min_clock;
};

// envelope of the incremental path (larger submits take the full re-merge)
#define HM_INC_MAX_NEW_C 8
#define HM_INC_MAX_NEW_O 64
#define HM_INC_MAX_TGT 64        // allDeps fold steps of a submit's new changes
#define HM_INC_MAX_REGS 256
#define HM_INC_MAX_SURV 256
#define HM_INC_MAX_STAGE 512     // old change rows staged in LDS (longer logs are searched in HBM)
#define HM_INC_SLOTS 8
#define HM_INC_SLOT_CAP 32

// per-launch LDS tiles, sized to the launch's largest document (dynamic LDS)
struct IncDims {
    uint32_t S, new_c, tgt, stage, regs, surv, slots;
    uint32_t o_nc, o_dep, o_tkey, o_tsrc, o_tad, o_adn, o_skey, o_sof, o_reg, o_sold, o_wl, o_wls, o_wla, o_scnt, bytes;
};
IncDims hm_inc_dims(uint32_t S, uint32_t new_c, uint32_t tgt, uint32_t stage, uint32_t regs, uint32_t surv,
                    uint32_t slots);

hipError_t hm_launch_inc_apply(const AppendDesc *descs, uint32_t n, const IncArenas &A, const IncDims &M,
                               uint32_t *bail, hipStream_t s);
hipError_t hm_launch_append(const AppendDesc *descs, uint32_t n_desc, const StoreArenas &src, const StoreArenas &dst,
                            const hm_change_row *st_changes, const hm_dep_row *st_deps, const hm_op_row *st_ops,
                            const uint8_t *remap, uint32_t S, hipStream_t s);
hipError_t hm_launch_read_regs(uint32_t n, const uint32_t *abs_reg, const uint32_t *surv_base, const hm_reg_result *regs,
                               const hm_surv_result *surv, hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t cap,
                               uint32_t *counter, hipStream_t s);
hipError_t hm_launch_gather(const uint32_t *handles, uint32_t n, uint32_t S, const hm_doc_result *res_docs,
                            const uint32_t *clock, const uint32_t *back_clock, const uint32_t *heads, uint8_t *out,
                            hipStream_t s);
hipError_t hm_launch_clock_update(const uint32_t *docs, uint32_t n, uint32_t S, const uint32_t *back_clock,
                                  uint32_t *stored, uint8_t *written, uint8_t *differs, uint32_t *out_stored,
                                  hipStream_t s);
hipError_t hm_launch_sync_ranges(const uint64_t *present, const uint64_t *word_off, const uint32_t *lo,
                                 const uint32_t *hi, uint32_t *out_end, uint32_t n, hipStream_t s);
