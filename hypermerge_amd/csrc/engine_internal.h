// engine_internal.h — what store.cpp needs from the engine (not part of the C-ABI)
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/hypermerge_amd.h"

// row extents of the tables a launch's document rows index (the store's arenas)
struct hm_extents { uint32_t n_changes, n_deps, n_ops, n_regs; };

// launch the merge kernels on the engine stream; doc_slot maps launch rows to the rows of
// the per-document outputs (NULL = identity); ext = table extents (NULL = the batch's counts);
// epos (optional, indexed like o->regs) receives every list element's document-order position
int hm_engine_launch_merge(hm_engine *e, const hm_batch *b, const hm_results *o, const uint32_t *doc_slot,
                           const hm_extents *ext, uint32_t *epos = nullptr);
hipStream_t hm_engine_stream(hm_engine *e);
int hm_engine_device(hm_engine *e);
int hm_engine_fail(hm_engine *e, int status, const char *msg);
