// store_kernels.hip — device side of the resident document store (store.cpp).
//
//  append_kernel        one workgroup per document of a submit: moves the document's
//                       log segments when they outgrow their capacity (or on arena
//                       compaction), applies an actor-rank remap to the old rows and to
//                       the rank-indexed per-document rows (minimumClock, stored clock),
//                       and appends the new change/dep/op rows with their offsets rebased
//                       from batch-local to arena positions.
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

__global__ __launch_bounds__(SWG) void append_kernel(const AppendDesc *descs, uint32_t n_desc, StoreArenas src,
                                                     StoreArenas dst, const hm_change_row *st_changes,
                                                     const hm_dep_row *st_deps, const hm_op_row *st_ops,
                                                     const uint8_t *remap, uint32_t S) {
    const uint32_t t = threadIdx.x;
    for (uint32_t di = blockIdx.x; di < n_desc; di += gridDim.x) {
        const AppendDesc D = descs[di];
        const bool moved = D.src_c != D.dst_c || D.src_d != D.dst_d || D.src_o != D.dst_o || src.changes != dst.changes;
        const bool rm = D.remap_row != 0xFFFFFFFFu;
        const uint8_t *mp = rm ? remap + (size_t)D.remap_row * S : nullptr;
        // old rows: moved (rebased) and/or re-ranked
        if (moved || rm) {
            const int64_t dd = (int64_t)D.dst_d - (int64_t)D.src_d, dop = (int64_t)D.dst_o - (int64_t)D.src_o;
            for (uint32_t i = t; i < D.n_old_c; i += SWG) {
                hm_change_row c = src.changes[D.src_c + i];
                c.dep_off = (uint32_t)((int64_t)c.dep_off + dd);
                c.op_first = (uint32_t)((int64_t)c.op_first + dop);
                if (rm && c.actor < S) c.actor = mp[c.actor];
                dst.changes[D.dst_c + i] = c;
            }
            for (uint32_t i = t; i < D.n_old_d; i += SWG) {
                hm_dep_row r = src.deps[D.src_d + i];
                if (rm && r.actor < S) r.actor = mp[r.actor];
                dst.deps[D.dst_d + i] = r;
            }
        }
        if (moved) {
            // 32-byte op rows as two 16-byte words per thread
            const uint4 *so = reinterpret_cast<const uint4 *>(src.ops + D.src_o);
            uint4 *dop = reinterpret_cast<uint4 *>(dst.ops + D.dst_o);
            for (uint32_t i = t; i < 2 * D.n_old_o; i += SWG) dop[i] = so[i];
        }
        // new rows: batch-local offsets -> arena offsets
        const uint32_t c_at = D.dst_c + D.n_old_c, d_at = D.dst_d + D.n_old_d, o_at = D.dst_o + D.n_old_o;
        for (uint32_t i = t; i < D.n_new_c; i += SWG) {
            hm_change_row c = st_changes[D.new_c + i];
            c.dep_off = d_at + (c.dep_off - D.new_d);
            c.op_first = o_at + (c.op_first - D.new_o);
            dst.changes[c_at + i] = c;
        }
        for (uint32_t i = t; i < D.n_new_d; i += SWG) dst.deps[d_at + i] = st_deps[D.new_d + i];
        {
            const uint4 *so = reinterpret_cast<const uint4 *>(st_ops + D.new_o);
            uint4 *dop = reinterpret_cast<uint4 *>(dst.ops + o_at);
            for (uint32_t i = t; i < 2 * D.n_new_o; i += SWG) dop[i] = so[i];
        }
        // rank-indexed per-document rows follow the remap
        if (rm && t == 0) {
            uint32_t *rows[2] = {dst.min_clock + (size_t)D.handle * S, dst.stored_clock + (size_t)D.handle * S};
            for (int w = 0; w < 2; w++) {
                uint32_t tmp[32];
                for (uint32_t a = 0; a < S && a < 32; a++) tmp[a] = 0;
                for (uint32_t a = 0; a < S && a < 32; a++) {
                    const uint32_t na = mp[a];
                    if (na < S && na < 32) tmp[na] = rows[w][a];
                }
                for (uint32_t a = 0; a < S && a < 32; a++) rows[w][a] = tmp[a];
            }
        }
        __syncthreads();
    }
}

// out = [n x hm_doc_result][n x S clock][n x S back_clock][n x S heads]
__global__ void gather_kernel(const uint32_t *handles, uint32_t n, uint32_t S, const hm_doc_result *res_docs,
                              const uint32_t *clock, const uint32_t *back_clock, const uint32_t *heads,
                              uint8_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = handles[i];
    reinterpret_cast<hm_doc_result *>(out)[i] = res_docs[h];
    uint32_t *oc = reinterpret_cast<uint32_t *>(out + (size_t)n * sizeof(hm_doc_result));
    for (uint32_t a = 0; a < S; a++) {
        oc[(size_t)i * S + a] = clock[(size_t)h * S + a];
        oc[(size_t)n * S + (size_t)i * S + a] = back_clock[(size_t)h * S + a];
        oc[(size_t)2 * n * S + (size_t)i * S + a] = heads[(size_t)h * S + a];
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

}  // namespace hms

hipError_t hm_launch_append(const AppendDesc *descs, uint32_t n_desc, const StoreArenas &src, const StoreArenas &dst,
                            const hm_change_row *st_changes, const hm_dep_row *st_deps, const hm_op_row *st_ops,
                            const uint8_t *remap, uint32_t S, hipStream_t s) {
    if (!n_desc) return hipSuccess;
    const uint32_t grid = n_desc < 65535u ? n_desc : 65535u;
    hipLaunchKernelGGL(hms::append_kernel, dim3(grid), dim3(SWG), 0, s, descs, n_desc, src, dst, st_changes, st_deps,
                       st_ops, remap, S);
    return hipGetLastError();
}

hipError_t hm_launch_gather(const uint32_t *handles, uint32_t n, uint32_t S, const hm_doc_result *res_docs,
                            const uint32_t *clock, const uint32_t *back_clock, const uint32_t *heads, uint8_t *out,
                            hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::gather_kernel, dim3((n + 255) / 256), dim3(256), 0, s, handles, n, S, res_docs, clock,
                       back_clock, heads, out);
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
