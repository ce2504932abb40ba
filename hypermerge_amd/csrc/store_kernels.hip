// store_kernels.hip — device side of the resident document store (store.cpp).
//
//  append_kernel        one workgroup per document of a submit: moves the document's
//                       log segments when they outgrow their capacity (or on arena
//                       compaction), applies an actor-rank remap to the old rows and to
//                       the rank-indexed per-document rows (minimumClock, stored clock),
//                       and appends the new change/dep/op rows with their offsets rebased
//                       from batch-local to arena positions.
//  inc_apply_kernel     incremental applyRemoteChanges: new changes applied on the resident
//                       state of documents whose submit is causally ready (see below).
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
    // one wave per document (a submit's appends are a few rows each; a 256-lane group per
    // document would idle most of its lanes), four documents per workgroup
    const uint32_t t = threadIdx.x & 63, W = 64;
    for (uint32_t di = blockIdx.x * 4 + (threadIdx.x >> 6); di < n_desc; di += gridDim.x * 4) {
        const AppendDesc D = descs[di];
        const bool moved = D.src_c != D.dst_c || D.src_d != D.dst_d || D.src_o != D.dst_o || src.changes != dst.changes;
        const bool rm = D.remap_row != 0xFFFFFFFFu;
        const uint8_t *mp = rm ? remap + (size_t)D.remap_row * S : nullptr;
        // old rows: moved (rebased) and/or re-ranked
        if (moved || rm) {
            const int64_t dd = (int64_t)D.dst_d - (int64_t)D.src_d, dop = (int64_t)D.dst_o - (int64_t)D.src_o;
            for (uint32_t i = t; i < D.n_old_c; i += W) {
                hm_change_row c = src.changes[D.src_c + i];
                c.dep_off = (uint32_t)((int64_t)c.dep_off + dd);
                c.op_first = (uint32_t)((int64_t)c.op_first + dop);
                if (rm && c.actor < S) c.actor = mp[c.actor];
                dst.changes[D.dst_c + i] = c;
            }
            for (uint32_t i = t; i < D.n_old_d; i += W) {
                hm_dep_row r = src.deps[D.src_d + i];
                if (rm && r.actor < S) r.actor = mp[r.actor];
                dst.deps[D.dst_d + i] = r;
            }
        }
        if (moved) {
            // 32-byte op rows as two 16-byte words per thread
            const uint4 *so = reinterpret_cast<const uint4 *>(src.ops + D.src_o);
            uint4 *dop = reinterpret_cast<uint4 *>(dst.ops + D.dst_o);
            for (uint32_t i = t; i < 2 * D.n_old_o; i += W) dop[i] = so[i];
        }
        // new rows: batch-local offsets -> arena offsets
        const uint32_t c_at = D.dst_c + D.n_old_c, d_at = D.dst_d + D.n_old_d, o_at = D.dst_o + D.n_old_o;
        for (uint32_t i = t; i < D.n_new_c; i += W) {
            hm_change_row c = st_changes[D.new_c + i];
            c.dep_off = d_at + (c.dep_off - D.new_d);
            c.op_first = o_at + (c.op_first - D.new_o);
            dst.changes[c_at + i] = c;
        }
        for (uint32_t i = t; i < D.n_new_d; i += W) dst.deps[d_at + i] = st_deps[D.new_d + i];
        {
            const uint4 *so = reinterpret_cast<const uint4 *>(st_ops + D.new_o);
            uint4 *dop = reinterpret_cast<uint4 *>(dst.ops + o_at);
            for (uint32_t i = t; i < 2 * D.n_new_o; i += W) dop[i] = so[i];
        }
        // rank-indexed per-document rows follow the remap: lane t gathers the new ranks t + 64k
        // (k < 4: S <= HM_MAX_STRIDE) from every old rank, all loads before any store (one wave)
        if (rm) {
            uint32_t *rows[2] = {dst.min_clock + (size_t)D.handle * S, dst.stored_clock + (size_t)D.handle * S};
            for (int w = 0; w < 2; w++) {
                uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
                for (uint32_t a = 0; a < S; a++) {
                    const uint32_t na = mp[a];
                    if (na >= S || (na & 63) != t) continue;
                    const uint32_t x = rows[w][a];
                    const uint32_t k = na >> 6;
                    v0 = k == 0 ? x : v0; v1 = k == 1 ? x : v1; v2 = k == 2 ? x : v2; v3 = k == 3 ? x : v3;
                }
                __builtin_amdgcn_wave_barrier();
                if (t < S) rows[w][t] = v0;
                if (t + 64 < S) rows[w][t + 64] = v1;
                if (t + 128 < S) rows[w][t + 128] = v2;
                if (t + 192 < S) rows[w][t + 192] = v3;
            }
        }
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

// ---------------- incremental applyRemoteChanges ----------------
// inc_apply_kernel: one wave per document whose new changes all apply in arrival order on
// the resident state (Automerge's applyQueuedOps applies them in its first pass when each is
// causally ready after the previous ones; DocBackend.ts:169-185 -> Backend.applyChanges).
// For each new change: causallyReady against the resident opSet.clock, allDeps by the
// transitiveDeps fold over the resident allDeps rows (each old fold source found by
// (actor, seq) in one scan of the log), history position, heads and clock.  For each new map
// op (set / del / link): the register's survivors filtered to the concurrent ones, the op
// pushed, sortBy(actor).reverse() — only the registers the new ops hit are recomputed; the
// rest of the register table is repacked as it was.  Anything outside that (a duplicate or
// not-yet-ready change, inc / counter / list / object-creation ops, an unknown object, tiles
// too small) lists the document in bail before any merged state is written, and the host re-merges that
// document's whole log with the batch kernels.  The loads that depend only on the
// descriptor (new rows, clock / heads, the old log's (actor, seq) keys, the register table,
// the survivors) are issued together; the remaining dependent steps are one scan of the log
// and one gather of allDeps rows.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t lane_bcast(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t key_of(const hm_change_row *r) {
    const uint2 w = *reinterpret_cast<const uint2 *>(r);          // actor | n_deps << 16, seq
    return ((uint64_t)(w.x & 0xFFFFu) << 32) | w.y;
}

// was object `o` created as a map/table by an op of the old log?
__device__ bool inc_obj_is_map(const AppendDesc &D, const IncArenas &A, uint32_t o, uint32_t lane) {
    for (uint32_t base = 0; base < D.n_old_o; base += 64) {
        const uint32_t i = base + lane;
        bool m = false;
        uint32_t act = 0;
        if (i < D.n_old_o) {
            const hm_op_row &r = A.ops[D.dst_o + i];
            act = r.action;
            m = act <= HM_MAKE_TEXT && r.obj == o;
        }
        const uint64_t b = wave_ballot(m);
        if (b) {
            const uint32_t first = lane_bcast(act, (uint32_t)__builtin_ctzll(b));
            return first == HM_MAKE_MAP || first == HM_MAKE_TABLE;
        }
    }
    return false;
}

__device__ bool inc_doc(const AppendDesc &D, const IncArenas &A, const IncDims &M, uint32_t lane, uint8_t *lds) {
    const uint32_t S = M.S, h = D.handle, NA = D.n_actors, nnc = D.n_new_c, nno = D.n_new_o;
    uint32_t *nc = reinterpret_cast<uint32_t *>(lds + M.o_nc);          // per new change: 8 words
    uint32_t *dep = reinterpret_cast<uint32_t *>(lds + M.o_dep);        // new deps: actor, seq
    uint64_t *tkey = reinterpret_cast<uint64_t *>(lds + M.o_tkey);      // fold steps: (actor, seq)
    int32_t *tsrc = reinterpret_cast<int32_t *>(lds + M.o_tsrc);        // new change index, or -1 (old)
    uint32_t *tidx = reinterpret_cast<uint32_t *>(tsrc + M.tgt), *tcnt = tidx + M.tgt;
    uint32_t *tad = reinterpret_cast<uint32_t *>(lds + M.o_tad);        // allDeps rows of old sources
    uint32_t *adn = reinterpret_cast<uint32_t *>(lds + M.o_adn);        // allDeps rows of the new changes
    uint64_t *skey = reinterpret_cast<uint64_t *>(lds + M.o_skey);      // staged old log: (actor, seq)
    uint32_t *sof = reinterpret_cast<uint32_t *>(lds + M.o_sof);        //                 first op
    uint32_t *r_cnt = reinterpret_cast<uint32_t *>(lds + M.o_reg), *r_off = r_cnt + M.regs, *r_obj = r_off + M.regs;
    uint8_t *r_slot = reinterpret_cast<uint8_t *>(r_obj + M.regs);
    hm_surv_result *sold = reinterpret_cast<hm_surv_result *>(lds + M.o_sold);
    hm_surv_result *wl = reinterpret_cast<hm_surv_result *>(lds + M.o_wl);
    uint32_t *wls = reinterpret_cast<uint32_t *>(lds + M.o_wls), *scnt = reinterpret_cast<uint32_t *>(lds + M.o_scnt);
    uint8_t *wla = lds + M.o_wla;

    const uint32_t hist_len = uni(A.res_docs[h].hist_len), n_old_surv = uni(A.res_docs[h].n_surv);
    // (lane-per-actor rows: wide strides re-merge; survivor actor bytes keep 7 bits)
    if (S > 64 || NA > S || nnc == 0 || nnc > M.new_c || nno > 64 || D.n_r > M.regs || n_old_surv > M.surv || D.n_old_r > D.n_r)
        return false;
    const bool staged = D.n_old_c <= M.stage;

    // ---- loads that depend only on the descriptor ----
    uint32_t clk = 0, hd = 0, mc = 0;
    if (lane < S) {
        clk = A.clock[(size_t)h * S + lane];
        hd = A.heads[(size_t)h * S + lane];
        mc = A.min_clock ? A.min_clock[(size_t)h * S + lane] : 0u;
    }
    uint32_t ca = 0, cq = 0, cnd = 0, cdo = 0, cno = 0, coo = 0;
    if (lane < nnc) {
        const hm_change_row c = A.changes[D.dst_c + D.n_old_c + lane];
        ca = c.actor; cq = c.seq; cnd = c.n_deps; cdo = c.dep_off - D.dst_d; cno = c.n_ops; coo = c.op_first - D.dst_o;
    }
    uint32_t o_act = 0, o_dt = 0, o_obj = 0, o_reg = 0, o_vt = 0, o_vlo = 0, o_vhi = 0;
    if (lane < nno) {
        const hm_op_row op = A.ops[D.dst_o + D.n_old_o + lane];
        o_act = op.action; o_dt = op.datatype; o_obj = op.obj; o_reg = op.reg; o_vt = op.vtag;
        o_vlo = (uint32_t)op.value; o_vhi = (uint32_t)(op.value >> 32);
    }
    if (staged)
        for (uint32_t i = lane; i < D.n_old_c; i += 64) {
            const hm_change_row *r = A.changes + D.dst_c + i;
            skey[i] = key_of(r);
            sof[i] = r->op_first - D.dst_o;
        }
    for (uint32_t g = lane; g < D.n_r; g += 64) {
        uint32_t c = 0, o = 0, ob = HM_NONE;
        if (g < D.n_old_r) {
            const hm_reg_result r = A.regs[D.src_r + g];
            c = r.n_surv; o = r.surv_off; ob = r.obj;
        }
        r_cnt[g] = c; r_off[g] = o; r_obj[g] = ob; r_slot[g] = 0xFF;
    }
    for (uint32_t i = lane; i < n_old_surv; i += 64) sold[i] = A.surv[D.src_o + i];

    // ---- the new rows: layout (grouped by change, in order, after the old rows) and values ----
    uint32_t sd = lane < nnc ? cnd : 0u, so = lane < nnc ? cno : 0u;
    for (uint32_t d = 1; d < 8; d <<= 1) {
        const uint32_t yd = __shfl_up(sd, d, 64), yo = __shfl_up(so, d, 64);
        if (lane >= d) { sd += yd; so += yo; }
    }
    const uint32_t xd = sd - (lane < nnc ? cnd : 0u), xo = so - (lane < nnc ? cno : 0u);
    const uint32_t total_d = lane_bcast(sd, nnc - 1), total_o = lane_bcast(so, nnc - 1);
    const bool bad_c = lane < nnc && (ca >= NA || cq == 0 || cdo != D.n_old_d + xd || coo != D.n_old_o + xo);
    // set / del / link, counter sets, and incs by a number (an inc of anything else is left to
    // the re-merge); an inc must stay inside the exact-integer envelope checked below
    const bool bad_o = lane < nno && ((o_act != HM_SET && o_act != HM_DEL && o_act != HM_LINK && o_act != HM_INC) ||
                                      (o_act == HM_INC && o_vt != HM_V_INT && o_vt != HM_V_FLOAT) ||
                                      (o_act == HM_INC && o_vt == HM_V_INT &&
                                       ((int64_t)(((uint64_t)o_vhi << 32) | o_vlo) >= (1ll << 43) ||
                                        (int64_t)(((uint64_t)o_vhi << 32) | o_vlo) <= -(1ll << 43))) ||
                                      (o_act == HM_INC && D.n_old_o + nno > 256) ||
                                      o_obj >= D.n_objs || o_reg >= D.n_r ||
                                      (o_vt == HM_V_INT && ((int64_t)(((uint64_t)o_vhi << 32) | o_vlo) > 9007199254740992ll ||
                                                            (int64_t)(((uint64_t)o_vhi << 32) | o_vlo) < -9007199254740992ll)));
    if (wave_ballot(bad_c || bad_o) || total_o != nno || total_d != D.n_new_d || total_d + nnc > M.tgt) return false;
    if (wave_ballot(lane < nno && o_act == HM_INC)) {
        // the exact-integer envelope over the whole log (the oracle's |partial sums| <= 2^53 rule):
        // every integer counter base |v| < 2^50 and inc |v| < 2^43 in <= 256 ops bound any sum
        bool big = false;
        for (uint32_t i = lane; i < D.n_old_o; i += 64) {
            const hm_op_row &r = A.ops[D.dst_o + i];
            const int64_t v = (int64_t)r.value;
            if (r.vtag == HM_V_INT && r.action == HM_INC) big |= v >= (1ll << 43) || v <= -(1ll << 43);
            if (r.vtag == HM_V_INT && r.action == HM_SET && r.datatype == HM_DT_COUNTER) big |= v >= (1ll << 50) || v <= -(1ll << 50);
        }
        if (lane < nno && o_act == HM_SET && o_dt == HM_DT_COUNTER && o_vt == HM_V_INT) {
            const int64_t v = (int64_t)(((uint64_t)o_vhi << 32) | o_vlo);
            big |= v >= (1ll << 50) || v <= -(1ll << 50);
        }
        if (wave_ballot(big)) return false;
    }
    if (lane < nnc) {
        uint32_t *w = nc + lane * 8;
        w[0] = ca; w[1] = cq; w[2] = cnd; w[3] = xd; w[4] = cno; w[5] = xo;
    }
    for (uint32_t t = lane; t < total_d; t += 64) {
        const hm_dep_row d = A.deps[D.dst_d + D.n_old_d + t];
        dep[2 * t] = d.actor; dep[2 * t + 1] = d.seq;
    }
    __syncthreads();

    // ---- causallyReady in arrival order; the transitiveDeps fold steps (A.1) ----
    uint32_t ck = clk, nt = 0;
    for (uint32_t j = 0; j < nnc; j++) {
        const uint32_t a = uni(nc[j * 8]), q = uni(nc[j * 8 + 1]), nd = uni(nc[j * 8 + 2]), d0 = uni(nc[j * 8 + 3]);
        if (lane_bcast(ck, a) + 1u != q) return false;          // a duplicate, or not ready: queue semantics
        const uint32_t t0 = nt;
        bool own = false;
        for (uint32_t t = 0; t <= nd; t++) {
            uint32_t da, dq;
            if (t < nd) {
                da = uni(dep[2 * (d0 + t)]); dq = uni(dep[2 * (d0 + t) + 1]);
                if (da >= NA) return false;
                if (da == a) { dq = q - 1; own = true; }
            } else {
                if (own) break;
                da = a; dq = q - 1;
            }
            if (lane_bcast(ck, da) < dq) return false;
            if (dq == 0) continue;
            int src = -1;
            for (uint32_t k = 0; k < j; k++)
                if (uni(nc[k * 8]) == da && uni(nc[k * 8 + 1]) == dq) src = (int)k;
            if (lane == 0) { tkey[nt] = ((uint64_t)da << 32) | dq; tsrc[nt] = src; tcnt[nt] = 0; tidx[nt] = 0; }
            nt++;
        }
        if (lane == 0) { nc[j * 8 + 6] = t0; nc[j * 8 + 7] = nt - t0; }
        if (lane == a) ck = q;
    }
    __syncthreads();

    // ---- old fold sources: exactly one applied row of the log per (actor, seq) ----
    bool any_old = false;
    for (uint32_t t = 0; t < nt; t++) any_old |= tsrc[t] < 0;
    if (any_old) {
        for (uint32_t base = 0; base < D.n_old_c; base += 64) {
            const uint32_t i = base + lane;
            uint64_t key = ~0ull;
            if (i < D.n_old_c) key = staged ? skey[i] : key_of(A.changes + D.dst_c + i);
            for (uint32_t t = 0; t < nt; t++) {
                if (tsrc[t] >= 0) continue;
                const uint64_t m = wave_ballot(key == tkey[t]);
                if (m && lane == 0) { tcnt[t] += (uint32_t)__builtin_popcountll(m); tidx[t] = base + (uint32_t)__builtin_ctzll(m); }
            }
        }
        __syncthreads();
        for (uint32_t t = 0; t < nt; t++)
            if (tsrc[t] < 0 && uni(tcnt[t]) != 1u) return false;       // duplicates in the log: re-merge
        for (uint32_t w = lane; w < nt * S; w += 64) {
            const uint32_t t = w / S, x = w - t * S;
            tad[w] = tsrc[t] < 0 ? A.all_deps[(size_t)(D.src_c + tidx[t]) * S + x] : 0u;
        }
        __syncthreads();
    }

    // ---- per new change: allDeps, heads, clock (applyChange) ----
    for (uint32_t j = 0; j < nnc; j++) {
        const uint32_t a = uni(nc[j * 8]), q = uni(nc[j * 8 + 1]), t0 = uni(nc[j * 8 + 6]), tn = uni(nc[j * 8 + 7]);
        uint32_t adv = 0;
        for (uint32_t t = t0; t < t0 + tn; t++) {
            const uint64_t key = tkey[t];
            const uint32_t da = uni((uint32_t)(key >> 32)), dq = uni((uint32_t)key);
            const int src = (int)uni((uint32_t)tsrc[t]);
            const uint32_t row = lane < S ? (src >= 0 ? adn[src * S + lane] : tad[t * S + lane]) : 0u;
            if (lane < NA && row > adv) adv = row;
            if (lane == da) adv = dq;
        }
        if (lane >= NA) adv = 0;
        if (lane < S) adn[j * S + lane] = adv;
        if (hd && hd <= adv) hd = 0;
        if (lane == a) { hd = q; clk = q; }
        __syncthreads();
    }

    // ---- objects other than the root must be maps created by the old log ----
    {
        uint64_t om = wave_ballot(lane < nno && o_obj != 0);
        uint32_t checked = 0;
        while (om) {
            const uint32_t l = (uint32_t)__builtin_ctzll(om);
            om &= om - 1;
            const uint32_t o = lane_bcast(o_obj, l);
            if (o == checked) continue;
            if (!inc_obj_is_map(D, A, o, lane)) return false;
            checked = o;
        }
    }

    // ---- the new ops in order (applyAssign, A.2) on the registers they hit ----
    uint32_t nslots = 0, j = 0, jend = uni(nc[4]);
    for (uint32_t k = 0; k < nno; k++) {
        while (k >= jend) { j++; jend += uni(nc[j * 8 + 4]); }
        const uint32_t a = uni(nc[j * 8]), q = uni(nc[j * 8 + 1]);
        const uint32_t act = lane_bcast(o_act, k), obj = lane_bcast(o_obj, k), g = lane_bcast(o_reg, k);
        const uint32_t vtag = lane_bcast(o_vt, k);
        const uint64_t val = ((uint64_t)lane_bcast(o_vhi, k) << 32) | lane_bcast(o_vlo, k);
        uint32_t slot = uni(r_slot[g]);
        if (slot == 0xFF) {
            if (nslots == M.slots) return false;
            slot = nslots++;
            const uint32_t c0 = uni(r_cnt[g]), o0 = uni(r_off[g]);
            if (c0 > HM_INC_SLOT_CAP || o0 + c0 > n_old_surv) return false;
            if (lane < c0) {
                const hm_surv_result x = sold[o0 + lane];
                // the old change owning op x.op: the last change whose first op is <= x.op
                uint32_t lo = 0, hi = D.n_old_c;
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    const uint32_t f = staged ? sof[mid] : A.changes[D.dst_c + mid].op_first - D.dst_o;
                    if (f <= x.op) lo = mid; else hi = mid;
                }
                const uint64_t kk = staged ? skey[lo] : key_of(A.changes + D.dst_c + lo);
                const hm_op_row &xo = A.ops[D.dst_o + x.op];
                const uint32_t cset = (xo.action == HM_SET && xo.datatype == HM_DT_COUNTER) ? 0x80u : 0u;
                wl[slot * HM_INC_SLOT_CAP + lane] = x;
                wla[slot * HM_INC_SLOT_CAP + lane] = (uint8_t)((kk >> 32) | cset);
                wls[slot * HM_INC_SLOT_CAP + lane] = (uint32_t)kk;
            }
            if (lane == 0) { scnt[slot] = c0; r_slot[g] = (uint8_t)slot; }
            __syncthreads();
        }
        const uint32_t base = slot * HM_INC_SLOT_CAP, cnt = uni(scnt[slot]);
        if (act == HM_INC) {
            // applyAssign for inc (A.2): every surviving counter set that is causally before the
            // inc (its change an ancestor of the inc's: allDeps(inc)[x.actor] >= x.seq) adds the
            // inc, integer + integer exactly, anything else in f64 (the application order); nothing
            // is removed or reordered.  Integer sums stay inside the exact range: |value| < 2^50,
            // |inc| < 2^43, at most 256 ops in the log (else the re-merge decides)
            bool out = false;
            if (lane < cnt) {
                hm_surv_result x = wl[base + lane];
                const uint32_t xa = wla[base + lane], xs = wls[base + lane];
                const bool numeric = x.vtag == HM_V_INT || x.vtag == HM_V_FLOAT;
                if ((xa & 0x80u) && numeric && adn[j * S + (xa & 0x7Fu)] >= xs) {
                    if (x.vtag == HM_V_INT && vtag == HM_V_INT) {
                        const int64_t cur = (int64_t)x.value;
                        out = cur >= (1ll << 50) || cur <= -(1ll << 50);
                        x.value = (uint64_t)(cur + (int64_t)val);
                    } else {
                        double xv, iv;
                        if (x.vtag == HM_V_INT) xv = (double)(int64_t)x.value; else __builtin_memcpy(&xv, &x.value, 8);
                        if (vtag == HM_V_INT) iv = (double)(int64_t)val; else __builtin_memcpy(&iv, &val, 8);
                        const double r = xv + iv;
                        __builtin_memcpy(&x.value, &r, 8);
                        x.vtag = HM_V_FLOAT;
                    }
                    wl[base + lane] = x;
                }
            }
            if (wave_ballot(out)) return false;
            __syncthreads();
            // (then, like every assign, the stable sortBy(actor).reverse() below: an inc flips
            // the order of a change's equal-actor survivors too)
        }
        // survivors concurrent with the new op stay (isConcurrent reduces to
        // allDeps(new)[x.actor] < x.seq: no resident change can depend on the new one)
        hm_surv_result x = {};
        uint32_t xa = 0, xs = 0;
        bool keep = false;
        if (lane < cnt) {
            x = wl[base + lane]; xa = wla[base + lane]; xs = wls[base + lane];
            keep = act == HM_INC || adn[j * S + (xa & 0x7Fu)] < xs;      // an inc removes nothing
        }
        const uint64_t km = wave_ballot(keep);
        const uint32_t nk = (uint32_t)__builtin_popcountll(km), pos = lanes_below(km);
        const bool push = act != HM_DEL && act != HM_INC;
        const uint32_t ncnt = nk + (push ? 1u : 0u);
        if (ncnt > HM_INC_SLOT_CAP) return false;
        __syncthreads();
        if (keep) { wl[base + pos] = x; wla[base + pos] = (uint8_t)xa; wls[base + pos] = xs; }
        if (push && lane == 0) {
            hm_surv_result y;
            y.op = D.n_old_o + k; y.vtag = vtag; y.value = val;
            const uint32_t cset = (act == HM_SET && lane_bcast(o_dt, k) == HM_DT_COUNTER) ? 0x80u : 0u;
            wl[base + nk] = y; wla[base + nk] = (uint8_t)(a | cset); wls[base + nk] = q;
        }
        __syncthreads();
        // sortBy(actor) (stable) then reverse
        if (lane < ncnt) { x = wl[base + lane]; xa = wla[base + lane]; xs = wls[base + lane]; }
        uint32_t rank = 0;
        for (uint32_t e = 0; e < ncnt; e++) {
            const uint32_t ea = wla[base + e] & 0x7Fu, xr = xa & 0x7Fu;
            rank += (ea < xr || (ea == xr && e < lane)) ? 1u : 0u;
        }
        __syncthreads();
        if (lane < ncnt) {
            const uint32_t d = ncnt - 1 - rank;
            wl[base + d] = x; wla[base + d] = (uint8_t)xa; wls[base + d] = xs;
        }
        if (lane == 0) { scnt[slot] = ncnt; r_obj[g] = obj; }
        __syncthreads();
    }

    // ---- write back: registers (repacked in register order), survivors ----
    const bool same_o = D.src_o == D.dst_o, same_r = D.src_r == D.dst_r;
    uint32_t carry = 0;
    for (uint32_t g0 = 0; g0 < D.n_r; g0 += 64) {
        const uint32_t g = g0 + lane;
        const bool valid = g < D.n_r;
        const uint32_t slot = valid ? r_slot[g] : 0xFFu;
        const uint32_t cnt = !valid ? 0u : (slot != 0xFF ? scnt[slot] : r_cnt[g]);
        uint32_t incl = cnt;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        const uint32_t off = carry + incl - cnt;
        carry += lane_bcast(incl, 63);
        if (valid) {
            const bool unchanged = slot == 0xFF && g < D.n_old_r && off == r_off[g];
            if (!(unchanged && same_r)) {
                hm_reg_result r;
                r.n_surv = cnt; r.surv_off = off; r.list_index = -1; r.obj = r_obj[g];
                A.regs[D.dst_r + g] = r;
            }
            if (!(unchanged && same_o))
                for (uint32_t i = 0; i < cnt; i++)
                    A.surv[D.dst_o + off + i] = slot != 0xFF ? wl[slot * HM_INC_SLOT_CAP + i] : sold[r_off[g] + i];
        }
    }

    // ---- history, allDeps, clocks, the document's result row ----
    if (D.src_c != D.dst_c) {
        for (uint32_t i = lane; i < D.n_old_c; i += 64) A.hist[D.dst_c + i] = A.hist[D.src_c + i];
        for (size_t w = lane; w < (size_t)D.n_old_c * S; w += 64)
            A.all_deps[(size_t)D.dst_c * S + w] = A.all_deps[(size_t)D.src_c * S + w];
    }
    if (lane < nnc) A.hist[D.dst_c + D.n_old_c + lane] = (int32_t)(hist_len + lane);
    for (uint32_t w = lane; w < nnc * S; w += 64) A.all_deps[(size_t)(D.dst_c + D.n_old_c) * S + w] = adn[w];
    if (lane < S) {
        A.clock[(size_t)h * S + lane] = clk;
        A.back_clock[(size_t)h * S + lane] = clk;                 // queue empty: every handed change applied
        A.heads[(size_t)h * S + lane] = hd;
    }
    const bool ag = wave_ballot(lane < S && clk < mc) == 0, bg = wave_ballot(lane < S && mc < clk) == 0;
    if (lane == 0) {
        hm_doc_result r = {};
        r.status = HM_OK; r.err_change = HM_NONE; r.err_op = HM_NONE;
        r.hist_len = hist_len + nnc; r.n_queued = 0; r.n_surv = carry;
        r.min_cmp = (ag && bg) ? 0u : (ag ? 1u : (bg ? 2u : 3u));
        A.res_docs[h] = r;
    }
    return true;
}

// bail[0] = count, bail[1 ..] = the handles handed back (any order)
__global__ __launch_bounds__(64, 8) void inc_apply_kernel(const AppendDesc *descs, uint32_t n, IncArenas A, IncDims M,
                                                       uint32_t *bail) {
    extern __shared__ __align__(16) uint8_t inc_lds[];
    const uint32_t lane = threadIdx.x;
    for (uint32_t di = blockIdx.x; di < n; di += gridDim.x) {
        if (!descs[di].inc) continue;
        const AppendDesc D = descs[di];
        const bool ok = inc_doc(D, A, M, lane, inc_lds);
        if (lane == 0 && !ok) bail[1 + atomicAdd(&bail[0], 1u)] = D.handle;
        __syncthreads();
    }
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
__device__ __forceinline__ uint32_t pow2c(uint32_t x) {
    x = x < 16u ? 16u : x;
    return x <= 1u ? 1u : 1u << (32 - __builtin_clz(x - 1));
}

// the submit's reductions go through LDS to one atomic per workgroup and value: same-address
// atomics from every wave of a million-document submit queue at one L2 channel (~10 ns each:
// ~1.2 ms of a 1M-document incremental plan, the same in doc_rows_kernel)
#define PLAN_WG 1024
__global__ __launch_bounds__(PLAN_WG) void plan_kernel(PlanArgs a) {
    __shared__ unsigned long long s_need[4][PLAN_WG / 64];
    __shared__ uint32_t s_inc[PLAN_WG / 64], s_mx[6][PLAN_WG / 64];
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    if (ln == 0) {
        for (int k = 0; k < 4; k++) s_need[k][wv] = 0;
        for (int k = 0; k < 6; k++) s_mx[k][wv] = 0;
        s_inc[wv] = 0;
    }
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i0 < a.n;
    const uint32_t i = live ? i0 : 0u;
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
    p.g[0] = live && m.n_c + r.n_changes > m.c_cap ? pow2c(m.n_c + r.n_changes) : 0u;
    p.g[1] = live && m.n_d + r.n_deps > m.d_cap ? pow2c(m.n_d + r.n_deps) : 0u;
    p.g[2] = live && m.n_o + r.n_ops > m.o_cap ? pow2c(m.n_o + r.n_ops) : 0u;
    p.g[3] = live && r.n_regs > m.r_cap ? pow2c(r.n_regs) : 0u;
    for (int k = 0; k < 4; k++) {
        unsigned long long g = p.g[k];
        for (int o = 32; o > 0; o >>= 1) g += (unsigned long long)__shfl_xor((long long)g, o);
        if (ln == 0) s_need[k][wv] = g;
    }
    // route: a clean resident state (last merge ok, nothing queued, no re-rank) and new rows that
    // fit the incremental tiles -> inc_apply_kernel; the rest re-merge their whole log
    const hm_doc_result last = a.res_docs[live ? h : 0u];
    const uint32_t tgt = r.n_deps + r.n_changes;
    const bool inc = live && a.incremental && last.status == HM_OK && last.n_queued == 0 && !remapped && r.n_changes > 0 &&
                     r.n_changes <= HM_INC_MAX_NEW_C && r.n_ops <= HM_INC_MAX_NEW_O && tgt <= HM_INC_MAX_TGT &&
                     r.n_regs <= HM_INC_MAX_REGS && last.n_surv <= HM_INC_MAX_SURV && m.n_r <= r.n_regs &&
                     r.n_actors <= a.S && !((m.flags | r.flags) & HM_DOC_HAS_LISTS);
    p.inc = inc ? 1u : 0u;
    p.remapped = remapped ? 1u : 0u;
    if (live) a.plan[i] = p;
    const unsigned long long im = __ballot(inc);
    if (ln == 0) s_inc[wv] = (uint32_t)__popcll(im);
    if (im) {
        uint32_t v[6] = {inc ? r.n_changes : 0u, inc ? tgt : 0u,
                         inc ? (m.n_c < HM_INC_MAX_STAGE ? m.n_c : (uint32_t)HM_INC_MAX_STAGE) : 0u, inc ? r.n_regs : 0u,
                         inc ? last.n_surv : 0u, inc ? (r.n_ops < HM_INC_SLOTS ? r.n_ops : (uint32_t)HM_INC_SLOTS) : 0u};
        for (int k = 0; k < 6; k++) {
            for (int o = 32; o > 0; o >>= 1) { const uint32_t y = (uint32_t)__shfl_xor((int)v[k], o); v[k] = v[k] > y ? v[k] : y; }
            if (ln == 0) s_mx[k][wv] = v[k];
        }
    }
    }
    __syncthreads();
    if (threadIdx.x < 11) {                                        // one lane per reduced value
        const uint32_t k = threadIdx.x, nw = PLAN_WG / 64;
        if (k < 4) {
            unsigned long long g = 0;
            for (uint32_t w = 0; w < nw; w++) g += s_need[k][w];
            if (g) atomicAdd(&a.st->need[k], g);
        } else if (k == 4) {
            uint32_t c = 0;
            for (uint32_t w = 0; w < nw; w++) c += s_inc[w];
            if (c) atomicAdd(&a.st->n_inc, c);
        } else {
            uint32_t x = 0;
            for (uint32_t w = 0; w < nw; w++) x = x > s_mx[k - 5][w] ? x : s_mx[k - 5][w];
            if (x) atomicMax(&a.st->mx[k - 5], x);
        }
    }
}

// alloc_kernel: segments for the rows that outgrow theirs (bump allocation at the arenas'
// ends), the append descriptor, the document's new totals, and the re-merge list
__global__ void alloc_kernel(PlanArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t h = a.handles[i];
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
    D.n_r = m.n_r; D.n_actors = m.n_actors; D.n_objs = m.n_objs;
    D.inc = (uint16_t)p.inc;
    a.descs[i] = D;
    a.dm[h] = m;
    if (!p.inc) a.list[atomicAdd(&a.st->n_cold, 1u)] = h;
}

__global__ __launch_bounds__(PLAN_WG) void doc_rows_kernel(const uint32_t *list, uint32_t n, const DevDoc *dm, hm_doc_row *rows,
                                                          PlanStats *st) {
    // per workgroup: 5 maxima, the flags OR, 4 sums -> LDS, then one atomic each
    __shared__ uint32_t s_mx[6];
    __shared__ unsigned long long s_tot[4];
    if (threadIdx.x < 6) s_mx[threadIdx.x] = 0;
    if (threadIdx.x < 4) s_tot[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const DevDoc m = dm[list[i]];
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
    __syncthreads();
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
    default: break;
    }
}

__global__ void rollback_kernel(const uint32_t *handles, uint32_t n, const hm_doc_result *res_docs, const PlanRow *plan,
                                const uint8_t *remap, uint32_t S, DevDoc *dm, AppendDesc *descs, uint8_t *inv,
                                uint32_t *list, PlanStats *st) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = handles[i];
    if (res_docs[h].status == HM_OK) return;
    const PlanRow p = plan[i];
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
    hipLaunchKernelGGL(hms::alloc_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t hm_launch_doc_rows(const uint32_t *list, uint32_t n, const DevDoc *dm, hm_doc_row *rows, PlanStats *st,
                              hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::doc_rows_kernel, dim3((n + PLAN_WG - 1) / PLAN_WG), dim3(PLAN_WG), 0, s, list, n, dm, rows, st);
    return hipGetLastError();
}
hipError_t hm_launch_rollback(const uint32_t *handles, uint32_t n, const hm_doc_result *res_docs, const PlanRow *plan,
                              const uint8_t *remap, uint32_t S, DevDoc *dm, AppendDesc *descs, uint8_t *inv,
                              uint32_t *list, PlanStats *st, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::rollback_kernel, dim3((n + 255) / 256), dim3(256), 0, s, handles, n, res_docs, plan, remap, S, dm,
                       descs, inv, list, st);
    return hipGetLastError();
}
hipError_t hm_launch_init_docs(DevDoc *dm, uint32_t h0, uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hms::init_docs_kernel, dim3((n + 255) / 256), dim3(256), 0, s, dm, h0, n);
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
                            const uint8_t *remap, uint32_t S, hipStream_t s) {
    if (!n_desc) return hipSuccess;
    const uint32_t grid = (n_desc + 3) / 4 < 65535u ? (n_desc + 3) / 4 : 65535u;
    hipLaunchKernelGGL(hms::append_kernel, dim3(grid), dim3(SWG), 0, s, descs, n_desc, src, dst, st_changes, st_deps,
                       st_ops, remap, S);
    return hipGetLastError();
}

IncDims hm_inc_dims(uint32_t S, uint32_t new_c, uint32_t tgt, uint32_t stage, uint32_t regs, uint32_t surv,
                    uint32_t slots) {
    IncDims M = {};
    M.S = S; M.new_c = new_c ? new_c : 1; M.tgt = tgt ? tgt : 1; M.stage = stage; M.regs = regs ? regs : 1;
    M.surv = surv ? surv : 1; M.slots = slots ? slots : 1;
    uint32_t o = 0;
    auto take = [&](size_t bytes) { const uint32_t r = o; o += (uint32_t)((bytes + 15) & ~(size_t)15); return r; };
    M.o_nc = take((size_t)M.new_c * 32);
    M.o_dep = take((size_t)M.tgt * 8);
    M.o_tkey = take((size_t)M.tgt * 8);
    M.o_tsrc = take((size_t)M.tgt * 12);
    M.o_tad = take((size_t)M.tgt * S * 4);
    M.o_adn = take((size_t)M.new_c * S * 4);
    M.o_skey = take((size_t)M.stage * 8);
    M.o_sof = take((size_t)M.stage * 4);
    M.o_reg = take((size_t)M.regs * 13);
    M.o_sold = take((size_t)M.surv * 16);
    M.o_wl = take((size_t)M.slots * HM_INC_SLOT_CAP * 16);
    M.o_wls = take((size_t)M.slots * HM_INC_SLOT_CAP * 4);
    M.o_wla = take((size_t)M.slots * HM_INC_SLOT_CAP);
    M.o_scnt = take((size_t)M.slots * 4);
    M.bytes = o;
    return M;
}

hipError_t hm_launch_inc_apply(const AppendDesc *descs, uint32_t n, const IncArenas &A, const IncDims &M,
                               uint32_t *bail, hipStream_t s) {
    if (!n) return hipSuccess;
    hipError_t z = hipMemsetAsync(bail, 0, 4, s);
    if (z != hipSuccess) return z;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&hms::inc_apply_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const uint32_t grid = n < (1u << 20) ? n : (1u << 20);
    hipLaunchKernelGGL(hms::inc_apply_kernel, dim3(grid), dim3(64), M.bytes, s, descs, n, A, M, bail);
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
