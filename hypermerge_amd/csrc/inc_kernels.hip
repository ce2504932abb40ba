// inc_kernels.hip — incremental applyRemoteChanges on the resident store (store.cpp).
//
// The reference applies only the new changes to the live opSet (src/DocBackend.ts:169-185 ->
// Automerge Backend.applyChanges): a change that is causallyReady against
// opSet.clock is applied at once (the first applyQueuedOps pass), its allDeps is the
// transitiveDeps fold over its deps' allDeps rows, and each of its ops runs applyAssign on one
// register: the survivors not causally before the op stay, the op is pushed (set / link), and
// the list is sorted by actor descending (sortBy(actor).reverse(), stable).  A document whose new
// changes all apply in arrival order on its resident state is advanced here; its cost is the new
// rows plus the registers they hit — the rest of the document is not read.
//
//   inc_group_kernel<G>  G lanes per document (G >= the store's actor stride: lane = actor for
//                        clock / allDeps rows, lane = survivor for a register's list), 256 / G
//                        documents per workgroup.  Loads are issued in four dependent levels:
//                        the descriptor; the document's clock rows, new change / dep / op rows and
//                        the log's last rows (the fold sources are found there by (actor, seq));
//                        the fold sources' allDeps rows and the hit registers' rows; their
//                        survivors with their (actor, seq) metadata (IncState / smeta: no log
//                        search).  A document outside the group's limits is handed to the
//                        G = 64 instantiation (defer), anything outside the incremental envelope
//                        to the re-merge (bail) — both before the first store.
//   inc_meta_kernel      after a re-merge: the survivors' (actor, seq, counter-set) metadata, the
//                        objects created as maps and the counter bound of each document.
// All of it is integer row work, HBM / latency bound.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/hypermerge_amd.h"
#include "store_kernels.h"

namespace hmi {

enum { INC_DONE = 0, INC_DEFER = 1, INC_BAIL = 2 };
constexpr uint32_t NC = HM_INC_MAX_NEW_C;     // new changes per document and submit (allDeps rows in registers)
constexpr uint32_t TB = 8;                    // fold sources whose allDeps rows are loaded together

// lanes [base, base + G) of the wave hold one document; every group-level branch is uniform
// within the group (shuffles and ballots are then well defined for it)
template <int G>
struct Grp {
    uint32_t lane, gl, base;
    __device__ Grp() {
        lane = __lane_id();
        gl = lane & (G - 1);
        base = lane & ~(uint32_t)(G - 1);
    }
    __device__ __forceinline__ uint64_t bits(bool p) const {
        const uint64_t b = __ballot(p);
        if constexpr (G == 64) return b;
        else return (b >> base) & ((1ull << G) - 1);
    }
    __device__ __forceinline__ uint32_t below(uint64_t m) const { return (uint32_t)__popcll(m & ((1ull << gl) - 1)); }
    __device__ __forceinline__ uint32_t sh(uint32_t x, uint32_t l) const { return (uint32_t)__shfl((int)x, (int)l, G); }
    __device__ __forceinline__ uint32_t up(uint32_t x, uint32_t d) const { return (uint32_t)__shfl_up((int)x, d, G); }
    // lane l of the group receives x from the lane that names it (dst must be a permutation of the group)
    __device__ __forceinline__ uint32_t to(uint32_t x, uint32_t dst) const {
        return (uint32_t)__builtin_amdgcn_ds_permute((int)((base + dst) << 2), (int)x);
    }
};

// v[j] by selects over opaque elements (a select between two loads of one array is otherwise
// folded into a load through a selected pointer, which puts the array in scratch memory)
__device__ __forceinline__ uint32_t sel_nc(const uint32_t (&v)[NC], uint32_t j) {
    uint32_t r = v[0];
    asm volatile("" : "+v"(r));
#pragma unroll
    for (uint32_t x = 1; x < NC; x++) {
        uint32_t t = v[x];
        asm volatile("" : "+v"(t));
        r = j == x ? t : r;
    }
    return r;
}
__device__ __forceinline__ void set_nc(uint32_t (&v)[NC], uint32_t j, uint32_t y) {
#pragma unroll
    for (uint32_t x = 0; x < NC; x++) v[x] = j == x ? y : v[x];
}
__device__ __forceinline__ uint64_t abs64(int64_t v) { return v < 0 ? (uint64_t)(-v) : (uint64_t)v; }

constexpr unsigned long long TWO53 = 1ull << 53;

// ---------------- list / text ops (G = 64: one document per wave) ----------------
// The document's lists have their order resident (lorder / epos / epar / ekey and the list
// directory, HM_IST_LIST): the lists end to end in object-id order, so an element's position is
// global and list k occupies [base_k, base_k + count_k).  A round's `ins` ops take the fast path
// of applyInsert when every new element hangs off an element of its own list that exists (or
// one this round inserted earlier) or off the list's '_head'.  Under an old parent its insertion
// point is right after the parent when it sorts before the parent's current first child
// (lamportCompare (elem, actor) DESCENDING: the typing case, a new element with the largest elem
// counter), else before the parent's first child with a smaller key or after the parent's
// subtree (a group scan of the order).  The new elements then form blocks, one per anchor, in
// pre-order of their own forest, placed at the anchor's insertion point; every old element after
// an insertion point (later lists' included) shifts by the blocks before it.  Anything else (an
// insert after an element not inserted yet, a duplicate elemId, anchors of different parents at
// one point) goes to the re-merge.  Sets /
// deletes on elements are applyAssign as for map keys; the visible indices (per list) are then
// rewritten from the first position that changed.
// per document (a group of G lanes): anchors (G), cumulative block sizes (G), subtree sizes (G)
template <int G> constexpr uint32_t lscr_words() { return 3u * (uint32_t)G; }
constexpr uint32_t LMAX = HM_INC_LISTS;

struct ListPlan {
    uint32_t n_el0, n_el;                      // elements before / after the submit, all lists (uniform)
    uint32_t na, pmin, q0;                     // anchors, first old position that moves, first position that changes
    uint32_t npos, key;                        // ins lanes: the new element's position and lamport key
    uint32_t nl;                               // lists (uniform)
    uint32_t bnew, cnew;                       // lane k < nl: list k's base and elements after the submit
};

template <int G>
__device__ __forceinline__ uint32_t list_shift(const uint32_t *lscr, uint32_t na, uint32_t i) {
    uint32_t s = 0;
    for (uint32_t k = 0; k < na; k++)
        if ((int)lscr[k] - 1 < (int)i) s = lscr[G + k];      // blocks of the anchors at or before position i
    return s;
}

// the list (directory index) holding global position i, from the lanes' (base, count)
template <int G>
__device__ __forceinline__ uint32_t list_at(const Grp<G> &g, uint32_t nl, uint32_t b, uint32_t c, uint32_t i) {
    uint32_t l = HM_NONE;
    for (uint32_t k = 0; k < nl; k++) {
        const uint32_t bk = g.sh(b, k), ck = g.sh(c, k);
        if (i >= bk && i < bk + ck) l = k;
    }
    return l;
}

// li: the op's list (directory index; HM_NONE for other ops); dir: lane k < nl holds list k's
// directory entry (object, elements)
template <int G>
__device__ int list_plan(const Grp<G> &g, const AppendDesc &D, const IncArgs &A, const IncState &I, uint32_t nno,
                         uint32_t o_act, uint32_t o_reg, uint32_t o_par, uint32_t o_elem, bool lst, uint32_t li,
                         uint32_t opactor, uint2 dir, uint32_t *lscr, ListPlan &lp) {
    const uint32_t gl = g.gl, n_el = I.pad[0], nl = I.pad[1];
    // the lists' bases (lane k): the counts before list k
    const uint32_t ck = gl < nl ? dir.y : 0u;
    uint32_t bk = 0;
    for (uint32_t k = 0; k < nl; k++) { const uint32_t x = g.sh(ck, k); bk += k < gl ? x : 0u; }   // (every lane shuffles)
    const uint32_t lix = li < nl ? li : 0u;
    const uint32_t lb = g.sh(bk, lix), lc = g.sh(ck, lix);            // this op's list
    const bool ins = lst && o_act == HM_INS, eop = lst && o_act != HM_INS;
    const uint64_t insm = g.bits(ins);
    const uint32_t nins = (uint32_t)__popcll(insm);
    const uint32_t key = (o_elem << 8) | (opactor & 0xFFu);
    // a new element's register is fresh (checked by the caller: no op touched it before); its
    // parent exists in its own list: an old element, '_head', or an element inserted earlier in
    // this round; an assign hits an element that exists
    bool bad = false;
    uint32_t pnew = HM_NONE, ecr = HM_NONE;
    for (uint32_t k = 0; k < nno; k++) {
        if (!((insm >> k) & 1ull)) continue;
        const uint32_t rk = g.sh(o_reg, k), lk = g.sh(li, k);
        if (k < gl && ins && rk == o_reg) bad = true;
        if (k < gl && ins && rk == o_par) { pnew = k; bad |= lk != li; }
        if (k < gl && eop && rk == o_reg) { ecr = k; bad |= lk != li; }
    }
    const bool root = ins && pnew == HM_NONE;
    uint32_t pold = HM_NONE, eold = HM_NONE;
    if (root && o_par != HM_HEAD) pold = o_par < D.n_old_r ? A.epos[D.src_r + o_par] : HM_NONE;
    if (eop && ecr == HM_NONE) eold = o_reg < D.n_old_r ? A.epos[D.src_r + o_reg] : HM_NONE;
    bad |= (root && o_par != HM_HEAD && (pold < lb || pold >= lb + lc)) || (eop && ecr == HM_NONE && (eold < lb || eold >= lb + lc));
    if (g.bits(bad)) return INC_BAIL;
    // the anchor: its insertion point (after the old parent, or the list's start for '_head') and a
    // key that orders anchors by insertion point, then an element's before the '_head's at the same
    // point (the end of one list is the start of the next), then '_head's by list (empty lists
    // share their base with the next list): insertion point << 4 | head << 3 | list
    uint32_t ins_at = root ? (o_par == HM_HEAD ? lb : pold + 1u) : 0u;
    // the positions read back name the registers (a register that is no element has a stale slot)
    uint32_t at_p = HM_NONE, at_e = HM_NONE, nxt = HM_NONE;
    if (root && o_par != HM_HEAD) at_p = A.lorder[D.src_r + pold];
    if (root && ins_at < lb + lc) nxt = A.lorder[D.src_r + ins_at];
    if (eop && ecr == HM_NONE) at_e = A.lorder[D.src_r + eold];
    bad = (root && o_par != HM_HEAD && at_p != o_par) || (eop && ecr == HM_NONE && at_e != o_reg);
    if (g.bits(bad)) return INC_BAIL;
    // under an old parent (or '_head') a new element that does not sort before the parent's first
    // child (a concurrent insert at the same place with a smaller lamport key) goes before the
    // parent's first child with a smaller key, or at the end of the parent's subtree: the group
    // scans the order from the parent on, G positions a step — an element whose parent is the
    // parent and whose key is smaller stops it, and so does one whose parent sits before the
    // parent (or is '_head'): the first element after the parent's subtree in pre-order
    const bool hard = root && nxt != HM_NONE && A.epar[D.src_r + nxt] == o_par && !(key > A.ekey[D.src_r + nxt]);
    for (uint64_t hm = g.bits(hard); hm; hm &= hm - 1) {
        const uint32_t k = (uint32_t)__builtin_ctzll(hm);
        const uint32_t p = g.sh(o_par, k), kk = g.sh(key, k), pp = g.sh(pold, k);
        const uint32_t start = g.sh(ins_at, k), end = g.sh(lb, k) + g.sh(lc, k);
        uint32_t found = end;
        bool dup = false;
        for (uint32_t j0 = start; j0 < end && found == end; j0 += G) {
            const uint32_t j = j0 + gl;
            bool stop = false;
            if (j < end) {
                const uint32_t y = A.lorder[D.src_r + j];
                const uint32_t py = A.epar[D.src_r + y];
                if (py == p) {
                    const uint32_t ky = A.ekey[D.src_r + y];
                    dup |= ky == kk;
                    stop = ky < kk;
                } else if (p != HM_HEAD) {
                    stop = py == HM_HEAD || A.epos[D.src_r + py] < pp;
                }
            }
            const uint64_t sm = g.bits(stop);
            if (sm) found = j0 + (uint32_t)__builtin_ctzll(sm);
        }
        if (g.bits(dup)) return INC_BAIL;                     // (the same elemId twice: the re-merge reports it)
        if (gl == k) ins_at = found;
    }
    const uint32_t akey = root ? (ins_at << 4) | (o_par == HM_HEAD ? 8u | lix : 0u) : 0u;
    // an insertion point the scan found may coincide with another anchor's (a deeper element's
    // child placed at the same point): the anchors' order there is not the key order — re-merge
    {
        bool clash = false;
        for (uint64_t rm = g.bits(root); rm; rm &= rm - 1) {
            const uint32_t k = (uint32_t)__builtin_ctzll(rm);
            const uint32_t ak = g.sh(akey, k), pk = g.sh(o_par, k);
            clash |= root && ak == akey && pk != o_par;
        }
        if (g.bits(clash)) return INC_BAIL;
    }

    // subtree sizes in the round's forest: every element counts itself at each of its ancestors
    uint32_t *sz = lscr + 2 * G;
    sz[gl] = 0;
    __builtin_amdgcn_wave_barrier();
    {
        uint32_t a = ins ? gl : HM_NONE;
        for (uint32_t st = 0; st < nins; st++) {
            if (a != HM_NONE) atomicAdd(&sz[a], 1u);
            const uint32_t up = g.sh(pnew, a == HM_NONE ? 0u : a);
            a = a == HM_NONE ? HM_NONE : up;
        }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t size = ins ? sz[gl] : 0u;
    // rank in the anchor's block: siblings (same new parent, or the same anchor for roots) with a
    // larger key come first with their subtrees; a child follows its parent
    uint32_t r0 = ins && !root ? 1u : 0u;
    for (uint32_t k = 0; k < nno; k++) {
        if (!((insm >> k) & 1ull)) continue;
        const uint32_t pk = g.sh(pnew, k), ak = g.sh(akey, k), kk = g.sh(key, k), sk = g.sh(size, k);
        const bool same = pnew != HM_NONE ? pk == pnew : (pk == HM_NONE && ak == akey);
        if (ins && k != gl && same && kk > key) r0 += sk;
    }
    uint32_t rank = r0, ranc = akey;
    {
        uint32_t a = ins ? pnew : HM_NONE;
        for (uint32_t st = 0; st < nins; st++) {
            const uint32_t src = a == HM_NONE ? 0u : a;
            const uint32_t ra = g.sh(r0, src), pp = g.sh(pnew, src), an = g.sh(akey, src);
            if (a != HM_NONE) { rank += ra; ranc = an; a = pp; }
        }
    }
    // anchors (distinct root anchors) in anchor-key order with their cumulative block sizes
    bool leader = root;
    uint32_t bsize = 0, before = 0;
    for (uint32_t k = 0; k < nno; k++) {
        if (!((insm >> k) & 1ull)) continue;
        const uint32_t pk = g.sh(pnew, k), ak = g.sh(akey, k), sk = g.sh(size, k);
        if (pk != HM_NONE) continue;
        if (root && k < gl && ak == akey) leader = false;
        if (root && ak == akey) bsize += sk;
        if (ins && ak < ranc) before += sk;                   // blocks of the anchors before this element's
    }
    const uint64_t lm = g.bits(leader);
    const uint32_t na = (uint32_t)__popcll(lm);
    uint32_t idx = 0, cum = 0;
    for (uint32_t k = 0; k < nno; k++) {
        if (!((lm >> k) & 1ull)) continue;
        const uint32_t ak = g.sh(akey, k), bk2 = g.sh(bsize, k);
        if (leader && ak < akey) idx++;
        if (leader && ak <= akey) cum += bk2;
    }
    if (leader) { lscr[idx] = ins_at; lscr[G + idx] = cum; }
    __builtin_amdgcn_wave_barrier();
    uint32_t pmin = ins ? (ranc >> 4) : HM_NONE;
    for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) { const uint32_t y = g.sh(pmin, gl ^ d); pmin = y < pmin ? y : pmin; }
    lp.n_el0 = n_el; lp.n_el = n_el + nins; lp.na = na; lp.pmin = nins ? pmin : n_el;
    lp.key = key;
    lp.npos = ins ? (ranc >> 4) + before + rank : HM_NONE;
    lp.nl = nl;
    // the lists after the submit: counts grow by their inserts, bases follow
    uint32_t cn = ck;
    for (uint32_t k = 0; k < nl; k++) {
        const uint32_t m = (uint32_t)__popcll(g.bits(ins && li == k));
        if (gl == k) cn += m;
    }
    uint32_t bn = 0;
    for (uint32_t k = 0; k < nl; k++) { const uint32_t x = g.sh(cn, k); bn += k < gl ? x : 0u; }
    lp.cnew = cn; lp.bnew = bn;
    // the first position whose visible index may change: the first moved one, or an element an
    // assign hits (at its new position)
    uint32_t qe = HM_NONE;
    {
        const uint32_t cnp = g.sh(lp.npos, ecr == HM_NONE ? 0u : ecr);
        const uint32_t sh = list_shift<G>(lscr, na, eold == HM_NONE ? 0u : eold);
        if (eop) qe = ecr != HM_NONE ? cnp : eold + sh;
    }
    uint32_t q0 = qe < lp.pmin ? qe : lp.pmin;
    for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) { const uint32_t y = g.sh(q0, gl ^ d); q0 = y < q0 ? y : q0; }
    lp.q0 = q0;
    return INC_DONE;
}

// the order rewritten: old elements from pmin on shift right (from the end, 64 at a time: every
// move goes up, so nothing is overwritten before it is read), then the new elements land
template <int G>
__device__ void list_insert(const Grp<G> &g, const AppendDesc &D, const IncArgs &A, const IncState &I, uint32_t o_act,
                            uint32_t o_reg, uint32_t o_par, const uint32_t *lscr, const ListPlan &lp) {
    const uint32_t gl = g.gl;
    if (lp.n_el > lp.n_el0)
        for (int top = (int)lp.n_el0 - 1; top >= (int)lp.pmin; top -= G) {
            const int i = top - (int)gl;
            const bool v = i >= (int)lp.pmin;
            const uint32_t e = v ? A.lorder[D.dst_r + i] : 0u;
            if (v) {
                const uint32_t np = (uint32_t)i + list_shift<G>(lscr, lp.na, (uint32_t)i);
                A.lorder[D.dst_r + np] = e;
                A.epos[D.dst_r + e] = np;
            }
        }
    if (lp.npos != HM_NONE && o_act == HM_INS) {
        A.lorder[D.dst_r + lp.npos] = o_reg;
        A.epos[D.dst_r + o_reg] = lp.npos;
        A.epar[D.dst_r + o_reg] = o_par;
        A.ekey[D.dst_r + o_reg] = lp.key;
    }
}

// visible indices (hm_reg_result.list_index, counted per list) from the first position that
// changed to the end of the last list
template <int G>
__device__ void list_indices(const Grp<G> &g, const AppendDesc &D, const IncArgs &A, const ListPlan &lp) {
    const uint32_t gl = g.gl, nl = lp.nl, bn = lp.bnew, cn = lp.cnew;
    if (lp.q0 >= lp.n_el) return;
    const uint32_t l0 = list_at(g, nl, bn, cn, lp.q0);
    const uint32_t b0 = g.sh(bn, l0 < nl ? l0 : 0u);
    const uint32_t start = l0 < nl ? b0 : lp.q0;
    uint32_t c = 0;                                           // visible elements of q0's list before q0
    for (int top = (int)lp.q0 - 1; top >= (int)start; top -= G) {
        const int i = top - (int)gl;
        bool v = false;
        int32_t li = -1;
        if (i >= (int)start) {
            const hm_reg_result &r = A.regs[D.dst_r + A.lorder[D.dst_r + i]];
            v = r.n_surv > 0;
            li = r.list_index;
        }
        const uint64_t m = g.bits(v);
        if (m) { c = (uint32_t)g.sh((uint32_t)li, (uint32_t)__builtin_ctzll(m)) + 1u; break; }
    }
    for (uint32_t q = lp.q0; q < lp.n_el; q += G) {
        const uint32_t i = q + gl;
        hm_reg_result *r = nullptr;
        bool v = false;
        int32_t old = -1;
        uint32_t s = 0;                                       // the first lane of this lane's list in the chunk
        bool cont = true;                                     // this lane's list began before the chunk
        if (i < lp.n_el) {
            r = A.regs + D.dst_r + A.lorder[D.dst_r + i];
            v = r->n_surv > 0;
            old = r->list_index;
        }
        {
            const uint32_t l = list_at(g, nl, bn, cn, i < lp.n_el ? i : lp.n_el - 1u);
            const uint32_t bl = g.sh(bn, l < nl ? l : 0u);        // (every lane shuffles)
            const uint32_t b = l < nl ? bl : q;
            cont = b < q;
            s = cont ? 0u : b - q;
        }
        const uint64_t m = g.bits(v);
        const uint64_t mine = m & ((1ull << gl) - 1) & ~((1ull << s) - 1);     // (gl, s < 64)
        const int32_t li = v ? (int32_t)((cont ? c : 0u) + (uint32_t)__popcll(mine)) : -1;
        if (r && li != old) r->list_index = li;
        // the carry: the visible elements of the chunk's last list, this chunk's included
        const uint32_t last = lp.n_el - 1u - q < (uint32_t)G - 1u ? lp.n_el - 1u - q : (uint32_t)G - 1u;
        const uint32_t sl = g.sh(s, last);
        const bool cl = g.sh(cont ? 1u : 0u, last) != 0u;
        const uint64_t tail = m & (last >= 63 ? ~0ull : ((1ull << (last + 1)) - 1)) & ~((1ull << sl) - 1);
        c = (cl ? c : 0u) + (uint32_t)__popcll(tail);
    }
}

// The submit's gathered results (what hm_batch_wait hands out: the result rows, then the clock,
// back-clock and heads rows, by batch row) written straight from the registers of a document
// finished here; gather_kernel then copies only the rows of the documents the re-merge took
// (gdone[bi] = 0).
__device__ __forceinline__ void gather_rows(const IncArgs &A, uint32_t bi, uint32_t a, uint32_t ck, uint32_t bk, uint32_t hd) {
    if (!A.gout) return;
    uint32_t *o = reinterpret_cast<uint32_t *>(A.gout) + (size_t)A.n * 8;
    const size_t ns = (size_t)A.n * A.S, k = (size_t)bi * A.S + a;
    o[k] = ck; o[ns + k] = bk; o[2 * ns + k] = hd;
}
__device__ __forceinline__ void gather_result(const IncArgs &A, uint32_t bi, const hm_doc_result &r) {
    if (!A.gout) return;
    reinterpret_cast<hm_doc_result *>(A.gout)[bi] = r;
}

// the new rows of a document whose segments did not move, from the submit's staged tables
// (batch-local offsets) to the log, rebased (append_kernel skips such documents)
template <int G>
__device__ __forceinline__ void inc_append(const Grp<G> &g, const AppendDesc &D, const IncArgs &A) {
    const uint32_t gl = g.gl, nnc = D.n_new_c, nno = D.n_new_o, nnd = D.n_new_d;
    for (uint32_t i = gl; i < nnc; i += G) {
        hm_change_row c = A.st_changes[D.new_c + i];
        c.dep_off = D.dst_d + D.n_old_d + (c.dep_off - D.new_d);
        c.op_first = D.dst_o + D.n_old_o + (c.op_first - D.new_o);
        A.changes[D.dst_c + D.n_old_c + i] = c;
    }
    for (uint32_t i = gl; i < nnd; i += G) A.deps[D.dst_d + D.n_old_d + i] = A.st_deps[D.new_d + i];
    const uint4 *so4 = reinterpret_cast<const uint4 *>(A.st_ops + D.new_o);
    uint4 *do4 = reinterpret_cast<uint4 *>(A.ops + D.dst_o + D.n_old_o);
    for (uint32_t i = gl; i < 2 * nno; i += G) do4[i] = so4[i];
}

template <int G, bool LS = false>
__device__ int inc_doc(const AppendDesc &D, const IncArgs &A, uint4 *ssv, uint2 *smt, uint32_t *lscr, bool appended = false,
                        uint32_t bi = HM_NONE) {
    const Grp<G> g;
    const uint32_t gl = g.gl;
    const uint32_t S = A.S, h = D.handle, NA = D.n_actors, nnc = D.n_new_c, nno = D.n_new_o, nnd = D.n_new_d;
    constexpr int FAILG = G < 64 ? INC_DEFER : INC_BAIL;     // a limit of this group size only
    constexpr bool LST = G == 64 || (HM_INC_LIST_GROUPS && LS);   // list / text ops taken by this instantiation
    constexpr uint32_t KT = G >= 32 ? 1u : 32u / G;           // the log's last KT * G rows are searched first
    // the new rows: a document whose segments did not move gets them appended here — before
    // anything can hand the document over, since the re-merge reads them from the log
    const bool moved = D.src_c != D.dst_c || D.src_d != D.dst_d || D.src_o != D.dst_o;
    if (!moved && !appended) inc_append<G>(g, D, A);
    if (nnc == 0 || NA > S || S > G || D.n_old_r > D.n_r) return INC_BAIL;
    if (nnc > NC || nno > G || nnd > G) return FAILG;       // (the tiled wave pass takes longer rounds)

    // ---- level 2: everything that depends only on the descriptor ----
    const IncState I = A.ist[h];
    const hm_doc_result R0 = A.res_docs[h];
    // the list directory (lane k < HM_INC_LISTS holds entry k)
    uint2 dir = make_uint2(HM_NONE, 0u);
    if constexpr (LST) { if (A.ldir && gl < LMAX) dir = A.ldir[(size_t)h * LMAX + gl]; }
    uint32_t ck = 0, hd = 0, mc = 0;
    if (gl < S) {
        ck = A.clock[(size_t)h * S + gl];
        hd = A.heads[(size_t)h * S + gl];
        mc = (A.min_clock && (D.inc & HM_DINC_MINC)) ? A.min_clock[(size_t)h * S + gl] : 0u;   // (no row: zeros)
    }
    uint32_t ca = 0, cq = 0, cnd = 0, cdo = 0, cno = 0, coo = 0;
    if (gl < nnc) {
        const hm_change_row c = A.st_changes[D.new_c + gl];
        ca = c.actor; cq = c.seq; cnd = c.n_deps; cdo = c.dep_off - D.new_d; cno = c.n_ops; coo = c.op_first - D.new_o;
    }
    uint32_t o_act = 0, o_dt = 0, o_obj = 0, o_reg = 0xFFFFFFFFu, o_vt = 0, o_vlo = 0, o_vhi = 0, o_par = 0, o_elem = 0;
    if (gl < nno) {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.st_ops + D.new_o + gl);
        const uint4 w0 = src[0], w1 = src[1];
        // hm_op_row: obj, reg, parent, elem | action, datatype, vtag, pad, key, value lo, value hi
        o_obj = w0.x; o_reg = w0.y; o_par = w0.z; o_elem = w0.w;
        o_act = w1.x & 0xFFu; o_dt = (w1.x >> 8) & 0xFFu; o_vt = (w1.x >> 16) & 0xFFu;
        o_vlo = w1.z; o_vhi = w1.w;
    }
    uint32_t dpa = 0, dpq = 0;
    if (gl < nnd) {
        const hm_dep_row d = A.st_deps[D.new_d + gl];
        dpa = d.actor; dpq = d.seq;
    }
    // the log's last rows, newest first, as packed (actor, seq, applied) keys: the applied copy of a
    // change is the one a fold finds (duplicates and queued copies are not applied)
    uint32_t tk[KT];
#pragma unroll
    for (uint32_t k = 0; k < KT; k++) {
        const int idx = (int)D.n_old_c - 1 - (int)(k * G + gl);
        tk[k] = idx >= 0 ? A.ckey[D.src_c + idx] : 0u;
    }
    if ((I.flags & (HM_IST_VALID | HM_IST_NOCKEY)) != HM_IST_VALID) return INC_BAIL;

    // ---- the new rows: grouped by change, in order, after the old rows; supported ops ----
    uint32_t sd = gl < nnc ? cnd : 0u, so = gl < nnc ? cno : 0u;
#pragma unroll
    for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) {
        const uint32_t yd = g.up(sd, d), yo = g.up(so, d);
        if (gl >= d) { sd += yd; so += yo; }
    }
    const uint32_t xd = sd - (gl < nnc ? cnd : 0u), xo = so - (gl < nnc ? cno : 0u);
    const uint32_t total_d = g.sh(sd, nnc - 1), total_o = g.sh(so, nnc - 1);
    const bool bad_c = gl < nnc && (ca >= NA || cq == 0 || cq >= (1u << 24) || cdo != xd || coo != xo);
    const int64_t oval = (int64_t)(((uint64_t)o_vhi << 32) | o_vlo);
    // an op on one of the document's list / text objects (their order is resident: HM_IST_LIST);
    // li = its list in the directory.  (Without HM_INC_LIST_GROUPS a group of 8 / 16 lanes has no
    // directory: an op on an object that is not a map of the log marks the document for the
    // one-document-per-wave pass)
    const uint32_t nl = (I.flags & HM_IST_LIST) ? (I.pad[1] < LMAX ? I.pad[1] : LMAX) : 0u;
    uint32_t li = HM_NONE;
    if constexpr (LST) {
        for (uint32_t k = 0; k < nl; k++) li = g.sh(dir.x, k) == o_obj ? k : li;
    } else {
        li = nl && o_obj != 0 && (o_obj >= 64 || !((I.mapmask >> o_obj) & 1ull)) ? 0u : HM_NONE;
    }
    // makeMap / makeTable (A.0): a fresh object id (a duplicate throws: the re-merge reports it);
    // documents with lists hand object creation to the re-merge (their list ids are not in mapmask).
    // `made` = the maps this round created before each op (an exclusive prefix OR over the group)
    const bool mk = gl < nno && (o_act == HM_MAKE_MAP || o_act == HM_MAKE_TABLE);
    unsigned long long made = mk && o_obj < 64 ? (1ull << o_obj) : 0ull;
#pragma unroll
    for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) {
        const unsigned long long y = (unsigned long long)__shfl_up((long long)made, d, G);
        if (gl >= d) made |= y;
    }
    const unsigned long long made_all = (unsigned long long)__shfl((long long)made, G - 1, G);
    made = (unsigned long long)__shfl_up((long long)made, 1, G);
    if (gl == 0) made = 0;
    const unsigned long long known = I.mapmask | made;
    const bool lst = gl < nno && !mk && li != HM_NONE;
    const bool bad_o = gl < nno && ((o_act != HM_SET && o_act != HM_DEL && o_act != HM_LINK && o_act != HM_INC && !mk &&
                                     !(lst && o_act == HM_INS)) ||
                                    (mk && ((D.inc & HM_DINC_LISTS) || o_obj == 0 || o_obj >= 64 || ((known >> o_obj) & 1ull))) ||
                                    (o_act == HM_INC && o_vt != HM_V_INT && o_vt != HM_V_FLOAT) ||
                                    o_obj >= D.n_objs || (!mk && o_reg >= D.n_r) ||
                                    (o_vt == HM_V_INT && abs64(oval) > TWO53) ||
                                    (o_act == HM_INS && (o_elem >= (1u << 24) || (o_par != HM_HEAD && o_par >= D.n_r))) ||
                                    // an object other than ROOT must be a map / table the log (or an
                                    // earlier op of this round) created
                                    (!mk && !lst && o_obj != 0 && (o_obj >= 64 || !((known >> o_obj) & 1ull))));
    if (g.bits(bad_c || bad_o) || total_o != nno || total_d != nnd) return INC_BAIL;
    const bool any_list = g.bits(lst) != 0;
    if (!LST && any_list) return INC_DEFER;                   // list / text ops: one document per wave
    // integer counters: |base| + sum|inc| of every counter stays <= 2^53 (the re-merge's exact rule)
    unsigned long long cadd = (gl < nno && o_vt == HM_V_INT &&
                               (o_act == HM_INC || (o_act == HM_SET && o_dt == HM_DT_COUNTER))) ? abs64(oval) : 0ull;
#pragma unroll
    for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) cadd += (unsigned long long)__shfl_xor((long long)cadd, d, G);
    const unsigned long long cabs = I.cabs + cadd;
    if (cabs > TWO53) return INC_BAIL;

    // ---- level 3a: the hit registers' rows (lane = op) ----
    hm_reg_result rr = {0u, 0u, -1, HM_NONE};
    if (gl < nno && o_reg < D.n_old_r) rr = A.regs[D.src_r + o_reg];

    // ---- causallyReady in arrival order; the transitiveDeps fold steps (A.1) ----
    // target t lives in lane t % G, slot t / G: actor | (new source + 1) << 8 | change << 16, seq, log index
    uint32_t tA0 = 0, tA1 = 0, tQ0 = 0, tQ1 = 0, tI0 = 0, tI1 = 0;
    uint32_t jt0 = 0, jtn = 0;                                 // lane j: change j's fold steps
    uint32_t ckr = ck, nt = 0;
    for (uint32_t j = 0; j < nnc; j++) {
        const uint32_t a = g.sh(ca, j), q = g.sh(cq, j), nd = g.sh(cnd, j), d0 = g.sh(xd, j);
        if (g.sh(ckr, a) + 1u != q) return INC_BAIL;           // a duplicate, or not ready: the queue decides
        const uint32_t t0 = nt;
        bool own = false;
        for (uint32_t t = 0; t <= nd; t++) {
            uint32_t da, dq;
            if (t < nd) {
                da = g.sh(dpa, d0 + t); dq = g.sh(dpq, d0 + t);
                if (da >= NA) return INC_BAIL;
                if (da == a) { dq = q - 1; own = true; }       // deps ∪ {actor: seq - 1}: the key keeps its place
            } else {
                if (own) break;
                da = a; dq = q - 1;
            }
            if (g.sh(ckr, da) < dq) return INC_BAIL;
            if (dq == 0) continue;
            const uint64_t m = g.bits(gl < j && ca == da && cq == dq);
            const uint32_t src1 = m ? (uint32_t)__builtin_ctzll(m) + 1u : 0u;
            if (nt >= 2u * G) return FAILG;
            const uint32_t w = da | (src1 << 8) | (j << 16);
            if (gl == (nt & (G - 1))) {
                if (nt < (uint32_t)G) { tA0 = w; tQ0 = dq; } else { tA1 = w; tQ1 = dq; }
            }
            nt++;
        }
        if (gl == j) { jt0 = t0; jtn = nt - t0; }
        if (gl == a) ckr = q;
    }

    // ---- fold sources in the old log: its applied row of (actor, seq), newest rows first ----
    for (uint32_t t = 0; t < nt; t++) {
        const uint32_t tl = t & (G - 1);
        const uint32_t w = g.sh(t < (uint32_t)G ? tA0 : tA1, tl);
        if ((w >> 8) & 0xFFu) continue;                        // a change of this submit
        const uint32_t da = w & 0xFFu, dq = g.sh(t < (uint32_t)G ? tQ0 : tQ1, tl);
        const uint32_t want = hm_ckey(da, dq, true);
        int found = -1;
#pragma unroll
        for (uint32_t k = 0; k < KT; k++) {
            const uint64_t m = g.bits(tk[k] == want);
            if (m && found < 0) found = (int)D.n_old_c - 1 - (int)(k * G + (uint32_t)__builtin_ctzll(m));
        }
        for (int top = (int)D.n_old_c - 1 - (int)(KT * G); found < 0 && top >= 0; top -= G) {
            const int idx = top - (int)gl;
            const uint64_t m = g.bits(idx >= 0 && A.ckey[D.src_c + idx] == want);
            if (m) found = top - (int)__builtin_ctzll(m);
        }
        if (found < 0) return INC_BAIL;
        if (gl == tl) { if (t < (uint32_t)G) tI0 = (uint32_t)found; else tI1 = (uint32_t)found; }
    }

    // ---- first-touch registers (lane = op): pushes, staging offsets, space ----
    bool first = gl < nno && o_act >= HM_SET;                 // (an ins creates its register, a make an object)
    uint32_t push = 0, oj = 0;
    for (uint32_t k = 0; k < nno; k++) {
        const uint32_t r = g.sh(o_reg, k), ak = g.sh(o_act, k);
        if (k < gl && r == o_reg && ak >= HM_SET) first = false;
        if (k >= gl && r == o_reg && (ak == HM_SET || ak == HM_LINK)) push++;
    }
    for (uint32_t j = 0; j < nnc; j++)
        if (g.sh(xo + cno, j) <= gl) oj++;                    // the op's change: ops are grouped by change
    const uint32_t n_old = first ? rr.n_surv : 0u;
    const uint32_t n_up = first ? n_old + push : 0u;           // the list's length after the submit, at most
    if (g.bits(first && n_up > (uint32_t)G)) return FAILG;
    uint32_t s_incl = n_old, g_incl = n_up;
#pragma unroll
    for (uint32_t d = 1; d < (uint32_t)G; d <<= 1) {
        const uint32_t y = g.up(s_incl, d), z = g.up(g_incl, d);
        if (gl >= d) { s_incl += y; g_incl += z; }
    }
    const uint32_t stage_off = s_incl - n_old, tot_old = g.sh(s_incl, G - 1), grow = g.sh(g_incl, G - 1);
    if (tot_old > 2u * G) return FAILG;
    if ((unsigned long long)I.s_used + grow > D.o_cap) return INC_BAIL;   // no room: the re-merge repacks

    // ---- level 3b: the fold sources' allDeps rows, TB at a time; allDeps / heads / clock of
    //      each new change (applyChange) ----
    uint32_t adn[NC];
#pragma unroll
    for (uint32_t x = 0; x < NC; x++) adn[x] = 0;
    uint32_t hdr = hd, ckf = ck;
    for (uint32_t j = 0; j < nnc; j++) {
        const uint32_t t0 = g.sh(jt0, j), tn = g.sh(jtn, j), a = g.sh(ca, j), q = g.sh(cq, j);
        uint32_t adv = 0;
        for (uint32_t tb = t0; tb < t0 + tn; tb += TB) {
            uint32_t row[TB], wv[TB], qv[TB];
#pragma unroll
            for (uint32_t u = 0; u < TB; u++) {
                const uint32_t t = tb + u < 2u * G ? tb + u : 0u, tl = t & (G - 1);
                wv[u] = g.sh(t < (uint32_t)G ? tA0 : tA1, tl);
                qv[u] = g.sh(t < (uint32_t)G ? tQ0 : tQ1, tl);
                const uint32_t ix = g.sh(t < (uint32_t)G ? tI0 : tI1, tl);
                row[u] = 0;
                if (tb + u < t0 + tn && !((wv[u] >> 8) & 0xFFu) && gl < S)
                    row[u] = A.all_deps[(size_t)(D.src_c + ix) * S + gl];
            }
#pragma unroll
            for (uint32_t u = 0; u < TB; u++) {
                if (tb + u >= t0 + tn) break;
                const uint32_t src1 = (wv[u] >> 8) & 0xFFu;
                const uint32_t r = src1 ? sel_nc(adn, src1 - 1) : row[u];
                if (gl < NA && r > adv) adv = r;
                if (gl == (wv[u] & 0xFFu)) adv = qv[u];         // then `a: s` (the literal fold)
            }
        }
        if (gl >= NA) adv = 0;
        set_nc(adn, j, adv);
        if (hdr && hdr <= adv) hdr = 0;
        if (gl == a) { hdr = q; ckf = q; }
    }

    // ---- list / text ops (applyInsert, A.3): the new elements' places in the resident order ----
    ListPlan lp;
    if constexpr (LST) {
        if (any_list) {
            // an inserted element's register was never touched: a fresh id, or one the document's
            // declared register count reserved (untouched registers have no object)
            if (g.bits(lst && o_act == HM_INS && o_reg < D.n_old_r && (rr.obj != HM_NONE || rr.n_surv != 0))) return INC_BAIL;
            const int rc = list_plan(g, D, A, I, nno, o_act, o_reg, o_par, o_elem, lst, li, g.sh(ca, oj), dir, lscr, lp);
            if (rc != INC_DONE) return rc;
        }
    }

    // ---- level 4: the hit registers' survivors and their metadata, staged per group ----
    {
        // slot p of the staging area (two per lane) <- survivor src of the register that owns p
        const uint32_t roff = first ? rr.surv_off : 0u, p0 = gl, p1 = gl + G;
        uint32_t s0 = 0xFFFFFFFFu, s1 = 0xFFFFFFFFu;
        for (uint32_t k = 0; k < nno; k++) {
            const uint32_t b = g.sh(stage_off, k), c = g.sh(n_old, k), o = g.sh(roff, k);
            if (p0 >= b && p0 < b + c) s0 = o + (p0 - b);
            if (p1 >= b && p1 < b + c) s1 = o + (p1 - b);
        }
        uint4 x0 = {}, x1 = {};
        uint2 m0 = {}, m1 = {};
        const bool v0 = p0 < tot_old && s0 != 0xFFFFFFFFu, v1 = p1 < tot_old && s1 != 0xFFFFFFFFu;
        if (v0) { x0 = *reinterpret_cast<const uint4 *>(A.surv + D.src_o + s0); m0 = A.smeta[D.src_o + s0]; }
        if (v1) { x1 = *reinterpret_cast<const uint4 *>(A.surv + D.src_o + s1); m1 = A.smeta[D.src_o + s1]; }
        if (v0) { ssv[p0] = x0; smt[p0] = m0; }
        if (v1) { ssv[p1] = x1; smt[p1] = m1; }
    }
    // segments the append moved: the per-change / survivor / register rows follow (rare: a
    // segment doubles)
    const bool mv = D.src_c != D.dst_c || D.src_o != D.dst_o || D.src_r != D.dst_r;
    if (D.src_c != D.dst_c) {
        for (uint32_t i = gl; i < D.n_old_c; i += G) { A.hist[D.dst_c + i] = A.hist[D.src_c + i]; A.ckey[D.dst_c + i] = A.ckey[D.src_c + i]; }
        for (size_t w = gl; w < (size_t)D.n_old_c * S; w += G) A.all_deps[(size_t)D.dst_c * S + w] = A.all_deps[(size_t)D.src_c * S + w];
    }
    if (D.src_o != D.dst_o)
        for (uint32_t i = gl; i < I.s_used; i += G) {
            const uint4 x = *reinterpret_cast<const uint4 *>(A.surv + D.src_o + i);
            const uint2 xm = A.smeta[D.src_o + i];
            *reinterpret_cast<uint4 *>(A.surv + D.dst_o + i) = x;
            A.smeta[D.dst_o + i] = xm;
        }
    if (D.src_r != D.dst_r) {
        for (uint32_t i = gl; i < D.n_old_r; i += G) A.regs[D.dst_r + i] = A.regs[D.src_r + i];
        if (I.flags & HM_IST_LIST) {
            for (uint32_t i = gl; i < D.n_old_r; i += G) {
                A.epos[D.dst_r + i] = A.epos[D.src_r + i];
                A.epar[D.dst_r + i] = A.epar[D.src_r + i];
                A.ekey[D.dst_r + i] = A.ekey[D.src_r + i];
            }
            for (uint32_t i = gl; i < I.pad[0]; i += G) A.lorder[D.dst_r + i] = A.lorder[D.src_r + i];
        }
    }
    if (mv) __threadfence_block();                            // the copies land before the writes below
    __builtin_amdgcn_wave_barrier();
    if constexpr (LST) {
        if (any_list) list_insert(g, D, A, I, o_act, o_reg, o_par, lscr, lp);
    }

    // ---- the new ops, register by register in first-touch order (applyAssign, A.2) ----
    uint64_t fm = g.bits(first);
    uint32_t acc = 0;
    int32_t dsurv = 0;
    while (fm) {
        const uint32_t k0 = (uint32_t)__builtin_ctzll(fm);
        fm &= fm - 1;
        const uint32_t greg = g.sh(o_reg, k0), cnt0 = g.sh(n_old, k0), sb = g.sh(stage_off, k0);
        const uint32_t off_old = g.sh(first ? rr.surv_off : 0u, k0), obj = g.sh(o_obj, k0);
        uint4 x = {0u, 0u, 0u, 0u};
        uint2 xm = {0u, 0u};
        if (gl < cnt0) { x = ssv[sb + gl]; xm = smt[sb + gl]; }
        uint32_t cnt = cnt0;
        for (uint32_t k = k0; k < nno; k++) {
            if (g.sh(o_reg, k) != greg || g.sh(o_act, k) < HM_SET) continue;
            const uint32_t act = g.sh(o_act, k), vt = g.sh(o_vt, k), dtk = g.sh(o_dt, k);
            const uint32_t vlo = g.sh(o_vlo, k), vhi = g.sh(o_vhi, k), j = g.sh(oj, k);
            const uint32_t a = g.sh(ca, j), q = g.sh(cq, j);
            // allDeps(new)[x.actor]: x is causally before the op iff that is >= x.seq
            const uint32_t anc = g.sh(sel_nc(adn, j), xm.y & 0xFFu);
            const bool live = gl < cnt;
            if (act == HM_INC && live && (xm.y & 0x100u) && (x.y == HM_V_INT || x.y == HM_V_FLOAT) && anc >= xm.x) {
                // every surviving counter set causally before the inc adds it: integer + integer
                // exactly (cabs bounds the sums), anything else in f64 in application order
                const uint64_t cur = ((uint64_t)x.w << 32) | x.z, inc = ((uint64_t)vhi << 32) | vlo;
                if (x.y == HM_V_INT && vt == HM_V_INT) {
                    const uint64_t s = (uint64_t)((int64_t)cur + (int64_t)inc);
                    x.z = (uint32_t)s; x.w = (uint32_t)(s >> 32);
                } else {
                    double xv, iv;
                    if (x.y == HM_V_INT) xv = (double)(int64_t)cur; else __builtin_memcpy(&xv, &cur, 8);
                    if (vt == HM_V_INT) iv = (double)(int64_t)inc; else __builtin_memcpy(&iv, &inc, 8);
                    const double r = xv + iv;
                    uint64_t rb;
                    __builtin_memcpy(&rb, &r, 8);
                    x.z = (uint32_t)rb; x.w = (uint32_t)(rb >> 32); x.y = HM_V_FLOAT;
                }
            }
            // the survivors concurrent with the op stay (an inc removes nothing)
            const bool keep = live && (act == HM_INC || anc < xm.x);
            const uint64_t km = g.bits(keep);
            const uint32_t nk = (uint32_t)__popcll(km), pos = g.below(km);
            const uint32_t dst = keep ? pos : nk + (gl - pos);  // a permutation of the group
            x.x = g.to(x.x, dst); x.y = g.to(x.y, dst); x.z = g.to(x.z, dst); x.w = g.to(x.w, dst);
            xm.x = g.to(xm.x, dst); xm.y = g.to(xm.y, dst);
            const bool pushes = act == HM_SET || act == HM_LINK;
            if (pushes && gl == nk) {
                x = make_uint4(D.n_old_o + k, vt, vlo, vhi);
                xm = make_uint2(q, a | ((act == HM_SET && dtk == HM_DT_COUNTER) ? 0x100u : 0u));
            }
            cnt = nk + (pushes ? 1u : 0u);
            // sortBy(actor) (stable) then reverse
            const uint32_t my = xm.y & 0xFFu;
            uint32_t rank = 0;
            for (uint32_t e = 0; e < cnt; e++) {
                const uint32_t ae = g.sh(my, e);
                rank += (ae < my || (ae == my && e < gl)) ? 1u : 0u;
            }
            const uint32_t d2 = gl < cnt ? cnt - 1 - rank : gl;
            x.x = g.to(x.x, d2); x.y = g.to(x.y, d2); x.z = g.to(x.z, d2); x.w = g.to(x.w, d2);
            xm.x = g.to(xm.x, d2); xm.y = g.to(xm.y, d2);
        }
        // a list that is no longer than before stays in its slots, a longer one moves to the end
        const uint32_t off = cnt <= cnt0 ? off_old : I.s_used + acc;
        if (cnt > cnt0) acc += cnt;
        dsurv += (int32_t)cnt - (int32_t)cnt0;
        if (gl < cnt) {
            *reinterpret_cast<uint4 *>(A.surv + D.dst_o + off + gl) = x;
            A.smeta[D.dst_o + off + gl] = xm;
        }
        if (gl == 0) {
            hm_reg_result r;
            r.n_surv = cnt; r.surv_off = off; r.list_index = -1; r.obj = obj;
            A.regs[D.dst_r + greg] = r;
        }
    }
    // registers new to the document and not hit (none for map ops; kept for the row contract)
    for (uint32_t r0 = D.n_old_r; r0 < D.n_r; r0 += G) {
        const uint32_t r = r0 + gl;
        bool hit = false;
        for (uint32_t k = 0; k < nno; k++) hit |= g.sh(o_reg, k) == r;
        if (r < D.n_r && !hit) {
            hm_reg_result z;
            z.n_surv = 0; z.surv_off = 0; z.list_index = -1; z.obj = HM_NONE;
            A.regs[D.dst_r + r] = z;
        }
    }
    // elements inserted and not assigned: no survivors, the list object (as the merge's op scan
    // records every op's object on its register)
    if (any_list) {
        bool asg = false;
        for (uint32_t k = 0; k < nno; k++) {
            const uint32_t rk = g.sh(o_reg, k), ak = g.sh(o_act, k);
            asg |= rk == o_reg && ak != HM_INS;
        }
        if (gl < nno && o_act == HM_INS && !asg) {
            hm_reg_result z;
            z.n_surv = 0; z.surv_off = 0; z.list_index = -1; z.obj = o_obj;
            A.regs[D.dst_r + o_reg] = z;
        }
    }

    if constexpr (LST) {
        if (any_list) {
            __threadfence_block();                            // the register rows above, then the visible indices
            __builtin_amdgcn_wave_barrier();
            list_indices(g, D, A, lp);
        }
    }

    // ---- history, allDeps, clocks, the document's result row and IncState ----
    if (gl < nnc) {
        A.hist[D.dst_c + D.n_old_c + gl] = (int32_t)(R0.hist_len + gl);
        A.ckey[D.dst_c + D.n_old_c + gl] = hm_ckey(ca, cq, true);
    }
    if (gl < S) {
#pragma unroll
        for (uint32_t j = 0; j < NC; j++)
            if (j < nnc) A.all_deps[(size_t)(D.dst_c + D.n_old_c + j) * S + gl] = adn[j];
        A.clock[(size_t)h * S + gl] = ckf;
        A.back_clock[(size_t)h * S + gl] = ckf;                // queue empty: every handed change applied
        A.heads[(size_t)h * S + gl] = hdr;
        if (bi != HM_NONE) gather_rows(A, bi, gl, ckf, ckf, hdr);
    }
    const bool ag = g.bits(gl < S && ckf < mc) == 0, bg = g.bits(gl < S && mc < ckf) == 0;
    if (gl == 0) {
        hm_doc_result r = {};
        r.status = HM_OK; r.err_change = HM_NONE; r.err_op = HM_NONE;
        r.hist_len = R0.hist_len + nnc; r.n_queued = 0; r.n_surv = (uint32_t)((int32_t)R0.n_surv + dsurv);
        r.min_cmp = (ag && bg) ? 0u : (ag ? 1u : (bg ? 2u : 3u));
        A.res_docs[h] = r;
        if (bi != HM_NONE) gather_result(A, bi, r);
        IncState s = I;
        s.s_used = I.s_used + acc; s.cabs = cabs; s.mapmask = I.mapmask | made_all;
        if (LST && any_list) s.pad[0] = lp.n_el;
        A.ist[h] = s;
    }
    if constexpr (LST) {
        if (any_list && gl < lp.nl) A.ldir[(size_t)h * LMAX + gl] = make_uint2(dir.x, lp.cnew);   // the lists' new lengths
    }
    return INC_DONE;
}

// A round longer than a group holds (more than NC changes, G ops or G dep rows) is applied in
// tiles: every row is appended first, then each tile — the most whole changes that fit — runs as a
// round of its own on the state the previous tile left (the rows before it are old rows to it).
// A tile after the first that cannot go incremental sends the document to the re-merge, which
// rewrites every row the earlier tiles wrote.
template <int G, bool LS = false>
__device__ int inc_doc_tiled(const AppendDesc &D, const IncArgs &A, uint4 *ssv, uint2 *smt, uint32_t *lscr, uint32_t bi) {
    const Grp<G> g;
    const uint32_t gl = g.gl;
    // (one call site of inc_doc: a second inlined copy costs the common round its occupancy)
    const bool tiled = D.n_new_c > NC || D.n_new_o > (uint32_t)G || D.n_new_d > (uint32_t)G;
    if (tiled && !(D.src_c != D.dst_c || D.src_d != D.dst_d || D.src_o != D.dst_o)) inc_append<G>(g, D, A);
    AppendDesc T = D;
    uint32_t c0 = 0, d0 = 0, o0 = 0;
    for (bool first = true;; first = false) {
        uint32_t k = D.n_new_c, to = D.n_new_o, td = D.n_new_d;
        if (tiled) {
            // the tile: changes c0 .. c0 + k - 1, at most NC of them with at most G ops and G dep rows
            uint32_t no = 0, nd = 0;
            if (gl < NC && c0 + gl < D.n_new_c) {
                const hm_change_row c = A.st_changes[D.new_c + c0 + gl];
                no = c.n_ops; nd = c.n_deps;
            }
            uint32_t so = no, sd = nd;
#pragma unroll
            for (uint32_t d = 1; d < NC; d <<= 1) {
                const uint32_t yo = g.up(so, d), yd = g.up(sd, d);
                if (gl >= d && gl < NC) { so += yo; sd += yd; }
            }
            k = (uint32_t)__popcll(g.bits(gl < NC && c0 + gl < D.n_new_c && so <= (uint32_t)G && sd <= (uint32_t)G));
            if (k == 0) return INC_BAIL;                      // a change larger than a group: the re-merge
            to = g.sh(so, k - 1); td = g.sh(sd, k - 1);
            T.new_c = D.new_c + c0; T.n_new_c = k; T.new_d = D.new_d + d0; T.n_new_d = td; T.new_o = D.new_o + o0; T.n_new_o = to;
            T.n_old_c = D.n_old_c + c0; T.n_old_d = D.n_old_d + d0; T.n_old_o = D.n_old_o + o0;
            if (!first) {
                T.src_c = D.dst_c; T.src_d = D.dst_d; T.src_o = D.dst_o; T.src_r = D.dst_r;
                T.n_old_r = D.n_r;                            // (the first tile wrote every new register's row)
            }
        }
        const int rc = inc_doc<G, LS>(T, A, ssv, smt, lscr, tiled, bi);
        if (rc != INC_DONE) return first ? rc : INC_BAIL;
        c0 += k; d0 += td; o0 += to;
        if (c0 >= D.n_new_c) return INC_DONE;
        __threadfence_block();                                // this tile's rows, then the next tile's reads
        __builtin_amdgcn_wave_barrier();
    }
}

// TL: the launch for rounds that need tiles (a separate instantiation: the tile loop around
// inc_doc costs the common round's register allocation half its occupancy)
#ifndef HM_INC_KARG_RELOAD
#define HM_INC_KARG_RELOAD 1 // inc_group_kernel: launch parameters re-read per document (see the kernel)
#endif
#ifndef HM_INC_WAVES
#define HM_INC_WAVES 1       // dev A/B: waves per SIMD the G = 8 / 16 instantiations are compiled for
#endif
// LS (G = 8 / 16, HM_INC_LIST_GROUPS): the instantiation for documents with lists (HM_DINC_LISTS);
// the other takes the map documents at the register budget the list code would cost them (116 vs
// 141 VGPRs: 4 waves per SIMD instead of 3)
template <int G, bool TL, bool LS = false>
__global__ __launch_bounds__(256, (G < 64 ? HM_INC_WAVES : 1)) void inc_group_kernel(IncArgs A_in) {
    constexpr uint32_t NG = 256 / G;
    __shared__ uint4 s_sv[NG][2 * G];
    __shared__ uint2 s_mt[NG][2 * G];
    constexpr bool LST = G == 64 || (HM_INC_LIST_GROUPS && LS);
    __shared__ uint32_t s_ls[LST ? NG : 1][LST ? lscr_words<G>() : 1];   // the list phase's anchors
    const uint32_t grp = threadIdx.x / G, gl = threadIdx.x & (G - 1);
    if (!A_in.list && A_in.pst && A_in.pst->n_inc == 0) return;     // (a submit with nothing incremental)
    if (LS && A_in.pst && A_in.pst->mx[4] == 0) return;              // (no list document routed to the groups)
    const uint32_t n = A_in.list ? A_in.list[0] : A_in.n;
    // the loop reads the launch parameters through an opaque pointer to the kernarg segment: a
    // document re-loads the fields it uses (scalar loads) rather than holding them in SGPRs
    // across the loop, where they were spilled to VGPR lanes (readlane / writelane VALU)
    typedef __attribute__((address_space(4))) const IncArgs KArgs;
    KArgs *kp = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    for (uint32_t q = blockIdx.x * NG + grp; q < n; q += gridDim.x * NG) {
        if (HM_INC_KARG_RELOAD) asm volatile("" : "+s"(kp));
        const IncArgs &A = HM_INC_KARG_RELOAD ? *(const IncArgs *)kp : A_in;
        const uint32_t di = A.list ? A.list[1 + q] : q;
        const AppendDesc D = A.descs[di];
        const uint32_t route = D.inc & HM_DINC_ROUTE;
        if (!route || route == 3 || (G < 64 && route == 2)) continue;   // (2: listed for the wave pass, 3: the lane pass)
        const bool tl = D.n_new_c > NC || D.n_new_o > (uint32_t)G || D.n_new_d > (uint32_t)G;
        if (G == 64 && tl != TL) continue;                             // (the other launch's document)
        if (HM_INC_LIST_GROUPS && G < 64 && ((D.inc & HM_DINC_LISTS) != 0) != LS) continue;   // (the other instantiation's)
        int rc;
        if constexpr (TL) rc = inc_doc_tiled<G, LS>(D, A, s_sv[grp], s_mt[grp], s_ls[LST ? grp : 0], di);
        else rc = inc_doc<G, LS>(D, A, s_sv[grp], s_mt[grp], s_ls[LST ? grp : 0], false, di);
        if (rc == INC_DONE && gl == 0 && A.gdone) A.gdone[di] = 1;
        if (rc != INC_DONE && gl == 0) {
            if (rc == INC_DEFER && A.defer) A.defer[1 + atomicAdd(&A.defer[0], 1u)] = di;
            else A.bail[1 + atomicAdd(&A.bail[0], 1u)] = D.handle;
        }
    }
}

// ---------------- one lane per document: map documents of strides <= 16 ----------------
// The group pass above spends most of its time exchanging values between the lanes of a group
// (every step of a document's short serial work is a ds_bpermute round trip).  A map document's
// round — a few new changes, a few ops on a few registers — is serial work over a few hundred
// bytes, so here ONE lane takes the whole document: its clock / heads / allDeps rows live in
// registers, the new changes apply one after the other in arrival order (no limit on their
// number: each change's allDeps row is folded, written and used by its own ops, and a later
// change finds it in the log like any older one), and each op runs applyAssign on its register's
// survivor list read from the slot and written back (in place when it does not grow).  Cross-
// lane work is only the wave-aggregated list appends at the end.
//   validation (before any store but the log append): every change causally ready in arrival
//   order against the resident clock, every op a map op on ROOT / a map of the log (or a
//   makeMap / makeTable of a new object), counters inside the exact-integer bound.  A document
//   that fails a check with a chance in the group / wave pass (list ops, a moved segment) is
//   deferred to it untouched; anything else goes to the re-merge (bail).  After the first store
//   the only exits are a register of more than LSV survivors, a full slot area or a fold source
//   missing from the log — the document is then re-merged, which rewrites every row the lane
//   wrote (the new rows are in the log before anything else happens).
constexpr uint32_t LSV = 8;    // survivors of a register the lane path holds (more: re-merge)
constexpr uint32_t LKF = 2;    // fold sources resolved and loaded together

// v[i] of a register array by selects (each element made opaque first: a select between two
// loads of one array is otherwise folded into a load through a selected pointer, which sends the
// whole array to scratch memory)
template <int N>
__device__ __forceinline__ uint32_t lsel(const uint32_t (&v)[N], uint32_t i) {
    uint32_t r = v[0];
    asm volatile("" : "+v"(r));
#pragma unroll
    for (int x = 1; x < N; x++) {
        uint32_t t = v[x];
        asm volatile("" : "+v"(t));
        r = i == (uint32_t)x ? t : r;
    }
    return r;
}
template <int N>
__device__ __forceinline__ void lput(uint32_t (&v)[N], uint32_t i, uint32_t y) {
#pragma unroll
    for (int x = 0; x < N; x++) v[x] = i == (uint32_t)x ? y : v[x];
}
template <int S>
__device__ __forceinline__ void lrow_load(const uint32_t *p, uint32_t (&v)[S]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int k = 0; k < S / 4; k++) {
        const uint4 w = q[k];
        v[4 * k] = w.x; v[4 * k + 1] = w.y; v[4 * k + 2] = w.z; v[4 * k + 3] = w.w;
    }
}
template <int S>
__device__ __forceinline__ void lrow_store(uint32_t *p, const uint32_t (&v)[S]) {
    uint4 *q = reinterpret_cast<uint4 *>(p);
#pragma unroll
    for (int k = 0; k < S / 4; k++) q[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
}

// applyAssign of one map op on its register (A.2): the register's survivors (at most LSV) read
// from its slot, filtered against the op's change's allDeps row `ad` (isConcurrent:
// allDeps(op)[x.actor] < x.seq), an inc added to every surviving counter set that is its ancestor,
// the op pushed (set / link), sortBy(actor) (stable) then reverse — each element written straight
// to its place, in the slot when the list does not grow, else at the end of the slot area
template <int S>
__device__ __forceinline__ int lane_assign(const AppendDesc &D, const IncArgs &A, const uint32_t (&ad)[S], uint32_t a, uint32_t q,
                                           uint32_t obj, uint32_t reg, uint32_t act, uint32_t dt, uint32_t vt, uint32_t vlo,
                                           uint32_t vhi, uint32_t op_local, const hm_reg_result &rr, uint32_t &used,
                                           int32_t &dsurv) {
    const uint32_t n = rr.n_surv;
    if (n > LSV) return INC_BAIL;
    uint4 x[LSV + 1];
    uint2 m[LSV + 1];
#pragma unroll
    for (uint32_t i = 0; i < LSV; i++) {
        x[i] = make_uint4(0u, 0u, 0u, 0u); m[i] = make_uint2(0u, 0u);
        if (i < n) {
            x[i] = *reinterpret_cast<const uint4 *>(A.surv + D.dst_o + rr.surv_off + i);
            m[i] = A.smeta[D.dst_o + rr.surv_off + i];
        }
    }
    uint32_t keep = 0, pos[LSV + 1], act8[LSV + 1], cnt = 0;
#pragma unroll
    for (uint32_t i = 0; i < LSV; i++) {
        pos[i] = 0; act8[i] = m[i].y & 0xFFu;
        if (i >= n) continue;
        const uint32_t anc = lsel<S>(ad, m[i].y & 0xFFu);
        if (act == HM_INC && (m[i].y & 0x100u) && (x[i].y == HM_V_INT || x[i].y == HM_V_FLOAT) && anc >= m[i].x) {
            const uint64_t cur = ((uint64_t)x[i].w << 32) | x[i].z, inc = ((uint64_t)vhi << 32) | vlo;
            if (x[i].y == HM_V_INT && vt == HM_V_INT) {
                const uint64_t sum = (uint64_t)((int64_t)cur + (int64_t)inc);
                x[i].z = (uint32_t)sum; x[i].w = (uint32_t)(sum >> 32);
            } else {
                double xv, iv;
                if (x[i].y == HM_V_INT) xv = (double)(int64_t)cur; else __builtin_memcpy(&xv, &cur, 8);
                if (vt == HM_V_INT) iv = (double)(int64_t)inc; else __builtin_memcpy(&iv, &inc, 8);
                const double rs = xv + iv;
                uint64_t rb;
                __builtin_memcpy(&rb, &rs, 8);
                x[i].z = (uint32_t)rb; x[i].w = (uint32_t)(rb >> 32); x[i].y = HM_V_FLOAT;
            }
        }
        if (act == HM_INC || anc < m[i].x) { keep |= 1u << i; pos[i] = cnt++; }
    }
    x[LSV] = make_uint4(D.n_old_o + op_local, vt, vlo, vhi);
    m[LSV] = make_uint2(q, a | ((act == HM_SET && dt == HM_DT_COUNTER) ? 0x100u : 0u));
    act8[LSV] = a; pos[LSV] = cnt;
    if (act == HM_SET || act == HM_LINK) { keep |= 1u << LSV; cnt++; }
    const uint32_t off = cnt <= n ? rr.surv_off : used;
    if (cnt > n) {
        if ((unsigned long long)used + cnt > D.o_cap) return INC_BAIL;    // no room: the re-merge repacks
        used += cnt;
    }
#pragma unroll
    for (uint32_t e = 0; e <= LSV; e++) {
        if (!((keep >> e) & 1u)) continue;
        uint32_t rank = 0;
#pragma unroll
        for (uint32_t f = 0; f <= LSV; f++)
            rank += ((keep >> f) & 1u) && (act8[f] < act8[e] || (act8[f] == act8[e] && pos[f] < pos[e])) ? 1u : 0u;
        const uint32_t dst = off + cnt - 1u - rank;
        *reinterpret_cast<uint4 *>(A.surv + D.dst_o + dst) = x[e];
        A.smeta[D.dst_o + dst] = m[e];
    }
    dsurv += (int32_t)cnt - (int32_t)n;
    hm_reg_result nr;
    nr.n_surv = cnt; nr.surv_off = off; nr.list_index = -1; nr.obj = obj;
    A.regs[D.dst_r + reg] = nr;
    return INC_DONE;
}

// the document's clocks (back_clock = clock: the queue is empty), result row and IncState
template <int S>
__device__ __forceinline__ void lane_finish(const AppendDesc &D, const IncArgs &A, const IncState &I, const hm_doc_result &R0,
                                            const uint32_t (&ck)[S], const uint32_t (&hd)[S], uint32_t used, int32_t dsurv,
                                            unsigned long long cabs, unsigned long long mm, uint32_t bi) {
    const uint32_t h = D.handle;
    lrow_store<S>(A.clock + (size_t)h * S, ck);
    lrow_store<S>(A.back_clock + (size_t)h * S, ck);
    lrow_store<S>(A.heads + (size_t)h * S, hd);
    uint32_t mc[S];
#pragma unroll
    for (int x = 0; x < S; x++) mc[x] = 0;
    if (D.inc & HM_DINC_MINC) lrow_load<S>(A.min_clock + (size_t)h * S, mc);
    bool ag = true, bg = true;
#pragma unroll
    for (int x = 0; x < S; x++) { ag &= ck[x] >= mc[x]; bg &= mc[x] >= ck[x]; }
    hm_doc_result r = {};
    r.status = HM_OK; r.err_change = HM_NONE; r.err_op = HM_NONE;
    r.hist_len = R0.hist_len + D.n_new_c; r.n_queued = 0; r.n_surv = (uint32_t)((int32_t)R0.n_surv + dsurv);
    r.min_cmp = (ag && bg) ? 0u : (ag ? 1u : (bg ? 2u : 3u));
    A.res_docs[h] = r;
    IncState st = I;
    st.s_used = used; st.cabs = cabs; st.mapmask = mm;
    A.ist[h] = st;
#pragma unroll
    for (int x = 0; x < S; x++) gather_rows(A, bi, (uint32_t)x, ck[x], ck[x], hd[x]);
    gather_result(A, bi, r);
}

template <int S>
__device__ int inc_lane(const AppendDesc &D, const IncArgs &A, uint32_t bi) {
    const uint32_t h = D.handle, NA = D.n_actors, nnc = D.n_new_c, nnd = D.n_new_d, nno = D.n_new_o;
    const bool rows_moved = D.src_c != D.dst_c || D.src_d != D.dst_d || D.src_o != D.dst_o;
    if (!rows_moved) {
        // the new rows into the log first (append_kernel skipped this document): whatever
        // happens below, the re-merge finds them there
#pragma unroll 4
        for (uint32_t i = 0; i < nnc; i++) {
            hm_change_row c = A.st_changes[D.new_c + i];
            c.dep_off = D.dst_d + D.n_old_d + (c.dep_off - D.new_d);
            c.op_first = D.dst_o + D.n_old_o + (c.op_first - D.new_o);
            A.changes[D.dst_c + D.n_old_c + i] = c;
        }
#pragma unroll 4
        for (uint32_t i = 0; i < nnd; i++) A.deps[D.dst_d + D.n_old_d + i] = A.st_deps[D.new_d + i];
        const uint4 *so4 = reinterpret_cast<const uint4 *>(A.st_ops + D.new_o);
        uint4 *do4 = reinterpret_cast<uint4 *>(A.ops + D.dst_o + D.n_old_o);
#pragma unroll 4
        for (uint32_t i = 0; i < 2 * nno; i++) do4[i] = so4[i];
    }
    if (nnc == 0 || NA > (uint32_t)S || D.n_old_r > D.n_r) return INC_BAIL;
    const IncState I = A.ist[h];
    if ((I.flags & (HM_IST_VALID | HM_IST_NOCKEY | HM_IST_LIST)) != HM_IST_VALID) return INC_BAIL;
    // segments the append moved (append_kernel copied the log rows, the new ones included): the
    // per-change, survivor and register rows follow
    if (D.src_c != D.dst_c) {
#pragma unroll 4
        for (uint32_t i = 0; i < D.n_old_c; i++) { A.hist[D.dst_c + i] = A.hist[D.src_c + i]; A.ckey[D.dst_c + i] = A.ckey[D.src_c + i]; }
        const uint4 *sa = reinterpret_cast<const uint4 *>(A.all_deps + (size_t)D.src_c * S);
        uint4 *da = reinterpret_cast<uint4 *>(A.all_deps + (size_t)D.dst_c * S);
#pragma unroll 4
        for (uint32_t w = 0; w < D.n_old_c * (uint32_t)(S / 4); w++) da[w] = sa[w];
    }
    if (D.src_o != D.dst_o) {
#pragma unroll 4
        for (uint32_t i = 0; i < I.s_used; i++) {
            *reinterpret_cast<uint4 *>(A.surv + D.dst_o + i) = *reinterpret_cast<const uint4 *>(A.surv + D.src_o + i);
            A.smeta[D.dst_o + i] = A.smeta[D.src_o + i];
        }
    }
    if (D.src_r != D.dst_r) {
#pragma unroll 4
        for (uint32_t i = 0; i < D.n_old_r; i++) A.regs[D.dst_r + i] = A.regs[D.src_r + i];
    }
    const bool lists = (D.inc & HM_DINC_LISTS) != 0;
    const hm_doc_result R0 = A.res_docs[h];
    uint32_t ck[S], hd[S];
    lrow_load<S>(A.clock + (size_t)h * S, ck);
    lrow_load<S>(A.heads + (size_t)h * S, hd);
    // the log's last 8 change keys, oldest first (the fold sources are almost always there)
    uint32_t tail[8];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const int idx = (int)D.n_old_c - 8 + t;
        tail[t] = idx >= 0 ? A.ckey[D.dst_c + idx] : 0u;
    }

    // ---- validation: readiness in arrival order, supported ops, counter bound ----
    unsigned long long mm = I.mapmask, cadd = 0;
    {
        uint32_t cur[S];
#pragma unroll
        for (int x = 0; x < S; x++) cur[x] = ck[x];
        uint32_t xd = 0, xo = 0;
        int defer = 0;
        for (uint32_t j = 0; j < nnc; j++) {
            const hm_change_row c = A.st_changes[D.new_c + j];
            if (c.actor >= NA || c.seq == 0 || c.seq >= (1u << 24) || c.dep_off - D.new_d != xd || c.op_first - D.new_o != xo ||
                xd + c.n_deps > nnd || xo + c.n_ops > nno)
                return INC_BAIL;
            if (lsel<S>(cur, c.actor) + 1u != c.seq) return INC_BAIL;      // a duplicate, or not ready: the queue decides
            for (uint32_t t = 0; t < c.n_deps; t++) {
                const hm_dep_row d = A.st_deps[D.new_d + xd + t];
                if (d.actor >= NA) return INC_BAIL;
                if (d.actor != c.actor && lsel<S>(cur, d.actor) < d.seq) return INC_BAIL;
            }
            for (uint32_t k = 0; k < c.n_ops; k++) {
                const uint4 *src = reinterpret_cast<const uint4 *>(A.st_ops + D.new_o + xo + k);
                const uint4 w0 = src[0], w1 = src[1];
                const uint32_t obj = w0.x, reg = w0.y, act = w1.x & 0xFFu, dt = (w1.x >> 8) & 0xFFu, vt = (w1.x >> 16) & 0xFFu;
                const int64_t v = (int64_t)(((uint64_t)w1.w << 32) | w1.z);
                if (act == HM_MAKE_MAP || act == HM_MAKE_TABLE) {
                    // a new map: its id must be fresh (a list's id is not in mapmask: documents with
                    // lists take the group pass, which hands object creation to the re-merge)
                    if (lists) { defer = 1; continue; }
                    if (obj == 0 || obj >= 64 || obj >= D.n_objs || ((mm >> obj) & 1ull)) return INC_BAIL;
                    mm |= 1ull << obj;
                    continue;
                }
                if (act == HM_INS || act == HM_MAKE_LIST || act == HM_MAKE_TEXT) { defer = 1; continue; }
                if (act != HM_SET && act != HM_DEL && act != HM_LINK && act != HM_INC) return INC_BAIL;
                if (obj >= D.n_objs || reg >= D.n_r) return INC_BAIL;
                if (obj != 0 && (obj >= 64 || !((mm >> obj) & 1ull))) {
                    if (lists) { defer = 1; continue; }              // a list element: the wave pass
                    return INC_BAIL;
                }
                if (act == HM_INC && vt != HM_V_INT && vt != HM_V_FLOAT) return INC_BAIL;
                if (vt == HM_V_INT && abs64(v) > TWO53) return INC_BAIL;
                if (vt == HM_V_INT && (act == HM_INC || (act == HM_SET && dt == HM_DT_COUNTER))) cadd += abs64(v);
            }
            xd += c.n_deps; xo += c.n_ops;
            lput<S>(cur, c.actor, c.seq);
        }
        if (xd != nnd || xo != nno) return INC_BAIL;
        if (defer) return INC_DEFER;
    }
    const unsigned long long cabs = I.cabs + cadd;
    if (cabs > TWO53) return INC_BAIL;

    // ---- apply: registers new to the document start empty (the ops below read their rows) ----
    for (uint32_t r = D.n_old_r; r < D.n_r; r++) {
        hm_reg_result z;
        z.n_surv = 0; z.surv_off = 0; z.list_index = -1; z.obj = HM_NONE;
        A.regs[D.dst_r + r] = z;
    }
    uint32_t used = I.s_used;
    int32_t dsurv = 0;
    uint32_t xd = 0, xo = 0;
    for (uint32_t j = 0; j < nnc; j++) {
        const hm_change_row c = A.st_changes[D.new_c + j];
        const uint32_t a = c.actor, q = c.seq, nd = c.n_deps, end = D.n_old_c + j;
        // transitiveDeps: the literal fold over deps in key order, then {actor: seq - 1} unless a
        // dep names the actor (A.1); each source is the applied row of (actor, seq) in the log
        uint32_t ad[S];
#pragma unroll
        for (int x = 0; x < S; x++) ad[x] = 0;
        bool own = false;
        for (uint32_t t0 = 0; t0 <= nd; t0 += LKF) {
            uint32_t sa[LKF], sq[LKF], si[LKF];
#pragma unroll
            for (uint32_t u = 0; u < LKF; u++) {
                const uint32_t t = t0 + u;
                sa[u] = 0; sq[u] = 0; si[u] = HM_NONE;
                if (t < nd) {
                    const hm_dep_row d = A.st_deps[D.new_d + xd + t];
                    sa[u] = d.actor; sq[u] = d.seq;
                    if (d.actor == a) { sq[u] = q - 1u; own = true; }
                } else if (t == nd && !own) {
                    sa[u] = a; sq[u] = q - 1u;
                }
            }
            // positions: the last 8 rows in registers, then older rows 8 at a time
            uint32_t miss = 0;
#pragma unroll
            for (uint32_t u = 0; u < LKF; u++) {
                if (!sq[u]) continue;
                const uint32_t want = hm_ckey(sa[u], sq[u], true);
#pragma unroll
                for (int t = 0; t < 8; t++) if (tail[t] == want && (int)end - 8 + t >= 0) si[u] = end - 8u + (uint32_t)t;
                if (si[u] == HM_NONE) miss |= 1u << u;
            }
            for (int top = (int)end - 9; miss && top >= 0; top -= 8) {
                uint32_t kk[8];
#pragma unroll
                for (int t = 0; t < 8; t++) kk[t] = top - t >= 0 ? A.ckey[D.dst_c + top - t] : 0u;
#pragma unroll
                for (uint32_t u = 0; u < LKF; u++) {
                    if (!((miss >> u) & 1u)) continue;
                    const uint32_t want = hm_ckey(sa[u], sq[u], true);
#pragma unroll
                    for (int t = 7; t >= 0; t--) if (kk[t] == want && top - t >= 0) si[u] = (uint32_t)(top - t);
                    if (si[u] != HM_NONE) miss &= ~(1u << u);
                }
            }
            if (miss) return INC_BAIL;
            uint32_t row[LKF][S];
#pragma unroll
            for (uint32_t u = 0; u < LKF; u++) {
                if (sq[u]) lrow_load<S>(A.all_deps + (size_t)(D.dst_c + si[u]) * S, row[u]);
                else {
#pragma unroll
                    for (int x = 0; x < S; x++) row[u][x] = 0;
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < LKF; u++) {
                if (!sq[u]) continue;
#pragma unroll
                for (int x = 0; x < S; x++) if ((uint32_t)x < NA && row[u][x] > ad[x]) ad[x] = row[u][x];
                lput<S>(ad, sa[u], sq[u]);
            }
        }
        // the change enters history
        const uint32_t key = hm_ckey(a, q, true);
        A.hist[D.dst_c + end] = (int32_t)(R0.hist_len + j);
        A.ckey[D.dst_c + end] = key;
        lrow_store<S>(A.all_deps + (size_t)(D.dst_c + end) * S, ad);
#pragma unroll
        for (int t = 0; t < 7; t++) tail[t] = tail[t + 1];
        tail[7] = key;
#pragma unroll
        for (int x = 0; x < S; x++) if (hd[x] && hd[x] <= ad[x]) hd[x] = 0;
        lput<S>(hd, a, q);
        lput<S>(ck, a, q);

        // its ops: applyAssign on each register (A.2)
        for (uint32_t k = 0; k < c.n_ops; k++) {
            const uint4 *src = reinterpret_cast<const uint4 *>(A.st_ops + D.new_o + xo + k);
            const uint4 w0 = src[0], w1 = src[1];
            const uint32_t act = w1.x & 0xFFu;
            if (act == HM_MAKE_MAP || act == HM_MAKE_TABLE) continue;    // (mapmask updated above)
            const hm_reg_result rr = A.regs[D.dst_r + w0.y];
            if (lane_assign<S>(D, A, ad, a, q, w0.x, w0.y, act, (w1.x >> 8) & 0xFFu, (w1.x >> 16) & 0xFFu, w1.z, w1.w, xo + k, rr,
                               used, dsurv) != INC_DONE)
                return INC_BAIL;
        }
        xd += nd; xo += c.n_ops;
    }

    lane_finish<S>(D, A, I, R0, ck, hd, used, dsurv, cabs, mm, bi);
    return INC_DONE;
}

// wave-aggregated append of the lanes' entries to list[1..] (list[0] = count)
__device__ __forceinline__ void lane_list_push(uint32_t *list, bool p, uint32_t v) {
    const uint64_t m = __ballot(p);
    if (!m) return;
    const uint32_t lane = __lane_id(), lead = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(&list[0], (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, (int)lead);
    if (p) list[1 + base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = v;
}

template <int S>
__global__ __launch_bounds__(256) void inc_lane_kernel(IncArgs A) {
    if (A.pst && A.pst->mx[0] == 0) return;                   // (no document routed to this pass)
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    int rc = -1;
    uint32_t hnd = 0;
    if (i < A.n) {
        const AppendDesc D = A.descs[i];
        if ((D.inc & HM_DINC_ROUTE) == 3u) {
            hnd = D.handle;
            rc = inc_lane<S>(D, A, i);
            if (rc == INC_DONE && A.gdone) A.gdone[i] = 1;
        }
    }
    // (the group passes hold a round in registers: what the lane pass hands over re-merges)
    lane_list_push(A.bail, rc == INC_BAIL || rc == INC_DEFER, hnd);
}

// the change that owns doc-local op k: the last change whose first op is <= k (ops are grouped
// by change in log order; a change without ops shares its first op with the next)
__device__ __forceinline__ uint32_t change_of_op(const hm_change_row *ch, uint32_t n_c, uint32_t o_off, uint32_t k) {
    uint32_t lo = 0, hi = n_c;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ch[mid].op_first - o_off <= k) lo = mid; else hi = mid;
    }
    return lo;
}

// After a re-merge (one wave per listed document): survivor metadata (the survivor's change by
// a binary search over the change rows' first ops), the packed change keys, the objects created
// as maps / tables, the counter bound, and — for a document with up to HM_INC_LISTS list / text
// objects — the resident list order from the element positions the merge wrote: the lists end to
// end in object-id order in lorder (epos global, epar, ekey per element), indexed by the per-handle
// directory ldir = (object, elements) per list.
// Documents that are not clean (an error, queued changes) get flags = 0: their next submit
// re-merges.
// a document of at most META_LCH changes keeps its changes' first ops (and applied bits) in LDS
// for the op -> change searches: from HBM / L2 each of their ~8 steps is a dependent round trip,
// which made one 3.7k-op text document's rebuild 236 us (a C3 round re-merging one or two
// documents spent that on top of the merge)
constexpr uint32_t META_LCH = 1024;
#ifndef HM_META_STAMPS
#define HM_META_STAMPS 0     // diagnostic builds: inc_meta_kernel's per-phase wave time (hm_debug_meta_stamps)
#endif
#if HM_META_STAMPS
__device__ unsigned long long hm_meta_st[8];
#define MSTAMP(k) do { const unsigned long long t_ = wall_clock64(); if (lane == 0) atomicAdd(&hm_meta_st[k], t_ - t_ms); t_ms = t_; } while (0)
#else
#define MSTAMP(k) do { } while (0)
#endif
__device__ __forceinline__ uint32_t change_of_op_lds(const uint32_t *s_of, uint32_t n_c, uint32_t k) {
    uint32_t lo = 0, hi = n_c;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((s_of[mid] & 0x7FFFFFFFu) <= k) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void inc_meta_kernel(MetaArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    __shared__ uint32_t s_of4[4][META_LCH];                  // per wave: op_first - o_off | applied << 31
    uint32_t *s_of = s_of4[threadIdx.x >> 6];
    // the change in PlanStats.n_valid, summed per wave, then per workgroup into part[], then by
    // valid_sum_kernel: device-scope atomics on one word from every document (or workgroup)
    // serialize across the XCDs (~10 ns each: 0.3-1.8 ms for 65k-1M of them)
    __shared__ int s_dv[4];
    int dv = 0;
    // one wave per listed document: the re-merged documents of a submit are few and large (their
    // state is rebuilt from whole logs) or many and small (a few loads each, then skipped), and a
    // wave per document keeps the large ones in parallel (a round-6 variant that let one lane per
    // document decide first and a wave build the kept ones serially cost a C3 round the sum of its
    // few re-merged documents' rebuilds: 0.35 -> 1.07 ms)
    for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < a.n; q += gridDim.x * 4) {
#if HM_META_STAMPS
        unsigned long long t_ms = wall_clock64();
#endif
        const uint32_t h = a.list[q];
        const DevDoc m = a.dm[h];
        const hm_doc_result r = a.res_docs[h];
        const bool was = HM_IST_COUNTS(a.ist[h].flags);      // (PlanStats.n_valid follows the change)
        // (mode 1: a small document with lists re-merges every round — one small-kernel wave either
        // way — so it keeps no incremental state at all)
        if (r.status != HM_OK || r.n_queued != 0 || r.n_surv > m.o_cap ||
            ((m.flags & HM_DOC_HAS_LISTS) && m.n_o <= a.small_lists)) {
            if (lane == 0) {
                IncState z = {};
                a.ist[h] = z;
            }
            dv -= was ? 1 : 0;
            continue;
        }
        const hm_change_row *ch = a.changes + m.c_off;
        const bool lch = m.n_c <= META_LCH;
        bool wide = false;                                   // a seq the packed keys cannot hold
        for (uint32_t i = lane; i < m.n_c; i += 64) {
            const hm_change_row c = ch[i];
            const bool app = a.hist[m.c_off + i] >= 0;
            wide |= c.seq >= (1u << 24);
            a.ckey[m.c_off + i] = hm_ckey(c.actor, c.seq, app);
            if (lch) s_of[i] = (c.op_first - m.o_off) | (app ? 0x80000000u : 0u);
        }
        wide = __ballot(wide) != 0;
        __threadfence_block();                               // (s_of: this wave's writes, then its reads)
        __builtin_amdgcn_wave_barrier();
        MSTAMP(0);
        // (the next chunk's survivor rows are loaded before this chunk's lookups)
        uint32_t sop = lane < r.n_surv ? a.surv[m.o_off + lane].op : 0u;
        for (uint32_t i = lane; i < r.n_surv; i += 64) {
            const uint32_t op = sop;
            if (i + 64 < r.n_surv) sop = a.surv[m.o_off + i + 64].op;
            const uint32_t ow = reinterpret_cast<const uint4 *>(a.ops + m.o_off + op)[1].x;   // action | datatype << 8
            const uint32_t c = lch ? change_of_op_lds(s_of, m.n_c, op) : change_of_op(ch, m.n_c, m.o_off, op);
            const uint2 kw = *reinterpret_cast<const uint2 *>(ch + c);
            const uint32_t cset = ((ow & 0xFFu) == HM_SET && ((ow >> 8) & 0xFFu) == HM_DT_COUNTER) ? 0x100u : 0u;
            a.smeta[m.o_off + i] = make_uint2(kw.y, (kw.x & 0xFFu) | cset);
        }
        MSTAMP(1);
        unsigned long long mask = 1ull, cabs = 0;
        // the op scans below load the next chunk's rows before working on this one (a large
        // document's scans are dozens of chunks, each otherwise waiting on its loads)
        auto ldop = [&](uint32_t i) -> hm_op_row {
            hm_op_row o = {};
            o.action = 0xFF;
            if (i < m.n_o) o = a.ops[m.o_off + i];
            return o;
        };
        // the list / text objects created: distinct, ascending, at most LMAX (lane k holds list k)
        uint32_t lobj = HM_NONE, nlst = 0;
        bool over = false;
        hm_op_row nx = ldop(lane);
        for (uint32_t i0 = 0; i0 < m.n_o; i0 += 64) {
            const hm_op_row o = nx;
            nx = ldop(i0 + 64 + lane);
            if ((o.action == HM_MAKE_MAP || o.action == HM_MAKE_TABLE) && o.obj < 64) mask |= 1ull << o.obj;
            if (o.vtag == HM_V_INT && (o.action == HM_INC || (o.action == HM_SET && o.datatype == HM_DT_COUNTER))) {
                const unsigned long long v = abs64((int64_t)o.value);
                cabs = cabs + v < cabs || cabs + v > (1ull << 62) ? (1ull << 62) : cabs + v;
            }
            // (a duplicate of the creating change repeats its make op: the same object)
            for (unsigned long long mk = __ballot(o.action == HM_MAKE_LIST || o.action == HM_MAKE_TEXT); mk; mk &= mk - 1) {
                const uint32_t ob = (uint32_t)__shfl((int)o.obj, (int)__builtin_ctzll(mk));
                if (__ballot(lane < nlst && lobj == ob)) continue;
                if (nlst == LMAX) { over = true; continue; }
                const uint32_t at = (uint32_t)__popcll(__ballot(lane < nlst && lobj < ob));
                const uint32_t prev = (uint32_t)__shfl((int)lobj, (int)(lane ? lane - 1 : 0));
                if (lane == at) lobj = ob;
                else if (lane > at && lane <= nlst) lobj = prev;
                nlst++;
            }
        }
        for (uint32_t d = 1; d < 64; d <<= 1) {
            mask |= (unsigned long long)__shfl_xor((long long)mask, d);
            const unsigned long long y = (unsigned long long)__shfl_xor((long long)cabs, d);
            cabs = cabs + y > (1ull << 62) ? (1ull << 62) : cabs + y;
        }
        MSTAMP(2);
        // the lists' order from the element positions of the merge (within each list), laid end
        // to end: every applied insert counted per list, then placed at its list's base
        uint32_t flags = HM_IST_VALID | (wide ? HM_IST_NOCKEY : 0u), n_el = 0;
        if (nlst == 1 && !over && a.lorder && a.ldir) {
            // one list (a text document): its base is 0, so the element positions the merge wrote
            // are already global — one pass counts the applied inserts, places each at its
            // position, and checks every insert's position against the count (the two counting /
            // placing passes and the hole check of the general case below, fused: C3's rebuild)
            const uint32_t lo0 = (uint32_t)__shfl((int)lobj, 0);
            bool bad = false, any_ins = false;
            uint32_t cnt1 = 0, maxpos = 0, c_lo = 0;                  // c_lo: the change of the chunk's first op
            hm_op_row px = ldop(lane);
            for (uint32_t i0 = 0; i0 < m.n_o; i0 += 64) {
                const uint32_t i = i0 + lane;
                const hm_op_row o = px;
                px = ldop(i0 + 64 + lane);
                // the changes that start inside the chunk (ops are grouped by change): lane j holds
                // the first op of change c_lo + 1 + j; an op's change is c_lo plus those starting at
                // or before it — one LDS read and a readlane per such change, no dependent search
                uint32_t cc = 0;
                bool chunk_ok = false;
                if (lch) {
                    const uint32_t cj = c_lo + 1 + lane;
                    const uint32_t ofj = cj < m.n_c ? (s_of[cj] & 0x7FFFFFFFu) : 0xFFFFFFFFu;
                    const unsigned long long in = __ballot(ofj <= i0 + 63);
                    chunk_ok = ~in != 0;                                  // (64 changes starting: search instead)
                    if (chunk_ok) {
                        cc = c_lo;
                        for (uint32_t j = 0, K = (uint32_t)__popcll(in); j < K; j++)
                            cc += (uint32_t)__builtin_amdgcn_readlane((int)ofj, (int)j) <= i ? 1u : 0u;
                    }
                }
                bool applied_ins = false;
                uint32_t c = 0;
                if (o.action == HM_INS) {
                    if (lch) {
                        c = chunk_ok ? cc : change_of_op_lds(s_of, m.n_c, i);
                        applied_ins = (s_of[c] >> 31) != 0;              // (a duplicate's copy: its twin counts)
                    } else {
                        c = change_of_op(ch, m.n_c, m.o_off, i);
                        applied_ins = a.hist[m.c_off + c] >= 0;
                    }
                }
                if (lch) {                                                // the next chunk's first change
                    const uint32_t cl = chunk_ok ? cc : change_of_op_lds(s_of, m.n_c, i < m.n_o ? i : m.n_o - 1);
                    c_lo = (uint32_t)__builtin_amdgcn_readlane((int)cl, 63);
                }
                const bool mine = o.obj == lo0;
                bad |= applied_ins && !(mine && o.elem < (1u << 24));
                cnt1 += (uint32_t)__popcll(__ballot(applied_ins && mine));
                if (o.action == HM_INS && o.reg < m.n_r) {
                    const uint32_t pos = a.epos[m.r_off + o.reg];
                    any_ins = true;
                    maxpos = pos > maxpos ? pos : maxpos;               // (HM_NONE: a hole)
                    if (applied_ins && mine && pos < m.n_r) {
                        a.lorder[m.r_off + pos] = o.reg;
                        a.epar[m.r_off + o.reg] = o.parent;
                        a.ekey[m.r_off + o.reg] = (o.elem << 8) | (ch[c].actor & 0xFFu);
                    }
                }
            }
            for (uint32_t d = 1; d < 64; d <<= 1) maxpos = max(maxpos, (uint32_t)__shfl_xor((int)maxpos, d));
            MSTAMP(3);
            n_el = cnt1;
            // every applied insert in the list, every insert's element placed inside it
            if (__ballot(bad) == 0 && (__ballot(any_ins) == 0 || maxpos < cnt1)) {
                flags |= HM_IST_LIST;
                if (lane == 0) a.ldir[(size_t)h * LMAX] = make_uint2(lo0, cnt1);
            }
        } else if (nlst && !over && a.lorder && a.ldir) {
            bool ok = true;
            uint32_t cnt = 0;                                  // lane k < nlst: list k's elements
            for (uint32_t pass = 0; pass < 2 && ok; pass++) {
                uint32_t bk = 0;                               // pass 1: lane k holds list k's base
                if (pass)
                    for (uint32_t k = 0; k < nlst; k++) {
                        const uint32_t x = (uint32_t)__shfl((int)cnt, (int)k);     // (every lane shuffles)
                        bk += k < lane ? x : 0u;
                    }
                hm_op_row px = ldop(lane);
                for (uint32_t i0 = 0; i0 < m.n_o; i0 += 64) {
                    const uint32_t i = i0 + lane;
                    const hm_op_row o = px;
                    px = ldop(i0 + 64 + lane);
                    bool applied_ins = false;
                    uint32_t c = 0, lk = HM_NONE;
                    if (o.action == HM_INS) {
                        if (lch) {
                            c = change_of_op_lds(s_of, m.n_c, i);
                            applied_ins = (s_of[c] >> 31) != 0;          // (a duplicate's copy: its twin counts)
                        } else {
                            c = change_of_op(ch, m.n_c, m.o_off, i);
                            applied_ins = a.hist[m.c_off + c] >= 0;
                        }
                    }
                    for (uint32_t k = 0; k < nlst; k++) lk = (uint32_t)__shfl((int)lobj, (int)k) == o.obj ? k : lk;
                    // (every lane shuffles: a lane that places nothing still serves as a source)
                    const uint32_t lkc = lk < nlst ? lk : 0u;
                    const uint32_t lb = (uint32_t)__shfl((int)bk, (int)lkc), lc = (uint32_t)__shfl((int)cnt, (int)lkc);
                    if (!pass) {
                        ok &= !applied_ins || (lk != HM_NONE && o.elem < (1u << 24));
                        for (uint32_t k = 0; k < nlst; k++) {
                            const uint32_t nk = (uint32_t)__popcll(__ballot(applied_ins && lk == k));
                            if (lane == k) cnt += nk;
                        }
                    } else if (applied_ins) {
                        const uint32_t pos = o.reg < m.n_r ? a.epos[m.r_off + o.reg] : HM_NONE;
                        ok &= pos < lc;
                        if (pos < lc) {
                            a.lorder[m.r_off + lb + pos] = o.reg;
                            a.epos[m.r_off + o.reg] = lb + pos;           // global from here on
                            a.epar[m.r_off + o.reg] = o.parent;
                            a.ekey[m.r_off + o.reg] = (o.elem << 8) | (ch[c].actor & 0xFFu);
                        }
                    }
                }
                ok = __ballot(!ok) == 0;
                MSTAMP(3 + pass);
            }
            for (uint32_t k = 0; k < nlst; k++) n_el += (uint32_t)__shfl((int)cnt, (int)k);
            // every element placed, at positions 0 .. n_el - 1 (detached elements have none)
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            if (ok) {
                bool hole = false;
                hm_op_row hx = ldop(lane);
                for (uint32_t i0 = 0; i0 < m.n_o; i0 += 64) {
                    const hm_op_row o = hx;
                    hx = ldop(i0 + 64 + lane);
                    if (o.action == HM_INS && o.reg < m.n_r) hole |= a.epos[m.r_off + o.reg] >= n_el;
                }
                ok = __ballot(hole) == 0;
            }
            MSTAMP(5);
            if (ok) {
                flags |= HM_IST_LIST;
                if (lane < nlst) a.ldir[(size_t)h * LMAX + lane] = make_uint2(lobj, cnt);
            }
        }
        if (lane == 0) {
            IncState st = {};
            st.s_used = r.n_surv; st.flags = flags; st.cabs = cabs; st.mapmask = mask;
            st.pad[0] = (flags & HM_IST_LIST) ? n_el : 0u; st.pad[1] = (flags & HM_IST_LIST) ? nlst : 0u;
            a.ist[h] = st;
        }
        dv += (HM_IST_COUNTS(flags) ? 1 : 0) - (was ? 1 : 0);
    }
    if (lane == 0) s_dv[threadIdx.x >> 6] = dv;
    __syncthreads();
    if (threadIdx.x == 0 && a.part) a.part[blockIdx.x] = s_dv[0] + s_dv[1] + s_dv[2] + s_dv[3];
}

// n_valid += the sum of inc_meta_kernel's per-workgroup changes (one workgroup, one atomic)
__global__ __launch_bounds__(1024) void valid_sum_kernel(const int *part, uint32_t n, uint32_t *n_valid) {
    __shared__ int s[16];
    int t = 0;
    for (uint32_t i = threadIdx.x; i < n; i += 1024) t += part[i];
    for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        int u = 0;
        for (int w = 0; w < 16; w++) u += s[w];
        if (u) atomicAdd(n_valid, (uint32_t)u);
    }
}

__global__ __launch_bounds__(256) void epos_clear_kernel(const uint32_t *list, uint32_t n, const DevDoc *dm, uint32_t *epos) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < n; q += gridDim.x * 4) {
        const DevDoc m = dm[list[q]];
        if (!(m.flags & HM_DOC_HAS_LISTS)) continue;
        for (uint32_t g = lane; g < m.n_r; g += 64) epos[m.r_off + g] = HM_NONE;
    }
}

}  // namespace hmi

hipError_t hm_launch_inc_apply(const IncArgs &A, hipStream_t s) {
    if (!A.n) return hipSuccess;
    const uint32_t S = A.S;
    if (S > 64) return hipErrorInvalidValue;
    // (the defer and bail lists' counts were zeroed by plan_kernel: alloc_kernel lists the list
    // documents in defer)
    auto grid = [](uint32_t n, uint32_t per) { const uint32_t g = (n + per - 1) / per; return g < 65535u ? g : 65535u; };
    if (S <= 16 && A.n_lane) {                                // (n_lane: the pass may have work; it checks on the device)
        // rounds longer than the group passes hold (route 3): one lane per document, first
        const uint32_t gl = (A.n + 255) / 256;
        if (S <= 8) hipLaunchKernelGGL(hmi::inc_lane_kernel<8>, dim3(gl), dim3(256), 0, s, A);
        else hipLaunchKernelGGL(hmi::inc_lane_kernel<16>, dim3(gl), dim3(256), 0, s, A);
    }
    if (S <= 8) hipLaunchKernelGGL((hmi::inc_group_kernel<8, false>), dim3(grid(A.n, 32)), dim3(256), 0, s, A);
    else if (S <= 16) hipLaunchKernelGGL((hmi::inc_group_kernel<16, false>), dim3(grid(A.n, 16)), dim3(256), 0, s, A);
    if (HM_INC_LIST_GROUPS) {
        // the documents with lists (the launch returns at once when the plan routed none here)
        if (S <= 8) hipLaunchKernelGGL((hmi::inc_group_kernel<8, false, true>), dim3(grid(A.n, 32)), dim3(256), 0, s, A);
        else if (S <= 16) hipLaunchKernelGGL((hmi::inc_group_kernel<16, false, true>), dim3(grid(A.n, 16)), dim3(256), 0, s, A);
    }
    if (S <= 16 && A.defer) {
        // the documents handed over, one per wave (their count is read on the device); rounds that
        // need tiles in a launch of their own
        IncArgs B = A;
        B.list = A.defer;
        B.defer = nullptr;
        const uint32_t gw = grid(A.n, 4) < 1024u ? grid(A.n, 4) : 1024u;
        hipLaunchKernelGGL((hmi::inc_group_kernel<64, false>), dim3(gw), dim3(256), 0, s, B);
        hipLaunchKernelGGL((hmi::inc_group_kernel<64, true>), dim3(gw), dim3(256), 0, s, B);
    } else if (S > 16) {
        IncArgs B = A;
        B.defer = nullptr;
        hipLaunchKernelGGL((hmi::inc_group_kernel<64, false>), dim3(grid(A.n, 4)), dim3(256), 0, s, B);
        hipLaunchKernelGGL((hmi::inc_group_kernel<64, true>), dim3(grid(A.n, 4) < 1024u ? grid(A.n, 4) : 1024u), dim3(256), 0, s, B);
    }
    return hipGetLastError();
}

extern "C" int hm_debug_meta_stamps(unsigned long long *out8, int reset) {
#if HM_META_STAMPS
    if (!out8 || hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(hmi::hm_meta_st), 64) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hmi::hm_meta_st), z, 64) != hipSuccess) return -1;
    }
    return 1;
#else
    (void)out8; (void)reset;
    return 0;
#endif
}

hipError_t hm_launch_inc_meta(const MetaArgs &a, hipStream_t s) {
    if (!a.n) return hipSuccess;
    const uint32_t grid = (a.n + 3) / 4 < HM_META_GRID ? (a.n + 3) / 4 : HM_META_GRID;
    hipLaunchKernelGGL(hmi::inc_meta_kernel, dim3(grid), dim3(256), 0, s, a);
    if (a.part && a.n_valid) hipLaunchKernelGGL(hmi::valid_sum_kernel, dim3(1), dim3(1024), 0, s, a.part, grid, a.n_valid);
    return hipGetLastError();
}

hipError_t hm_launch_epos_clear(const uint32_t *list, uint32_t n, const DevDoc *dm, uint32_t *epos, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t grid = (n + 3) / 4 < 65535u ? (n + 3) / 4 : 65535u;
    hipLaunchKernelGGL(hmi::epos_clear_kernel, dim3(grid), dim3(256), 0, s, list, n, dm, epos);
    return hipGetLastError();
}
