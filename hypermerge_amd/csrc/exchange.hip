// exchange.hip — the cross-GPU clock exchange of the sharded engine (include/hypermerge_amd.h,
// "Clock exchange"), over RCCL on the node's xGMI links.
//
// Documents shard by FNV-1a64(docId) % G, so the merge itself never communicates.  What crosses
// GPUs is the ClockStore feed: every document's clock entries as repo-global records
// (docId key, actorId key, seq) — actor *ranks* are per-document and encoder-local, so a record
// must name the actor by a key every rank's host can resolve ({actorId: seq}, the form
// ClockStore.update and CursorMessage carry: src/RepoBackend.ts:374-392,402,412-418).
//
//   hm_clock_records_device   dense per-document clock rows -> compacted records (order kept:
//                             document-major, actor rank within a document), device-side
//   hm_clock_count_allgather  every rank's record count (ncclAllGather, 8 B per rank)
//   hm_clock_allgather        every rank's records, back to back in rank order: one grouped
//                             ncclBroadcast per rank with that rank's exact count (no padding)
//   hm_clock_min_allreduce    Clock.intersection across replicas (src/Clock.ts:103-113) over
//                             rank-aligned rows: ncclAllReduce(MIN) with HM_CLOCK_NOT_HELD as
//                             the identity of a rank that does not hold the document
//
// RCCL is loaded on first use (dlopen "librccl.so.1": the copy the process already mapped, e.g.
// PyTorch's, or /opt/rocm's), so the merge library itself has no RCCL dependency.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <stdint.h>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>
#include "../../include/hypermerge_amd.h"
#include "engine_internal.h"

static_assert(sizeof(hm_clock_rec) == 24, "hm_clock_rec is 24 bytes");
static_assert(HM_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

namespace {

struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *);
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*Broadcast)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*GroupStart)();
    ncclResult_t (*GroupEnd)();
    const char *(*GetErrorString)(ncclResult_t);
    bool ok = false;
    std::string err;
};

Rccl &rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) { R.err = std::string("dlopen librccl.so.1: ") + dlerror(); return; }
#define SYM(f, n) if (!(*(void **)&R.f = dlsym(h, n))) { R.err = "librccl lacks " n; return; }
        SYM(GetUniqueId, "ncclGetUniqueId") SYM(CommInitRank, "ncclCommInitRank") SYM(CommDestroy, "ncclCommDestroy")
        SYM(AllGather, "ncclAllGather") SYM(Broadcast, "ncclBroadcast") SYM(AllReduce, "ncclAllReduce")
        SYM(GroupStart, "ncclGroupStart") SYM(GroupEnd, "ncclGroupEnd") SYM(GetErrorString, "ncclGetErrorString")
#undef SYM
        R.ok = true;
    });
    return R;
}

constexpr uint32_t XT = 256;          // threads per block of the record kernels
constexpr uint32_t XPER = 8;          // entries per thread
constexpr uint32_t XTILE = XT * XPER; // entries per block

__device__ __forceinline__ bool rec_live(const uint64_t *actor_keys, const uint32_t *clock, const uint32_t *base, size_t i) {
    const uint32_t v = clock[i];
    return actor_keys[i] != 0 && v > (base ? base[i] : 0u);
}

// per block: live entries of its tile
__global__ __launch_bounds__(XT) void rec_count_kernel(const uint64_t *actor_keys, const uint32_t *clock,
                                                       const uint32_t *base, size_t n, uint32_t *block_cnt) {
    __shared__ uint32_t part[XT / 64];
    const size_t t0 = (size_t)blockIdx.x * XTILE;
    uint32_t c = 0;
    for (uint32_t k = 0; k < XPER; k++) {
        const size_t i = t0 + (size_t)k * XT + threadIdx.x;
        c += (i < n && rec_live(actor_keys, clock, base, i)) ? 1u : 0u;
    }
    for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (uint32_t w = 0; w < XT / 64; w++) s += part[w];
        block_cnt[blockIdx.x] = s;
    }
}

// exclusive scan of the block counts (one workgroup; a few thousand blocks at most per 10M entries)
__global__ __launch_bounds__(1024) void rec_scan_kernel(uint32_t *block_cnt, uint32_t nb, uint32_t *total) {
    __shared__ uint32_t carry, wsum[16];
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t v = b < nb ? block_cnt[b] : 0u;
        uint32_t x = v;                                   // inclusive scan in the wave
        for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(x, o); if ((threadIdx.x & 63) >= (uint32_t)o) x += y; }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = x;
        __syncthreads();
        uint32_t wo = 0;
        for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) wo += wsum[w];
        const uint32_t c0 = carry;
        if (b < nb) block_cnt[b] = c0 + wo + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = c0 + wo + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

// records in entry order: a block's live entries at its scanned offset, ordered within the tile
__global__ __launch_bounds__(XT) void rec_write_kernel(const uint64_t *doc_keys, const uint64_t *actor_keys,
                                                       const uint32_t *clock, const uint32_t *base, size_t n,
                                                       uint32_t S, const uint32_t *block_off, hm_clock_rec *out) {
    __shared__ uint32_t wcnt[XT / 64];
    __shared__ uint32_t running;
    const size_t t0 = (size_t)blockIdx.x * XTILE;
    if (threadIdx.x == 0) running = block_off[blockIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t k = 0; k < XPER; k++) {
        const size_t i = t0 + (size_t)k * XT + threadIdx.x;
        const bool live = i < n && rec_live(actor_keys, clock, base, i);
        const unsigned long long m = __ballot(live);
        if (lane == 0) wcnt[w] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t off = running;
        for (uint32_t v = 0; v < w; v++) off += wcnt[v];
        if (live) {
            hm_clock_rec r;
            r.doc_key = doc_keys[i / S];
            r.actor_key = actor_keys[i];
            r.seq = clock[i];
            r.flags = 0;
            out[off + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = r;
        }
        __syncthreads();
        if (threadIdx.x == 0) { uint32_t s = 0; for (uint32_t v = 0; v < XT / 64; v++) s += wcnt[v]; running += s; }
        __syncthreads();
    }
}

}  // namespace

struct hm_comm {
    hm_engine *e = nullptr;
    ncclComm_t comm = nullptr;
    int world = 0, rank = 0;
};

namespace {

int nccl_fail(hm_engine *e, ncclResult_t r, const char *what) {
    std::string m = std::string(what) + ": " + (rccl().GetErrorString ? rccl().GetErrorString(r) : "rccl error");
    return hm_engine_fail(e, HM_ERR_DEVICE, m.c_str());
}

}  // namespace

extern "C" {

int hm_comm_unique_id(uint8_t *out) {
    if (!out) return HM_ERR_INVALID;
    Rccl &R = rccl();
    if (!R.ok) return HM_ERR_DEVICE;
    ncclUniqueId id;
    if (R.GetUniqueId(&id) != ncclSuccess) return HM_ERR_DEVICE;
    memcpy(out, id.internal, HM_COMM_ID_BYTES);
    return HM_OK;
}

int hm_comm_create(hm_engine *e, int world, int rank, const uint8_t *unique_id, hm_comm **out) {
    if (!e || !out || !unique_id || world < 1 || rank < 0 || rank >= world) return HM_ERR_INVALID;
    *out = nullptr;
    Rccl &R = rccl();
    if (!R.ok) return hm_engine_fail(e, HM_ERR_DEVICE, R.err.c_str());
    if (hipSetDevice(hm_engine_device(e)) != hipSuccess) return hm_engine_fail(e, HM_ERR_DEVICE, "hipSetDevice");
    hm_comm *c = new (std::nothrow) hm_comm();
    if (!c) return HM_ERR_NOMEM;
    ncclUniqueId id;
    memcpy(id.internal, unique_id, HM_COMM_ID_BYTES);
    ncclResult_t r = R.CommInitRank(&c->comm, world, id, rank);
    if (r != ncclSuccess) { delete c; return nccl_fail(e, r, "ncclCommInitRank"); }
    c->e = e; c->world = world; c->rank = rank;
    *out = c;
    return HM_OK;
}

void hm_comm_destroy(hm_comm *c) {
    if (!c) return;
    if (c->comm && rccl().ok) (void)rccl().CommDestroy(c->comm);
    delete c;
}

int hm_comm_group_start(void) {
    Rccl &R = rccl();
    return R.ok && R.GroupStart() == ncclSuccess ? HM_OK : HM_ERR_DEVICE;
}

int hm_comm_group_end(void) {
    Rccl &R = rccl();
    return R.ok && R.GroupEnd() == ncclSuccess ? HM_OK : HM_ERR_DEVICE;
}

int hm_clock_records_device(hm_engine *e, const uint64_t *doc_keys, const uint64_t *actor_keys, const uint32_t *clock,
                            const uint32_t *base, uint32_t n_docs, uint32_t a_stride, hm_clock_rec *out,
                            uint32_t *out_count, void *scratch, void *stream) {
    if (!e || !a_stride || (n_docs && (!doc_keys || !actor_keys || !clock || !out || !scratch)) || !out_count)
        return HM_ERR_INVALID;
    hipStream_t s = stream ? (hipStream_t)stream : hm_engine_stream(e);
    const size_t n = (size_t)n_docs * a_stride;
    const uint32_t nb = (uint32_t)((n + XTILE - 1) / XTILE);
    uint32_t *blk = (uint32_t *)scratch;
    if (nb == 0) {
        return hipMemsetAsync(out_count, 0, 4, s) == hipSuccess ? HM_OK : hm_engine_fail(e, HM_ERR_DEVICE, "memset");
    }
    hipLaunchKernelGGL(rec_count_kernel, dim3(nb), dim3(XT), 0, s, actor_keys, clock, base, n, blk);
    hipLaunchKernelGGL(rec_scan_kernel, dim3(1), dim3(1024), 0, s, blk, nb, out_count);
    hipLaunchKernelGGL(rec_write_kernel, dim3(nb), dim3(XT), 0, s, doc_keys, actor_keys, clock, base, n, a_stride,
                       (const uint32_t *)blk, out);
    hipError_t r = hipGetLastError();
    return r == hipSuccess ? HM_OK : hm_engine_fail(e, HM_ERR_DEVICE, hipGetErrorString(r));
}

size_t hm_clock_records_scratch_bytes(uint32_t n_docs, uint32_t a_stride) {
    const size_t n = (size_t)n_docs * a_stride;
    return ((n + XTILE - 1) / XTILE + 1) * 4;
}

int hm_clock_count_allgather(hm_comm *c, uint64_t n_local, uint64_t *d_counts, void *stream) {
    if (!c || !d_counts) return HM_ERR_INVALID;
    Rccl &R = rccl();
    hipStream_t s = stream ? (hipStream_t)stream : hm_engine_stream(c->e);
    // the own count goes through the output row: RCCL's in-place all-gather form
    if (hipMemcpyAsync(d_counts + c->rank, &n_local, 8, hipMemcpyHostToDevice, s) != hipSuccess)
        return hm_engine_fail(c->e, HM_ERR_DEVICE, "count upload");
    ncclResult_t r = R.AllGather(d_counts + c->rank, d_counts, 1, ncclUint64, c->comm, s);
    if (r != ncclSuccess) return nccl_fail(c->e, r, "ncclAllGather(counts)");
    // the pageable upload above must land before n_local leaves scope
    if (hipStreamSynchronize(s) != hipSuccess) return hm_engine_fail(c->e, HM_ERR_DEVICE, "sync");
    return HM_OK;
}

int hm_clock_allgather(hm_comm *c, const hm_clock_rec *d_recs, const uint64_t *counts, hm_clock_rec *d_out,
                       void *stream) {
    if (!c || !counts || (counts[c->rank] && !d_recs)) return HM_ERR_INVALID;
    Rccl &R = rccl();
    hipStream_t s = stream ? (hipStream_t)stream : hm_engine_stream(c->e);
    uint64_t total = 0;
    for (int q = 0; q < c->world; q++) total += counts[q];
    if (total && !d_out) return HM_ERR_INVALID;
    ncclResult_t r = R.GroupStart();
    if (r != ncclSuccess) return nccl_fail(c->e, r, "ncclGroupStart");
    uint64_t off = 0;
    for (int q = 0; q < c->world; q++) {
        const size_t words = (size_t)counts[q] * (sizeof(hm_clock_rec) / 8);
        if (words) {
            r = R.Broadcast(q == c->rank ? (const void *)d_recs : nullptr, d_out + off, words, ncclUint64, q, c->comm, s);
            if (r != ncclSuccess) { (void)R.GroupEnd(); return nccl_fail(c->e, r, "ncclBroadcast(records)"); }
        }
        off += counts[q];
    }
    r = R.GroupEnd();
    if (r != ncclSuccess) return nccl_fail(c->e, r, "ncclGroupEnd");
    return HM_OK;
}

int hm_clock_min_allreduce(hm_comm *c, uint32_t *d_seq, uint64_t n, void *stream) {
    if (!c || (n && !d_seq)) return HM_ERR_INVALID;
    if (!n) return HM_OK;
    hipStream_t s = stream ? (hipStream_t)stream : hm_engine_stream(c->e);
    ncclResult_t r = rccl().AllReduce(d_seq, d_seq, n, ncclUint32, ncclMin, c->comm, s);
    return r == ncclSuccess ? HM_OK : nccl_fail(c->e, r, "ncclAllReduce(min)");
}

// ---- one process driving several GPUs (the Node host's GpuEngine): host-buffer helpers ----

int hm_comm_create_local(hm_engine *const *engines, int n, hm_comm **out) {
    if (!engines || !out || n < 1) return HM_ERR_INVALID;
    for (int i = 0; i < n; i++) out[i] = nullptr;
    uint8_t id[HM_COMM_ID_BYTES];
    int st = hm_comm_unique_id(id);
    if (st) return st;
    int rc = hm_comm_group_start();
    if (rc) return rc;
    for (int i = 0; i < n && !st; i++) st = hm_comm_create(engines[i], n, i, id, &out[i]);
    rc = hm_comm_group_end();
    if (st || rc) {
        for (int i = 0; i < n; i++) { hm_comm_destroy(out[i]); out[i] = nullptr; }
        return st ? st : rc;
    }
    return HM_OK;
}

int hm_clock_exchange_host(hm_comm *const *comms, int n, const hm_clock_rec *const *recs, const uint64_t *n_recs,
                           hm_clock_rec *out, uint64_t out_cap, uint64_t *out_total) {
    if (!comms || n < 1 || !n_recs || !out_total) return HM_ERR_INVALID;
    uint64_t total = 0;
    for (int i = 0; i < n; i++) total += n_recs[i];
    *out_total = total;
    if (total > out_cap || (total && !out)) return HM_ERR_INVALID;
    std::vector<hm_clock_rec *> dsend(n, nullptr), drecv(n, nullptr);
    std::vector<uint64_t *> dcnt(n, nullptr);
    int st = HM_OK;
    auto cleanup = [&] {
        for (int i = 0; i < n; i++) {
            (void)hipSetDevice(hm_engine_device(comms[i]->e));
            (void)hipStreamSynchronize(hm_engine_stream(comms[i]->e));
            if (dsend[i]) (void)hipFree(dsend[i]);
            if (drecv[i]) (void)hipFree(drecv[i]);
            if (dcnt[i]) (void)hipFree(dcnt[i]);
        }
    };
    for (int i = 0; i < n && !st; i++) {
        hm_comm *c = comms[i];
        if (hipSetDevice(hm_engine_device(c->e)) != hipSuccess ||
            hipMalloc(&dsend[i], (n_recs[i] + 1) * sizeof(hm_clock_rec)) != hipSuccess ||
            hipMalloc(&drecv[i], (total + 1) * sizeof(hm_clock_rec)) != hipSuccess ||
            hipMalloc(&dcnt[i], 8 * (size_t)c->world) != hipSuccess) { st = HM_ERR_NOMEM; break; }
        if (n_recs[i] && hipMemcpy(dsend[i], recs[i], n_recs[i] * sizeof(hm_clock_rec), hipMemcpyHostToDevice) != hipSuccess)
            st = HM_ERR_DEVICE;
    }
    // the counts are the callers' own (one process): every communicator gathers the same records
    std::vector<uint64_t> counts(n_recs, n_recs + n);
    if (!st) st = hm_comm_group_start();
    if (!st) {
        for (int i = 0; i < n && !st; i++) {
            (void)hipSetDevice(hm_engine_device(comms[i]->e));
            st = hm_clock_allgather(comms[i], dsend[i], counts.data(), drecv[i], hm_engine_stream(comms[i]->e));
        }
        const int rc = hm_comm_group_end();
        st = st ? st : rc;
    }
    if (!st && total) {
        (void)hipSetDevice(hm_engine_device(comms[0]->e));
        if (hipMemcpyAsync(out, drecv[0], total * sizeof(hm_clock_rec), hipMemcpyDeviceToHost,
                           hm_engine_stream(comms[0]->e)) != hipSuccess) st = HM_ERR_DEVICE;
    }
    cleanup();
    return st;
}

int hm_clock_min_host(hm_comm *const *comms, int n, uint32_t *const *seq, uint64_t len) {
    if (!comms || n < 1 || !seq) return HM_ERR_INVALID;
    if (!len) return HM_OK;
    std::vector<uint32_t *> d(n, nullptr);
    int st = HM_OK;
    for (int i = 0; i < n && !st; i++) {
        (void)hipSetDevice(hm_engine_device(comms[i]->e));
        if (hipMalloc(&d[i], len * 4) != hipSuccess) { st = HM_ERR_NOMEM; break; }
        if (hipMemcpy(d[i], seq[i], len * 4, hipMemcpyHostToDevice) != hipSuccess) st = HM_ERR_DEVICE;
    }
    if (!st) st = hm_comm_group_start();
    if (!st) {
        for (int i = 0; i < n && !st; i++) {
            (void)hipSetDevice(hm_engine_device(comms[i]->e));
            st = hm_clock_min_allreduce(comms[i], d[i], len, hm_engine_stream(comms[i]->e));
        }
        const int rc = hm_comm_group_end();
        st = st ? st : rc;
    }
    for (int i = 0; i < n; i++) {
        (void)hipSetDevice(hm_engine_device(comms[i]->e));
        (void)hipStreamSynchronize(hm_engine_stream(comms[i]->e));
        if (!st && d[i] && hipMemcpy(seq[i], d[i], len * 4, hipMemcpyDeviceToHost) != hipSuccess) st = HM_ERR_DEVICE;
        if (d[i]) (void)hipFree(d[i]);
    }
    return st;
}

}  // extern "C"
