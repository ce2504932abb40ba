/*
 * hypermerge_amd.h — C-ABI boundary of the MI355X batched CRDT merge engine.
 *
 * The engine replaces the L5 -> L0 edge of hypermerge: everything that
 * Automerge 0.12's `Backend.applyChanges(state, changes)` computes when
 * `DocBackend.applyRemoteChanges` / `DocBackend.init` hand it a batch of
 * decoded `Change` objects, plus the vector-clock bookkeeping around it.
 *
 *   reference call sites replaced (paths relative to the reference repo):
 *     src/DocBackend.ts:115-117  applyRemoteChanges(changes)  -> remoteChangesQ
 *     src/DocBackend.ts:169-185  Backend.applyChanges(back, changes) + updateClock
 *     src/DocBackend.ts:144-167  init(changes): Backend.applyChanges(Backend.init(), changes)
 *     src/DocBackend.ts:135-142  updateClock (clock includes queued changes)
 *     src/DocBackend.ts:90-100   testMinimumClockSatisfied -> Clock.cmp
 *     src/Clock.ts:13-38,87-113  gte / cmp / union / intersection
 *     src/RepoBackend.ts:570-579 MaterializeMsg (history-prefix replay)
 *   Automerge 0.12.2-beta.0 (yarn.lock:178-185; NOT vendored) backend/op_set.js:
 *     addChange/applyQueuedOps/causallyReady, applyChange/transitiveDeps,
 *     applyAssign (map registers, counters, conflicts), applyInsert +
 *     updateListElement (RGA lists/text).  Restated in SURVEY.md Appendix A.
 *
 * A batch is columnar: plain little-endian tables, no strings.  Strings
 * (actor ids, object UUIDs, keys, string values) are interned by the host
 * encoder; the engine only needs their identity, except actor ids, whose
 * JS UTF-16 string order is encoded as the per-document actor *rank*.
 *
 * No C++ exception crosses this boundary.  Every call returns an hm_status;
 * per-document failures are reported per document (hm_doc_result.status),
 * never as a whole-batch failure (the reference aborts only the throwing
 * document's applyChanges; SURVEY.md §5, §8b "Errors").
 */
#ifndef HYPERMERGE_AMD_H
#define HYPERMERGE_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HM_ABI_VERSION 4u

/* ------------------------------------------------------------------ */
/* Status codes                                                        */
/* ------------------------------------------------------------------ */
typedef enum {
    HM_OK = 0,
    /* per-document Automerge errors (the message each maps to is what the
     * reference would throw; see hm_status_message) */
    HM_ERR_INCONSISTENT_SEQ = 1,   /* 'Inconsistent reuse of sequence number <seq> by <actor>' */
    HM_ERR_UNKNOWN_OBJECT = 2,     /* 'Modification of unknown object <obj>' */
    HM_ERR_DUPLICATE_OBJECT = 3,   /* 'Duplicate creation of object <obj>' */
    HM_ERR_DUPLICATE_ELEM = 4,     /* 'Duplicate list element ID <elemId>' */
    HM_ERR_MISSING_ELEM = 5,       /* 'Missing index entry for list element <elemId>' */
    /* engine-side limits / preconditions (not reference errors) */
    HM_ERR_UNSUPPORTED = 16,       /* document outside the engine's supported envelope */
    /* call-level errors */
    HM_ERR_INVALID = 32,           /* malformed batch (bad offsets, sizes) */
    HM_ERR_DEVICE = 33,            /* HIP runtime failure */
    HM_ERR_NOMEM = 34
} hm_status;

/* ------------------------------------------------------------------ */
/* Op actions / datatypes / value tags (Automerge 0.12 op vocabulary)   */
/* ------------------------------------------------------------------ */
enum {
    HM_MAKE_MAP = 0, HM_MAKE_TABLE = 1, HM_MAKE_LIST = 2, HM_MAKE_TEXT = 3,
    HM_INS = 4, HM_SET = 5, HM_DEL = 6, HM_LINK = 7, HM_INC = 8
};
enum { HM_DT_NONE = 0, HM_DT_COUNTER = 1, HM_DT_TIMESTAMP = 2 };
enum {
    HM_V_NULL = 0, HM_V_FALSE = 1, HM_V_TRUE = 2,
    HM_V_INT = 3,    /* integral JS number, |v| < 2^53, stored as int64 */
    HM_V_FLOAT = 4,  /* any other JS number, stored as IEEE-754 f64 bits */
    HM_V_STR = 5,    /* string-pool id */
    HM_V_OBJ = 6     /* doc-local object id (link target) */
};
#define HM_HEAD 0xFFFFFFFFu      /* ins parent '_head' */
#define HM_NONE 0xFFFFFFFFu

/* ------------------------------------------------------------------ */
/* Columnar batch tables                                               */
/* ------------------------------------------------------------------ */

/* One row per document (48 B).  Every input range of a document is in its row,
 * so all of a document's loads can be issued as soon as the row is read. */
typedef struct {
    uint32_t change_off;  /* first row of this doc in changes[] */
    uint32_t n_changes;   /* changes handed to applyChanges, in array (arrival) order */
    uint32_t dep_off;     /* first row of this doc in deps[] (= changes[change_off].dep_off) */
    uint32_t n_deps;      /* dep rows of all its changes (contiguous) */
    uint32_t op_off;      /* first row of this doc in ops[]; ops are grouped by change, in op order */
    uint32_t n_ops;
    uint32_t reg_off;     /* first row of this doc in the per-register output table */
    uint32_t n_regs;      /* registers = interned (obj, key) pairs; for lists key = elemId */
    uint32_t n_objs;      /* interned object ids, 0 = ROOT '00000000-0000-0000-0000-000000000000' */
    uint16_t n_actors;    /* actor ranks 0..n_actors-1 (rank = order of the actor id strings) */
    uint16_t flags;       /* HM_DOC_* bits set by the encoder */
    uint32_t reserved[2]; /* not read by the engine (the synthetic feeds keep the doc's global index here) */
} hm_doc_row;
#define HM_DOC_HAS_LISTS 1u     /* the doc creates a list/text object (launch sizing hint only) */
#define HM_DOC_HAS_COUNTERS 2u  /* the doc has counter sets or incs (launch sizing hint only) */

/* One row per change (24 B), in the order the changes are handed over. */
typedef struct {
    uint16_t actor;       /* actor rank within the doc */
    uint16_t n_deps;
    uint32_t seq;         /* 1-based */
    uint32_t dep_off;     /* first row in deps[] (global) */
    uint32_t n_ops;       /* ops of this change: rows [op_first, op_first+n_ops) */
    uint32_t op_first;    /* global op row */
    uint32_t content_id;  /* equal <=> the two changes are deep-equal (host-interned) */
} hm_change_row;

/* One row per dependency entry (8 B), in the change's `deps` key order. */
typedef struct {
    uint16_t actor;
    uint16_t pad;
    uint32_t seq;
} hm_dep_row;

/* One row per op (32 B). */
typedef struct {
    uint32_t obj;         /* doc-local object id the op modifies (make*: the created object) */
    uint32_t reg;         /* set/del/link/inc: register of (obj,key); ins: register of the new element */
    uint32_t parent;      /* ins: register of the predecessor element, or HM_HEAD */
    uint32_t elem;        /* ins: element counter */
    uint8_t  action;      /* HM_MAKE_* / HM_INS / HM_SET / HM_DEL / HM_LINK / HM_INC */
    uint8_t  datatype;    /* HM_DT_* */
    uint8_t  vtag;        /* HM_V_* */
    uint8_t  pad;
    uint32_t key;         /* string-pool id of the map key (rendering only) */
    uint64_t value;       /* int64 / f64 bits / string id / object id, by vtag */
} hm_op_row;

/* Widest per-actor row (actors per document): the reference mints one actor per writer
 * (src/RepoBackend.ts:286-293), so a shared document can have many.  Documents of more than
 * 8 actors merge in the general kernel; rows wider than 64 are the "wide" strides. */
#define HM_MAX_STRIDE 256u

typedef struct {
    uint32_t n_docs, n_changes, n_deps, n_ops, n_regs;
    uint32_t a_stride;    /* >= max n_actors; stride of every per-actor output row (1..HM_MAX_STRIDE) */
    /* per-document maxima over the batch (launch sizing hints); 0 = unknown,
     * computed by the engine from the doc table */
    uint32_t max_changes, max_ops, max_regs, max_objs;
    uint32_t doc_flags;   /* OR of every docs[d].flags (launch hint; 0 when unknown -> computed) */
    uint32_t max_deps;    /* max docs[d].n_deps (launch hint, sizes the LDS dep table) */
    const hm_doc_row    *docs;
    const hm_change_row *changes;
    const hm_dep_row    *deps;
    const hm_op_row     *ops;
    const uint32_t      *min_clock;  /* optional [n_docs*a_stride] minimumClock (0 = absent) or NULL */
} hm_batch;

/* ------------------------------------------------------------------ */
/* Results                                                             */
/* ------------------------------------------------------------------ */
typedef struct {          /* 32 B */
    int32_t  status;      /* hm_status for this document */
    uint32_t err_change;  /* doc-local change index where the first error fired (HM_NONE if ok) */
    uint32_t err_op;      /* op index within that change, HM_NONE for change-level errors */
    uint32_t hist_len;    /* opSet.history.size after the merge */
    uint32_t n_queued;    /* changes left in opSet.queue (causally blocked) */
    uint32_t n_surv;      /* survivors written for this doc */
    uint32_t min_cmp;     /* Clock.cmp(DocBackend.clock, minimumClock): 0 EQ 1 GT 2 LT 3 CONCUR */
    uint32_t pad;
} hm_doc_result;

typedef struct {          /* 16 B per register */
    uint32_t n_surv;      /* surviving ops (winner + conflicts) */
    uint32_t surv_off;    /* doc-local offset into the survivor table (doc base = docs[d].op_off) */
    int32_t  list_index;  /* list/text element: index among visible elements, else -1 */
    uint32_t obj;         /* object the register belongs to (HM_NONE if never touched) */
} hm_reg_result;

typedef struct {          /* 16 B per survivor, winner first then conflicts */
    uint32_t op;          /* doc-local op index (ops[docs[d].op_off + op]) */
    uint32_t vtag;        /* value tag of the resolved value (counters may turn INT -> FLOAT) */
    uint64_t value;       /* resolved value (counter: base + causally-later incs) */
} hm_surv_result;

typedef struct {
    hm_doc_result  *docs;       /* [n_docs] */
    uint32_t       *clock;      /* [n_docs*a_stride] opSet.clock (applied changes only) */
    uint32_t       *back_clock; /* [n_docs*a_stride] DocBackend.clock (max over handed changes, quirk) */
    uint32_t       *heads;      /* [n_docs*a_stride] opSet.deps (0 = no entry) */
    int32_t        *hist;       /* [n_changes] history position, -1 queued, -2 duplicate (no-op) */
    uint32_t       *all_deps;   /* [n_changes*a_stride] opSet.states[actor][seq-1].allDeps (0 if not applied) */
    hm_reg_result  *regs;       /* [n_regs] */
    hm_surv_result *surv;       /* [n_ops] */
} hm_results;

/* ------------------------------------------------------------------ */
/* Engine                                                              */
/* ------------------------------------------------------------------ */
typedef struct hm_engine hm_engine;

typedef struct {
    int device;           /* HIP device ordinal */
    int flags;            /* HM_CFG_* */
} hm_config;
#define HM_CFG_GENERAL_ONLY 1   /* route every document through the general (workgroup) kernel */

/* Version of the ABI compiled into the library. */
uint32_t hm_abi_version(void);
const char *hm_status_message(int status);

int  hm_engine_create(const hm_config *cfg, hm_engine **out);
void hm_engine_destroy(hm_engine *e);
const char *hm_engine_last_error(const hm_engine *e);

/* Host batch -> device -> merge -> host results (synchronous).  All host
 * buffers are owned by the caller; the engine stages copies.  A batch of
 * >= 128k documents whose tables are in document order is processed in up to
 * 16 document ranges with upload, merge and download overlapped on three
 * streams; page-locked caller buffers (hipHostMalloc / torch pin_memory) let
 * those copies run at PCIe DMA rate.  Results are identical either way. */
int hm_merge_host(hm_engine *e, const hm_batch *batch, const hm_results *out);

/* Device-resident merge: every pointer in `batch` and `out` is a device
 * pointer on the engine's device; work is enqueued on `stream` (hipStream_t,
 * NULL = the engine's stream) and the call returns without synchronising.
 * `scratch` is device memory of at least hm_scratch_bytes(batch) bytes. */
size_t hm_scratch_bytes(const hm_batch *batch);
int hm_merge_device(hm_engine *e, const hm_batch *batch, const hm_results *out,
                    void *scratch, void *stream);

/* Per-kernel launch timing of the last hm_merge_* call on `stream`,
 * measured with HIP events on that stream (ms).  Returns number filled. */
int hm_last_kernel_ms(hm_engine *e, float *ms, int max_kernels);
/* Documents the last hm_merge_* launch routed to the general (workgroup) kernel: waits
 * for that launch, copies up to `cap` of their launch-row indices (in hand-over order)
 * and returns their count (negative hm_status on failure; -HM_ERR_INVALID after a
 * hm_merge_device with caller scratch, whose list the engine cannot know is still valid).
 * Diagnostics / roofline attribution: the two kernels' algorithmic bytes are split by it. */
int hm_last_deferred(hm_engine *e, uint32_t *out_docs, uint32_t cap);

/* ------------------------------------------------------------------ */
/* Clock algebra (src/Clock.ts) over dense per-doc rows (a_stride wide) */
/* ------------------------------------------------------------------ */
/* out[d] = Clock.cmp(a[d], b[d]) coded 0 EQ, 1 GT, 2 LT, 3 CONCUR  (src/Clock.ts:27-38) */
int hm_clock_cmp_device(hm_engine *e, const uint32_t *a, const uint32_t *b, uint8_t *out,
                        uint32_t n_docs, uint32_t a_stride, void *stream);
/* c[d] = Clock.union(a[d], b[d]) elementwise max (src/Clock.ts:87-95) */
int hm_clock_union_device(hm_engine *e, const uint32_t *a, const uint32_t *b, uint32_t *c,
                          uint32_t n_docs, uint32_t a_stride, void *stream);
/* c[d] = Clock.intersection(a[d], b[d]) elementwise min, zeros dropped (src/Clock.ts:103-113) */
int hm_clock_intersection_device(hm_engine *e, const uint32_t *a, const uint32_t *b, uint32_t *c,
                                 uint32_t n_docs, uint32_t a_stride, void *stream);

/* ------------------------------------------------------------------ */
/* Resident document store: the per-document Automerge BackendState    */
/* (`DocBackend.back`, src/DocBackend.ts:50) kept on the device.       */
/* ------------------------------------------------------------------ */
/*
 * Every open document owns device segments holding its change log (the
 * change/dep/op rows of every change handed to applyChanges so far, in
 * arrival order) and its merged state (history, allDeps, registers,
 * survivors, clocks).  `Backend.applyChanges(back, changes)` is a left fold of
 * addChange over `changes`, so applyChanges(applyChanges(s, A), B) is
 * applyChanges(s, A ++ B): a submit appends each document's new rows to its
 * log and either applies them on the resident state (hm_store_set_incremental)
 * or re-merges the log with the batch kernels.  A document whose merge
 * throws is rolled back to its previous log, exactly as a throwing
 * applyChanges leaves `DocBackend.back` (and `DocBackend.clock`) unchanged
 * (src/DocBackend.ts:170-184).
 *
 *   replaces: src/DocBackend.ts:144-167 init(changes)  (hm_doc_open + submit)
 *             src/DocBackend.ts:115-117,169-185 applyRemoteChanges
 *             src/DocBackend.ts:90-113 testMinimumClockSatisfied / updateMinimumClock
 *             src/DocBackend.ts:135-142 updateClock (hm_batch_wait back_clock)
 *             src/RepoBackend.ts:572-576 history.slice(0, n) (hm_doc_history_prefix)
 *             src/ClockStore.ts:78-91 update (hm_store_clock_update)
 *             src/RepoBackend.ts:506-531 syncChanges contiguity (hm_sync_ranges_device)
 */
typedef struct hm_store hm_store;

typedef struct {
    uint32_t a_stride;      /* per-actor row width of every document (1..64) */
    uint32_t reserved;
} hm_store_config;

int  hm_store_create(hm_engine *e, const hm_store_config *cfg, hm_store **out);
void hm_store_destroy(hm_store *s);

/* A new, empty document (Backend.init()).  Handles are dense from 0. */
int hm_doc_open(hm_store *s, uint32_t *out_doc);

/* n new, empty documents with consecutive handles starting at *out_first. */
int hm_doc_open_n(hm_store *s, uint32_t n, uint32_t *out_first);

/* Release n documents: each handle becomes an empty document again (as hm_doc_open made it,
 * ready for reuse) and its old rows are dead space that the next compaction reclaims.
 * Not while a batch is in flight; the handles must be distinct.  (No reference counterpart:
 * the docset's restride (a document moving to a wider actor class) releases its old handle
 * with it instead of leaking its rows.) */
int hm_doc_reset(hm_store *s, const uint32_t *doc_handles, uint32_t n);

/* Append new changes to documents and re-merge them.  `b` is a batch in the
 * hm_batch layout whose rows are only the NEW changes (offsets local to `b`);
 * for each row i, docs[i].n_actors / n_regs / n_objs are document totals
 * after the append and doc_handles[i] names the document (each at most once
 * per batch).  actor_remap (optional, [n_docs * a_stride]) gives, for each row,
 * the new rank of every previously used actor rank (identity rows allowed;
 * NULL = no document's ranks moved) — ranks are actor-id string order, so a
 * new actor can shift the ranks of the document's existing rows.
 * Asynchronous: results are collected by hm_batch_wait.  One batch in flight. */
int hm_batch_submit(hm_store *s, const hm_batch *b, const uint32_t *doc_handles,
                    const uint8_t *actor_remap, uint64_t *out_batch_id);

/* Wait for a submitted batch (from any one host thread; the store is not otherwise
 * thread-safe: no other call on it until the wait returns); per batch row: the merge result of the
 * document's whole log, and (each optional) its opSet.clock, DocBackend.clock
 * and opSet.deps rows ([n_docs * a_stride]).  Documents whose merge threw are
 * reported with their error status and rolled back before this returns. */
int hm_batch_wait(hm_store *s, uint64_t batch_id, hm_doc_result *out_docs,
                  uint32_t *out_clock, uint32_t *out_back_clock, uint32_t *out_heads);

/* hm_batch_submit with the batch already in HBM: b->docs / changes / deps / ops, doc_handles
 * and actor_remap are device pointers on the store's device (counts in b as usual), read
 * in place — they must stay unchanged until the batch's wait returns.  (A host that decodes
 * blocks into device buffers on a copy stream, or a GPU producer, hands rows over without a
 * host round trip.) */
int hm_batch_submit_device(hm_store *s, const hm_batch *b, const uint32_t *doc_handles,
                           const uint8_t *actor_remap, uint64_t *out_batch_id);

/* Wait for a batch and leave its results on the device: out_dev (device memory) receives
 * [n_docs hm_doc_result][n_docs*a_stride clock][n_docs*a_stride back_clock][n_docs*a_stride heads]
 * by one device-to-device copy; out_n_failed (optional, host) = rows whose status is not OK
 * (those documents are rolled back before this returns, as in hm_batch_wait). */
int hm_batch_wait_device(hm_store *s, uint64_t batch_id, void *out_dev, uint32_t *out_n_failed);

/* Undo the last waited batch: every document of it back to its log and state before the
 * submit (its new rows dropped, actor ranks mapped back, the previous state re-merged), as if
 * the batch had thrown for all of them.  Only the last batch waited for, and only until the
 * store's next submit.  (The docset undoes the batches of a call whose later step failed, so a
 * call is applied to every store or to none.) */
int hm_batch_undo(hm_store *s, uint64_t batch_id);

/* Incremental applyRemoteChanges (on by default): a document whose new changes are each
 * causally ready in arrival order on its resident state (nothing queued, no actor re-rank,
 * map set/del/link/inc ops, small submits) is advanced in place — history, allDeps, heads and
 * clock appended, only the registers its new ops hit read and rewritten — instead of
 * re-merging its whole log.  Results are identical either way; off = always re-merge.
 * on = 1: a document with list / text objects whose log fits the small merge kernel (<= 256
 * ops) re-merges: it is one wave either way, and such a document then keeps no incremental
 * state to maintain; on = 2: every eligible document takes the incremental path (tests).
 * (A register's survivors may then sit anywhere in its document's op segment; hm_doc_read
 * hands them out packed, as a merge writes them.) */
int hm_store_set_incremental(hm_store *s, int on);
/* Routing of the last submit: out3 = {incremental, re-merged, incremental handed back to
 * the re-merge}. */
int hm_store_last_routing(const hm_store *s, uint32_t *out3);
/* Device time of the last submit, from HIP events on the engine stream: out2[0] = the
 * incremental kernels (lane / group / wave passes), out2[1] = the re-merge of the documents
 * they did not take (row build, merge kernels, metadata), in ms; read once hm_batch_wait(_device)
 * has returned for that submit (the submit itself does not wait for its kernels). */
int hm_store_last_kernel_ms(const hm_store *s, float *out2);
/* Documents whose resident incremental state a submit can use (kept on the device by every step
 * that builds or drops a state; a store with none plans its submits as whole re-merges and
 * launches no incremental kernel).  Synchronous; no batch may be in flight. */
int hm_store_inc_states(hm_store *s, uint32_t *out);

/* Diagnostics of check builds (libhmgpu_check.so, built beside libhmgpu.so): out2[0] = documents
 * whose next rows merge_small_kernel loaded asynchronously and re-read with counted loads,
 * out2[1] = those whose two reads differed (the asynchronous wait was too short); reset zeroes
 * both.  Returns 1 in a check build, 0 in the product build (out2 untouched), < 0 on a HIP error. */
int hm_debug_async_check(unsigned long long *out2, int reset);

/* Sizes of a document's log and merged state. */
typedef struct {
    uint32_t n_changes, n_deps, n_ops, n_regs, n_objs, n_actors;
    uint32_t hist_len, n_queued, n_surv;
    int32_t  status;
} hm_doc_info_t;
int hm_doc_info(hm_store *s, uint32_t doc, hm_doc_info_t *out);

/* Read a document's merged state (any pointer may be NULL):
 * hist [n_changes], all_deps [n_changes*a_stride], regs [n_regs],
 * surv [n_ops] (first n_surv valid), clock/back_clock/heads [a_stride]. */
int hm_doc_read(hm_store *s, uint32_t doc, int32_t *hist, uint32_t *all_deps, hm_reg_result *regs,
                hm_surv_result *surv, uint32_t *clock, uint32_t *back_clock, uint32_t *heads);

/* Chosen registers of resident documents (incremental patches: only the registers a submit's
 * ops hit are read).  Request i = (doc_handles[i], regs[i]); out_regs[i] is that register's row
 * with surv_off rewritten to an offset into out_surv, where its n_surv survivors are copied
 * (request order of the survivor blocks is unspecified).  surv_cap = rows of out_surv; the
 * survivors of a document's registers never exceed its hm_doc_result.n_surv.  *out_n_surv =
 * rows needed; HM_ERR_NOMEM (nothing copied to out_surv) when that exceeds surv_cap. */
int hm_store_read_regs(hm_store *s, uint32_t n, const uint32_t *doc_handles, const uint32_t *regs,
                       hm_reg_result *out_regs, hm_surv_result *out_surv, uint32_t surv_cap, uint32_t *out_n_surv);

/* The log rows of a document (debug / materialize): changes [n_changes]
 * with dep_off/op_first local to the document, deps [n_deps], ops [n_ops]. */
int hm_doc_log(hm_store *s, uint32_t doc, hm_change_row *changes, hm_dep_row *deps, hm_op_row *ops);

/* history.slice(0, n): log indices of the first n applied changes, in history
 * order (src/RepoBackend.ts:572-576).  Returns the count written (<= n). */
int hm_doc_history_prefix(hm_store *s, uint32_t doc, uint32_t n, uint32_t *out_log_index);

/* history.slice(from[i], to[i]) of many documents at once (the changes one applyChanges round
 * applied, in application order; patch rendering): request i writes
 * rows out_off[i] .. out_off[i+1]-1 (out_off[i+1] - out_off[i] = to[i] - from[i]): the log index
 * of each change and (out_all_deps optional, [rows * a_stride]) its allDeps row.
 * HM_ERR_INVALID if a slice runs past the document's history. */
int hm_store_read_history(hm_store *s, uint32_t n, const uint32_t *doc_handles, const uint32_t *from, const uint32_t *to,
                          const uint32_t *out_off, uint32_t *out_log_index, uint32_t *out_all_deps);

/* minimumClock row of a document (rank-indexed, 0 = absent); used for the
 * min_cmp of the next merges (Clock.cmp(DocBackend.clock, minimumClock)). */
int hm_doc_set_min_clock(hm_store *s, uint32_t doc, const uint32_t *clock);

/* ClockStore.update(repoId=self, docId, doc.clock) for n documents
 * (src/ClockStore.ts:78-91, called at src/RepoBackend.ts:343-345): the stored
 * row becomes max(stored, DocBackend.clock) per entry.  out_written[i] = 1 if any
 * stored entry changed (the rows SQLite must persist); out_differs[i] = 1 if
 * !Clock.equal(input, stored) (ClockStore pushes updateQ).  out_stored
 * (optional, [n*a_stride]) receives the stored rows. */
int hm_store_clock_update(hm_store *s, uint32_t n, const uint32_t *docs, uint8_t *out_written,
                          uint8_t *out_differs, uint32_t *out_stored);

/* ------------------------------------------------------------------ */
/* CursorStore (src/CursorStore.ts:19-79) on the device                 */
/* ------------------------------------------------------------------ */
/* One repo's Cursors table (schema src/migrations/0001_initial_schema.sql:15-21): per
 * document row (dense indices the caller assigns), up to max_actors_per_doc entries of
 * (actor key, seq); actor key = FNV-1a64 of the actor id (as hm_clock_rec), seq stored
 * boundedSeq-clamped to [0, INFINITY_SEQ = 2^53 - 1].  Entries keep insertion order.
 * It gates syncChanges (src/RepoBackend.ts:506-531): docsWithActor picks the documents of
 * a synced actor and entry bounds each one's range; every call here is a batch. */
typedef struct hm_cursors hm_cursors;
int  hm_cursors_create(hm_engine *e, uint32_t max_actors_per_doc, hm_cursors **out);
void hm_cursors_destroy(hm_cursors *c);
/* rows 0 .. n_rows-1 exist (new rows empty) */
int  hm_cursors_reserve(hm_cursors *c, uint32_t n_rows);
/* CursorStore.update(repoId, docId, cursor) for n_docs documents (src/CursorStore.ts:51-64):
 * document d's entries are [entry_off[d], entry_off[d+1]) of actor_keys / seqs (distinct
 * actors per document; seqs as JS numbers, Infinity allowed); each is an upsert-max
 * (ON CONFLICT DO UPDATE ... WHERE excluded.seq > seq).  out_differs[d] (optional) = 1 if
 * !Clock.equal(cursor, stored cursor after the update), i.e. updateQ is pushed.
 * All or nothing: HM_ERR_INVALID with nothing written if a row would outgrow
 * max_actors_per_doc, a row appears twice in the call, or an actor twice in one row's entries. */
int  hm_cursors_update(hm_cursors *c, uint32_t n_docs, const uint32_t *rows, const uint32_t *entry_off,
                       const uint64_t *actor_keys, const double *seqs, uint8_t *out_differs);
/* CursorStore.get for n rows: out_count[i] entries in out_actor/out_seq [i * max_actors_per_doc ...] */
int  hm_cursors_get(hm_cursors *c, uint32_t n, const uint32_t *rows, uint32_t *out_count, uint64_t *out_actor,
                    uint64_t *out_seq);
/* CursorStore.entry (src/CursorStore.ts:68-70) for n (row, actor) pairs: stored seq or 0 */
int  hm_cursors_entry(hm_cursors *c, uint32_t n, const uint32_t *rows, const uint64_t *actor_keys, uint64_t *out_seq);
/* CursorStore.docsWithActor(repoId, actor, seq) (src/CursorStore.ts:73-75) for n_actors
 * actors at once: every stored entry of one of the actors with seq >= boundedSeq(min_seqs[q])
 * (min_seqs may be NULL = 0) -> (row, query index q, stored seq); order unspecified.
 * *out_n = matches; HM_ERR_NOMEM (nothing copied) when that exceeds cap. */
int  hm_cursors_docs_with_actors(hm_cursors *c, uint32_t n_actors, const uint64_t *actor_keys, const double *min_seqs,
                                 uint32_t cap, uint32_t *out_row, uint32_t *out_actor, uint64_t *out_seq,
                                 uint32_t *out_n);

/* syncChanges contiguity (src/RepoBackend.ts:513-522) over many (doc, actor)
 * pairs on the device: for pair i, walk seq indices j = lo[i] .. hi[i]-1 while
 * bit j of the actor feed's present bitmap (words from present + word_off[i])
 * is set; out_end[i] = first missing index (or hi[i]).  Device pointers. */
int hm_sync_ranges_device(hm_engine *e, const uint64_t *present, const uint64_t *word_off,
                          const uint32_t *lo, const uint32_t *hi, uint32_t *out_end, uint32_t n,
                          void *stream);
/* The same from host arrays (present: n_words u64 bitmap words; staged through the device,
 * synchronous): the syncChanges plan of a batch of (doc, actor) pairs. */
int hm_sync_ranges_host(hm_engine *e, const uint64_t *present, const uint64_t *word_off, const uint32_t *lo,
                        const uint32_t *hi, uint32_t *out_end, uint32_t n, uint32_t n_words);

/* ------------------------------------------------------------------ */
/* Blocks -> columnar rows (host, multi-threaded)                      */
/* ------------------------------------------------------------------ */
/*
 * The host front of the path: hypercore blocks -> Change objects -> the rows above.
 *   replaces: src/Block.ts:18-29 Block.unpack ('{"' raw JSON | 'BR' + brotli(JSON), else throw)
 *             src/JsonBuffer.ts:1-4 JsonBuffer.parse, src/Actor.ts:137-141 Actor.parseBlock
 *             + the host encoder (hypermerge_amd/js/columnar.js), row for row.
 * Blocks of all documents lie back to back in `data`: block i is data[block_off[i] ..
 * block_off[i+1]); document d's blocks (one Change each, in arrival order) are blocks
 * doc_block[d] .. doc_block[d+1]-1.  Documents decode on `threads` threads; the rows do not
 * depend on the thread count.  A document with an undecodable block (the reference's
 * Block.unpack / JSON.parse throw) is reported HM_ERR_INVALID in hm_decoded_status with no
 * rows.  a_stride 0 = the batch's widest document.  Brotli uses the system libbrotlidec.
 */
typedef struct hm_decoded hm_decoded;
int hm_decode_blocks(const uint8_t *data, const uint64_t *block_off, const uint32_t *doc_block, uint32_t n_docs,
                     uint32_t a_stride, int threads, hm_decoded **out);
/* The decoded tables as a host hm_batch (pointers valid until hm_decoded_free). */
int hm_decoded_batch(const hm_decoded *d, hm_batch *out);
const int32_t *hm_decoded_status(const hm_decoded *d);            /* [n_docs] HM_OK / HM_ERR_INVALID */
uint32_t hm_decoded_n_strings(const hm_decoded *d);               /* the string pool (keys, string values) */
const char *hm_decoded_string(const hm_decoded *d, uint32_t i, size_t *len);
const char *hm_decoded_actor(const hm_decoded *d, uint32_t doc, uint32_t rank, size_t *len);
const char *hm_decoded_obj(const hm_decoded *d, uint32_t doc, uint32_t obj, size_t *len);       /* object uuid */
const char *hm_decoded_reg(const hm_decoded *d, uint32_t doc, uint32_t reg, uint32_t *obj, size_t *len); /* key | elemId */
void hm_decoded_free(hm_decoded *d);

/* ------------------------------------------------------------------ */
/* Docset: the Node drop-in's host engine (raw blocks in, patches out)  */
/* ------------------------------------------------------------------ */
/*
 * The documents of one device with everything the JS host used to keep per document: their
 * interners (actor ids ranked in JS string order, object UUIDs, registers, string values,
 * change content identity), their placement in resident stores (one hm_store per actor-stride
 * class 8/16/32/64; a document moves to a wider class when a new actor outgrows its rows) and
 * their patch base.  One hm_docset_apply = one applyChanges round of every listed document:
 *
 *   replaces: src/Actor.ts:137-141 parseBlock, src/Block.ts:18-29 unpack, src/JsonBuffer.ts:1-4
 *             src/DocBackend.ts:169-185 applyRemoteChanges -> Backend.applyChanges -> updateClock
 *             src/DocBackend.ts:144-167 init(changes) (the first call on a document)
 *             Automerge makePatch: {clock, deps, canUndo, canRedo, diffs}
 *
 * Input: the blocks of each document (one Change per block, '{"' JSON or 'BR' + brotli JSON),
 * laid out as in hm_decode_blocks; docs[i] is the docset document of doc_block[i]..[i+1]-1
 * (each at most once per call).  Output (hm_text): per document an hm_doc_result (status:
 * HM_ERR_INVALID with err_change = the block index in this call when a block does not decode
 * (the reference's Block.unpack / JSON.parse throw); an Automerge error status with err_change
 * = the log index (blocks of all successful calls, in order) when applyChanges throws; the
 * document is rolled back either way) and one JSON text
 *   {"p": [patch | null, ...], "b": [clock of the whole log | null, ...], "c": [clock of this call's changes | null, ...]}
 * patch.clock / deps are opSet.clock / opSet.deps; diffs take the document from the previous
 * successful call's patch to this one (objects created, map keys set / removed, list elements
 * removed / inserted / set) in the Automerge 0.12 diff vocabulary; "b" is the max seq per actor
 * over every change of the document's log and "c" over this call's changes (queued ones
 * included: DocBackend.updateClock(changes), src/DocBackend.ts:135-142).
 * Calls on one docset are serialised (a second concurrent call fails); hm_docset_open may run
 * while a call is in flight (it allocates host state only).
 */
typedef struct hm_docset hm_docset;
typedef struct hm_text hm_text;
typedef struct {
    uint32_t threads;     /* host threads for decode / render (0 = min(16, hardware)) */
    uint32_t flags;       /* HM_DOCSET_* */
} hm_docset_config;
#define HM_DOCSET_NO_PATCHES 1u   /* patches carry clock / deps only (no diffs, no register reads) */
#define HM_DOCSET_BINARY 2u       /* hm_docset_apply's text is the binary form below instead of JSON */
#define HM_DOCSET_NET_DIFFS 4u    /* diffs take the previous patch's document to the new one (one per changed
                                     register) instead of Automerge's per-op sequence (the default) */
/* Binary results ('HMP1', for a host that builds the patch objects itself instead of parsing
 * JSON; a call whose strings hold a lone surrogate falls back to the JSON form, first byte '{'):
 *   u32 header[8] = {0x31504D48, n_docs, n_strings, n_words, n_nums, blob_bytes, ascii, 0}
 *   u32 doc_word_off[n_docs + 1], doc_str_base[n_docs + 1], doc_num_base[n_docs + 1]
 *   u32 str_off[n_strings + 1] (byte offsets into blob), u32 words[n_words], pad to 8,
 *   f64 nums[n_nums], u8 blob[blob_bytes]
 * A document's words (string and number indices local to the document): opSet.clock, opSet.deps,
 * the log's clock, this call's clock, each as n then n x (actor string, seq); then n_diffs and
 * per diff a head word (action 0 create | 1 set | 2 remove | 3 insert, type << 3 with type 0 map
 * | 1 table | 2 list | 3 text) followed by: create: obj; map set: obj, key, entry; map remove:
 * obj, key; list remove: obj, index; list insert: obj, index, elemId, entry; list set: obj,
 * index, entry.  entry = n_surv, the winner's value word, then per conflict (actor string, value
 * word); value word = vtag | datatype << 3 | payload << 5 (STR / OBJ: string index, INT / FLOAT:
 * number index). */

int  hm_docset_create(hm_engine *e, const hm_docset_config *cfg, hm_docset **out);
void hm_docset_destroy(hm_docset *ds);
hm_engine *hm_docset_engine(hm_docset *ds);
/* n new, empty documents (Backend.init()) with consecutive ids from *out_first */
int  hm_docset_open(hm_docset *ds, uint32_t n, uint32_t *out_first);
int  hm_docset_apply(hm_docset *ds, const uint8_t *data, const uint64_t *block_off, const uint32_t *doc_block,
                     const uint32_t *docs, uint32_t n_docs, hm_text **out);
const char *hm_text_data(const hm_text *t, size_t *len);
const hm_doc_result *hm_text_results(const hm_text *t, uint32_t *n);
void hm_text_free(hm_text *t);

typedef struct {
    uint32_t a_stride;    /* class of the store the document lives in (0 = not placed yet) */
    uint32_t n_changes, n_ops, n_actors, n_objs, n_regs, hist_len, n_queued;
} hm_docset_doc_info_t;
int hm_docset_doc_info(hm_docset *ds, uint32_t doc, hm_docset_doc_info_t *out);
/* history.slice(0, n) (src/RepoBackend.ts:572-576): log indices in history order; returns the count */
int hm_docset_history_prefix(hm_docset *ds, uint32_t doc, uint32_t n, uint32_t *out_log_index);
/* ClockStore.update(self, docId, doc.clock) for n documents (hm_store_clock_update per class);
 * *out_stored (optional) = JSON array of the stored clocks, in call order */
int hm_docset_clock_update(hm_docset *ds, uint32_t n, const uint32_t *docs, uint8_t *out_written, uint8_t *out_differs,
                           hm_text **out_stored);
/* the merged document: {uuid: {"type", "keys": [[key, entry]], "elems": [[elemId, entry]]}} */
int hm_docset_view(hm_docset *ds, uint32_t doc, hm_text **out);
/* counters: calls, documents, class moves, net patches from the hit registers, net patches from every
 * register, per-op patches, per-op replays whose registers differ from the device's merged state
 * (always 0 unless the renderer and the kernels disagree) */
int hm_docset_stats(const hm_docset *ds, uint64_t *out8);
/* How the docset's stores merged its document rounds so far (hm_store_last_routing summed over
 * every submit): out3 = {incremental, re-merged, incremental handed back to the re-merge}. */
int hm_docset_routing(const hm_docset *ds, uint64_t *out3);
/* The store of class a_stride (8, 16, 32, 64, 128, 256): handles opened in it and handles
 * released (a document moved to a wider class; empty, reused before new ones are opened) */
int hm_docset_handles(const hm_docset *ds, uint32_t a_stride, uint32_t *out_opened, uint32_t *out_free);

/* ------------------------------------------------------------------ */
/* Clock exchange across the node's GPUs (RCCL over xGMI)              */
/* ------------------------------------------------------------------ */
/*
 * Documents shard by FNV-1a64(docId) % G; each GPU (engine) owns its documents' state and the
 * merge never communicates.  What crosses GPUs is the ClockStore feed: per-document clock
 * entries as repo-global records, the analogue of the `clocks` a CursorMessage carries
 * ({docId, clock: {actorId: seq}}, src/PeerMsg.ts:12-16, assembled from ClockStore at
 * src/RepoBackend.ts:374-392 and applied at :397-418).  Actor ranks are per-document and
 * encoder-local, so records name documents and actors by 64-bit keys (FNV-1a64 of the docId /
 * actorId strings; 0 = no actor); the host keeps the key -> string tables.
 *
 *   replaces: src/RepoBackend.ts:374-392 onDiscovery clocks = ClockStore.get per doc
 *             src/RepoBackend.ts:402,412-418 ClockStore.update(sender, doc, clock) + minimumClock
 *             src/Clock.ts:103-113 intersection (the min-clock across replicas)
 *
 * One process per GPU: rank 0 makes a unique id (hm_comm_unique_id), the host distributes it
 * (any channel), every rank calls hm_comm_create.  One thread driving several GPUs: create
 * (and later issue each collective on) every communicator between hm_comm_group_start/_end.
 */
#define HM_COMM_ID_BYTES 128
#define HM_CLOCK_NOT_HELD 0xFFFFFFFFu   /* min-allreduce identity: "this rank does not hold the doc" */

typedef struct {          /* 24 B */
    uint64_t doc_key;     /* FNV-1a64(docId) */
    uint64_t actor_key;   /* FNV-1a64(actorId) */
    uint32_t seq;         /* the clock entry (DocBackend.clock / ClockStore row) */
    uint32_t flags;       /* 0 (reserved) */
} hm_clock_rec;

typedef struct hm_comm hm_comm;
int  hm_comm_unique_id(uint8_t *out /* HM_COMM_ID_BYTES */);
int  hm_comm_create(hm_engine *e, int world, int rank, const uint8_t *unique_id, hm_comm **out);
void hm_comm_destroy(hm_comm *c);
int  hm_comm_group_start(void);
int  hm_comm_group_end(void);

/* Dense per-document clock rows (device: doc_keys[n_docs], actor_keys / clock / base
 * [n_docs*a_stride], base optional) -> records of every entry with actor_key != 0 and
 * clock > base (base NULL: > 0), document-major, rank order within a document.
 * *out_count (device u32) receives the count; `scratch` = hm_clock_records_scratch_bytes. */
size_t hm_clock_records_scratch_bytes(uint32_t n_docs, uint32_t a_stride);
int hm_clock_records_device(hm_engine *e, const uint64_t *doc_keys, const uint64_t *actor_keys,
                            const uint32_t *clock, const uint32_t *base, uint32_t n_docs, uint32_t a_stride,
                            hm_clock_rec *out, uint32_t *out_count, void *scratch, void *stream);

/* d_counts[world] (device u64) <- every rank's record count (all-gather; returns after it). */
int hm_clock_count_allgather(hm_comm *c, uint64_t n_local, uint64_t *d_counts, void *stream);
/* d_out <- every rank's records back to back in rank order; counts (host, [world]) from
 * hm_clock_count_allgather; d_out holds sum(counts) records.  Enqueued on `stream`. */
int hm_clock_allgather(hm_comm *c, const hm_clock_rec *d_recs, const uint64_t *counts, hm_clock_rec *d_out,
                       void *stream);
/* In place, elementwise MIN over every rank of rank-aligned seq rows (row = a (doc, actor) key
 * of the gathered key universe): a rank that holds the document contributes its entry (0 =
 * absent), one that does not HM_CLOCK_NOT_HELD.  After it, 0 and HM_CLOCK_NOT_HELD are absent
 * entries and the rest is Clock.intersection over the replicas holding the document. */
int hm_clock_min_allreduce(hm_comm *c, uint32_t *d_seq, uint64_t n, void *stream);

/* One process driving n GPUs (the Node host's GpuEngine, one engine per device): an n-rank
 * communicator over the engines, and host-buffer forms of the two collectives (staged
 * through each device; every engine's records / seq row is one rank's contribution).
 * hm_clock_exchange_host: out <- all records in rank order (*out_total of them, <= out_cap).
 * hm_clock_min_host: every seq[i] row (len entries) <- the MIN over the n rows. */
int hm_comm_create_local(hm_engine *const *engines, int n, hm_comm **out);
int hm_clock_exchange_host(hm_comm *const *comms, int n, const hm_clock_rec *const *recs, const uint64_t *n_recs,
                           hm_clock_rec *out, uint64_t out_cap, uint64_t *out_total);
int hm_clock_min_host(hm_comm *const *comms, int n, uint32_t *const *seq, uint64_t len);

#ifdef __cplusplus
}
#endif
#endif /* HYPERMERGE_AMD_H */
