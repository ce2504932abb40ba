/*
 * hmgpu_node.c — N-API addon: the Node face of the C-ABI in include/hypermerge_amd.h.
 *
 * Thin by design: every function unpacks Buffers / TypedArrays into the C-ABI's plain
 * pointers and sizes and throws a JS Error carrying hm_status_message() on failure
 * (no C++ and no exceptions cross the ABI).  GpuDocBackend.js (same directory) is the
 * only caller; it mirrors the reference's DocBackend API (src/DocBackend.ts:46-213).
 *
 * waitAsync: each store owns one host thread that runs hm_batch_wait for it; completion is
 * delivered to JS on the main thread through a napi_threadsafe_function (SURVEY.md §8b:
 * N-API calls only from the main thread, one engine host thread per GPU store), so the
 * event loop never blocks on the device.
 *
 * Build (hypermerge_amd/build.py):
 *   gcc -shared -fPIC -I/usr/include/node -Iinclude hmgpu_node.c -Lhypermerge_amd/_lib -lhmgpu
 *       -Wl,-rpath,'$ORIGIN' -o hypermerge_amd/_lib/hmgpu.node
 */
#define NAPI_VERSION 4
#include <node_api.h>
#include <pthread.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "hypermerge_amd.h"

#define CHECK_NAPI(call)                                          \
    do {                                                          \
        if ((call) != napi_ok) {                                  \
            napi_throw_error(env, NULL, "N-API call failed: " #call); \
            return NULL;                                          \
        }                                                         \
    } while (0)

static napi_value throw_status(napi_env env, hm_engine *e, int st, const char *what) {
    char msg[512];
    snprintf(msg, sizeof msg, "%s: %s%s%s", what, hm_status_message(st), e ? " — " : "", e ? hm_engine_last_error(e) : "");
    napi_throw_error(env, NULL, msg);
    return NULL;
}

typedef struct Job {
    struct Job *next;
    uint64_t id;
    uint32_t n, S;
    int st;
    char err[512];
    uint8_t *buf;                 /* results: docs | clock | backClock | heads */
    napi_threadsafe_function tsfn;
} Job;

typedef struct {
    hm_engine *engine;
    hm_store *store;
    uint32_t a_stride;
    uint32_t pending_n;   /* documents of the batch in flight (sizes Wait's buffers) */
    /* the store's host thread (waitAsync) */
    pthread_t thread;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    Job *head, *tail;
    int started, stop;
    int busy;             /* a waitAsync job is in flight: every other call on the store throws */
} Store;

static void *store_thread(void *arg) {
    Store *s = (Store *)arg;
    for (;;) {
        pthread_mutex_lock(&s->mu);
        while (!s->head && !s->stop) pthread_cond_wait(&s->cv, &s->mu);
        if (!s->head) { pthread_mutex_unlock(&s->mu); return NULL; }
        Job *j = s->head;
        s->head = j->next;
        if (!s->head) s->tail = NULL;
        pthread_mutex_unlock(&s->mu);
        const size_t rb = (size_t)j->n * sizeof(hm_doc_result), cb = (size_t)j->n * j->S * 4;
        j->buf = (uint8_t *)malloc(rb + 3 * cb + 16);
        j->st = j->buf ? hm_batch_wait(s->store, j->id, (hm_doc_result *)j->buf, (uint32_t *)(j->buf + rb),
                                       (uint32_t *)(j->buf + rb + cb), (uint32_t *)(j->buf + rb + 2 * cb))
                       : HM_ERR_NOMEM;
        if (j->st) snprintf(j->err, sizeof j->err, "hm_batch_wait: %s — %s", hm_status_message(j->st), hm_engine_last_error(s->engine));
        napi_call_threadsafe_function(j->tsfn, j, napi_tsfn_blocking);
        napi_release_threadsafe_function(j->tsfn, napi_tsfn_release);
    }
}

static void store_finalize(napi_env env, void *data, void *hint) {
    (void)env; (void)hint;
    Store *s = (Store *)data;
    if (s->started) {
        pthread_mutex_lock(&s->mu);
        s->stop = 1;
        pthread_cond_signal(&s->cv);
        pthread_mutex_unlock(&s->mu);
        pthread_join(s->thread, NULL);
        pthread_mutex_destroy(&s->mu);
        pthread_cond_destroy(&s->cv);
    }
    if (s->store) hm_store_destroy(s->store);
    if (s->engine) hm_engine_destroy(s->engine);
    free(s);
}

static int get_args(napi_env env, napi_callback_info info, size_t want, napi_value *argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < want) {
        napi_throw_type_error(env, NULL, "missing arguments");
        return 0;
    }
    return 1;
}

static Store *get_store_any(napi_env env, napi_value v) {
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, NULL, "expected a store handle");
        return NULL;
    }
    return (Store *)p;
}

/* the store for a call that touches its state: refused while an async wait runs on its host
 * thread (hm_batch_wait copies out and rolls back documents there) */
static Store *get_store(napi_env env, napi_value v) {
    Store *s = get_store_any(env, v);
    if (s && s->busy) {
        napi_throw_error(env, NULL, "store busy: a batch is in flight (wait for its waitAsync callback)");
        return NULL;
    }
    return s;
}

/* bytes of a Buffer / TypedArray / ArrayBuffer view; null/undefined -> NULL */
static int get_bytes(napi_env env, napi_value v, void **data, size_t *len) {
    napi_valuetype t;
    *data = NULL; *len = 0;
    if (napi_typeof(env, v, &t) != napi_ok) return 0;
    if (t == napi_null || t == napi_undefined) return 1;
    bool is;
    if (napi_is_buffer(env, v, &is) == napi_ok && is) return napi_get_buffer_info(env, v, data, len) == napi_ok;
    if (napi_is_typedarray(env, v, &is) == napi_ok && is) {
        napi_typedarray_type tt; size_t n, off; napi_value ab;
        if (napi_get_typedarray_info(env, v, &tt, &n, data, &ab, &off) != napi_ok) return 0;
        size_t el = 1;
        switch (tt) {
        case napi_int16_array: case napi_uint16_array: el = 2; break;
        case napi_int32_array: case napi_uint32_array: case napi_float32_array: el = 4; break;
        case napi_float64_array: el = 8; break;
        default: el = 1;
        }
        *len = n * el;
        return 1;
    }
    napi_throw_type_error(env, NULL, "expected a Buffer or TypedArray");
    return 0;
}

static uint32_t get_u32(napi_env env, napi_value v) {
    uint32_t x = 0;
    napi_get_value_uint32(env, v, &x);
    return x;
}

static napi_value buf_copy(napi_env env, const void *p, size_t n) {
    napi_value out; void *dst;
    if (napi_create_buffer_copy(env, n, n ? p : "", &dst, &out) != napi_ok) return NULL;
    return out;
}

static void set(napi_env env, napi_value obj, const char *k, napi_value v) { napi_set_named_property(env, obj, k, v); }
static napi_value u32v(napi_env env, uint32_t x) { napi_value v; napi_create_uint32(env, x, &v); return v; }
static napi_value i32v(napi_env env, int32_t x) { napi_value v; napi_create_int32(env, x, &v); return v; }

/* createStore(device, aStride) -> store */
static napi_value CreateStore(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Store *s = (Store *)calloc(1, sizeof(Store));
    hm_config cfg = {(int)get_u32(env, argv[0]), 0};
    int st = hm_engine_create(&cfg, &s->engine);
    if (st) { free(s); return throw_status(env, NULL, st, "hm_engine_create"); }
    hm_store_config sc = {get_u32(env, argv[1]), 0};
    st = hm_store_create(s->engine, &sc, &s->store);
    if (st) { napi_value r = throw_status(env, s->engine, st, "hm_store_create"); hm_engine_destroy(s->engine); free(s); return r; }
    s->a_stride = sc.a_stride;
    napi_value out;
    CHECK_NAPI(napi_create_external(env, s, store_finalize, NULL, &out));
    return out;
}

/* openDoc(store) -> handle */
static napi_value OpenDoc(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    uint32_t h;
    int st = hm_doc_open(s->store, &h);
    if (st) return throw_status(env, s->engine, st, "hm_doc_open");
    return u32v(env, h);
}

/* submit(store, docs, changes, deps, ops, handles, remap|null) -> batch id (number) */
static napi_value Submit(napi_env env, napi_callback_info info) {
    napi_value argv[7];
    if (!get_args(env, info, 7, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    void *p[6]; size_t n[6];
    for (int i = 0; i < 6; i++) if (!get_bytes(env, argv[1 + i], &p[i], &n[i])) return NULL;
    hm_batch b;
    memset(&b, 0, sizeof b);
    b.n_docs = (uint32_t)(n[0] / sizeof(hm_doc_row));
    b.n_changes = (uint32_t)(n[1] / sizeof(hm_change_row));
    b.n_deps = (uint32_t)(n[2] / sizeof(hm_dep_row));
    b.n_ops = (uint32_t)(n[3] / sizeof(hm_op_row));
    b.a_stride = s->a_stride;
    b.docs = (const hm_doc_row *)p[0]; b.changes = (const hm_change_row *)p[1];
    b.deps = (const hm_dep_row *)p[2]; b.ops = (const hm_op_row *)p[3];
    for (uint32_t i = 0; i < b.n_docs; i++) b.n_regs += b.docs[i].n_regs;
    if (n[4] / 4 != b.n_docs) { napi_throw_range_error(env, NULL, "handles length != documents"); return NULL; }
    if (p[5] && n[5] != (size_t)b.n_docs * s->a_stride) { napi_throw_range_error(env, NULL, "remap must be n_docs * aStride bytes"); return NULL; }
    uint64_t id = 0;
    int st = hm_batch_submit(s->store, &b, (const uint32_t *)p[4], (const uint8_t *)p[5], &id);
    if (st) return throw_status(env, s->engine, st, "hm_batch_submit");
    s->pending_n = b.n_docs;
    napi_value out;
    CHECK_NAPI(napi_create_double(env, (double)id, &out));
    return out;
}

/* wait(store, id[, nDocs]) -> {docs, clock, backClock, heads} (Buffers).  The buffers are
 * sized from the submitted batch's document count, never from the caller's nDocs. */
static napi_value Wait(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    double idd; napi_get_value_double(env, argv[1], &idd);
    const uint32_t n = s->pending_n, S = s->a_stride;
    size_t rb = (size_t)n * sizeof(hm_doc_result), cb = (size_t)n * S * 4;
    uint8_t *buf = (uint8_t *)malloc(rb + 3 * cb + 16);
    int st = hm_batch_wait(s->store, (uint64_t)idd, (hm_doc_result *)buf, (uint32_t *)(buf + rb),
                           (uint32_t *)(buf + rb + cb), (uint32_t *)(buf + rb + 2 * cb));
    if (st) { free(buf); return throw_status(env, s->engine, st, "hm_batch_wait"); }
    napi_value o;
    napi_create_object(env, &o);
    set(env, o, "docs", buf_copy(env, buf, rb));
    set(env, o, "clock", buf_copy(env, buf + rb, cb));
    set(env, o, "backClock", buf_copy(env, buf + rb + cb, cb));
    set(env, o, "heads", buf_copy(env, buf + rb + 2 * cb, cb));
    free(buf);
    return o;
}

static napi_value result_object(napi_env env, const uint8_t *buf, uint32_t n, uint32_t S) {
    const size_t rb = (size_t)n * sizeof(hm_doc_result), cb = (size_t)n * S * 4;
    napi_value o;
    napi_create_object(env, &o);
    set(env, o, "docs", buf_copy(env, buf, rb));
    set(env, o, "clock", buf_copy(env, buf + rb, cb));
    set(env, o, "backClock", buf_copy(env, buf + rb + cb, cb));
    set(env, o, "heads", buf_copy(env, buf + rb + 2 * cb, cb));
    return o;
}

/* main thread: callback(err, result) for a finished job */
static void job_call_js(napi_env env, napi_value cb, void *context, void *data) {
    Job *j = (Job *)data;
    if (context) ((Store *)context)->busy = 0;
    if (env && cb) {
        napi_value argv[2], undef, ret;
        napi_get_undefined(env, &undef);
        if (j->st) {
            napi_value msg;
            napi_create_string_utf8(env, j->err, NAPI_AUTO_LENGTH, &msg);
            napi_create_error(env, NULL, msg, &argv[0]);
            argv[1] = undef;
        } else {
            napi_get_null(env, &argv[0]);
            argv[1] = result_object(env, j->buf, j->n, j->S);
        }
        napi_call_function(env, undef, cb, 2, argv, &ret);
    }
    free(j->buf);
    free(j);
}

/* waitAsync(store, id, callback(err, {docs, clock, backClock, heads})): hm_batch_wait on the
 * store's host thread; no other call on the store until the callback runs */
static napi_value WaitAsync(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    double idd;
    napi_get_value_double(env, argv[1], &idd);
    Job *j = (Job *)calloc(1, sizeof(Job));
    if (!j) { napi_throw_error(env, NULL, "out of memory"); return NULL; }
    j->id = (uint64_t)idd; j->n = s->pending_n; j->S = s->a_stride;
    napi_value name;
    napi_create_string_utf8(env, "hmgpu.waitAsync", NAPI_AUTO_LENGTH, &name);
    if (napi_create_threadsafe_function(env, argv[2], NULL, name, 0, 1, NULL, NULL, s, job_call_js, &j->tsfn) != napi_ok) {
        free(j);
        napi_throw_error(env, NULL, "napi_create_threadsafe_function failed");
        return NULL;
    }
    if (!s->started) {
        pthread_mutex_init(&s->mu, NULL);
        pthread_cond_init(&s->cv, NULL);
        if (pthread_create(&s->thread, NULL, store_thread, s) != 0) {
            napi_release_threadsafe_function(j->tsfn, napi_tsfn_abort);
            free(j);
            napi_throw_error(env, NULL, "pthread_create failed");
            return NULL;
        }
        s->started = 1;
    }
    s->busy = 1;
    pthread_mutex_lock(&s->mu);
    if (s->tail) s->tail->next = j; else s->head = j;
    s->tail = j;
    pthread_cond_signal(&s->cv);
    pthread_mutex_unlock(&s->mu);
    return NULL;
}

/* readRegs(store, docs Uint32Array, regs Uint32Array, survCap) -> {regs, surv} (Buffers): the
 * rows of the chosen registers, surv_off rewritten to offsets into `surv` */
static napi_value ReadRegs(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    void *pd, *pr; size_t nd, nr;
    if (!get_bytes(env, argv[1], &pd, &nd) || !get_bytes(env, argv[2], &pr, &nr)) return NULL;
    if (nd != nr) { napi_throw_range_error(env, NULL, "docs and regs differ in length"); return NULL; }
    const uint32_t n = (uint32_t)(nd / 4), cap = get_u32(env, argv[3]);
    hm_reg_result *rr = (hm_reg_result *)malloc((size_t)n * sizeof(hm_reg_result) + 16);
    hm_surv_result *sv = (hm_surv_result *)malloc((size_t)cap * sizeof(hm_surv_result) + 16);
    uint32_t got = 0;
    int st = (rr && sv) ? hm_store_read_regs(s->store, n, (const uint32_t *)pd, (const uint32_t *)pr, rr, sv, cap, &got)
                        : HM_ERR_NOMEM;
    napi_value o = NULL;
    if (!st) {
        napi_create_object(env, &o);
        set(env, o, "regs", buf_copy(env, rr, (size_t)n * sizeof(hm_reg_result)));
        set(env, o, "surv", buf_copy(env, sv, (size_t)got * sizeof(hm_surv_result)));
    }
    free(rr); free(sv);
    if (st) return throw_status(env, s->engine, st, "hm_store_read_regs");
    return o;
}

/* info(store, h) -> {nChanges, ..., status} */
static napi_value Info(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    hm_doc_info_t d;
    int st = hm_doc_info(s->store, get_u32(env, argv[1]), &d);
    if (st) return throw_status(env, s->engine, st, "hm_doc_info");
    napi_value o;
    napi_create_object(env, &o);
    set(env, o, "nChanges", u32v(env, d.n_changes)); set(env, o, "nDeps", u32v(env, d.n_deps));
    set(env, o, "nOps", u32v(env, d.n_ops)); set(env, o, "nRegs", u32v(env, d.n_regs));
    set(env, o, "nObjs", u32v(env, d.n_objs)); set(env, o, "nActors", u32v(env, d.n_actors));
    set(env, o, "histLen", u32v(env, d.hist_len)); set(env, o, "nQueued", u32v(env, d.n_queued));
    set(env, o, "nSurv", u32v(env, d.n_surv)); set(env, o, "status", i32v(env, d.status));
    return o;
}

/* read(store, h) -> {hist, allDeps, regs, surv, clock, backClock, heads} (Buffers) */
static napi_value Read(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    const uint32_t h = get_u32(env, argv[1]), S = s->a_stride;
    hm_doc_info_t d;
    int st = hm_doc_info(s->store, h, &d);
    if (st) return throw_status(env, s->engine, st, "hm_doc_info");
    size_t sz[7] = {(size_t)d.n_changes * 4, (size_t)d.n_changes * S * 4, (size_t)d.n_regs * sizeof(hm_reg_result),
                    (size_t)d.n_ops * sizeof(hm_surv_result), S * 4, S * 4, S * 4};
    void *p[7];
    for (int i = 0; i < 7; i++) p[i] = calloc(1, sz[i] + 8);
    st = hm_doc_read(s->store, h, (int32_t *)p[0], (uint32_t *)p[1], (hm_reg_result *)p[2], (hm_surv_result *)p[3],
                     (uint32_t *)p[4], (uint32_t *)p[5], (uint32_t *)p[6]);
    napi_value o = NULL;
    if (!st) {
        static const char *names[7] = {"hist", "allDeps", "regs", "surv", "clock", "backClock", "heads"};
        napi_create_object(env, &o);
        for (int i = 0; i < 7; i++) set(env, o, names[i], buf_copy(env, p[i], sz[i]));
    }
    for (int i = 0; i < 7; i++) free(p[i]);
    if (st) return throw_status(env, s->engine, st, "hm_doc_read");
    return o;
}

/* historyPrefix(store, h, n) -> Buffer of u32 log indices */
static napi_value HistoryPrefix(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    const uint32_t n = get_u32(env, argv[2]);
    uint32_t *out = (uint32_t *)malloc((size_t)n * 4 + 4);
    int k = hm_doc_history_prefix(s->store, get_u32(env, argv[1]), n, out);
    if (k < 0) { free(out); return throw_status(env, s->engine, k, "hm_doc_history_prefix"); }
    napi_value r = buf_copy(env, out, (size_t)k * 4);
    free(out);
    return r;
}

/* setMinClock(store, h, Uint32Array[aStride]) */
static napi_value SetMinClock(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    void *p; size_t n;
    if (!get_bytes(env, argv[2], &p, &n)) return NULL;
    if (n != (size_t)s->a_stride * 4) { napi_throw_range_error(env, NULL, "clock row must be aStride u32"); return NULL; }
    int st = hm_doc_set_min_clock(s->store, get_u32(env, argv[1]), (const uint32_t *)p);
    if (st) return throw_status(env, s->engine, st, "hm_doc_set_min_clock");
    return NULL;
}

/* clockUpdate(store, Uint32Array handles) -> {written, differs, stored} */
static napi_value ClockUpdate(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Store *s = get_store(env, argv[0]);
    if (!s) return NULL;
    void *p; size_t n;
    if (!get_bytes(env, argv[1], &p, &n)) return NULL;
    const uint32_t k = (uint32_t)(n / 4), S = s->a_stride;
    uint8_t *w = (uint8_t *)calloc(1, k + 8), *df = (uint8_t *)calloc(1, k + 8);
    uint32_t *stv = (uint32_t *)calloc(1, (size_t)k * S * 4 + 8);
    int st = hm_store_clock_update(s->store, k, (const uint32_t *)p, w, df, stv);
    napi_value o = NULL;
    if (!st) {
        napi_create_object(env, &o);
        set(env, o, "written", buf_copy(env, w, k));
        set(env, o, "differs", buf_copy(env, df, k));
        set(env, o, "stored", buf_copy(env, stv, (size_t)k * S * 4));
    }
    free(w); free(df); free(stv);
    if (st) return throw_status(env, s->engine, st, "hm_store_clock_update");
    return o;
}

/* ---- clock exchange across the devices of one process (include/hypermerge_amd.h) ---- */
typedef struct { int n; hm_comm *comms[64]; } Comms;

static void comms_finalize(napi_env env, void *data, void *hint) {
    (void)env; (void)hint;
    Comms *c = (Comms *)data;
    for (int i = 0; i < c->n; i++) hm_comm_destroy(c->comms[i]);
    free(c);
}

/* commCreateLocal([store per device]) -> comm: one rank per store's engine (distinct GPUs) */
static napi_value CommCreateLocal(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    uint32_t n = 0;
    if (napi_get_array_length(env, argv[0], &n) != napi_ok || n < 1 || n > 64) {
        napi_throw_range_error(env, NULL, "expected 1..64 stores");
        return NULL;
    }
    hm_engine *engines[64];
    for (uint32_t i = 0; i < n; i++) {
        napi_value v;
        CHECK_NAPI(napi_get_element(env, argv[0], i, &v));
        Store *s = get_store(env, v);
        if (!s) return NULL;
        engines[i] = s->engine;
    }
    Comms *c = (Comms *)calloc(1, sizeof(Comms));
    c->n = (int)n;
    int st = hm_comm_create_local(engines, (int)n, c->comms);
    if (st) { free(c); return throw_status(env, engines[0], st, "hm_comm_create_local"); }
    napi_value out;
    CHECK_NAPI(napi_create_external(env, c, comms_finalize, NULL, &out));
    return out;
}

static Comms *get_comms(napi_env env, napi_value v) {
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) { napi_throw_type_error(env, NULL, "expected a comm handle"); return NULL; }
    return (Comms *)p;
}

/* clockExchange(comm, [Buffer of 24 B hm_clock_rec per rank]) -> Buffer: every rank's
 * records in rank order (hm_clock_exchange_host: RCCL over the devices) */
static napi_value ClockExchange(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Comms *c = get_comms(env, argv[0]);
    if (!c) return NULL;
    const hm_clock_rec *recs[64];
    uint64_t n[64], total = 0;
    for (int i = 0; i < c->n; i++) {
        napi_value v; void *p; size_t len;
        CHECK_NAPI(napi_get_element(env, argv[1], (uint32_t)i, &v));
        if (!get_bytes(env, v, &p, &len)) return NULL;
        recs[i] = (const hm_clock_rec *)p; n[i] = len / sizeof(hm_clock_rec); total += n[i];
    }
    hm_clock_rec *out = (hm_clock_rec *)malloc((total + 1) * sizeof(hm_clock_rec));
    uint64_t got = 0;
    int st = hm_clock_exchange_host(c->comms, c->n, recs, n, out, total, &got);
    if (st) { free(out); return throw_status(env, NULL, st, "hm_clock_exchange_host"); }
    napi_value r = buf_copy(env, out, got * sizeof(hm_clock_rec));
    free(out);
    return r;
}

/* clockMin(comm, [Uint32Array per rank, equal lengths]): every row <- the MIN over the rows
 * (hm_clock_min_host) */
static napi_value ClockMin(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Comms *c = get_comms(env, argv[0]);
    if (!c) return NULL;
    uint32_t *rows[64];
    size_t len0 = 0;
    for (int i = 0; i < c->n; i++) {
        napi_value v; void *p; size_t len;
        CHECK_NAPI(napi_get_element(env, argv[1], (uint32_t)i, &v));
        if (!get_bytes(env, v, &p, &len)) return NULL;
        if (i && len != len0) { napi_throw_range_error(env, NULL, "rows differ in length"); return NULL; }
        rows[i] = (uint32_t *)p; len0 = len;
    }
    int st = hm_clock_min_host(c->comms, c->n, rows, len0 / 4);
    if (st) return throw_status(env, NULL, st, "hm_clock_min_host");
    return NULL;
}

static napi_value StatusMessage(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    int32_t c = 0;
    napi_get_value_int32(env, argv[0], &c);
    napi_value out;
    napi_create_string_utf8(env, hm_status_message(c), NAPI_AUTO_LENGTH, &out);
    return out;
}

/* ---------------- docset: raw blocks in, results + patches out (hm_docset_*) ---------------- */
typedef struct DsJob {
    struct DsJob *next;
    uint8_t *data;
    napi_ref data_ref;                  /* packed calls: data is the caller's Buffer, held by this reference */
    int borrowed;                       /* synchronous packed calls: data is the caller's Buffer, read before returning */
    uint64_t *bo;
    uint32_t *db, *ids, n;
    int st;
    char err[512];
    hm_text *out;
    napi_threadsafe_function tsfn;
} DsJob;

typedef struct {
    hm_engine *engine;
    hm_docset *ds;
    pthread_t thread;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    DsJob *head, *tail;
    int started, stop, busy;
} Docset;

/* env NULL (the environment is going away): a held Buffer reference is left to it */
static void ds_job_free(napi_env env, DsJob *j) {
    if (!j) return;
    if (j->data_ref) { if (env) napi_delete_reference(env, j->data_ref); }
    else if (!j->borrowed) free(j->data);
    free(j->bo); free(j->db); free(j->ids);
    if (j->out) hm_text_free(j->out);
    free(j);
}

static void *docset_thread(void *arg) {
    Docset *d = (Docset *)arg;
    for (;;) {
        pthread_mutex_lock(&d->mu);
        while (!d->head && !d->stop) pthread_cond_wait(&d->cv, &d->mu);
        if (!d->head) { pthread_mutex_unlock(&d->mu); return NULL; }
        DsJob *j = d->head;
        d->head = j->next;
        if (!d->head) d->tail = NULL;
        pthread_mutex_unlock(&d->mu);
        j->st = hm_docset_apply(d->ds, j->data, j->bo, j->db, j->ids, j->n, &j->out);
        if (j->st) snprintf(j->err, sizeof j->err, "hm_docset_apply: %s — %s", hm_status_message(j->st), hm_engine_last_error(d->engine));
        napi_call_threadsafe_function(j->tsfn, j, napi_tsfn_blocking);
        napi_release_threadsafe_function(j->tsfn, napi_tsfn_release);
    }
}

static void docset_finalize(napi_env env, void *data, void *hint) {
    (void)env; (void)hint;
    Docset *d = (Docset *)data;
    if (d->started) {
        pthread_mutex_lock(&d->mu);
        d->stop = 1;
        pthread_cond_signal(&d->cv);
        pthread_mutex_unlock(&d->mu);
        pthread_join(d->thread, NULL);
        pthread_mutex_destroy(&d->mu);
        pthread_cond_destroy(&d->cv);
    }
    if (d->ds) hm_docset_destroy(d->ds);
    if (d->engine) hm_engine_destroy(d->engine);
    free(d);
}

static Docset *get_docset_any(napi_env env, napi_value v) {
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) { napi_throw_type_error(env, NULL, "expected a docset handle"); return NULL; }
    return (Docset *)p;
}

static Docset *get_docset(napi_env env, napi_value v) {
    Docset *d = get_docset_any(env, v);
    if (d && d->busy) { napi_throw_error(env, NULL, "docset busy: an applyAsync round is in flight"); return NULL; }
    return d;
}

/* docsetCreate(device, threads, patches[, binary]) -> docset (binary: results in the HMP1 form) */
static napi_value DocsetCreate(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    size_t argc = 5;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 3) {
        napi_throw_type_error(env, NULL, "missing arguments");
        return NULL;
    }
    bool binary = false, net = false;
    if (argc >= 4) napi_get_value_bool(env, argv[3], &binary);
    if (argc >= 5) napi_get_value_bool(env, argv[4], &net);
    Docset *d = (Docset *)calloc(1, sizeof(Docset));
    hm_config cfg = {(int)get_u32(env, argv[0]), 0};
    int st = hm_engine_create(&cfg, &d->engine);
    if (st) { free(d); return throw_status(env, NULL, st, "hm_engine_create"); }
    bool patches = true;
    napi_get_value_bool(env, argv[2], &patches);
    hm_docset_config dc = {get_u32(env, argv[1]), (patches ? 0u : HM_DOCSET_NO_PATCHES) | (binary ? HM_DOCSET_BINARY : 0u) |
                                              (net ? HM_DOCSET_NET_DIFFS : 0u)};
    st = hm_docset_create(d->engine, &dc, &d->ds);
    if (st) { napi_value r = throw_status(env, d->engine, st, "hm_docset_create"); hm_engine_destroy(d->engine); free(d); return r; }
    napi_value out;
    CHECK_NAPI(napi_create_external(env, d, docset_finalize, NULL, &out));
    return out;
}

/* docsetOpen(docset, n) -> first document id (allowed while a round is in flight) */
static napi_value DocsetOpen(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Docset *d = get_docset_any(env, argv[0]);
    if (!d) return NULL;
    uint32_t first = 0;
    int st = hm_docset_open(d->ds, get_u32(env, argv[1]), &first);
    if (st) return throw_status(env, d->engine, st, "hm_docset_open");
    return u32v(env, first);
}

/* the blocks of every document of a call (Array of Arrays of Buffer | string) -> one
 * contiguous copy + offsets owned by the job (the JS values need not outlive the call) */
static int gather_blocks(napi_env env, napi_value ids_v, napi_value blocks_v, DsJob *j) {
    void *ip; size_t il;
    if (!get_bytes(env, ids_v, &ip, &il)) return 0;
    uint32_t n = (uint32_t)(il / 4), nd = 0;
    if (napi_get_array_length(env, blocks_v, &nd) != napi_ok || nd != n) {
        napi_throw_range_error(env, NULL, "blocks must be an array with one array of blocks per document");
        return 0;
    }
    j->n = n;
    j->ids = (uint32_t *)malloc((size_t)n * 4 + 4);
    j->db = (uint32_t *)malloc(((size_t)n + 1) * 4);
    memcpy(j->ids, ip, (size_t)n * 4);
    size_t cap_b = 1024, nb = 0, cap = 1 << 16, used = 0;
    j->bo = (uint64_t *)malloc(cap_b * 8);
    j->data = (uint8_t *)malloc(cap);
    j->bo[0] = 0;
    for (uint32_t i = 0; i < n; i++) {
        j->db[i] = (uint32_t)nb;
        napi_value arr;
        uint32_t k = 0;
        if (napi_get_element(env, blocks_v, i, &arr) != napi_ok || napi_get_array_length(env, arr, &k) != napi_ok) {
            napi_throw_type_error(env, NULL, "each document's blocks must be an array");
            return 0;
        }
        for (uint32_t b = 0; b < k; b++) {
            napi_value v;
            napi_get_element(env, arr, b, &v);
            napi_valuetype t;
            napi_typeof(env, v, &t);
            size_t len = 0;
            void *src = NULL;
            if (t == napi_string) napi_get_value_string_utf8(env, v, NULL, 0, &len);
            else if (!get_bytes(env, v, &src, &len)) return 0;
            if (used + len + 1 > cap) {
                while (used + len + 1 > cap) cap *= 2;
                j->data = (uint8_t *)realloc(j->data, cap);
            }
            if (t == napi_string) { size_t w = 0; napi_get_value_string_utf8(env, v, (char *)j->data + used, len + 1, &w); len = w; }
            else if (len) memcpy(j->data + used, src, len);
            used += len;
            if (nb + 2 > cap_b) { cap_b *= 2; j->bo = (uint64_t *)realloc(j->bo, cap_b * 8); }
            j->bo[++nb] = used;
        }
    }
    j->db[n] = (uint32_t)nb;
    return 1;
}

/* the packed form: ids (Uint32Array n), data (one Buffer of every block back to back),
 * ends (Uint32Array: end offset of each block), docBlock (Uint32Array n + 1: first block of each
 * document) — one copy, no per-block N-API calls (1.3M blocks per 20k-document round cost the
 * main thread ~1 s through napi_get_element / typeof / buffer info) */
/* mode 0: copy `data`; 1: hold it by a reference and read it in place (async); 2: read it in
 * place (synchronous: the call is done before JS runs again) */
static int gather_packed(napi_env env, napi_value ids_v, napi_value data_v, napi_value ends_v, napi_value db_v, int mode,
                         DsJob *j) {
    void *ip, *dp, *ep, *bp; size_t il, dl, el, bl;
    if (!get_bytes(env, ids_v, &ip, &il) || !get_bytes(env, data_v, &dp, &dl) || !get_bytes(env, ends_v, &ep, &el) ||
        !get_bytes(env, db_v, &bp, &bl))
        return 0;
    const uint32_t n = (uint32_t)(il / 4), nb = (uint32_t)(el / 4);
    const uint32_t *ends = (const uint32_t *)ep, *db = (const uint32_t *)bp;
    if (bl / 4 != (size_t)n + 1 || db[0] != 0 || db[n] != nb) {
        napi_throw_range_error(env, NULL, "docBlock must hold n + 1 ascending block indices ending at the block count");
        return 0;
    }
    for (uint32_t i = 0; i < n; i++)
        if (db[i] > db[i + 1]) { napi_throw_range_error(env, NULL, "docBlock not ascending"); return 0; }
    for (uint32_t b = 0; b < nb; b++)
        if (ends[b] > dl || (b && ends[b] < ends[b - 1])) { napi_throw_range_error(env, NULL, "block ends outside the data"); return 0; }
    j->n = n;
    j->ids = (uint32_t *)malloc((size_t)n * 4 + 4);
    j->db = (uint32_t *)malloc(((size_t)n + 1) * 4);
    j->bo = (uint64_t *)malloc(((size_t)nb + 1) * 8);
    memcpy(j->ids, ip, (size_t)n * 4);
    memcpy(j->db, db, ((size_t)n + 1) * 4);
    j->bo[0] = 0;
    for (uint32_t b = 0; b < nb; b++) j->bo[b + 1] = ends[b];
    /* copied by default; in place only when the caller promises the Buffer is its own and is
     * neither written nor transferred until the call has called back (GpuEngine.prepare builds
     * it for this call and never touches it again) — the Buffer is then held by a reference */
    if (mode == 2) { j->borrowed = 1; j->data = (uint8_t *)dp; }
    else if (mode == 1 && dl && napi_create_reference(env, data_v, 1, &j->data_ref) == napi_ok) j->data = (uint8_t *)dp;
    else {
        j->data_ref = NULL;
        j->data = (uint8_t *)malloc(dl + 1);
        if (dl) memcpy(j->data, dp, dl);
    }
    return 1;
}

static void text_finalize(napi_env env, void *data, void *hint) { (void)env; (void)data; hm_text_free((hm_text *)hint); }

/* {results, data}: results copied, data handed over without a copy (an external Buffer over the
 * hm_text, freed when the Buffer is collected; *tp is then NULL) */
static napi_value text_object(napi_env env, hm_text **tp) {
    hm_text *t = *tp;
    size_t len = 0;
    const char *p = hm_text_data(t, &len);
    uint32_t n = 0;
    const hm_doc_result *r = hm_text_results(t, &n);
    napi_value o, dv;
    napi_create_object(env, &o);
    set(env, o, "results", buf_copy(env, r, (size_t)n * sizeof(hm_doc_result)));
    if (len && napi_create_external_buffer(env, len, (void *)p, text_finalize, t, &dv) == napi_ok) *tp = NULL;
    else dv = buf_copy(env, p, len);
    set(env, o, "data", dv);
    return o;
}

static void ds_call_js(napi_env env, napi_value cb, void *context, void *data) {
    DsJob *j = (DsJob *)data;
    if (context) ((Docset *)context)->busy--;
    if (env && cb) {
        napi_value argv[2], undef, ret;
        napi_get_undefined(env, &undef);
        if (j->st) {
            napi_value msg;
            napi_create_string_utf8(env, j->err, NAPI_AUTO_LENGTH, &msg);
            napi_create_error(env, NULL, msg, &argv[0]);
            argv[1] = undef;
        } else {
            napi_get_null(env, &argv[0]);
            argv[1] = text_object(env, &j->out);
        }
        napi_call_function(env, undef, cb, 2, argv, &ret);
    }
    ds_job_free(env, j);
}

/* docsetApply(docset, ids Uint32Array, blocks[][], callback?) -> {results, data} | undefined
 * (data: the JSON text, or the HMP1 binary form when the docset was created binary):
 * one applyChanges round of every listed document (hm_docset_apply); with a callback the
 * round runs on the docset's host thread and callback(err, {results, data}) runs on the main
 * thread when it is done; further async calls queue behind it (run in call order), any other
 * docset call except docsetOpen throws until every queued round has called back */
static napi_value docset_apply(napi_env env, napi_callback_info info, int packed) {
    napi_value argv[7];
    size_t argc = 7;
    const size_t need = packed ? 5 : 3;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < need) {
        napi_throw_type_error(env, NULL, "missing arguments");
        return NULL;
    }
    napi_value cbv = argv[need];
    napi_valuetype cbt = napi_undefined;
    if (argc > need) napi_typeof(env, cbv, &cbt);
    /* async calls queue behind the ones in flight (the host thread runs them in order); a
     * synchronous call needs the docset idle */
    Docset *d = cbt == napi_function ? get_docset_any(env, argv[0]) : get_docset(env, argv[0]);
    if (!d) return NULL;
    DsJob *j = (DsJob *)calloc(1, sizeof(DsJob));
    bool in_place = false;
    if (packed && argc > need + 1) napi_get_value_bool(env, argv[need + 1], &in_place);
    if (!(packed ? gather_packed(env, argv[1], argv[2], argv[3], argv[4], cbt != napi_function ? 2 : in_place ? 1 : 0, j)
                 : gather_blocks(env, argv[1], argv[2], j))) {
        ds_job_free(env, j);
        return NULL;
    }
    if (cbt != napi_function) {
        int st = hm_docset_apply(d->ds, j->data, j->bo, j->db, j->ids, j->n, &j->out);
        if (st) { ds_job_free(env, j); return throw_status(env, d->engine, st, "hm_docset_apply"); }
        napi_value o = text_object(env, &j->out);
        ds_job_free(env, j);
        return o;
    }
    napi_value name;
    napi_create_string_utf8(env, "hmgpu.docsetApply", NAPI_AUTO_LENGTH, &name);
    if (napi_create_threadsafe_function(env, cbv, NULL, name, 0, 1, NULL, NULL, d, ds_call_js, &j->tsfn) != napi_ok) {
        ds_job_free(env, j);
        napi_throw_error(env, NULL, "napi_create_threadsafe_function failed");
        return NULL;
    }
    if (!d->started) {
        pthread_mutex_init(&d->mu, NULL);
        pthread_cond_init(&d->cv, NULL);
        if (pthread_create(&d->thread, NULL, docset_thread, d) != 0) {
            napi_release_threadsafe_function(j->tsfn, napi_tsfn_abort);
            ds_job_free(env, j);
            napi_throw_error(env, NULL, "pthread_create failed");
            return NULL;
        }
        d->started = 1;
    }
    d->busy++;
    pthread_mutex_lock(&d->mu);
    if (d->tail) d->tail->next = j; else d->head = j;
    d->tail = j;
    pthread_cond_signal(&d->cv);
    pthread_mutex_unlock(&d->mu);
    return NULL;
}

static napi_value DocsetApply(napi_env env, napi_callback_info info) { return docset_apply(env, info, 0); }
/* docsetApplyPacked(docset, ids, data, blockEnds, docBlock, callback?, inPlace?): docsetApply
 * with the blocks packed by the caller (gather_packed).  A synchronous call reads `data` in
 * place; an async call copies it unless inPlace is true: then the caller must neither write nor
 * transfer it until the callback has run */
static napi_value DocsetApplyPacked(napi_env env, napi_callback_info info) { return docset_apply(env, info, 1); }

/* docsetHistoryPrefix(docset, doc, n) -> Buffer of u32 log indices (history order) */
static napi_value DocsetHistoryPrefix(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    Docset *d = get_docset(env, argv[0]);
    if (!d) return NULL;
    const uint32_t n = get_u32(env, argv[2]);
    uint32_t *out = (uint32_t *)malloc((size_t)n * 4 + 4);
    int k = hm_docset_history_prefix(d->ds, get_u32(env, argv[1]), n, out);
    if (k < 0) { free(out); return throw_status(env, d->engine, -k, "hm_docset_history_prefix"); }
    napi_value r = buf_copy(env, out, (size_t)k * 4);
    free(out);
    return r;
}

/* docsetClockUpdate(docset, ids Uint32Array) -> {written, differs, json} */
static napi_value DocsetClockUpdate(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Docset *d = get_docset(env, argv[0]);
    if (!d) return NULL;
    void *p; size_t n;
    if (!get_bytes(env, argv[1], &p, &n)) return NULL;
    const uint32_t k = (uint32_t)(n / 4);
    uint8_t *w = (uint8_t *)calloc(1, k + 8), *df = (uint8_t *)calloc(1, k + 8);
    hm_text *t = NULL;
    int st = hm_docset_clock_update(d->ds, k, (const uint32_t *)p, w, df, &t);
    napi_value o = NULL;
    if (!st) {
        size_t len = 0;
        const char *s = hm_text_data(t, &len);
        napi_value js;
        napi_create_object(env, &o);
        set(env, o, "written", buf_copy(env, w, k));
        set(env, o, "differs", buf_copy(env, df, k));
        napi_create_string_utf8(env, s, len, &js);
        set(env, o, "json", js);
    }
    free(w); free(df);
    if (t) hm_text_free(t);
    if (st) return throw_status(env, d->engine, st, "hm_docset_clock_update");
    return o;
}

/* docsetView(docset, doc) -> JSON text of the merged document */
static napi_value DocsetView(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Docset *d = get_docset(env, argv[0]);
    if (!d) return NULL;
    hm_text *t = NULL;
    int st = hm_docset_view(d->ds, get_u32(env, argv[1]), &t);
    if (st) return throw_status(env, d->engine, st, "hm_docset_view");
    size_t len = 0;
    const char *s = hm_text_data(t, &len);
    napi_value js;
    napi_create_string_utf8(env, s, len, &js);
    hm_text_free(t);
    return js;
}

/* docsetInfo(docset, doc) -> {aStride, nChanges, nOps, nActors, nObjs, nRegs, histLen, nQueued} */
static napi_value DocsetInfo(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Docset *d = get_docset(env, argv[0]);
    if (!d) return NULL;
    hm_docset_doc_info_t x;
    int st = hm_docset_doc_info(d->ds, get_u32(env, argv[1]), &x);
    if (st) return throw_status(env, d->engine, st, "hm_docset_doc_info");
    napi_value o;
    napi_create_object(env, &o);
    set(env, o, "aStride", u32v(env, x.a_stride)); set(env, o, "nChanges", u32v(env, x.n_changes));
    set(env, o, "nOps", u32v(env, x.n_ops)); set(env, o, "nActors", u32v(env, x.n_actors));
    set(env, o, "nObjs", u32v(env, x.n_objs)); set(env, o, "nRegs", u32v(env, x.n_regs));
    set(env, o, "histLen", u32v(env, x.hist_len)); set(env, o, "nQueued", u32v(env, x.n_queued));
    return o;
}

/* docsetStats(docset) -> {calls, docs, moves, hitPatches, fullPatches, opPatches, replayMismatch, incremental,
 * remerged, handedBack} (the last three: document rounds by store route, hm_docset_routing) */
static napi_value DocsetStats(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    Docset *d = get_docset_any(env, argv[0]);
    if (!d) return NULL;
    uint64_t x[8];
    hm_docset_stats(d->ds, x);
    napi_value o;
    napi_create_object(env, &o);
    const char *names[7] = {"calls", "docs", "moves", "hitPatches", "fullPatches", "opPatches", "replayMismatch"};
    for (int i = 0; i < 7; i++) { napi_value v; napi_create_double(env, (double)x[i], &v); set(env, o, names[i], v); }
    uint64_t r3[3] = {0, 0, 0};
    hm_docset_routing(d->ds, r3);
    const char *rn[3] = {"incremental", "remerged", "handedBack"};
    for (int i = 0; i < 3; i++) { napi_value v; napi_create_double(env, (double)r3[i], &v); set(env, o, rn[i], v); }
    return o;
}

/* commCreateLocalDocsets([docset per device]) -> comm: one rank per docset's engine (distinct GPUs) */
static napi_value CommCreateLocalDocsets(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return NULL;
    uint32_t n = 0;
    if (napi_get_array_length(env, argv[0], &n) != napi_ok || n < 1 || n > 64) {
        napi_throw_range_error(env, NULL, "expected 1..64 docsets");
        return NULL;
    }
    hm_engine *engines[64];
    for (uint32_t i = 0; i < n; i++) {
        napi_value v;
        CHECK_NAPI(napi_get_element(env, argv[0], i, &v));
        Docset *d = get_docset(env, v);
        if (!d) return NULL;
        engines[i] = d->engine;
    }
    Comms *c = (Comms *)calloc(1, sizeof(Comms));
    c->n = (int)n;
    int st = hm_comm_create_local(engines, (int)n, c->comms);
    if (st) { free(c); return throw_status(env, engines[0], st, "hm_comm_create_local"); }
    napi_value out;
    CHECK_NAPI(napi_create_external(env, c, comms_finalize, NULL, &out));
    return out;
}

/* ---------------- CursorStore on the device (hm_cursors_*) and the syncChanges plan ---------------- */
typedef struct { hm_cursors *c; hm_engine *e; uint32_t K; } Cursors;

static void cursors_finalize(napi_env env, void *data, void *hint) {
    (void)env; (void)hint;
    Cursors *c = (Cursors *)data;
    if (c->c) hm_cursors_destroy(c->c);
    free(c);
}

static Cursors *get_cursors(napi_env env, napi_value v) {
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) { napi_throw_type_error(env, NULL, "expected a cursors handle"); return NULL; }
    return (Cursors *)p;
}

/* cursorsCreate(docset, maxActorsPerDoc) -> cursors (one repo's Cursors table on the docset's device).
 * The table must not outlive its docset. */
static napi_value CursorsCreate(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Docset *d = get_docset(env, argv[0]);
    if (!d) return NULL;
    Cursors *c = (Cursors *)calloc(1, sizeof(Cursors));
    c->e = d->engine; c->K = get_u32(env, argv[1]);
    int st = hm_cursors_create(c->e, c->K, &c->c);
    if (st) { free(c); return throw_status(env, d->engine, st, "hm_cursors_create"); }
    napi_value out;
    CHECK_NAPI(napi_create_external(env, c, cursors_finalize, NULL, &out));
    return out;
}

static napi_value CursorsReserve(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Cursors *c = get_cursors(env, argv[0]);
    if (!c) return NULL;
    int st = hm_cursors_reserve(c->c, get_u32(env, argv[1]));
    if (st) return throw_status(env, c->e, st, "hm_cursors_reserve");
    return NULL;
}

/* cursorsUpdate(c, rows u32[n], entryOff u32[n+1], actorKeys u64[], seqs f64[]) -> Buffer differs[n] */
static napi_value CursorsUpdate(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return NULL;
    Cursors *c = get_cursors(env, argv[0]);
    if (!c) return NULL;
    void *p[4]; size_t n[4];
    for (int i = 0; i < 4; i++) if (!get_bytes(env, argv[1 + i], &p[i], &n[i])) return NULL;
    const uint32_t nd = (uint32_t)(n[0] / 4);
    if (n[1] / 4 != (size_t)nd + 1 || n[2] / 8 != n[3] / 8 || (nd && ((uint32_t *)p[1])[nd] != n[2] / 8)) {
        napi_throw_range_error(env, NULL, "cursorsUpdate: rows / entryOff / keys / seqs disagree");
        return NULL;
    }
    uint8_t *df = (uint8_t *)calloc(1, nd + 8);
    int st = hm_cursors_update(c->c, nd, (const uint32_t *)p[0], (const uint32_t *)p[1], (const uint64_t *)p[2],
                               (const double *)p[3], df);
    napi_value r = st ? NULL : buf_copy(env, df, nd);
    free(df);
    if (st) return throw_status(env, c->e, st, "hm_cursors_update");
    return r;
}

/* cursorsGet(c, rows u32[n]) -> {count: u32[n], actors: u64[n*K], seqs: u64[n*K]} */
static napi_value CursorsGet(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return NULL;
    Cursors *c = get_cursors(env, argv[0]);
    if (!c) return NULL;
    void *p; size_t n;
    if (!get_bytes(env, argv[1], &p, &n)) return NULL;
    const uint32_t k = (uint32_t)(n / 4);
    uint32_t *cnt = (uint32_t *)calloc(1, (size_t)k * 4 + 4);
    uint64_t *ak = (uint64_t *)calloc(1, (size_t)k * c->K * 8 + 8), *sq = (uint64_t *)calloc(1, (size_t)k * c->K * 8 + 8);
    int st = hm_cursors_get(c->c, k, (const uint32_t *)p, cnt, ak, sq);
    napi_value o = NULL;
    if (!st) {
        napi_create_object(env, &o);
        set(env, o, "count", buf_copy(env, cnt, (size_t)k * 4));
        set(env, o, "actors", buf_copy(env, ak, (size_t)k * c->K * 8));
        set(env, o, "seqs", buf_copy(env, sq, (size_t)k * c->K * 8));
    }
    free(cnt); free(ak); free(sq);
    if (st) return throw_status(env, c->e, st, "hm_cursors_get");
    return o;
}

/* cursorsEntry(c, rows u32[n], actorKeys u64[n]) -> Buffer u64[n] (CursorStore.entry) */
static napi_value CursorsEntry(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    Cursors *c = get_cursors(env, argv[0]);
    if (!c) return NULL;
    void *pr, *pk; size_t nr, nk;
    if (!get_bytes(env, argv[1], &pr, &nr) || !get_bytes(env, argv[2], &pk, &nk)) return NULL;
    const uint32_t k = (uint32_t)(nr / 4);
    if (nk / 8 != k) { napi_throw_range_error(env, NULL, "rows and keys differ in length"); return NULL; }
    uint64_t *out = (uint64_t *)calloc(1, (size_t)k * 8 + 8);
    int st = hm_cursors_entry(c->c, k, (const uint32_t *)pr, (const uint64_t *)pk, out);
    napi_value r = st ? NULL : buf_copy(env, out, (size_t)k * 8);
    free(out);
    if (st) return throw_status(env, c->e, st, "hm_cursors_entry");
    return r;
}

/* cursorsDocsWithActors(c, actorKeys u64[q], minSeqs f64[q]|null) -> {rows u32[], actors u32[], seqs u64[]} */
static napi_value CursorsDocsWithActors(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    Cursors *c = get_cursors(env, argv[0]);
    if (!c) return NULL;
    void *pk, *pm; size_t nk, nm;
    if (!get_bytes(env, argv[1], &pk, &nk) || !get_bytes(env, argv[2], &pm, &nm)) return NULL;
    const uint32_t q = (uint32_t)(nk / 8);
    if (pm && nm / 8 != q) { napi_throw_range_error(env, NULL, "keys and minSeqs differ in length"); return NULL; }
    uint32_t cap = 1024, got = 0;
    for (;;) {
        uint32_t *rows = (uint32_t *)malloc((size_t)cap * 4), *act = (uint32_t *)malloc((size_t)cap * 4);
        uint64_t *seq = (uint64_t *)malloc((size_t)cap * 8);
        int st = hm_cursors_docs_with_actors(c->c, q, (const uint64_t *)pk, (const double *)pm, cap, rows, act, seq, &got);
        if (st == HM_ERR_NOMEM && got > cap) { free(rows); free(act); free(seq); cap = got; continue; }
        napi_value o = NULL;
        if (!st) {
            napi_create_object(env, &o);
            set(env, o, "rows", buf_copy(env, rows, (size_t)got * 4));
            set(env, o, "actors", buf_copy(env, act, (size_t)got * 4));
            set(env, o, "seqs", buf_copy(env, seq, (size_t)got * 8));
        }
        free(rows); free(act); free(seq);
        if (st) return throw_status(env, c->e, st, "hm_cursors_docs_with_actors");
        return o;
    }
}

/* syncRanges(docset, present u64 words, wordOff u64[n], lo u32[n], hi u32[n]) -> Buffer u32[n]:
 * the first missing block of each (doc, actor) range (RepoBackend.syncChanges contiguity) */
static napi_value SyncRanges(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return NULL;
    Docset *d = get_docset(env, argv[0]);
    if (!d) return NULL;
    void *p[4]; size_t n[4];
    for (int i = 0; i < 4; i++) if (!get_bytes(env, argv[1 + i], &p[i], &n[i])) return NULL;
    const uint32_t k = (uint32_t)(n[2] / 4);
    if (n[1] / 8 != k || n[3] / 4 != k) { napi_throw_range_error(env, NULL, "syncRanges: lengths disagree"); return NULL; }
    uint32_t *out = (uint32_t *)calloc(1, (size_t)k * 4 + 4);
    int st = hm_sync_ranges_host(d->engine, (const uint64_t *)p[0], (const uint64_t *)p[1], (const uint32_t *)p[2],
                                 (const uint32_t *)p[3], out, k, (uint32_t)(n[0] / 8));
    napi_value r = st ? NULL : buf_copy(env, out, (size_t)k * 4);
    free(out);
    if (st) return throw_status(env, d->engine, st, "hm_sync_ranges_host");
    return r;
}

/* decodeBlocks(blocks[][], aStride, threads) -> {status, docs, changes, deps, ops}: the
 * stateless decoder (hm_decode_blocks) for cold batches, tables as Buffers */
static napi_value DecodeBlocks(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return NULL;
    uint32_t n = 0;
    if (napi_get_array_length(env, argv[0], &n) != napi_ok) { napi_throw_type_error(env, NULL, "expected an array"); return NULL; }
    uint32_t *ids = (uint32_t *)calloc(1, (size_t)n * 4 + 4);
    napi_value idv;
    void *idp;
    napi_create_buffer_copy(env, (size_t)n * 4, ids, &idp, &idv);
    free(ids);
    DsJob *j = (DsJob *)calloc(1, sizeof(DsJob));
    if (!gather_blocks(env, idv, argv[0], j)) { ds_job_free(env, j); return NULL; }
    hm_decoded *dd = NULL;
    int st = hm_decode_blocks(j->data, j->bo, j->db, n, get_u32(env, argv[1]), (int)get_u32(env, argv[2]), &dd);
    ds_job_free(env, j);
    if (st) return throw_status(env, NULL, st, "hm_decode_blocks");
    hm_batch b;
    hm_decoded_batch(dd, &b);
    napi_value o;
    napi_create_object(env, &o);
    set(env, o, "status", buf_copy(env, hm_decoded_status(dd), (size_t)n * 4));
    set(env, o, "docs", buf_copy(env, b.docs, (size_t)b.n_docs * sizeof(hm_doc_row)));
    set(env, o, "changes", buf_copy(env, b.changes, (size_t)b.n_changes * sizeof(hm_change_row)));
    set(env, o, "deps", buf_copy(env, b.deps, (size_t)b.n_deps * sizeof(hm_dep_row)));
    set(env, o, "ops", buf_copy(env, b.ops, (size_t)b.n_ops * sizeof(hm_op_row)));
    set(env, o, "aStride", u32v(env, b.a_stride));
    hm_decoded_free(dd);
    return o;
}

static napi_value Init(napi_env env, napi_value exports) {
    struct { const char *name; napi_callback fn; } fns[] = {
        {"createStore", CreateStore}, {"openDoc", OpenDoc}, {"submit", Submit}, {"wait", Wait},
        {"info", Info}, {"read", Read}, {"historyPrefix", HistoryPrefix}, {"setMinClock", SetMinClock},
        {"clockUpdate", ClockUpdate}, {"statusMessage", StatusMessage},
        {"commCreateLocal", CommCreateLocal}, {"clockExchange", ClockExchange}, {"clockMin", ClockMin},
        {"waitAsync", WaitAsync}, {"readRegs", ReadRegs},
        {"docsetCreate", DocsetCreate}, {"docsetOpen", DocsetOpen}, {"docsetApply", DocsetApply}, {"docsetApplyPacked", DocsetApplyPacked},
        {"docsetHistoryPrefix", DocsetHistoryPrefix}, {"docsetClockUpdate", DocsetClockUpdate},
        {"docsetView", DocsetView}, {"docsetInfo", DocsetInfo}, {"docsetStats", DocsetStats},
        {"cursorsCreate", CursorsCreate}, {"cursorsReserve", CursorsReserve}, {"cursorsUpdate", CursorsUpdate},
        {"cursorsGet", CursorsGet}, {"cursorsEntry", CursorsEntry}, {"cursorsDocsWithActors", CursorsDocsWithActors},
        {"syncRanges", SyncRanges}, {"decodeBlocks", DecodeBlocks}, {"commCreateLocalDocsets", CommCreateLocalDocsets},
    };
    for (size_t i = 0; i < sizeof fns / sizeof fns[0]; i++) {
        napi_value f;
        napi_create_function(env, fns[i].name, NAPI_AUTO_LENGTH, fns[i].fn, NULL, &f);
        napi_set_named_property(env, exports, fns[i].name, f);
    }
    napi_value v;
    napi_create_uint32(env, hm_abi_version(), &v);
    napi_set_named_property(env, exports, "abiVersion", v);
    return exports;
}

#ifndef NODE_GYP_MODULE_NAME
#define NODE_GYP_MODULE_NAME hmgpu
#endif
NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
