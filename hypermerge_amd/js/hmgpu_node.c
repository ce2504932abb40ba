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

static Store *get_store(napi_env env, napi_value v) {
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, NULL, "expected a store handle");
        return NULL;
    }
    return (Store *)p;
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
    (void)context;
    Job *j = (Job *)data;
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
    if (napi_create_threadsafe_function(env, argv[2], NULL, name, 0, 1, NULL, NULL, NULL, job_call_js, &j->tsfn) != napi_ok) {
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

static napi_value Init(napi_env env, napi_value exports) {
    struct { const char *name; napi_callback fn; } fns[] = {
        {"createStore", CreateStore}, {"openDoc", OpenDoc}, {"submit", Submit}, {"wait", Wait},
        {"info", Info}, {"read", Read}, {"historyPrefix", HistoryPrefix}, {"setMinClock", SetMinClock},
        {"clockUpdate", ClockUpdate}, {"statusMessage", StatusMessage},
        {"commCreateLocal", CommCreateLocal}, {"clockExchange", ClockExchange}, {"clockMin", ClockMin},
        {"waitAsync", WaitAsync}, {"readRegs", ReadRegs},
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
