/*
 * oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * merge path, used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the CHECKER.  Nothing in hypermerge_amd/ links,
 * loads or calls this file; the product path is the HIP library.
 *
 * It restates, literally and sequentially (one document at a time, one
 * change at a time, one op at a time), over the columnar batch of
 * include/hypermerge_amd.h:
 *
 *   hypermerge (reference repo, TypeScript):
 *     src/DocBackend.ts:135-142  updateClock: clock[actor] = max(., seq) over
 *                                *every* handed change, queued ones included;
 *                                not reached when applyChanges throws
 *     src/DocBackend.ts:90-100   testMinimumClockSatisfied -> Clock.cmp
 *     src/Clock.ts:13-38         gte / cmp (a missing entry counts as 0)
 *   Automerge 0.12.2-beta.0 backend (third-party, NOT vendored in the
 *   reference; yarn.lock:178-185, github:automerge/automerge#opaque-strings
 *   @340ca073b716f28426175e221766352e52d84daf).  Its rules are restated
 *   from SURVEY.md Appendix A (a restatement of upstream backend/op_set.js
 *   made without the source); PARITY FOR THESE RULES IS UNPINNED by any
 *   reference output — only by the hand-derived known-answer tests in
 *   tests/test_oracle_kat.py:
 *     A.1 addChange / applyQueuedOps pass order, causallyReady,
 *         applyChange duplicate check, transitiveDeps (a fold in deps key
 *         order then {actor: seq-1}, whose `.set` overrides the max),
 *         deps heads, clock, history.
 *     A.2 applyAssign: survivors = concurrent prior ops, push set/link,
 *         `sortBy(actor).reverse()` after EVERY assign (stable sort, so
 *         equal-actor ties flip each time), `inc` adds to causally-prior
 *         counter sets.
 *     A.3 applyInsert / updateListElement / getPrevious / insertionsAfter
 *         (children ordered by lamportCompare (elem, actor) descending).
 *
 * Error model: the first throw aborts the document's applyChanges; we
 * record (status, change, op) and stop processing that document.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "../include/hypermerge_amd.h"

#define NONE 0xFFFFFFFFu

typedef struct { uint32_t op; uint32_t vtag; uint64_t value; double absum; } surv_t;
typedef struct { surv_t *v; uint32_t n, cap; } survlist_t;
typedef struct { uint32_t *v; uint32_t n, cap; } u32vec_t;

static void u32_push(u32vec_t *a, uint32_t x) {
    if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 4; a->v = (uint32_t *)realloc(a->v, a->cap * sizeof(uint32_t)); }
    a->v[a->n++] = x;
}
static void u32_insert(u32vec_t *a, uint32_t at, uint32_t x) {
    u32_push(a, 0);
    memmove(a->v + at + 1, a->v + at, (a->n - 1 - at) * sizeof(uint32_t));
    a->v[at] = x;
}
static void u32_remove(u32vec_t *a, uint32_t at) {
    memmove(a->v + at, a->v + at + 1, (a->n - 1 - at) * sizeof(uint32_t));
    a->n--;
}
static int64_t u32_index_of(const u32vec_t *a, uint32_t x) {
    for (uint32_t i = 0; i < a->n; i++) if (a->v[i] == x) return i;
    return -1;
}
static void surv_push(survlist_t *a, surv_t x) {
    if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 4; a->v = (surv_t *)realloc(a->v, a->cap * sizeof(surv_t)); }
    a->v[a->n++] = x;
}

/* per-document working state (the "opSet") */
typedef struct {
    const hm_batch *b;
    const hm_doc_row *doc;
    const hm_results *out;
    uint32_t A, S;            /* actors, a_stride */
    uint32_t *clock;          /* opSet.clock (applied) */
    uint32_t *heads;          /* opSet.deps */
    u32vec_t *states;         /* opSet.states[actor] -> doc-local change index, in seq order */
    uint32_t *ad;             /* allDeps rows (doc-local change index * S) */
    int8_t   *objtype;        /* byObject[obj]._init.action, -1 = not created */
    survlist_t *keys;         /* byObject[obj]._keys[key], one list per register */
    uint32_t *insertion;      /* _insertion[elemId] -> doc-local op index of the ins, or NONE */
    u32vec_t *following;      /* _following[parent]: regs 0..R-1, then '_head' of obj o at R+o */
    u32vec_t *elemids;        /* _elemIds per object (visible elements, in order) */
    uint32_t *reg_obj;
    uint32_t *op_change;      /* doc-local op -> doc-local change */
    uint32_t *op_actor;       /* doc-local op -> actor rank of its change */
    uint32_t *kids;           /* scratch for insertionsAfter */
    uint32_t hist_len;
    int status; uint32_t err_change, err_op;
    int unsupported;
} docst_t;

static inline const hm_change_row *CH(docst_t *s, uint32_t i) { return &s->b->changes[s->doc->change_off + i]; }
static inline const hm_op_row *OP(docst_t *s, uint32_t k) { return &s->b->ops[s->doc->op_off + k]; }

/* isConcurrent(opSet, op1, op2): allDeps1[actor2] < seq2 && allDeps2[actor1] < seq1 */
static int is_concurrent(docst_t *s, uint32_t c1, uint32_t c2) {
    const hm_change_row *x = CH(s, c1), *y = CH(s, c2);
    const uint32_t *ad1 = s->ad + (size_t)c1 * s->S, *ad2 = s->ad + (size_t)c2 * s->S;
    return ad1[y->actor] < y->seq && ad2[x->actor] < x->seq;
}

/* causallyReady: every (a, s) of deps.set(actor, seq-1) has clock[a] >= s */
static int causally_ready(docst_t *s, uint32_t ci) {
    const hm_change_row *c = CH(s, ci);
    for (uint32_t j = 0; j < c->n_deps; j++) {
        const hm_dep_row *d = &s->b->deps[c->dep_off + j];
        uint32_t need = (d->actor == c->actor) ? c->seq - 1 : d->seq;
        if (s->clock[d->actor] < need) return 0;
    }
    return s->clock[c->actor] >= c->seq - 1;
}

static void fail(docst_t *s, int st, uint32_t ci, uint32_t op) {
    if (s->status == HM_OK) { s->status = st; s->err_change = ci; s->err_op = op; }
}

/* ---------------- lists (A.3) ---------------- */

/* insertionsAfter(obj, parent): child registers sorted by lamportCompare
 * (elem, then actor string) DESCENDING.  Returns the count. */
static uint32_t insertions_after(docst_t *s, uint32_t pkey, uint32_t *out) {
    u32vec_t *f = &s->following[pkey];
    uint32_t n = f->n;
    for (uint32_t i = 0; i < n; i++) {               /* insertion sort, descending */
        uint32_t x = f->v[i], j = i;
        const hm_op_row *ox = OP(s, x);
        while (j > 0) {
            uint32_t y = out[j - 1];
            const hm_op_row *oy = OP(s, y);
            int y_less = (oy->elem < ox->elem) || (oy->elem == ox->elem && s->op_actor[y] < s->op_actor[x]);
            if (!y_less) break;
            out[j] = y; j--;
        }
        out[j] = x;
    }
    for (uint32_t i = 0; i < n; i++) out[i] = OP(s, out[i])->reg;
    return n;
}

/* getParent: parent key (reg, or R+obj for '_head'); -1 = 'Missing index entry' */
static int64_t get_parent(docst_t *s, uint32_t obj, uint32_t reg) {
    uint32_t ins = s->insertion[reg];
    if (ins == NONE) return -1;
    uint32_t p = OP(s, ins)->parent;
    return p == HM_HEAD ? (int64_t)(s->doc->n_regs + obj) : (int64_t)p;
}

/* getPrevious: returns the predecessor element reg, NONE for the head.  *steps counts the
 * elements visited: a walk over an acyclic insertion tree visits each at most twice, so a walk
 * past the bound is going round a cycle of inserts (each after the next, all detached from
 * '_head'), on which the reference's getPrevious never returns: *err = 2 */
static uint32_t get_previous(docst_t *s, uint32_t obj, uint32_t reg, int *err, uint64_t *steps) {
    const uint64_t bound = 4 * (uint64_t)s->doc->n_regs + 8;
    int64_t parent = get_parent(s, obj, reg);
    if (parent < 0) { *err = 1; return NONE; }
    uint32_t *kids = s->kids;
    uint32_t n = insertions_after(s, (uint32_t)parent, kids);
    if (n > 0 && kids[0] == reg)
        return parent >= (int64_t)s->doc->n_regs ? NONE : (uint32_t)parent;
    uint32_t prev = NONE;
    for (uint32_t i = 0; i < n; i++) { if (kids[i] == reg) break; prev = kids[i]; }
    while (1) {
        if (++*steps > bound) { *err = 2; return NONE; }
        uint32_t m = insertions_after(s, prev, kids);
        if (m == 0) return prev;
        prev = kids[m - 1];
    }
}

/* updateListElement */
static int update_list_element(docst_t *s, uint32_t obj, uint32_t reg) {
    survlist_t *ops = &s->keys[reg];
    u32vec_t *el = &s->elemids[obj];
    int64_t index = u32_index_of(el, reg);
    if (index >= 0) {
        if (ops->n == 0) u32_remove(el, (uint32_t)index);   /* 'remove' */
        return 0;                                           /* else 'set' */
    }
    if (ops->n == 0) return 0;                              /* deleting a non-existent element */
    uint32_t prev = reg;
    uint64_t steps = 0;
    while (1) {
        index = -1;
        int err = 0;
        prev = get_previous(s, obj, prev, &err, &steps);
        if (err == 2) { s->unsupported = 1; return HM_ERR_UNSUPPORTED; }   /* the reference loops forever */
        if (err) return HM_ERR_MISSING_ELEM;
        if (++steps > 4 * (uint64_t)s->doc->n_regs + 8) { s->unsupported = 1; return HM_ERR_UNSUPPORTED; }
        if (prev == NONE) break;
        index = u32_index_of(el, prev);
        if (index >= 0) break;
    }
    u32_insert(el, (uint32_t)(index + 1), reg);             /* 'insert' */
    return 0;
}

static const double TWO53 = 9007199254740992.0;

static double num_of(uint32_t vtag, uint64_t v) {
    if (vtag == HM_V_INT) return (double)(int64_t)v;
    double d; memcpy(&d, &v, 8); return d;
}

/* ---------------- applyAssign (A.2) ---------------- */
static int apply_assign(docst_t *s, uint32_t ci, uint32_t k) {
    const hm_op_row *op = OP(s, k);
    if (op->obj >= s->doc->n_objs || s->objtype[op->obj] < 0) return HM_ERR_UNKNOWN_OBJECT;
    if (op->reg >= s->doc->n_regs) { s->unsupported = 1; return 0; }
    survlist_t *L = &s->keys[op->reg];
    s->reg_obj[op->reg] = op->obj;
    if (op->action == HM_INC) {
        /* ops.map(other => counter set && !isConcurrent ? value + inc : other) */
        for (uint32_t i = 0; i < L->n; i++) {
            surv_t *x = &L->v[i];
            const hm_op_row *xo = OP(s, x->op);
            int numeric = (x->vtag == HM_V_INT || x->vtag == HM_V_FLOAT);
            if (xo->action == HM_SET && numeric && xo->datatype == HM_DT_COUNTER &&
                !is_concurrent(s, s->op_change[x->op], ci)) {
                double inc = num_of(op->vtag, op->value);
                x->absum += fabs(inc);
                if (x->vtag == HM_V_INT && op->vtag == HM_V_INT) {
                    x->value = (uint64_t)((int64_t)x->value + (int64_t)op->value);
                } else {
                    double r = num_of(x->vtag, x->value) + inc;
                    memcpy(&x->value, &r, 8);
                    x->vtag = HM_V_FLOAT;
                }
            }
        }
    } else {
        /* groupBy(isConcurrent): keep only the concurrent prior ops */
        uint32_t w = 0;
        for (uint32_t i = 0; i < L->n; i++)
            if (is_concurrent(s, s->op_change[L->v[i].op], ci)) L->v[w++] = L->v[i];
        L->n = w;
    }
    if (op->action == HM_SET || op->action == HM_LINK) {
        surv_t x = { k, op->vtag, op->value, op->vtag == HM_V_INT ? fabs((double)(int64_t)op->value) : 0.0 };
        surv_push(L, x);
    }
    /* remaining.sortBy(op => op.actor).reverse(): stable ascending, then reverse */
    for (uint32_t i = 1; i < L->n; i++) {
        surv_t x = L->v[i];
        uint32_t ax = s->op_actor[x.op], j = i;
        while (j > 0 && s->op_actor[L->v[j - 1].op] > ax) { L->v[j] = L->v[j - 1]; j--; }
        L->v[j] = x;
    }
    if (L->n > 1)
        for (uint32_t i = 0, j = L->n - 1; i < j; i++, j--) { surv_t t = L->v[i]; L->v[i] = L->v[j]; L->v[j] = t; }
    int t = s->objtype[op->obj];
    if (t == HM_MAKE_LIST || t == HM_MAKE_TEXT) return update_list_element(s, op->obj, op->reg);
    return 0;
}

/* ---------------- applyChange (A.1) ---------------- */
static void apply_change(docst_t *s, uint32_t ci) {
    const hm_change_row *c = CH(s, ci);
    u32vec_t *prior = &s->states[c->actor];
    if (c->seq <= prior->n) {                                /* already applied */
        uint32_t stored = prior->v[c->seq - 1];
        if (CH(s, stored)->content_id != c->content_id) fail(s, HM_ERR_INCONSISTENT_SEQ, ci, NONE);
        s->out->hist[s->doc->change_off + ci] = -2;
        return;
    }
    /* transitiveDeps(deps.set(actor, seq-1)): reduce in key order,
     * deps.mergeWith(max, states[a][s-1].allDeps).set(a, s) */
    uint32_t *ad = s->ad + (size_t)ci * s->S;
    memset(ad, 0, s->S * sizeof(uint32_t));
    int own_seen = 0;
    for (uint32_t j = 0; j <= c->n_deps; j++) {
        uint32_t a, q;
        if (j < c->n_deps) {
            const hm_dep_row *d = &s->b->deps[c->dep_off + j];
            a = d->actor; q = d->seq;
            if (a == c->actor) { q = c->seq - 1; own_seen = 1; }
        } else {
            if (own_seen) break;
            a = c->actor; q = c->seq - 1;
        }
        if (q == 0) continue;
        uint32_t dc = s->states[a].v[q - 1];
        const uint32_t *t = s->ad + (size_t)dc * s->S;
        for (uint32_t x = 0; x < s->A; x++) if (t[x] > ad[x]) ad[x] = t[x];
        ad[a] = q;
    }
    u32_push(prior, ci);
    /* applyOps, each op tagged with the change's actor and seq */
    for (uint32_t j = 0; j < c->n_ops; j++) {
        uint32_t k = c->op_first - s->doc->op_off + j;
        const hm_op_row *op = OP(s, k);
        int err = 0;
        switch (op->action) {
        case HM_MAKE_MAP: case HM_MAKE_TABLE: case HM_MAKE_LIST: case HM_MAKE_TEXT:
            if (op->obj >= s->doc->n_objs) { s->unsupported = 1; break; }
            if (s->objtype[op->obj] >= 0) { err = HM_ERR_DUPLICATE_OBJECT; break; }
            s->objtype[op->obj] = (int8_t)op->action;
            break;
        case HM_INS:
            if (op->obj >= s->doc->n_objs || s->objtype[op->obj] < 0) { err = HM_ERR_UNKNOWN_OBJECT; break; }
            if (op->reg >= s->doc->n_regs || (op->parent != HM_HEAD && op->parent >= s->doc->n_regs)) { s->unsupported = 1; break; }
            if (s->insertion[op->reg] != NONE) { err = HM_ERR_DUPLICATE_ELEM; break; }
            /* an insert after an element not inserted yet waits in its parent's _following
             * (applyInsert does not look the parent up); getPrevious throws later if a set
             * lands on an element whose insertion chain is still incomplete */
            s->reg_obj[op->reg] = op->obj;
            u32_push(&s->following[op->parent == HM_HEAD ? s->doc->n_regs + op->obj : op->parent], k);
            s->insertion[op->reg] = k;
            break;
        case HM_SET: case HM_DEL: case HM_LINK: case HM_INC:
            err = apply_assign(s, ci, k);
            break;
        default:
            s->unsupported = 1;
        }
        if (err) { fail(s, err, ci, j); return; }
    }
    /* deps = deps.filter((seq, a) => seq > allDeps.get(a, 0)).set(actor, seq) */
    for (uint32_t a = 0; a < s->A; a++) if (s->heads[a] && s->heads[a] <= ad[a]) s->heads[a] = 0;
    s->heads[c->actor] = c->seq;
    s->clock[c->actor] = c->seq;
    s->out->hist[s->doc->change_off + ci] = (int32_t)s->hist_len++;
}

static void merge_doc(const hm_batch *b, const hm_results *out, uint32_t d) {
    docst_t s; memset(&s, 0, sizeof(s));
    s.b = b; s.doc = &b->docs[d]; s.out = out;
    s.A = s.doc->n_actors; s.S = b->a_stride;
    const uint32_t n = s.doc->n_changes, m = s.doc->n_ops, R = s.doc->n_regs, O = s.doc->n_objs;
    s.clock = out->clock + (size_t)d * s.S;
    s.heads = out->heads + (size_t)d * s.S;
    uint32_t *bclock = out->back_clock + (size_t)d * s.S;
    memset(s.clock, 0, s.S * 4); memset(s.heads, 0, s.S * 4); memset(bclock, 0, s.S * 4);
    s.ad = out->all_deps + (size_t)s.doc->change_off * s.S;
    memset(s.ad, 0, (size_t)n * s.S * 4);
    s.states = (u32vec_t *)calloc(s.A ? s.A : 1, sizeof(u32vec_t));
    s.objtype = (int8_t *)malloc(O ? O : 1);
    memset(s.objtype, -1, O ? O : 1);
    if (O) s.objtype[0] = HM_MAKE_MAP;                          /* ROOT */
    s.keys = (survlist_t *)calloc(R ? R : 1, sizeof(survlist_t));
    s.insertion = (uint32_t *)malloc((R ? R : 1) * 4);
    for (uint32_t i = 0; i < R; i++) s.insertion[i] = NONE;
    s.following = (u32vec_t *)calloc(R + O + 1, sizeof(u32vec_t));
    s.elemids = (u32vec_t *)calloc(O ? O : 1, sizeof(u32vec_t));
    s.reg_obj = (uint32_t *)malloc((R ? R : 1) * 4);
    for (uint32_t i = 0; i < R; i++) s.reg_obj[i] = NONE;
    s.op_change = (uint32_t *)malloc((m ? m : 1) * 4);
    s.op_actor = (uint32_t *)malloc((m ? m : 1) * 4);
    s.kids = (uint32_t *)malloc((m ? m : 1) * 4);
    for (uint32_t k = 0; k < m; k++) { s.op_change[k] = NONE; s.op_actor[k] = 0; }
    /* engine envelope: op and dep rows grouped by change in arrival order, without gaps
     * (the layout include/hypermerge_amd.h prescribes) */
    uint32_t op_next = s.doc->op_off, dep_next = s.doc->dep_off;
    for (uint32_t i = 0; i < n; i++) {
        const hm_change_row *c = CH(&s, i);
        if (c->op_first != op_next || c->dep_off != dep_next) s.unsupported = 1;
        op_next = c->op_first + c->n_ops; dep_next = c->dep_off + c->n_deps;
    }
    if (op_next != s.doc->op_off + m || dep_next != s.doc->dep_off + s.doc->n_deps) s.unsupported = 1;
    for (uint32_t i = 0; i < n; i++) {
        const hm_change_row *c = CH(&s, i);
        if (c->actor >= s.A || c->seq == 0) s.unsupported = 1;
        for (uint32_t j = 0; j < c->n_deps; j++) if (b->deps[c->dep_off + j].actor >= s.A) s.unsupported = 1;
        for (uint32_t j = 0; j < c->n_ops; j++) {
            uint32_t k = c->op_first - s.doc->op_off + j;
            if (k < m) { s.op_change[k] = i; s.op_actor[k] = c->actor; } else s.unsupported = 1;
        }
        out->hist[s.doc->change_off + i] = -1;
    }
    /* engine envelope: malformed op rows (ids outside the doc's tables, unknown actions)
     * put the whole document outside, whatever would throw first */
    for (uint32_t k = 0; k < m; k++) {
        const hm_op_row *op = OP(&s, k);
        if (op->action <= HM_MAKE_TEXT) { if (op->obj >= O) s.unsupported = 1; }
        else if (op->action <= HM_INC) {
            if (op->reg >= R) s.unsupported = 1;
            if (op->action == HM_INS && op->parent != HM_HEAD && op->parent >= R) s.unsupported = 1;
        } else s.unsupported = 1;
    }

    uint32_t qn = 0;
    uint32_t *queue = (uint32_t *)malloc((n ? n : 1) * 4);
    uint32_t *nq = (uint32_t *)malloc((n ? n : 1) * 4);
    /* Backend.applyChanges: addChange for each change in array order */
    for (uint32_t i = 0; i < n && s.status == HM_OK && !s.unsupported; i++) {
        queue[qn++] = i;
        while (s.status == HM_OK) {                             /* applyQueuedOps */
            uint32_t nn = 0;
            for (uint32_t q = 0; q < qn && s.status == HM_OK; q++) {
                if (causally_ready(&s, queue[q])) apply_change(&s, queue[q]);
                else nq[nn++] = queue[q];
            }
            if (nn == qn) break;
            memcpy(queue, nq, nn * 4); qn = nn;
        }
    }
    hm_doc_result *r = &out->docs[d];
    memset(r, 0, sizeof(*r));
    r->err_change = NONE; r->err_op = NONE;
    if (s.unsupported && s.status == HM_OK) s.status = HM_ERR_UNSUPPORTED;
    r->status = s.status;
    if (s.status != HM_OK && s.status != HM_ERR_UNSUPPORTED) { r->err_change = s.err_change; r->err_op = s.err_op; }
    r->hist_len = s.hist_len;
    r->n_queued = qn;
    /* DocBackend.updateClock (reached only when applyChanges did not throw) */
    if (s.status == HM_OK)
        for (uint32_t i = 0; i < n; i++) {
            const hm_change_row *c = CH(&s, i);
            if (c->seq > bclock[c->actor]) bclock[c->actor] = c->seq;
        }
    /* Clock.cmp(DocBackend.clock, minimumClock): 0 EQ, 1 GT, 2 LT, 3 CONCUR */
    if (b->min_clock) {
        const uint32_t *mc = b->min_clock + (size_t)d * s.S;
        int ag = 1, bg = 1;
        for (uint32_t a = 0; a < s.S; a++) { if (bclock[a] < mc[a]) ag = 0; if (mc[a] < bclock[a]) bg = 0; }
        r->min_cmp = (ag && bg) ? 0 : (ag ? 1 : (bg ? 2 : 3));
    }
    /* registers: survivors laid out in register-id order */
    uint32_t off = 0;
    for (uint32_t g = 0; g < R; g++) {
        hm_reg_result *rr = &out->regs[s.doc->reg_off + g];
        rr->n_surv = s.keys[g].n; rr->surv_off = off; rr->list_index = -1; rr->obj = s.reg_obj[g];
        for (uint32_t i = 0; i < s.keys[g].n; i++) {
            const surv_t *x = &s.keys[g].v[i];
            hm_surv_result *o = &out->surv[s.doc->op_off + off + i];
            o->op = x->op; o->vtag = x->vtag; o->value = x->value;
            /* an integer counter is exact in JS only while every partial sum is < 2^53 */
            if (x->vtag == HM_V_INT && x->absum > TWO53 && r->status == HM_OK) r->status = HM_ERR_UNSUPPORTED;
        }
        off += s.keys[g].n;
    }
    r->n_surv = off;
    for (uint32_t o = 0; o < O; o++)
        for (uint32_t i = 0; i < s.elemids[o].n; i++)
            out->regs[s.doc->reg_off + s.elemids[o].v[i]].list_index = (int32_t)i;

    for (uint32_t a = 0; a < s.A; a++) free(s.states[a].v);
    for (uint32_t g = 0; g < R; g++) free(s.keys[g].v);
    for (uint32_t g = 0; g < R + O + 1; g++) free(s.following[g].v);
    for (uint32_t o = 0; o < O; o++) free(s.elemids[o].v);
    free(s.states); free(s.objtype); free(s.keys); free(s.insertion); free(s.following);
    free(s.elemids); free(s.reg_obj); free(s.op_change); free(s.op_actor); free(s.kids);
    free(queue); free(nq);
}

/* Merge documents [doc_begin, doc_end) of the batch (thread-safe across
 * disjoint document ranges). */
int oracle_merge(const hm_batch *b, const hm_results *out, uint32_t doc_begin, uint32_t doc_end) {
    if (doc_end > b->n_docs) doc_end = b->n_docs;
    for (uint32_t d = doc_begin; d < doc_end; d++) merge_doc(b, out, d);
    return 0;
}

uint32_t oracle_abi_version(void) { return HM_ABI_VERSION; }
