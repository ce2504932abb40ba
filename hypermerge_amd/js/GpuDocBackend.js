'use strict'
// GpuDocBackend.js — the Node host side of the MI355X merge engine, a drop-in for the
// reference's remote-change path:
//
//   Backend      Automerge's functional API as DocBackend/RepoBackend use it
//                (Backend.init, Backend.applyChanges(state, changes) -> [state, patch],
//                state.getIn(['opSet','history']).size / .slice(0, n).toArray();
//                src/DocBackend.ts:79,148,157,172,175, src/RepoBackend.ts:572-576).
//   DocBackend   the reference class (src/DocBackend.ts:46-213): same constructor, fields
//                (id, actorId, clock, back, changes, ready) and methods (init, initActor,
//                applyRemoteChanges, applyLocalChange, updateMinimumClock), same
//                ReadyMsg / ActorIdMsg / RemotePatchMsg / LocalPatchMsg messages.
//   GpuEngine    owns the device store (N-API addon -> include/hypermerge_amd.h) and runs
//                every document's applyChanges calls as batched GPU submits: per-document
//                FIFO job queues, one submit per round over all documents with work.
//                mode 'sync' flushes inside the caller's stack (the reference's Queue
//                semantics: a push runs the merge synchronously); mode 'batched' flushes
//                once per event-loop turn (setImmediate), merging every document that
//                received changes during the turn in one launch; mode 'async' does the
//                same but waits for the device on the store's host thread (waitAsync,
//                completion through a napi_threadsafe_function), so the event loop never
//                blocks on the GPU.
//                Patches are incremental: after a round in which a document's new changes
//                all applied, only the registers its new ops hit are read back
//                (hm_store_read_regs, one call per store and round) and diffed against the
//                document's previous view; otherwise the whole document is re-read.
//   ClockStore   the reference's clock table semantics (src/ClockStore.ts:24-112) kept in
//                host memory, with updateDocs(): ClockStore.update(repo, doc, doc.clock)
//                for many documents from one GPU upsert-max (hm_store_clock_update).
//
// A document's applyChanges that throws (e.g. 'Inconsistent reuse of sequence number')
// is rolled back on the device and rethrown here, like the reference's throw out of
// Backend.applyChanges leaves DocBackend.back unchanged.

const path = require('path')
const addon = require(path.join(__dirname, '..', '_lib', 'hmgpu.node'))
const C = require('./columnar')
const Clock = require('./clocks')
const Channel = require('./channel')

const ERR_TEXT = {
  1: 'Inconsistent reuse of sequence number',
  2: 'Modification of unknown object',
  3: 'Duplicate creation of object',
  4: 'Duplicate list element ID',
  5: 'Missing index entry for list element',
  16: 'Document outside the engine envelope',
}

class History {
  constructor(state) { this.state = state; this.size = state.histLen }
  slice(a, b) {
    const st = this.state
    const lo = a || 0
    const hi = b === undefined ? this.size : Math.min(b, this.size)
    const idx = addon.historyPrefix(st.store, st.handle, Math.max(hi, 0))
    const out = []
    for (let i = lo; i < idx.length / 4; i++) out.push(st.log[idx.readUInt32LE(4 * i)])
    return { toArray: () => out, size: out.length }
  }
}

// FNV-1a 64 over the UTF-8 bytes of an id string: the shard key (and the clock exchange's
// record key) of hypermerge_amd/exchange.py and include/hypermerge_amd.h.
const FNV_OFFSET = 0xcbf29ce484222325n, FNV_PRIME = 0x100000001b3n, M64 = (1n << 64n) - 1n
function fnv1a64(s) {
  let h = FNV_OFFSET
  for (const b of Buffer.from(s, 'utf8')) h = ((h ^ BigInt(b)) * FNV_PRIME) & M64
  return h
}

// Row widths of the stores a document can live in: a document starts in the narrowest that
// holds its actors and moves to a wider one when a new actor outgrows it (its whole log is
// re-merged there, once).
const STRIDES = [8, 16, 32, 64]

// The per-document BackendState: a handle into one device store (its shard's, at its stride)
// plus the host-side interner and the change objects of the log (for history slices and
// re-striding).  States are linear: applyChanges advances the document in place and returns
// the same state object.
class GpuBackendState {
  constructor(engine, docId) {
    this.engine = engine
    this.docId = docId
    this.shard = docId === undefined ? 0 : engine.shardOf(docId)
    this.stride = engine.minStride
    this.store = engine.storeFor(this.shard, this.stride)
    this.handle = addon.openDoc(this.store)
    this.enc = new C.DocEncoder(engine.pool)
    this.log = []
    this.opActor = []                // doc-local op index -> [op, actor] (the log's ops in order)
    this.view = null                 // materialized view of the last patch (diff base)
    this.objType = new Map([[0, 0]]) // obj id -> make action (ROOT = map), kept per round
    this.newObjs = []                // objects the last round created
    this.roundSeq = 0                // rounds applied ...
    this.patchedSeq = 0              // ... and the round the view reflects
    this.pendingRegs = null          // registers the last round's ops hit, read back (incremental patch)
    this.histLen = 0
    this.nQueued = 0
    this.clock = {}
    this.deps = {}
    this.backClock = {}              // DocBackend.clock as the engine computed it (queued included)
  }

  getIn(p) {
    if (p.length === 2 && p[0] === 'opSet' && p[1] === 'history') return new History(this)
    if (p.length === 2 && p[0] === 'opSet' && p[1] === 'clock') return Object.assign({}, this.clock)
    if (p.length === 2 && p[0] === 'opSet' && p[1] === 'deps') return Object.assign({}, this.deps)
    throw new Error(`GpuBackendState.getIn: unsupported path ${JSON.stringify(p)}`)
  }
}

class GpuEngine {
  // opts: devices (HIP ordinals; documents shard over them by FNV-1a64(docId) % devices.length),
  // aStride (narrowest store stride), mode 'sync' | 'batched', onError, patches
  constructor(opts) {
    const o = opts || {}
    this.devices = o.devices || [o.device || 0]
    this.minStride = o.aStride || 8
    this.aStride = this.minStride
    this.mode = o.mode || 'batched'
    this.shards = this.devices.map((d) => ({ device: d, stores: new Map() }))
    this.store = this.storeFor(0, this.minStride)
    this.pool = new C.StringPool()
    this.queues = new Map()          // state -> FIFO of jobs
    this.flushing = false
    this.scheduled = false
    this.onError = o.onError || null
    this.submits = 0
    this.restrides = 0
    this.patches = o.patches !== false  // emit patch diffs (one device read per patch)
    this.comm = null
  }

  shardOf(docId) { return Number(fnv1a64(docId) % BigInt(this.shards.length)) }

  storeFor(shard, stride) {
    const sh = this.shards[shard]
    let st = sh.stores.get(stride)
    if (!st) { st = addon.createStore(sh.device, stride); sh.stores.set(stride, st) }
    return st
  }

  init(docId) { return new GpuBackendState(this, docId) }

  // job: {changes|null, extraActors, done(result|null), fail(err)}
  enqueue(state, job) {
    let q = this.queues.get(state)
    if (!q) { q = []; this.queues.set(state, q) }
    q.push(job)
    if (this.mode === 'sync') this.flush()
    else if (!this.scheduled && !this.flushing) {
      this.scheduled = true
      setImmediate(() => { this.scheduled = false; this.flush() })
    }
  }

  // leading callbacks run; each document's head GPU job forms the round
  collectRound() {
    for (;;) {
      const round = []
      for (const [state, q] of Array.from(this.queues)) {
        while (q.length && q[0].changes === null) q.shift().done(null)
        if (q.length) round.push([state, q.shift()])
        else this.queues.delete(state)
      }
      if (round.length || this.queues.size === 0) return round
    }
  }

  flush() {
    if (this.mode === 'async') return this.flushAsync()
    if (this.flushing) return
    this.flushing = true
    try {
      for (;;) {
        const round = this.collectRound()
        if (!round.length) break
        this.runRound(round)
      }
    } finally {
      this.flushing = false
    }
  }

  flushAsync() {
    if (this.flushing) return
    this.flushing = true
    let round
    try {
      round = this.collectRound()
    } catch (e) {
      this.flushing = false
      throw e
    }
    if (!round.length) { this.flushing = false; return }
    this.runRoundAsync(round, () => { this.flushing = false; this.flushAsync() })
  }

  // resolves when every queued job has run
  idle() {
    return new Promise((resolve) => {
      const check = () => (this.queues.size || this.flushing || this.scheduled ? setImmediate(check) : resolve())
      check()
    })
  }

  // One applyChanges per document of the round: the documents of each store (device shard x
  // stride) go to that store as one batch; every store's batch is submitted before any is
  // waited for, so the devices merge at once.
  runRound(round) {
    const { pending, errors } = this.submitRound(round)
    for (const p of pending) this.finishStore(p, addon.wait(p.store, p.id), errors)
    this.raise(errors)
  }

  runRoundAsync(round, done) {
    let sub
    try {
      sub = this.submitRound(round)
    } catch (e) {
      done()
      throw e
    }
    const { pending, errors } = sub
    let left = pending.length
    const finish = () => { try { this.raise(errors) } finally { done() } }
    if (!left) { finish(); return }
    for (const p of pending) {
      addon.waitAsync(p.store, p.id, (err, r) => {
        try {
          if (err) {
            p.items.forEach(({ state, job, snap, moved }) => { if (!moved) state.enc.restore(snap); errors.push([job, err]) })
          } else this.finishStore(p, r, errors)
        } finally {
          if (--left === 0) finish()
        }
      })
    }
  }

  submitRound(round) {
    const groups = new Map()         // store -> [{state, job, snap, append, moved}]
    const errors = []
    for (const [state, job] of round) {
      const snap = state.enc.snapshot()
      let a = state.enc.encode(job.changes, job.extraActors)
      let moved = null
      if (a.nActors > state.stride) {
        // a new actor outgrew the document's store: re-merge its whole log in a wider one
        state.enc.restore(snap)
        const stride = STRIDES.find((x) => x >= a.nActors)
        if (stride === undefined) {
          errors.push([job, new Error(`document has ${a.nActors} actors > ${STRIDES[STRIDES.length - 1]}`)])
          continue
        }
        const enc = new C.DocEncoder(this.pool)
        const store = this.storeFor(state.shard, stride)
        a = enc.encode(state.log.concat(job.changes), job.extraActors)
        moved = { enc, store, stride, handle: addon.openDoc(store) }
      }
      const store = moved ? moved.store : state.store
      if (!groups.has(store)) groups.set(store, [])
      groups.get(store).push({ state, job, snap, append: a, moved })
    }
    const pending = []
    for (const [store, items] of groups) {
      const stride = items[0].moved ? items[0].moved.stride : items[0].state.stride
      const b = C.buildBatch(items.map((it) => it.append), stride)
      const handles = Uint32Array.from(items.map((it) => (it.moved ? it.moved.handle : it.state.handle)))
      pending.push({ store, stride, items, id: addon.submit(store, b.docs, b.changes, b.deps, b.ops, handles, b.remap) })
    }
    return { pending, errors }
  }

  finishStore({ store, stride: S, items }, r, errors) {
    this.submits++
    const ok = []
    items.forEach((it, i) => {
      const { state, job, snap, moved, append } = it
      const res = C.readDocResult(r.docs, i)
      if (res.status !== 0) {
        if (!moved) state.enc.restore(snap)
        errors.push([job, this.errorFor(state, job.changes, res)])
        return
      }
      if (moved) {
        Object.assign(state, { enc: moved.enc, store: moved.store, stride: moved.stride, handle: moved.handle })
        state.objType = null           // ids re-encoded: rebuilt from the log at the next patch
        this.restrides++
      }
      const base = state.log.length
      state.log.push(...job.changes)
      for (const c of job.changes) for (const op of c.ops || []) state.opActor.push([op, c.actor])
      // objects this round created (make ops, first creation wins)
      state.newObjs = []
      if (state.objType && !moved) {
        for (let k = 0; k < append.ops.length / C.OP_ROW; k++) {
          const act = append.ops[k * C.OP_ROW + 16]
          if (act > C.ACTIONS.makeText) continue
          const o = append.ops.readUInt32LE(k * C.OP_ROW)
          if (!state.objType.has(o)) { state.objType.set(o, act); state.newObjs.push(o) }
        }
      }
      const prevHist = state.histLen, prevQueued = state.nQueued, prevSeq = state.roundSeq
      state.roundSeq++
      state.histLen = res.histLen
      state.nQueued = res.nQueued
      state.clock = Clock.fromRow(r.clock, i * S * 4, state.enc.actors)
      state.deps = Clock.fromRow(r.heads, i * S * 4, state.enc.actors)
      const backClock = Clock.fromRow(r.backClock, i * S * 4, state.enc.actors)
      state.backClock = backClock
      // incremental patch: the view is current up to the previous round (a fresh document's
      // view is the empty root map) and every new change applied
      if (state.view === null && prevSeq === 0 && state.patchedSeq === 0)
        state.view = new Map([[C.ROOT_ID, { type: 'map', keys: new Map(), elems: [] }]])
      const simple = !moved && state.view !== null && state.objType !== null && state.patchedSeq === prevSeq &&
        prevQueued === 0 && res.nQueued === 0 && res.histLen - prevHist === job.changes.length
      ok.push({ state, job, res, append, simple, payload: { res, base, prevHist, backClock, minCmp: Clock.CMP_CODES[res.minCmp] } })
    })
    if (this.patches) this.prefetchRegs(store, ok)
    for (const e of ok) e.job.done(e.payload)
  }

  // one read of the registers the round's new ops hit, for every simple document of the store
  prefetchRegs(store, ok) {
    const docs = [], regs = [], owners = []
    let cap = 0
    for (const e of ok) {
      const st = e.state
      st.pendingRegs = null
      if (!e.simple) continue
      st.pendingRegs = []
      const seen = new Set()
      for (let k = 0; k < e.append.ops.length / C.OP_ROW; k++) {
        const act = e.append.ops[k * C.OP_ROW + 16]
        if (act < C.ACTIONS.set) continue                   // make / ins: no visible value of their own
        const g = e.append.ops.readUInt32LE(k * C.OP_ROW + 4)
        if (g === C.NONE || seen.has(g)) continue
        seen.add(g)
        docs.push(st.handle); regs.push(g); owners.push(st)
      }
      cap += e.res.nSurv
    }
    if (!regs.length) return
    const rr = addon.readRegs(store, Uint32Array.from(docs), Uint32Array.from(regs), cap)
    for (let q = 0; q < regs.length; q++) {
      const b = q * C.REG_RESULT
      const n = rr.regs.readUInt32LE(b), off = rr.regs.readUInt32LE(b + 4)
      const surv = []
      for (let x = 0; x < n; x++) {
        const sb = (off + x) * C.SURV_RESULT
        surv.push([rr.surv.readUInt32LE(sb), rr.surv.readUInt32LE(sb + 4), rr.surv.readUInt32LE(sb + 8), rr.surv.readUInt32LE(sb + 12)])
      }
      owners[q].pendingRegs.push({ g: regs[q], n, li: rr.regs.readInt32LE(b + 8), o: rr.regs.readUInt32LE(b + 12), surv })
    }
  }

  raise(errors) {
    for (const [job, err] of errors) {
      if (job.fail) job.fail(err)
      else if (this.onError) this.onError(err)
      else throw err
    }
  }

  errorFor(state, changes, res) {
    const text = ERR_TEXT[res.status] || `engine status ${res.status}`
    const all = state.log.concat(changes)
    const c = res.errChange < all.length ? all[res.errChange] : null
    let detail = ''
    if (c && res.status === 1) detail = ` ${c.seq} by ${c.actor}`
    else if (c && res.errOp !== C.NONE && c.ops && c.ops[res.errOp]) {
      const op = c.ops[res.errOp]
      detail = res.status === 4 ? ` ${c.actor}:${op.elem}` : res.status === 5 ? ` ${op.key}` : ` ${op.obj}`
    }
    const e = new Error(text + detail)
    e.status = res.status
    return e
  }

  // Synchronous single-document applyChanges (Backend.applyChanges)
  applyChanges(state, changes) {
    if (this.mode === 'async' && this.flushing) throw new Error('GpuEngine.applyChanges while an async round is in flight')
    let out = null, err = null
    const prevMode = this.mode
    this.mode = 'sync'
    try {
      this.enqueue(state, { changes, done: (r) => { out = r }, fail: (e) => { err = e } })
    } finally {
      this.mode = prevMode
    }
    if (err) throw err
    return out
  }

  // ---- the node-wide ClockStore feed (CursorMessage clocks, src/RepoBackend.ts:374-392) ----
  // Every shard's documents' DocBackend.clock entries as repo-global records
  // (FNV-1a64(docId), FNV-1a64(actorId), seq) gathered across the devices over RCCL
  // (hm_comm_create_local + hm_clock_exchange_host) when they are distinct GPUs, and
  // turned back into {docId: {actorId: seq}} with the host's id tables.
  exchangeClocks(states) {
    const perShard = this.shards.map(() => [])
    const ids = new Map()
    for (const st of states) {
      const dk = fnv1a64(st.docId)
      ids.set(dk, st.docId)
      for (const [a, s] of Object.entries(st.backClock)) {
        const ak = fnv1a64(a)
        ids.set(ak, a)
        perShard[st.shard].push([dk, ak, s])
      }
    }
    const bufs = perShard.map((rows) => {
      const b = Buffer.alloc(rows.length * 24)
      rows.forEach(([dk, ak, s], i) => { b.writeBigUInt64LE(dk, 24 * i); b.writeBigUInt64LE(ak, 24 * i + 8); b.writeUInt32LE(s, 24 * i + 16) })
      return b
    })
    let all
    const distinct = new Set(this.devices).size === this.devices.length
    if (distinct) {
      if (!this.comm) this.comm = addon.commCreateLocal(this.shards.map((sh) => this.storeFor(this.shards.indexOf(sh), this.minStride)))
      all = addon.clockExchange(this.comm, bufs)
    } else all = Buffer.concat(bufs)           // shards sharing one device: the host holds them all
    const out = {}
    for (let i = 0; i < all.length / 24; i++) {
      const doc = ids.get(all.readBigUInt64LE(24 * i)), actor = ids.get(all.readBigUInt64LE(24 * i + 8))
      const c = out[doc] || (out[doc] = {})
      const s = all.readUInt32LE(24 * i + 16)
      if (!(actor in c) || s > c[actor]) c[actor] = s
    }
    return out
  }
}

// ---------------- patches (Automerge makePatch, consumed by Frontend.applyPatch) ----------------
// clock / deps are applied-only (queued changes excluded).  `diffs` turn the frontend's copy of
// the document from the state of the previous patch into the current one, in the Automerge 0.12
// diff vocabulary (SURVEY.md Appendix A.4): {action:'create', obj, type},
// {action:'set'|'remove', type:'map'|'table', obj, key, value, link?, datatype?, conflicts?},
// {action:'insert'|'set'|'remove', type:'list'|'text', obj, index, elemId?, value, ...}.
// They are derived from the GPU's merged registers (one diff per changed register / element,
// removals before insertions), not replayed op by op: the document a frontend builds from them
// equals the merged state, but the diff sequence is not Automerge's per-op sequence (parity of
// that sequence is unpinned: Automerge 0.12 is not available here).
const TYPE_OF = { 0: 'map', 1: 'table', 2: 'list', 3: 'text' }
const DT_NAME = { 1: 'counter', 2: 'timestamp' }
const TWO32 = 4294967296

function opValue(state, vtag, lo, hi) {
  switch (vtag) {
    case C.V.NULL: return { value: null }
    case C.V.FALSE: return { value: false }
    case C.V.TRUE: return { value: true }
    case C.V.INT: return { value: hi >= 0x80000000 ? (hi - TWO32) * TWO32 + lo : hi * TWO32 + lo }
    case C.V.FLOAT: { const b = Buffer.alloc(8); b.writeUInt32LE(lo, 0); b.writeUInt32LE(hi, 4); return { value: b.readDoubleLE(0) } }
    case C.V.STR: return { value: state.engine.pool.strings[lo] }
    case C.V.OBJ: return { value: state.enc.objList[lo], link: true }
    default: throw new Error(`unknown value tag ${vtag}`)
  }
}

function objTypes(state) {
  if (state.objType) return state.objType
  const objType = new Map([[0, 0]])
  for (const [op] of state.opActor) {
    const a = C.ACTIONS[op.action]
    if (a <= C.ACTIONS.makeText) { const o = state.enc.objs.get(op.obj); if (!objType.has(o)) objType.set(o, a) }
  }
  state.objType = objType
  return objType
}

// a register's survivors [[op, vtag, lo, hi]] -> a diff value with conflicts
function entryOf(state, surv) {
  const vals = surv.map(([k, vt, lo, hi]) => {
    const [op, actor] = state.opActor[k]
    const v = opValue(state, vt, lo, hi)
    if (op.datatype) v.datatype = op.datatype
    return [actor, v]
  })
  const entry = Object.assign({}, vals[0][1])
  if (vals.length > 1) entry.conflicts = vals.slice(1).map(([actor, v]) => Object.assign({ actor }, v))
  return entry
}

// the merged document as {objUuid -> {type, keys: Map(key -> entry) | elems: [[elemId, entry]]}}
function materialize(state) {
  const r = addon.read(state.store, state.handle)
  const objType = objTypes(state)
  const view = new Map()
  const nRegs = r.regs.length / C.REG_RESULT
  for (let g = 0; g < nRegs; g++) {
    const b = g * C.REG_RESULT
    const n = r.regs.readUInt32LE(b), off = r.regs.readUInt32LE(b + 4), li = r.regs.readInt32LE(b + 8), o = r.regs.readUInt32LE(b + 12)
    if (!n || o === C.NONE) continue
    const t = objType.has(o) ? objType.get(o) : 0
    const list = t === 2 || t === 3
    if (list && li < 0) continue
    const surv = []
    for (let q = 0; q < n; q++) {
      const sb = (off + q) * C.SURV_RESULT
      surv.push([r.surv.readUInt32LE(sb), r.surv.readUInt32LE(sb + 4), r.surv.readUInt32LE(sb + 8), r.surv.readUInt32LE(sb + 12)])
    }
    const entry = entryOf(state, surv)
    const uuid = state.enc.objList[o]
    let ov = view.get(uuid)
    if (!ov) { ov = { type: TYPE_OF[t], keys: new Map(), elems: [] }; view.set(uuid, ov) }
    const key = state.enc.regList[g][1]
    if (list) ov.elems[li] = [key, entry]
    else ov.keys.set(key, entry)
  }
  // objects created but still empty (a linked empty map/list)
  for (const [o, t] of objType) {
    const uuid = state.enc.objList[o]
    if (!view.has(uuid)) view.set(uuid, { type: TYPE_OF[t], keys: new Map(), elems: [] })
  }
  return view
}

// the previous view advanced by the registers the round's ops hit (state.pendingRegs): the
// same diffs diffViews would give for them — objects created, list removals (descending
// index), insertions (ascending final index), then value changes
function applyRegs(state) {
  const view = state.view, diffs = [], sig = (e) => JSON.stringify(e)
  for (const o of state.newObjs) {
    const uuid = state.enc.objList[o]
    if (view.has(uuid)) continue
    const t = TYPE_OF[state.objType.get(o)]
    view.set(uuid, { type: t, keys: new Map(), elems: [] })
    if (uuid !== C.ROOT_ID) diffs.push({ action: 'create', obj: uuid, type: t })
  }
  const lists = new Map()
  for (const r of state.pendingRegs) {
    if (r.o === C.NONE) continue
    const t = state.objType.has(r.o) ? state.objType.get(r.o) : 0
    const list = t === 2 || t === 3
    const uuid = state.enc.objList[r.o]
    let ov = view.get(uuid)
    if (!ov) { ov = { type: TYPE_OF[t], keys: new Map(), elems: [] }; view.set(uuid, ov) }
    const key = state.enc.regList[r.g][1]
    const entry = r.n ? entryOf(state, r.surv) : null
    if (!list) {
      const old = ov.keys.get(key)
      if (!entry) {
        if (old !== undefined) { ov.keys.delete(key); diffs.push({ action: 'remove', type: ov.type, obj: uuid, key }) }
      } else if (old === undefined || sig(old) !== sig(entry)) {
        ov.keys.set(key, entry)
        diffs.push(Object.assign({ action: 'set', type: ov.type, obj: uuid, key }, entry))
      }
      continue
    }
    let L = lists.get(uuid)
    if (!L) { L = { ov, rem: [], ins: [], set: [] }; lists.set(uuid, L) }
    const visible = r.n > 0 && r.li >= 0
    const oldIdx = ov.elems.findIndex((e) => e[0] === key)
    if (oldIdx >= 0 && !visible) L.rem.push(oldIdx)
    else if (oldIdx < 0 && visible) L.ins.push([r.li, key, entry])
    else if (visible && sig(ov.elems[oldIdx][1]) !== sig(entry)) L.set.push([key, entry])
  }
  for (const [uuid, L] of lists) {
    L.rem.sort((a, b) => b - a).forEach((i) => {
      L.ov.elems.splice(i, 1)
      diffs.push({ action: 'remove', type: L.ov.type, obj: uuid, index: i })
    })
    L.ins.sort((a, b) => a[0] - b[0]).forEach(([i, key, e]) => {
      L.ov.elems.splice(i, 0, [key, e])
      diffs.push(Object.assign({ action: 'insert', type: L.ov.type, obj: uuid, index: i, elemId: key }, e))
    })
    L.set.forEach(([key, e]) => {
      const i = L.ov.elems.findIndex((x) => x[0] === key)
      L.ov.elems[i] = [key, e]
      diffs.push(Object.assign({ action: 'set', type: L.ov.type, obj: uuid, index: i }, e))
    })
  }
  return diffs
}

function diffViews(prev, next) {
  const diffs = []
  const sig = (e) => JSON.stringify(e)
  for (const [uuid, ov] of next) if (uuid !== C.ROOT_ID && !prev.has(uuid)) diffs.push({ action: 'create', obj: uuid, type: ov.type })
  for (const [uuid, ov] of next) {
    const po = prev.get(uuid) || { keys: new Map(), elems: [] }
    if (ov.type === 'list' || ov.type === 'text') {
      const keep = new Set(ov.elems.map(([id]) => id))
      const was = new Map(po.elems.map(([id, e], i) => [id, [i, e]]))
      for (let i = po.elems.length - 1; i >= 0; i--)
        if (!keep.has(po.elems[i][0])) diffs.push({ action: 'remove', type: ov.type, obj: uuid, index: i })
      ov.elems.forEach(([id, e], i) => {
        if (!was.has(id)) diffs.push(Object.assign({ action: 'insert', type: ov.type, obj: uuid, index: i, elemId: id }, e))
      })
      ov.elems.forEach(([id, e], i) => {
        if (was.has(id) && sig(was.get(id)[1]) !== sig(e)) diffs.push(Object.assign({ action: 'set', type: ov.type, obj: uuid, index: i }, e))
      })
    } else {
      const keys = Array.from(new Set([...po.keys.keys(), ...ov.keys.keys()])).sort()
      for (const k of keys) {
        const a = po.keys.get(k), b = ov.keys.get(k)
        if (b === undefined) diffs.push({ action: 'remove', type: ov.type, obj: uuid, key: k })
        else if (a === undefined || sig(a) !== sig(b)) diffs.push(Object.assign({ action: 'set', type: ov.type, obj: uuid, key: k }, b))
      }
    }
  }
  return diffs
}

function makePatch(state) {
  let diffs = []
  if (state.engine.patches && state.patchedSeq !== state.roundSeq) {
    if (state.view && state.pendingRegs && state.objType) {
      diffs = applyRegs(state)
      state.incrementalPatches = (state.incrementalPatches || 0) + 1
    } else {
      const view = materialize(state)
      diffs = diffViews(state.view || new Map(), view)
      state.view = view
    }
    state.patchedSeq = state.roundSeq
    state.pendingRegs = null
  }
  return { clock: Object.assign({}, state.clock), deps: Object.assign({}, state.deps), canUndo: false, canRedo: false, diffs }
}

function makeBackend(engine) {
  return {
    init: (docId) => engine.init(docId),
    applyChanges: (state, changes) => {
      engine.applyChanges(state, changes)
      return [state, makePatch(state)]
    },
    getPatch: (state) => makePatch(state),
  }
}

class DocBackend {
  constructor(documentId, notify, back, engine) {
    this.id = documentId
    this.actorId = undefined
    this.clock = {}
    this.back = undefined
    this.changes = new Map()
    this.ready = new Channel('doc:back:readyQ')
    this.notify = notify
    this.minimumClock = undefined
    this.minimumClockSatisfied = false
    this.localChangeQ = new Channel('doc:back:localChangeQ')
    this.remoteChangesQ = new Channel('doc:back:remoteChangesQ')
    this.engine = engine || (back && back.engine) || DocBackend.defaultEngine()
    if (back) {
      this.back = back
      this.actorId = documentId                           // rootActorId(documentId)
      this.ready.subscribe((f) => f())
      this.minimumClockSatisfied = true
      this.subscribeToRemoteChanges()
      this.subscribeToLocalChanges()
      this.notify({ type: 'ReadyMsg', id: this.id, minimumClockSatisfied: this.minimumClockSatisfied,
        actorId: this.actorId, history: this.back.histLen })
    }
  }

  static defaultEngine() {
    if (!DocBackend._engine) DocBackend._engine = new GpuEngine({})
    return DocBackend._engine
  }

  testMinimumClockSatisfied() {
    if (this.minimumClock) {
      const t = Clock.cmp(this.clock, this.minimumClock)
      this.minimumClockSatisfied = t === 'GT' || t === 'EQ'
    }
  }

  updateMinimumClock(clock) {
    if (this.minimumClockSatisfied) return
    this.minimumClock = Clock.union(clock, this.minimumClock || {})
    this.testMinimumClockSatisfied()
  }

  applyRemoteChanges(changes) { this.remoteChangesQ.push(changes) }

  applyLocalChange(change) { this.localChangeQ.push(change) }

  initActor(actorId) {
    if (this.back) {
      this.actorId = this.actorId || actorId
      this.notify({ type: 'ActorIdMsg', id: this.id, actorId: this.actorId })
    }
  }

  updateClock(changes) {
    changes.forEach((change) => {
      const old = this.clock[change.actor] || 0
      this.clock[change.actor] = Math.max(old, change.seq)
    })
    if (!this.minimumClockSatisfied) this.testMinimumClockSatisfied()
  }

  init(changes, actorId) {
    const state = this.engine.init(this.id)
    this.engine.enqueue(state, { changes, done: () => {
      this.actorId = this.actorId || actorId
      this.back = state
      this.updateClock(changes)
      this.minimumClockSatisfied = changes.length > 0
      const patch = makePatch(state)
      this.ready.subscribe((f) => f())
      this.subscribeToLocalChanges()
      this.subscribeToRemoteChanges()
      // ReadyMsg after the buffered remote changes drained above (per-document FIFO)
      this.engine.enqueue(state, { changes: null, done: () => {
        this.notify({ type: 'ReadyMsg', id: this.id, minimumClockSatisfied: this.minimumClockSatisfied,
          actorId: this.actorId, patch, history: this.back.histLen })
      } })
    } })
  }

  subscribeToRemoteChanges() {
    this.remoteChangesQ.subscribe((changes) => {
      this.engine.enqueue(this.back, { changes, done: () => {
        this.updateClock(changes)
        this.notify({ type: 'RemotePatchMsg', id: this.id, minimumClockSatisfied: this.minimumClockSatisfied,
          patch: makePatch(this.back), history: this.back.histLen })
      } })
    })
  }

  subscribeToLocalChanges() {
    this.localChangeQ.subscribe((change) => {
      // Backend.applyLocalChange: the change must extend its actor's sequence
      const cur = this.back.clock[change.actor] || 0
      if (change.seq <= cur) throw new Error(`Change request has already been applied: ${change.actor}:${change.seq}`)
      this.engine.enqueue(this.back, { changes: [change], done: () => {
        this.updateClock([change])
        const patch = Object.assign(makePatch(this.back), { actor: change.actor, seq: change.seq })
        this.notify({ type: 'LocalPatchMsg', id: this.id, actorId: this.actorId,
          minimumClockSatisfied: this.minimumClockSatisfied, change, patch, history: this.back.histLen })
      } })
    })
  }
}

// ClockStore with the reference's semantics (src/ClockStore.ts:24-112, SQL upsert-max per
// entry, zero entries stored and returned, updateQ pushed when the input differs from the
// stored clock), in host memory (better-sqlite3 is not part of this engine).
class ClockStore {
  constructor(engine) {
    this.engine = engine || null
    this.rows = new Map()            // repoId \0 docId -> Map(actorId -> seq)
    this.updateQ = new Channel('clockstore:updateQ')
  }

  key(repoId, docId) { return repoId + '\u0000' + docId }

  get(repoId, docId) {
    const m = this.rows.get(this.key(repoId, docId))
    const c = {}
    if (m) Array.from(m.keys()).sort(byteOrder).forEach((a) => { c[a] = m.get(a) })
    return c
  }

  getMultiple(repoId, docIds) {
    return docIds.reduce((acc, d) => { acc[d] = this.get(repoId, d); return acc }, {})
  }

  update(repoId, docId, clock) {
    const k = this.key(repoId, docId)
    let m = this.rows.get(k)
    if (!m) { m = new Map(); this.rows.set(k, m) }
    for (const [a, s] of Object.entries(clock)) {
      if (!m.has(a) || s > m.get(a)) m.set(a, s)
    }
    const stored = this.get(repoId, docId)
    const d = [repoId, docId, stored]
    if (!Clock.equal(clock, stored)) this.updateQ.push(d)
    return d
  }

  set(repoId, docId, clock) {
    this.rows.delete(this.key(repoId, docId))
    return this.update(repoId, docId, clock)
  }

  getAllDocumentIds(repoId) {
    const out = []
    for (const k of this.rows.keys()) { const [r, d] = k.split('\u0000'); if (r === repoId) out.push(d) }
    return out
  }

  getAllRepoIds() { return Array.from(new Set(Array.from(this.rows.keys()).map((k) => k.split('\u0000')[0]))) }

  // ClockStore.update(repoId, doc.id, doc.clock) for many GPU documents at once
  // (src/RepoBackend.ts:343-345): the device upsert-max decides which rows change
  // (written) and which inputs differ from the stored clock (updateQ).
  updateDocs(repoId, docs) {
    if (!docs.length) return []
    // one device upsert-max per store holding some of the documents
    const byStore = new Map()
    docs.forEach((doc, i) => {
      const st = doc.back.store
      if (!byStore.has(st)) byStore.set(st, [])
      byStore.get(st).push(i)
    })
    const out = new Array(docs.length)
    for (const [store, idx] of byStore) {
      const handles = Uint32Array.from(idx.map((i) => docs[i].back.handle))
      const r = addon.clockUpdate(store, handles)
      const S = docs[idx[0]].back.stride
      idx.forEach((i, j) => {
        const doc = docs[i]
        const actors = doc.back.enc.actors
        const k = this.key(repoId, doc.id)
        if (r.written[j]) {
          const stored = Clock.fromRow(r.stored, j * S * 4, actors)
          let m = this.rows.get(k)
          if (!m) { m = new Map(); this.rows.set(k, m) }
          for (const [a, s] of Object.entries(stored)) if (!m.has(a) || s > m.get(a)) m.set(a, s)
        }
        const d = [repoId, doc.id, this.get(repoId, doc.id)]
        if (r.differs[j]) this.updateQ.push(d)
        out[i] = d
      })
    }
    return out
  }
}

// SQLite's BINARY collation (memcmp of UTF-8) orders the Clocks primary key
function byteOrder(a, b) { return Buffer.compare(Buffer.from(a, 'utf8'), Buffer.from(b, 'utf8')) }

module.exports = { GpuEngine, GpuBackendState, DocBackend, ClockStore, makeBackend, materialize, fnv1a64, addon }
