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
//   GpuEngine    one docset per device (N-API addon -> hm_docset_* in include/hypermerge_amd.h):
//                every document's applyChanges calls run as batched rounds, per-document FIFO
//                job queues, one hm_docset_apply per device and round over all documents
//                with work.  The docset does everything per document natively: the blocks'
//                JSON (Actor.parseBlock, src/Actor.ts:137-141), the interning, the merge on
//                the GPU, the patch diffs and clocks (rendered as JSON, one JSON.parse per
//                round here).  Changes may be handed over as Change objects (stringified
//                here), JSON strings or raw hypercore blocks (Buffers: '{"' JSON or 'BR' +
//                brotli), the last skipping Actor.parseBlock altogether.
//                mode 'sync' runs the round inside the caller's stack (the reference's Queue
//                semantics: a push runs the merge synchronously); mode 'batched' once per
//                event-loop turn (setImmediate) over every document that received changes
//                during the turn; mode 'async' the same with the round on the docset's host
//                thread (completion through a napi_threadsafe_function), so the event loop
//                never blocks on decode, the GPU or the patch rendering.
//   ClockStore   the reference's clock table semantics (src/ClockStore.ts:24-112) kept in
//                host memory, with updateDocs(): ClockStore.update(repo, doc, doc.clock)
//                for many documents from one GPU upsert-max per device.
//   CursorStore  the reference's cursor table (src/CursorStore.ts:19-91) on the device, batched,
//                and syncPlan(): RepoBackend.syncChanges' ranges (src/RepoBackend.ts:506-531).
//
// A document's applyChanges that throws (e.g. 'Inconsistent reuse of sequence number') is
// rolled back natively and rethrown here, like the reference's throw out of
// Backend.applyChanges leaves DocBackend.back unchanged.

const path = require('path')
const addon = require(path.join(__dirname, '..', '_lib', 'hmgpu.node'))
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
const NONE = 0xffffffff
const RESULT_U32 = 8                   // hm_doc_result: 32 B

// a log entry as the docset takes it: raw block (Buffer), JSON text, or a Change object
const toBlock = (c) => (Buffer.isBuffer(c) || typeof c === 'string' ? c : JSON.stringify(c))
// ... and as the reference's history holds it (Block.unpack, src/Block.ts:18-29)
const zlib = require('zlib')
function toChange(c) {
  if (typeof c === 'string') return JSON.parse(c)
  if (!Buffer.isBuffer(c)) return c
  const header = c.slice(0, 2).toString()
  if (header === '{"') return JSON.parse(c.toString())
  if (header === 'BR') return JSON.parse(zlib.brotliDecompressSync(c.slice(2)).toString())
  throw new Error(`fail to unpack blocks - head is '${header}'`)
}

// A round's results as the docset renders them: JSON text ('{"p": ...}') or the HMP1 binary
// form (include/hypermerge_amd.h, HM_DOCSET_BINARY) -> {p: [patch], b: [log clock], c: [call clock]}
// per document of the call.  The binary form builds the same objects JSON.parse would, without
// the parse (the round's strings decoded once, numbers read from a Float64Array).
const TYPES = ['map', 'table', 'list', 'text']
const ACTIONS = ['create', 'set', 'remove', 'insert']
// One round's decoder state (module level: no closures per document — the per-op diff form
// makes millions of small objects per round, and the garbage collector is the JS thread's
// largest cost)
const R = { w: null, nums: null, strs: null, p: 0, sb: 0, nb: 0, tag: 0, dt: 0 }
// Clock objects ({actorId: seq}).  Hypermerge mints an actor per document, so a process holds
// thousands of distinct actor ids; object literals keyed by them give V8 a hidden-class
// transition per new key from the empty shape, and past its transition limit every clock built
// falls to the slow path (C2 with base58 ids: clocks 4x slower than in dictionary mode, and the
// maps' garbage).  Once more than 1024 distinct actor ids have been seen, clocks start in
// dictionary mode (an object literal whose two placeholder keys are deleted: Object.prototype
// stays, insertion order stays); with a few shared actors the literal form is faster (3x) and stays.
const CK = { dict: false, seen: new Set(), probes: 0 }
function noteActor(a) {
  const s = CK.seen
  if (!s) return
  s.add(a)
  if (s.size > 1024) { CK.dict = true; CK.seen = null } else if (++CK.probes > 65536) CK.seen = null
}
function newClock() {
  if (!CK.dict) return {}
  const c = { _a: 0, _b: 0 }
  delete c._a
  delete c._b
  return c
}
// a long-lived clock made before the switch, moved to the dictionary form (once per object)
function dictCopy(o) {
  const c = newClock()
  for (const k in o) c[k] = o[k]
  return c
}
function rdClock() {
  const w = R.w, strs = R.strs, sb = R.sb
  const c = newClock()
  let p = R.p
  if (CK.seen) {
    for (let k = w[p]; k > 0; k--) noteActor(strs[sb + w[p + 2 * k - 1]])
  }
  for (let k = w[p++]; k > 0; k--) { c[strs[sb + w[p]]] = w[p + 1]; p += 2 }
  R.p = p
  return c
}
// into an existing object (a clock that only grows: every key it had stays)
function rdClockInto(c) {
  const w = R.w, strs = R.strs, sb = R.sb
  let p = R.p
  for (let k = w[p++]; k > 0; k--) { c[strs[sb + w[p]]] = w[p + 1]; p += 2 }
  R.p = p
}
function skipClock() { R.p += 1 + 2 * R.w[R.p] }
// One docset call's HMP1 results, read document by document: decodeRound(buf, n).advance(d,
// state) moves a document's state to the round's end (clocks, deps), .message(d, state) builds
// its patch (clock, deps, diffs) and the round's clock.  finish() advances every document first
// and builds each patch only when it is delivered, so a round's patch and diff objects die young
// instead of all being live at once (and promoted by the collector) across the delivery loop.
class RoundReader {
  constructor(buf, n) {
    if (buf.byteOffset % 8) buf = Buffer.from(buf)           // a fresh, aligned copy
    const u = new Uint32Array(buf.buffer, buf.byteOffset, buf.length >>> 2)
    if (u[0] !== 0x31504d48 || u[1] !== n) throw new Error('docset results: bad HMP1 header')
    const ns = u[2], nw = u[3], nn = u[4], blobBytes = u[5], ascii = u[6]
    let at = 8
    this.woff = u.subarray(at, at + n + 1); at += n + 1
    this.sbase = u.subarray(at, at + n + 1); at += n + 1
    this.nbase = u.subarray(at, at + n + 1); at += n + 1
    const soff = u.subarray(at, at + ns + 1); at += ns + 1
    this.w = u.subarray(at, at + nw); at += nw
    const numsAt = ((4 * at + 7) >> 3) << 3
    this.nums = new Float64Array(buf.buffer, buf.byteOffset + numsAt, nn)
    const blobAt = numsAt + 8 * nn
    const strs = this.strs = new Array(ns)
    if (ascii) {
      const text = buf.toString('latin1', blobAt, blobAt + blobBytes)
      for (let i = 0; i < ns; i++) strs[i] = text.substring(soff[i], soff[i + 1])
    } else {
      for (let i = 0; i < ns; i++) strs[i] = buf.toString('utf8', blobAt + soff[i], blobAt + soff[i + 1])
    }
    this.at = new Uint32Array(n)                             // each document's first diff word
  }

  enter(d, p) { R.w = this.w; R.nums = this.nums; R.strs = this.strs; R.p = p; R.sb = this.sbase[d]; R.nb = this.nbase[d] }
  leave() { R.w = R.nums = R.strs = null }

  // pass 1, every document of the call: its state advanced from its head — the opSet clock and
  // DocBackend.clock updated in place (they only grow), deps a fresh object — so nothing else
  // is held across the call's deliveries (objects that live through a young-generation
  // collection are promoted, and the old generation's collections cost the JS thread most)
  advance(d, state) {
    if (this.woff[d] === this.woff[d + 1]) return false
    if (CK.dict && !state.dictClocks) {
      state.clock = dictCopy(state.clock)
      state.backClock = dictCopy(state.backClock)
      state.dictClocks = true
    }
    this.enter(d, this.woff[d])
    rdClockInto(state.clock)
    state.deps = rdClock()
    rdClockInto(state.backClock)
    skipClock()
    this.at[d] = R.p
    this.leave()
    return true
  }

  // pass 2, just before the document's delivery: its patch and the round's clock
  message(d, state) {
    this.enter(d, this.woff[d])
    const clock = rdClock()
    skipClock(); skipClock()
    const c = rdClock()
    this.leave()
    return { patch: { clock, deps: state.deps, canUndo: state.canUndo, canRedo: state.canRedo, diffs: this.diffs(d) }, c }
  }

  diffs(d) {
    this.enter(d, this.at[d])
    const w = R.w, strs = R.strs, sb = R.sb
    const nd = w[R.p++]
    const diffs = new Array(nd)
    for (let k = 0; k < nd; k++) {
      const h = w[R.p++], action = h & 7, t = (h >>> 3) & 3
      const obj = strs[sb + w[R.p++]]
      let e
      if (action === 0) e = { action: 'create', obj, type: TYPES[t] }
      else if (t < 2) {
        if (action === 1) e = setDiff(TYPES[t], obj, strs[sb + w[R.p++]])
        else e = { action: ACTIONS[action], type: TYPES[t], obj, key: strs[sb + w[R.p++]] }
      } else if (action === 3) {
        const index = w[R.p++]
        e = insertDiff(TYPES[t], obj, index, strs[sb + w[R.p++]])
      } else if (action === 1) {
        e = setIndexDiff(TYPES[t], obj, w[R.p++])
      } else e = { action: ACTIONS[action], type: TYPES[t], obj, index: w[R.p++] }
      diffs[k] = e
    }
    this.leave()
    return diffs
  }
}

// The value-carrying diffs, built whole: the entry (value, datatype, link, conflicts) is read
// first and the object created with exactly its fields, so no property is added after the
// literal (an added property costs an out-of-object backing store per diff).
function rdVal() {
  const v = R.w[R.p++]
  const dt = (v >>> 3) & 3
  R.tag = v & 7; R.dt = dt === 3 ? 0 : dt
  const pay = v >>> 5
  switch (R.tag) {
    case 1: return false
    case 2: return true
    case 3: case 4: return R.nums[R.nb + pay]
    case 5: case 6: return R.strs[R.sb + pay]
    default: return null
  }
}
function rdConflicts(k) {
  const cs = new Array(k - 1)
  for (let i = 1; i < k; i++) {
    const actor = R.strs[R.sb + R.w[R.p++]]
    const value = rdVal()
    let c
    if (R.tag === 6) c = R.dt ? { actor, value, link: true, datatype: DTS[R.dt] } : { actor, value, link: true }
    else c = R.dt ? { actor, value, datatype: DTS[R.dt] } : { actor, value }
    cs[i - 1] = c
  }
  return cs
}
const DTS = [undefined, 'counter', 'timestamp', undefined]
function setDiff(type, obj, key) {
  const k = R.w[R.p++]
  const value = rdVal(), tag = R.tag, dt = R.dt
  const conflicts = k > 1 ? rdConflicts(k) : null
  if (conflicts === null) {
    if (tag === 6) return { action: 'set', type, obj, key, value, link: true }
    return dt ? { action: 'set', type, obj, key, value, datatype: DTS[dt] } : { action: 'set', type, obj, key, value }
  }
  if (tag === 6) return { action: 'set', type, obj, key, value, link: true, conflicts }
  return dt ? { action: 'set', type, obj, key, value, datatype: DTS[dt], conflicts } : { action: 'set', type, obj, key, value, conflicts }
}
function setIndexDiff(type, obj, index) {
  const k = R.w[R.p++]
  const value = rdVal(), tag = R.tag, dt = R.dt
  const conflicts = k > 1 ? rdConflicts(k) : null
  const e = tag === 6 ? { action: 'set', type, obj, index, value, link: true }
    : dt ? { action: 'set', type, obj, index, value, datatype: DTS[dt] } : { action: 'set', type, obj, index, value }
  if (conflicts !== null) e.conflicts = conflicts
  return e
}
function insertDiff(type, obj, index, elemId) {
  const k = R.w[R.p++]
  const value = rdVal(), tag = R.tag, dt = R.dt
  const e = tag === 6 ? { action: 'insert', type, obj, index, elemId, value, link: true }
    : dt ? { action: 'insert', type, obj, index, elemId, value, datatype: DTS[dt] } : { action: 'insert', type, obj, index, elemId, value }
  if (k > 1) e.conflicts = rdConflicts(k)
  return e
}

// a JSON results buffer (the docset's debug form) read through the same interface
class JsonRoundReader {
  constructor(j) { this.j = j }
  advance(d, state) {
    const p = this.j.p[d]
    if (!p) return false
    Object.assign(state.clock, p.clock)
    state.deps = p.deps
    Object.assign(state.backClock, this.j.b[d])
    return true
  }
  message(d, state) {
    return { patch: Object.assign({}, this.j.p[d], { deps: state.deps, canUndo: state.canUndo, canRedo: state.canRedo }), c: this.j.c[d] }
  }
}

function decodeRound(buf, n) {
  if (buf.length === 0 || buf[0] === 0x7b) return new JsonRoundReader(JSON.parse(buf.toString()))
  return new RoundReader(buf, n)
}

class History {
  constructor(state) { this.state = state; this.size = state.histLen }
  slice(a, b) {
    const st = this.state
    const lo = a || 0
    const hi = b === undefined ? this.size : Math.min(b, this.size)
    const idx = addon.docsetHistoryPrefix(st.ds, st.id, Math.max(hi, 0))
    const out = []
    for (let i = lo; i < idx.length / 4; i++) out.push(st.change(idx.readUInt32LE(4 * i)))
    return { toArray: () => out, size: out.length }
  }
}

// FNV-1a 64 over the UTF-8 bytes of an id string: the shard key (and the clock exchange's
// record key) of hypermerge_amd/exchange.py and include/hypermerge_amd.h.
// Computed on two 32-bit halves in plain Numbers (h * prime = h * 0x1b3 + h << 40; every partial
// product stays below 2^53), the BigInt only built at the end.
const TWO32 = 4294967296
function fnvHalves(s) {
  let lo = 0x84222325, hi = 0xcbf29ce4
  const step = (b) => {
    lo = (lo ^ b) >>> 0
    const pl = lo * 0x1b3
    const nlo = pl >>> 0
    hi = (hi * 0x1b3 + Math.floor(pl / TWO32) + (lo & 0xffffff) * 256) >>> 0
    lo = nlo
  }
  let ascii = true
  for (let i = 0; i < s.length && ascii; i++) ascii = s.charCodeAt(i) < 0x80
  if (ascii) for (let i = 0; i < s.length; i++) step(s.charCodeAt(i))
  else for (const b of Buffer.from(s, 'utf8')) step(b)
  return [hi, lo]
}
function fnv1a64(s) {
  const [hi, lo] = fnvHalves(s)
  return (BigInt(hi) << 32n) | BigInt(lo)
}
// fnv1a64(s) % n without the BigInt ((hi * 2^32 + lo) mod n, n < 2^21)
function fnvMod(s, n) {
  const [hi, lo] = fnvHalves(s)
  return ((hi % n) * (TWO32 % n) + (lo % n)) % n
}

// The per-document BackendState: a document of its shard's docset plus the log entries as
// they were handed over (history slices).  States are linear: applyChanges advances the
// document in place and returns the same state object.
// key -> id string of every id a host has keyed: a 64-bit key that two different ids share is
// an error, never a silent merge of two actors' cursors or clocks (the reference keys its
// Cursors / Clocks rows by the id strings themselves, src/CursorStore.ts, src/ClockStore.ts)
class KeyTable {
  constructor(hash) { this.hash = hash || fnv1a64; this.ids = new Map() }
  key(s) {
    const k = this.hash(s)
    const old = this.ids.get(k)
    if (old === undefined) this.ids.set(k, s)
    else if (old !== s) throw new Error(`FNV-1a64 key collision: ${JSON.stringify(old)} and ${JSON.stringify(s)} (key ${k})`)
    return k
  }
  id(k) { return this.ids.get(k) }
}

class GpuBackendState {
  constructor(engine, docId) {
    this.engine = engine
    this.docId = docId
    this.shard = docId === undefined ? 0 : engine.shardOf(docId)
    this.ds = engine.docsets[this.shard]
    this.id = addon.docsetOpen(this.ds, 1)
    this.log = []
    this.histLen = 0
    this.nQueued = 0
    this.clock = newClock()
    this.deps = newClock()
    this.backClock = newClock()      // max seq per actor over the whole log (queued included)
    this.dictClocks = CK.dict
    // Automerge's local undo history (applyLocalChange, SURVEY Appendix A.4): undoStack of op
    // lists, undoPos, redoStack; canUndo = undoPos > 0, canRedo = redoStack not empty
    this.undoStack = []
    this.undoPos = 0
    this.redoStack = []
  }

  get canUndo() { return this.undoPos > 0 }
  get canRedo() { return this.redoStack.length > 0 }

  change(i) {
    const c = this.log[i]
    if (c !== null && typeof c === 'object' && !Buffer.isBuffer(c)) return c
    const o = toChange(c)
    this.log[i] = o
    return o
  }

  get stride() { return addon.docsetInfo(this.ds, this.id).aStride }

  getIn(p) {
    if (p.length === 2 && p[0] === 'opSet' && p[1] === 'history') return new History(this)
    if (p.length === 2 && p[0] === 'opSet' && p[1] === 'clock') return Object.assign({}, this.clock)
    if (p.length === 2 && p[0] === 'opSet' && p[1] === 'deps') return Object.assign({}, this.deps)
    throw new Error(`GpuBackendState.getIn: unsupported path ${JSON.stringify(p)}`)
  }
}

class GpuEngine {
  // opts: devices (HIP ordinals; documents shard over them by FNV-1a64(docId) % devices.length),
  // mode 'sync' | 'batched' | 'async', patches (diffs on), threads (host threads per docset),
  // onError, hash (tests: a key function to force collisions)
  constructor(opts) {
    const o = opts || {}
    this.devices = o.devices || [o.device || 0]
    this.mode = o.mode || 'batched'
    this.patches = o.patches !== false
    // diffs: 'ops' (Automerge's per-op sequence in application order) or 'net' (the diffs that
    // take the previous patch's document to this one)
    this.diffs = o.diffs || 'ops'
    this.docsets = this.devices.map((d) => addon.docsetCreate(d, o.threads || 0, this.patches, o.binary !== false,
      this.diffs === 'net'))
    this.queues = new Map()          // state -> FIFO of jobs
    this.flushing = false
    this.scheduled = false
    this.onError = o.onError || null
    this.submits = 0
    this.comm = null
    this.slice = o.slice || 4096     // documents per docset call in async mode (pipelined)
    this.hash = o.hash || null       // the id -> 64-bit key function of the clock exchange (default FNV-1a64)
  }

  shardOf(docId) { return fnvMod(docId, this.docsets.length) }

  init(docId) { return new GpuBackendState(this, docId) }

  stats() {
    const t = { calls: 0, docs: 0, moves: 0, hitPatches: 0, fullPatches: 0, opPatches: 0, replayMismatch: 0,
      incremental: 0, remerged: 0, handedBack: 0 }
    for (const ds of this.docsets) { const s = addon.docsetStats(ds); for (const k in t) t[k] += s[k] }
    t.dictClocks = CK.dict                      // (clocks in dictionary form: > 1024 actor ids seen)
    return t
  }

  get restrides() { return this.stats().moves }

  // job: {entries|null, done(payload|null), fail(err)}
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
    const prepErrors = []            // (requests whose preparation threw: raised with the round)
    for (;;) {
      const round = []
      round.prepErrors = prepErrors
      for (const [state, q] of Array.from(this.queues)) {
        while (q.length && q[0].entries === null) q.shift().done(null)
        if (!q.length) { this.queues.delete(state); continue }
        const job = q.shift()
        if (job.prepare) {
          // (a local undo / redo request: its ops from the document as every earlier round left it)
          try {
            job.prepare()
          } catch (e) {
            prepErrors.push([job, e])
            continue
          }
        }
        round.push([state, job])
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
        if (!round.length) { this.raise(round.prepErrors); break }
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
    if (!round.length) { this.flushing = false; this.raise(round.prepErrors); return }
    this.runRoundAsync(round, () => { this.flushing = false; this.flushAsync() })
  }

  // resolves when every queued job has run
  idle() {
    return new Promise((resolve) => {
      const check = () => (this.queues.size || this.flushing || this.scheduled ? setImmediate(check) : resolve())
      check()
    })
  }

  // the round's documents grouped by docset (device shard), in slices of at most `slice`
  // documents (async mode queues the slices on the docset's host thread, so the main thread
  // hands over the next slice and builds the previous one's messages while a slice merges)
  groups(round, slice) {
    const g = new Map()
    for (const [state, job] of round) {
      let x = g.get(state.ds)
      if (!x) { x = []; g.set(state.ds, x) }
      x.push({ state, job })
    }
    const out = []
    for (const [ds, items] of g) {
      const k = slice || items.length
      for (let a = 0; a < items.length; a += k) out.push({ ds, items: items.slice(a, a + k) })
    }
    return out
  }

  // the call's blocks packed into one Buffer (block end offsets, first block per document):
  // the addon copies it once instead of visiting every block through N-API
  static prepare(g) {
    const n = g.items.length
    g.ids = Uint32Array.from(g.items, (it) => it.state.id)
    const bufs = []
    g.docBlock = new Uint32Array(n + 1)
    for (let i = 0; i < n; i++) {
      const e = g.items[i].job.entries
      for (let k = 0; k < e.length; k++) {
        const c = e[k]
        bufs.push(Buffer.isBuffer(c) ? c : Buffer.from(typeof c === 'string' ? c : JSON.stringify(c), 'utf8'))
      }
      g.docBlock[i + 1] = bufs.length
    }
    g.ends = new Uint32Array(bufs.length)
    let at = 0
    for (let b = 0; b < bufs.length; b++) { at += bufs[b].length; g.ends[b] = at }
    if (at >= 2 ** 32) throw new RangeError('docset call over 4 GB of blocks')
    g.data = Buffer.concat(bufs, at)
    return g
  }

  // One applyChanges per document of the round, one docset call per device
  runRound(round) {
    const errors = round.prepErrors ? round.prepErrors.slice() : []
    for (const g of this.groups(round, 0)) {
      GpuEngine.prepare(g)
      this.finish(g, addon.docsetApplyPacked(g.ds, g.ids, g.data, g.ends, g.docBlock), errors)
    }
    this.raise(errors)
  }

  runRoundAsync(round, done) {
    let gs
    try {
      gs = this.groups(round, this.slice)
    } catch (e) {
      done()
      throw e
    }
    const errors = round.prepErrors ? round.prepErrors.slice() : []
    let left = gs.length
    const finish = () => { try { this.raise(errors) } finally { done() } }
    for (const g of gs) {
      GpuEngine.prepare(g)
      // in place: prepare() built g.data for this call alone and nothing touches it again
      addon.docsetApplyPacked(g.ds, g.ids, g.data, g.ends, g.docBlock, (err, r) => {
        try {
          if (err) g.items.forEach(({ job }) => errors.push([job, err]))
          else this.finish(g, r, errors)
        } finally {
          if (--left === 0) finish()
        }
      }, true)
    }
  }

  finish({ items }, r, errors) {
    this.submits++
    const res = new Uint32Array(r.results.buffer, r.results.byteOffset, r.results.length / 4)
    const j = decodeRound(r.data, items.length)
    const ok = []
    items.forEach(({ state, job }, i) => {
      const status = res[RESULT_U32 * i] | 0
      if (status !== 0) {
        errors.push([job, this.errorFor(state, job.entries, status, res[RESULT_U32 * i + 1], res[RESULT_U32 * i + 2])])
        return
      }
      for (const c of job.entries) state.log.push(c)
      state.histLen = res[RESULT_U32 * i + 3]
      state.nQueued = res[RESULT_U32 * i + 4]
      if (j.advance(i, state)) ok.push(i)
    })
    // every state of the call is advanced before the first delivery; each patch is built just
    // before it is delivered
    for (const i of ok) {
      const { state, job } = items[i]
      const m = j.message(i, state)
      job.done({ patch: m.patch, roundClock: m.c, backClock: state.backClock, minCmp: null })
    }
  }

  raise(errors) {
    for (const [job, err] of errors) {
      if (job.fail) job.fail(err)
      else if (this.onError) this.onError(err)
      else throw err
    }
  }

  // the reference's Error for a document whose round failed (status, change index, op index)
  errorFor(state, entries, status, errChange, errOp) {
    if (status === 32) {
      // a block that does not decode: the throw of Block.unpack / JSON.parse (src/Block.ts:18-29)
      const c = entries[errChange]
      try {
        toChange(toBlock(c))
      } catch (e) {
        return e
      }
      const e = new Error('Malformed change: not an Automerge 0.12 change')
      e.status = status
      return e
    }
    const text = ERR_TEXT[status] || `engine status ${status}`
    const n = state.log.length
    let c = null
    try {
      c = errChange < n ? state.change(errChange) : errChange - n < entries.length ? toChange(entries[errChange - n]) : null
    } catch (_) { c = null }
    let detail = ''
    if (c && status === 1) detail = ` ${c.seq} by ${c.actor}`
    else if (c && errOp !== NONE && c.ops && c.ops[errOp]) {
      const op = c.ops[errOp]
      detail = status === 4 ? ` ${c.actor}:${op.elem}` : status === 5 ? ` ${op.key}` : ` ${op.obj}`
    }
    const e = new Error(text + detail)
    e.status = status
    return e
  }

  // Synchronous single-document applyChanges (Backend.applyChanges)
  applyChanges(state, changes) {
    if (this.mode === 'async' && this.flushing) throw new Error('GpuEngine.applyChanges while an async round is in flight')
    let out = null, err = null
    const prevMode = this.mode
    this.mode = 'sync'
    try {
      this.enqueue(state, { entries: changes, done: (r) => { out = r }, fail: (e) => { err = e } })
    } finally {
      this.mode = prevMode
    }
    if (err) throw err
    return out
  }

  // ---- the node-wide ClockStore feed (CursorMessage clocks, src/RepoBackend.ts:374-392) ----
  // Every shard's documents' clock entries as repo-global records (FNV-1a64(docId),
  // FNV-1a64(actorId), seq) gathered across the devices over RCCL (hm_comm_create_local +
  // hm_clock_exchange_host) when they are distinct GPUs, and turned back into
  // {docId: {actorId: seq}} with the host's id tables.
  exchangeClocks(states) {
    const perShard = this.docsets.map(() => [])
    const ids = this.keys || (this.keys = new KeyTable(this.hash))
    for (const st of states) {
      const dk = ids.key(st.docId)
      for (const [a, s] of Object.entries(st.backClock)) perShard[st.shard].push([dk, ids.key(a), s])
    }
    const bufs = perShard.map((rows) => {
      const b = Buffer.alloc(rows.length * 24)
      rows.forEach(([dk, ak, s], i) => { b.writeBigUInt64LE(dk, 24 * i); b.writeBigUInt64LE(ak, 24 * i + 8); b.writeUInt32LE(s, 24 * i + 16) })
      return b
    })
    let all
    const distinct = new Set(this.devices).size === this.devices.length
    if (distinct) {
      if (!this.comm) this.comm = addon.commCreateLocalDocsets(this.docsets)
      all = addon.clockExchange(this.comm, bufs)
    } else all = Buffer.concat(bufs)           // shards sharing one device: the host holds them all
    const out = {}
    for (let i = 0; i < all.length / 24; i++) {
      const doc = ids.id(all.readBigUInt64LE(24 * i)), actor = ids.id(all.readBigUInt64LE(24 * i + 8))
      const c = out[doc] || (out[doc] = {})
      const s = all.readUInt32LE(24 * i + 16)
      if (!(actor in c) || s > c[actor]) c[actor] = s
    }
    return out
  }
}

// ---------------- patches (Automerge makePatch, consumed by Frontend.applyPatch) ----------------
// Each round's patch comes from the docset: clock / deps are applied-only (queued changes
// excluded); `diffs` turn the frontend's copy of the document from the state of the previous
// patch into the current one, in the Automerge 0.12 diff vocabulary (SURVEY.md Appendix A.4):
// {action:'create', obj, type}, {action:'set'|'remove', type:'map'|'table', obj, key, value,
// link?, datatype?, conflicts?}, {action:'insert'|'set'|'remove', type:'list'|'text', obj,
// index, elemId?, value, ...}.  By default one diff per applied op, in application order (the
// sequence Automerge's applyChanges emits, Appendix A.4; the docset replays the round's ops over
// the patch base, csrc/docset.cpp Replay); with the docset's net-diff option (HM_DOCSET_NET_DIFFS)
// one diff per register whose rendered value changed instead.  The document a frontend builds
// from either equals the merged state; Automerge 0.12's own diff field set is unpinned (it is not
// available here).

// the merged document as {objUuid -> {type, keys: Map(key -> entry), elems: [[elemId, entry]]}}
function materialize(state) {
  const v = JSON.parse(addon.docsetView(state.ds, state.id))
  const view = new Map()
  for (const [uuid, ov] of Object.entries(v)) view.set(uuid, { type: ov.type, keys: new Map(ov.keys), elems: ov.elems })
  return view
}

// Backend.getPatch(state): the whole document as diffs from an empty one
function fullPatch(state) {
  const diffs = []
  for (const [uuid, ov] of materialize(state)) {
    if (uuid !== '00000000-0000-0000-0000-000000000000') diffs.push({ action: 'create', obj: uuid, type: ov.type })
  }
  for (const [uuid, ov] of materialize(state)) {
    for (const [key, e] of ov.keys) diffs.push(Object.assign({ action: 'set', type: ov.type, obj: uuid, key }, e))
    ov.elems.forEach(([elemId, e], index) => diffs.push(Object.assign({ action: 'insert', type: ov.type, obj: uuid, index, elemId }, e)))
  }
  return { clock: dictCopy(state.clock), deps: dictCopy(state.deps), canUndo: state.canUndo,
    canRedo: state.canRedo, diffs }
}

const emptyPatch = (state) => ({ clock: dictCopy(state.clock), deps: dictCopy(state.deps),
  canUndo: state.canUndo, canRedo: state.canRedo, diffs: [] })

// ---------------- local undo / redo (Backend.applyLocalChange, src/DocBackend.ts:187-205) ----------------
// Automerge 0.12 records, for every set / del / link / inc of an undoable local change, the ops
// that restore the field it touches: an inc's negation, else the field's current ops (action,
// obj, key, value, datatype) or a del when it has none; the list goes on undoStack at undoPos
// (the redo stack is cleared).  An 'undo' request applies undoStack[undoPos - 1] as its ops and
// pushes the ops that restore the fields they touch onto redoStack; a 'redo' request applies the
// top of redoStack.  (SURVEY Appendix A.4 [R]: recollected, parity unpinned.)  The field
// states come from the merged document (the docset's view, read when the request reaches the
// head of its document's queue: every earlier round of the document has applied); the fields a
// request touches twice see its own earlier ops, which are concurrent with later ones of the same
// change (so a later set keeps the earlier one as a conflict).
function viewField(view, obj, key) {
  const ov = view[obj]
  if (!ov) return []
  let e = null
  if (ov.type === 'list' || ov.type === 'text') { for (const [id, x] of ov.elems) if (id === key) { e = x; break } } else {
    for (const [k, x] of ov.keys) if (k === key) { e = x; break }
  }
  if (!e) return []
  const one = (x) => {
    const o = { action: x.link ? 'link' : 'set', obj, key, value: x.value }
    if (x.datatype) o.datatype = x.datatype
    return o
  }
  return [one(e)].concat((e.conflicts || []).map(one))
}

const UNDO_ACTIONS = new Set(['set', 'del', 'link', 'inc'])

// the undo ops of an undoable local change's ops, in op order
function undoOpsOf(view, ops) {
  const sim = new Map()                       // obj \0 key -> {prior: [...], own: [...]}
  const out = []
  for (const op of ops || []) {
    if (!UNDO_ACTIONS.has(op.action)) continue
    const k = op.obj + '\u0000' + op.key
    let f = sim.get(k)
    if (!f) { f = { prior: viewField(view, op.obj, op.key), own: [] }; sim.set(k, f) }
    if (op.action === 'inc') {
      out.push({ action: 'inc', obj: op.obj, key: op.key, value: -op.value })
      // the inc adds to the counters it causally follows: the field's earlier ops, not this change's
      f.prior = f.prior.map((o) => (o.datatype === 'counter' && typeof o.value === 'number' ? Object.assign({}, o, { value: o.value + op.value }) : o))
      continue
    }
    const cur = f.own.concat(f.prior)
    if (cur.length) for (const o of cur) out.push(Object.assign({}, o))
    else out.push({ action: 'del', obj: op.obj, key: op.key })
    // set / link / del remove the field's earlier ops (this change causally follows them) and keep
    // this change's own (concurrent with each other: one change)
    f.prior = []
    if (op.action === 'set' || op.action === 'link') {
      const o = { action: op.action, obj: op.obj, key: op.key, value: op.value }
      if (op.datatype) o.datatype = op.datatype
      f.own.unshift(o)
    }
  }
  return out
}

// the ops that restore the fields an undo change's ops touch (the redo ops), from the fields before it
function redoOpsOf(view, ops) {
  const out = []
  for (const op of ops) {
    if (op.action === 'inc') { out.push({ action: 'inc', obj: op.obj, key: op.key, value: -op.value }); continue }
    const cur = viewField(view, op.obj, op.key)
    if (cur.length) for (const o of cur) out.push(o)
    else out.push({ action: 'del', obj: op.obj, key: op.key })
  }
  return out
}

function makeBackend(engine) {
  return {
    init: (docId) => engine.init(docId),
    applyChanges: (state, changes) => {
      const r = engine.applyChanges(state, changes)
      return [state, r ? r.patch : emptyPatch(state)]
    },
    getPatch: (state) => fullPatch(state),
  }
}

class DocBackend {
  constructor(documentId, notify, back, engine) {
    this.id = documentId
    this.actorId = undefined
    this.clock = newClock()
    this.dictClock = CK.dict
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

  // changes: Change objects (the reference's), or raw hypercore blocks / JSON texts of them
  applyRemoteChanges(changes) { this.remoteChangesQ.push(changes) }

  // the blocks of an actor feed as downloaded (Actor.onDownload -> syncChanges without parseBlock)
  applyRemoteBlocks(blocks) { this.remoteChangesQ.push(blocks) }

  applyLocalChange(change) { this.localChangeQ.push(change) }

  initActor(actorId) {
    if (this.back) {
      this.actorId = this.actorId || actorId
      this.notify({ type: 'ActorIdMsg', id: this.id, actorId: this.actorId })
    }
  }

  // DocBackend.updateClock (src/DocBackend.ts:135-142) from the max seq per actor of the
  // handed changes (queued ones included), which the docset reports per round
  updateClock(roundClock) {
    if (CK.dict && !this.dictClock) { this.clock = dictCopy(this.clock); this.dictClock = true }
    for (const a in roundClock) {
      const old = this.clock[a] || 0
      this.clock[a] = Math.max(old, roundClock[a])
    }
    if (!this.minimumClockSatisfied) this.testMinimumClockSatisfied()
  }

  init(changes, actorId) {
    const state = this.engine.init(this.id)
    this.engine.enqueue(state, { entries: changes, done: (r) => {
      this.actorId = this.actorId || actorId
      this.back = state
      this.updateClock(r.roundClock)
      this.minimumClockSatisfied = changes.length > 0
      const patch = r.patch
      this.ready.subscribe((f) => f())
      this.subscribeToLocalChanges()
      this.subscribeToRemoteChanges()
      // ReadyMsg after the buffered remote changes drained above (per-document FIFO)
      this.engine.enqueue(state, { entries: null, done: () => {
        this.notify({ type: 'ReadyMsg', id: this.id, minimumClockSatisfied: this.minimumClockSatisfied,
          actorId: this.actorId, patch, history: this.back.histLen })
      } })
    } })
  }

  subscribeToRemoteChanges() {
    this.remoteChangesQ.subscribe((changes) => {
      this.engine.enqueue(this.back, { entries: changes, done: (r) => {
        this.updateClock(r.roundClock)
        this.notify({ type: 'RemotePatchMsg', id: this.id, minimumClockSatisfied: this.minimumClockSatisfied,
          patch: r.patch, history: this.back.histLen })
      } })
    })
  }

  subscribeToLocalChanges() {
    this.localChangeQ.subscribe((change) => {
      // Backend.applyLocalChange: the change must extend its actor's sequence
      const cur = this.back.clock[change.actor] || 0
      if (change.seq <= cur) throw new Error(`Change request has already been applied: ${change.actor}:${change.seq}`)
      // requestType 'change' (a request without one is taken as a change), 'undo' or 'redo'
      const type = change.requestType === undefined ? 'change' : change.requestType
      if (type !== 'change' && type !== 'undo' && type !== 'redo') throw new RangeError(`Unknown requestType: ${type}`)
      const state = this.back
      let after = null
      const job = { entries: [change], done: (r) => {
        if (after) after()
        this.updateClock(r.roundClock)
        const patch = Object.assign(r.patch, { actor: change.actor, seq: change.seq, canUndo: state.canUndo,
          canRedo: state.canRedo })
        this.notify({ type: 'LocalPatchMsg', id: this.id, actorId: this.actorId,
          minimumClockSatisfied: this.minimumClockSatisfied, change, patch, history: this.back.histLen })
      } }
      const undoable = type === 'change' && change.undoable !== false
      if (undoable || type !== 'change') {
        // run when the request heads its document's queue (every earlier round applied)
        job.prepare = () => {
          const view = JSON.parse(addon.docsetView(state.ds, state.id))
          if (type === 'change') {
            const ops = undoOpsOf(view, change.ops)
            after = () => {
              state.undoStack = state.undoStack.slice(0, state.undoPos).concat([ops])
              state.undoPos++
              state.redoStack = []
            }
            return
          }
          let ops
          if (type === 'undo') {
            ops = state.undoPos > 0 ? state.undoStack[state.undoPos - 1] : undefined
            if (!ops) throw new RangeError('Cannot undo: there is nothing to be undone')
            const redo = redoOpsOf(view, ops)
            after = () => { state.undoPos--; state.redoStack = state.redoStack.concat([redo]) }
          } else {
            ops = state.redoStack[state.redoStack.length - 1]
            if (!ops) throw new RangeError('Cannot redo: the last change was not an undo')
            after = () => { state.undoPos++; state.redoStack = state.redoStack.slice(0, -1) }
          }
          // the change the engine applies: the request's actor / seq / deps / message with these ops
          const c = { actor: change.actor, seq: change.seq, deps: change.deps || {} }
          if (change.message !== undefined) c.message = change.message
          c.ops = ops
          job.entries = [c]
        }
      }
      this.engine.enqueue(this.back, job)
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
    this.writes = []                 // rows written since the last takeBatch (the persistence batch)
  }

  // The Clocks rows this store wrote since the last call, in order, for one SQL transaction
  // (INTEGRATION.md §3): ['upsert', repoId, docId, actorId, seq] for every row an upsert-max
  // changed or inserted, ['delete', repoId, docId] for set()'s clear.  Replayed through the
  // reference's statements (src/ClockStore.ts:37-48) they give the table this store holds.
  takeBatch() { const b = this.writes; this.writes = []; return b }

  upsert(m, repoId, docId, a, s) {
    if (!m.has(a) || s > m.get(a)) { m.set(a, s); this.writes.push(['upsert', repoId, docId, a, s]) }
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
    for (const [a, s] of Object.entries(clock)) this.upsert(m, repoId, docId, a, s)
    const stored = this.get(repoId, docId)
    const d = [repoId, docId, stored]
    if (!Clock.equal(clock, stored)) this.updateQ.push(d)
    return d
  }

  set(repoId, docId, clock) {
    if (this.rows.delete(this.key(repoId, docId))) this.writes.push(['delete', repoId, docId])
    return this.update(repoId, docId, clock)
  }

  getAllDocumentIds(repoId) {
    const out = []
    for (const k of this.rows.keys()) { const [r, d] = k.split('\u0000'); if (r === repoId) out.push(d) }
    return out
  }

  getAllRepoIds() { return Array.from(new Set(Array.from(this.rows.keys()).map((k) => k.split('\u0000')[0]))) }

  // ClockStore.update(repoId, doc.id, doc.back's clock) for many GPU documents at once
  // (src/RepoBackend.ts:343-345): the device upsert-max decides which rows change
  // (written) and which inputs differ from the stored clock (updateQ).  Not while an async
  // round is in flight on the documents' device (the docset refuses the call).
  updateDocs(repoId, docs) {
    if (!docs.length) return []
    const byDs = new Map()
    docs.forEach((doc, i) => {
      const ds = doc.back.ds
      if (!byDs.has(ds)) byDs.set(ds, [])
      byDs.get(ds).push(i)
    })
    const out = new Array(docs.length)
    for (const [ds, idx] of byDs) {
      const r = addon.docsetClockUpdate(ds, Uint32Array.from(idx, (i) => docs[i].back.id))
      const stored = JSON.parse(r.json)
      idx.forEach((i, j) => {
        const doc = docs[i]
        const k = this.key(repoId, doc.id)
        if (r.written[j]) {
          let m = this.rows.get(k)
          if (!m) { m = new Map(); this.rows.set(k, m) }
          for (const [a, s] of Object.entries(stored[j])) this.upsert(m, repoId, doc.id, a, s)
        }
        const d = [repoId, doc.id, this.get(repoId, doc.id)]
        if (r.differs[j]) this.updateQ.push(d)
        out[i] = d
      })
    }
    return out
  }
}

// SQLite's BINARY collation (memcmp of UTF-8) orders the Clocks / Cursors primary keys
function byteOrder(a, b) { return Buffer.compare(Buffer.from(a, 'utf8'), Buffer.from(b, 'utf8')) }

// CursorStore (src/CursorStore.ts:19-91) on the device: one table per repo, documents as dense
// rows, actors as FNV-1a64 keys (the clock exchange's); every batched form is one launch.
const INFINITY_SEQ = Number.MAX_SAFE_INTEGER
class CursorStore {
  constructor(engine, maxActorsPerDoc, opts) {
    this.engine = engine
    this.K = maxActorsPerDoc || 64
    this.tables = new Map()          // repoId -> {c, rows: Map(docId -> row), docs: []}
    this.actors = new KeyTable(opts && opts.hash)
    this.updateQ = new Channel('cursorstore:updateQ')
    this.writes = []
  }

  // The Cursors upserts since the last call, for one SQL transaction (INTEGRATION.md §3):
  // ['upsert', repoId, docId, actorId, boundedSeq] per entry handed to update, in order — the
  // statements src/CursorStore.ts:51-64 runs, batched across calls.
  takeBatch() { const b = this.writes; this.writes = []; return b }

  table(repoId) {
    let t = this.tables.get(repoId)
    if (!t) { t = { c: addon.cursorsCreate(this.engine.docsets[0], this.K), rows: new Map(), docs: [] }; this.tables.set(repoId, t) }
    return t
  }

  row(t, docId) {
    let r = t.rows.get(docId)
    if (r === undefined) { r = t.docs.length; t.rows.set(docId, r); t.docs.push(docId); addon.cursorsReserve(t.c, t.docs.length) }
    return r
  }

  key(actorId) { return this.actors.key(actorId) }

  getMany(repoId, docIds) {
    const t = this.table(repoId)
    const have = docIds.filter((d) => t.rows.has(d))
    const out = new Map()
    if (have.length) {
      const g = addon.cursorsGet(t.c, Uint32Array.from(have, (d) => t.rows.get(d)))
      have.forEach((d, i) => {
        const n = g.count.readUInt32LE(4 * i)
        const ent = []
        for (let e = 0; e < n; e++) {
          const o = 8 * (i * this.K + e)
          ent.push([this.actors.id(g.actors.readBigUInt64LE(o)), Number(g.seqs.readBigUInt64LE(o))])
        }
        ent.sort((a, b) => byteOrder(a[0], b[0]))            // SELECT * in primary-key order
        out.set(d, Object.fromEntries(ent))
      })
    }
    return docIds.map((d) => out.get(d) || {})
  }

  get(repoId, docId) { return this.getMany(repoId, [docId])[0] }

  // CursorStore.update for many documents in one launch: {docId: cursor} -> descriptors
  updateMany(repoId, cursors) {
    const t = this.table(repoId)
    const docs = Object.keys(cursors)
    const off = new Uint32Array(docs.length + 1)
    const keys = [], seqs = []
    docs.forEach((d, i) => {
      for (const [a, s] of Object.entries(cursors[d])) { keys.push(this.key(a)); seqs.push(s) }
      off[i + 1] = keys.length
    })
    docs.forEach((d) => {
      for (const [a, s] of Object.entries(cursors[d]))
        this.writes.push(['upsert', repoId, d, a, Math.max(0, Math.min(s, INFINITY_SEQ))])
    })
    const rows = Uint32Array.from(docs, (d) => this.row(t, d))
    const differs = addon.cursorsUpdate(t.c, rows, off, BigUint64Array.from(keys), Float64Array.from(seqs))
    const stored = this.getMany(repoId, docs)
    return docs.map((d, i) => {
      const desc = [stored[i], d, repoId]
      if (differs[i]) this.updateQ.push(desc)
      return desc
    })
  }

  update(repoId, docId, cursor) { return this.updateMany(repoId, { [docId]: cursor })[0] }

  addActor(repoId, docId, actorId, seq) {
    const s = seq === undefined ? INFINITY_SEQ : Math.max(0, Math.min(seq, INFINITY_SEQ))
    return this.update(repoId, docId, { [actorId]: s })
  }

  // CursorStore.entry for many (docId, actorId) pairs in one launch
  entries(repoId, pairs) {
    const t = this.table(repoId)
    const idx = pairs.map(([d], i) => (t.rows.has(d) ? i : -1)).filter((i) => i >= 0)
    const out = new Array(pairs.length).fill(0)
    if (idx.length) {
      const got = addon.cursorsEntry(t.c, Uint32Array.from(idx, (i) => t.rows.get(pairs[i][0])),
        BigUint64Array.from(idx, (i) => this.key(pairs[i][1])))
      idx.forEach((i, j) => { out[i] = Number(got.readBigUInt64LE(8 * j)) })
    }
    return out
  }

  entry(repoId, docId, actorId) { return this.entries(repoId, [[docId, actorId]])[0] }

  // docsWithActor for many actors in one launch: [[docId, actorId, storedSeq]]
  docsWithActors(repoId, actorSeqs) {
    const t = this.table(repoId)
    const names = Object.keys(actorSeqs)
    if (!names.length || !t.docs.length) return []
    const r = addon.cursorsDocsWithActors(t.c, BigUint64Array.from(names, (a) => this.key(a)), Float64Array.from(names, (a) => actorSeqs[a]))
    const out = []
    for (let i = 0; i < r.rows.length / 4; i++)
      out.push([t.docs[r.rows.readUInt32LE(4 * i)], names[r.actors.readUInt32LE(4 * i)], Number(r.seqs.readBigUInt64LE(8 * i))])
    return out
  }

  docsWithActor(repoId, actorId, seq) {
    return this.docsWithActors(repoId, { [actorId]: seq || 0 }).map((x) => x[0]).sort(byteOrder)
  }
}

// RepoBackend.syncChanges (src/RepoBackend.ts:506-531) for many synced actors at once: for
// every open document whose cursor has the actor, the block range [min, end) it receives:
// min = doc.changes.get(actor) || 0, end = the first block missing from the actor's feed
// (present[actor]: downloaded flags) at or after min, below the cursor entry.  One
// docsWithActor launch and one contiguity launch; the caller sets doc.changes[actor] = end and
// hands the blocks [min, end) to applyRemoteChanges / applyRemoteBlocks when end > min.
function syncPlan(engine, cursors, repoId, actors, docs, present) {
  const hits = cursors.docsWithActors(repoId, Object.fromEntries(actors.map((a) => [a, 0]))).filter(([d]) => docs.has(d))
  if (!hits.length) return []
  const feeds = Array.from(new Set(hits.map((h) => h[1])))
  const fidx = new Map(feeds.map((a, i) => [a, i]))
  const wordOff = new BigUint64Array(feeds.length + 1)
  feeds.forEach((a, i) => { wordOff[i + 1] = wordOff[i] + BigInt(Math.ceil(present[a].length / 64)) })
  const words = new BigUint64Array(Number(wordOff[feeds.length]) + 1)
  feeds.forEach((a, i) => {
    const f = present[a], base = Number(wordOff[i])
    for (let j = 0; j < f.length; j++) if (f[j]) words[base + (j >> 6)] |= 1n << BigInt(j & 63)
  })
  const lo = Uint32Array.from(hits, ([d, a]) => docs.get(d).changes.get(a) || 0)
  const hi = Uint32Array.from(hits, ([, a, s], i) => Math.max(Math.min(s, present[a].length, 0xffffffff), lo[i]))
  const off = BigUint64Array.from(hits, ([, a]) => wordOff[fidx.get(a)])
  const end = addon.syncRanges(engine.docsets[0], words, off, lo, hi)
  return hits.map(([d, a], i) => [d, a, lo[i], end.readUInt32LE(4 * i)]).sort((x, y) => byteOrder(x[0] + '\0' + x[1], y[0] + '\0' + y[1]))
}

module.exports = { GpuEngine, GpuBackendState, DocBackend, ClockStore, CursorStore, KeyTable, syncPlan, makeBackend,
  materialize, fnv1a64, addon, toChange, decodeRound }
