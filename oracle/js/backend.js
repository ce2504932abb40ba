'use strict'
// oracle/js/backend.js — TEST / BASELINE INFRASTRUCTURE ONLY.  A from-scratch JavaScript
// restatement of the Automerge 0.12 backend the reference drives (Backend.init /
// Backend.applyChanges, called at src/DocBackend.ts:148,172), over plain JS Maps, plus a
// DocBackend restatement (src/DocBackend.ts:46-213) that calls it synchronously the way the
// reference's Queue does (push runs the subscriber, src/Queue.ts:38-57).  It is the
// "JS restatement" CPU baseline of BASELINE.md (baseline 2): one Node thread, the same
// DocBackend message API as the GPU drop-in.  Nothing in hypermerge_amd/ loads it.
//
// Rules (SURVEY.md Appendix A, the same restatement oracle/oracle.c follows; parity with
// Automerge itself is unpinned — Automerge 0.12 is not vendored in the reference):
//   A.1 addChange -> queue; applyQueuedOps passes until no change applies; causallyReady;
//       duplicate (actor, seq) must have equal content; allDeps = transitiveDeps fold in deps
//       key order then {actor: seq-1} whose set overrides the max; deps heads; clock; history.
//   A.2 applyAssign: survivors = the concurrent prior ops, push set/link, stable
//       sortBy(actor) then reverse after every assign; inc adds to causally prior counter sets.
//   A.3 applyInsert / updateListElement / getPrevious / insertionsAfter (lamport order desc).
// Actor order is JS string order, as Immutable's sortBy compares actor ids.

const ROOT = '00000000-0000-0000-0000-000000000000'

function canon(v) {
  if (v === null || typeof v !== 'object') return JSON.stringify(v === 0 ? 0 : v)
  if (Array.isArray(v)) return '[' + v.map(canon).join(',') + ']'
  return '{' + Object.keys(v).sort().map((k) => JSON.stringify(k) + ':' + canon(v[k])).join(',') + '}'
}

class OpSet {
  constructor() {
    this.clock = new Map()        // actor -> seq (applied)
    this.deps = new Map()         // heads
    this.states = new Map()       // actor -> [{change, allDeps: Map, text}]
    this.history = []
    this.queue = []
    this.objs = new Map([[ROOT, { type: 'map', keys: new Map(), following: new Map(), insertion: new Map(), elemIds: [] }]])
    // local undo history (Backend.applyLocalChange, Appendix A.4 [R]): undoLocal collects the undo
    // ops of the change being applied undoably
    this.undoStack = []
    this.undoPos = 0
    this.redoStack = []
    this.undoLocal = null
  }
}

// a field's current ops as undo / redo ops: action, obj, key, value, datatype
function fieldOps(s, objId, key) {
  const obj = s.objs.get(objId)
  const ops = obj ? obj.keys.get(key) || [] : []
  return ops.map((o) => {
    const r = { action: o.action, obj: o.obj, key: o.key, value: o.value }
    if (o.datatype) r.datatype = o.datatype
    return r
  })
}

// recordUndoHistory: the ops that restore the field an op of an undoable local change touches
function recordUndo(s, op) {
  if (!s.undoLocal) return
  if (op.action === 'inc') { s.undoLocal.push({ action: 'inc', obj: op.obj, key: op.key, value: -op.value }); return }
  const f = fieldOps(s, op.obj, op.key)
  if (f.length) s.undoLocal.push(...f)
  else s.undoLocal.push({ action: 'del', obj: op.obj, key: op.key })
}

function allDepsOf(s, actor, seq) { return s.states.get(actor)[seq - 1].allDeps }

function causallyReady(s, c) {
  const deps = Object.assign({}, c.deps || {})
  deps[c.actor] = c.seq - 1
  for (const a of Object.keys(deps)) if ((s.clock.get(a) || 0) < deps[a]) return false
  return true
}

// isConcurrent(opSet, op1, op2)
function isConcurrent(s, o1, o2) {
  const c1 = allDepsOf(s, o1.actor, o1.seq), c2 = allDepsOf(s, o2.actor, o2.seq)
  return (c1.get(o2.actor) || 0) < o2.seq && (c2.get(o1.actor) || 0) < o1.seq
}

function transitiveDeps(s, baseDeps) {
  let deps = new Map()
  for (const a of Object.keys(baseDeps)) {
    const q = baseDeps[a]
    if (q <= 0) continue
    const t = allDepsOf(s, a, q)
    for (const [x, v] of t) if (v > (deps.get(x) || 0)) deps.set(x, v)
    deps.set(a, q)
  }
  return deps
}

function lamportGreater(s, a, b) {             // element ops: (elem, actor) descending
  if (a.elem !== b.elem) return a.elem > b.elem
  return a.actor > b.actor
}

function insertionsAfter(obj, parent) {
  const kids = (obj.following.get(parent) || []).slice()
  kids.sort((x, y) => (lamportGreater(null, x, y) ? -1 : lamportGreater(null, y, x) ? 1 : 0))
  return kids.map((op) => `${op.actor}:${op.elem}`)
}

function getPrevious(obj, elemId) {
  const ins = obj.insertion.get(elemId)
  if (!ins) throw new Error(`Missing index entry for list element ${elemId}`)
  const parent = ins.key
  const kids = insertionsAfter(obj, parent)
  if (kids[0] === elemId) return parent === '_head' ? null : parent
  let prev = null
  for (const k of kids) { if (k === elemId) break; prev = k }
  for (;;) {
    const more = insertionsAfter(obj, prev)
    if (!more.length) return prev
    prev = more[more.length - 1]
  }
}

// a diff's value fields: the winner's value (link / datatype), the other survivors as conflicts
function valueFields(o) {
  const r = { value: o.value }
  if (o.action === 'link') r.link = true
  if (o.datatype) r.datatype = o.datatype
  return r
}
function entryFields(ops) {
  const r = valueFields(ops[0])
  if (ops.length > 1) r.conflicts = ops.slice(1).map((o) => Object.assign({ actor: o.actor }, valueFields(o)))
  return r
}

function updateListElement(s, obj, elemId, diffs, objId) {
  const ops = obj.keys.get(elemId) || []
  let index = obj.elemIds.indexOf(elemId)
  if (index >= 0) {
    if (!ops.length) { obj.elemIds.splice(index, 1); diffs.push({ action: 'remove', type: obj.type, obj: objId, index }) }
    else diffs.push(Object.assign({ action: 'set', type: obj.type, obj: objId, index }, entryFields(ops)))
    return
  }
  if (!ops.length) return
  let prev = elemId
  for (;;) {
    index = -1
    prev = getPrevious(obj, prev)
    if (prev === null) break
    index = obj.elemIds.indexOf(prev)
    if (index >= 0) break
  }
  obj.elemIds.splice(index + 1, 0, elemId)
  diffs.push(Object.assign({ action: 'insert', type: obj.type, obj: objId, index: index + 1, elemId }, entryFields(ops)))
}

function applyAssign(s, op, diffs) {
  const obj = s.objs.get(op.obj)
  if (!obj) throw new Error(`Modification of unknown object ${op.obj}`)
  recordUndo(s, op)
  const prior = obj.keys.get(op.key) || []
  let remaining
  if (op.action === 'inc') {
    remaining = prior.map((o) => (o.action === 'set' && typeof o.value === 'number' && o.datatype === 'counter' &&
      !isConcurrent(s, o, op)) ? Object.assign({}, o, { value: o.value + op.value }) : o)
  } else {
    remaining = prior.filter((o) => isConcurrent(s, o, op))
  }
  if (op.action === 'set' || op.action === 'link') remaining = remaining.concat([op])
  // sortBy(op => op.actor).reverse(): stable ascending by actor, then reversed
  remaining = remaining.map((o, i) => [o, i]).sort((x, y) => (x[0].actor < y[0].actor ? -1 : x[0].actor > y[0].actor ? 1 : x[1] - y[1]))
    .map((x) => x[0]).reverse()
  obj.keys.set(op.key, remaining)
  if (obj.type === 'list' || obj.type === 'text') updateListElement(s, obj, op.key, diffs, op.obj)
  else if (remaining.length) diffs.push(Object.assign({ action: 'set', type: obj.type, obj: op.obj, key: op.key }, entryFields(remaining)))
  else diffs.push({ action: 'remove', type: obj.type, obj: op.obj, key: op.key })
}

const MAKE = { makeMap: 'map', makeTable: 'table', makeList: 'list', makeText: 'text' }

function applyChange(s, c, diffs) {
  const prior = s.states.get(c.actor) || []
  if (c.seq <= prior.length) {
    if (prior[c.seq - 1].text !== canon(c)) throw new Error(`Inconsistent reuse of sequence number ${c.seq} by ${c.actor}`)
    return
  }
  const base = Object.assign({}, c.deps || {})
  base[c.actor] = c.seq - 1
  const allDeps = transitiveDeps(s, base)
  prior.push({ change: c, allDeps, text: canon(c) })
  s.states.set(c.actor, prior)
  for (const raw of c.ops || []) {
    const op = Object.assign({ actor: c.actor, seq: c.seq }, raw)
    if (MAKE[op.action]) {
      if (s.objs.has(op.obj)) throw new Error(`Duplicate creation of object ${op.obj}`)
      s.objs.set(op.obj, { type: MAKE[op.action], keys: new Map(), following: new Map(), insertion: new Map(), elemIds: [] })
      diffs.push({ action: 'create', obj: op.obj, type: MAKE[op.action] })
    } else if (op.action === 'ins') {
      const obj = s.objs.get(op.obj)
      if (!obj) throw new Error(`Modification of unknown object ${op.obj}`)
      const elemId = `${op.actor}:${op.elem}`
      if (obj.insertion.has(elemId)) throw new Error(`Duplicate list element ID ${elemId}`)
      const f = obj.following.get(op.key) || []
      f.push(op)
      obj.following.set(op.key, f)
      obj.insertion.set(elemId, op)
    } else {
      applyAssign(s, op, diffs)
    }
  }
  for (const [a, q] of Array.from(s.deps)) if (q <= (allDeps.get(a) || 0)) s.deps.delete(a)
  s.deps.set(c.actor, c.seq)
  s.clock.set(c.actor, c.seq)
  s.history.push(c)
}

function applyQueuedOps(s, diffs) {
  for (;;) {
    const next = []
    let applied = false
    for (const c of s.queue) {
      if (causallyReady(s, c)) { applyChange(s, c, diffs); applied = true } else next.push(c)
    }
    s.queue = next
    if (!applied) return
  }
}

const Backend = {
  init() { return new OpSet() },
  // applyChanges(state, changes) -> [state, patch]; the state is advanced in place (the
  // restatement's states are linear, like the GPU drop-in's)
  applyChanges(s, changes) {
    const diffs = []
    for (const c of changes) { s.queue.push(c); applyQueuedOps(s, diffs) }
    return [s, makePatch(s, diffs)]
  },
  // applyLocalChange(state, request) -> [state, patch]: requestType 'change' (undoable unless
  // `undoable: false`; a request without a type is taken as a change), 'undo', 'redo'
  applyLocalChange(s, change) {
    if (change.seq <= (s.clock.get(change.actor) || 0)) throw new RangeError('Change request has already been applied')
    const type = change.requestType === undefined ? 'change' : change.requestType
    const diffs = []
    if (type === 'change') {
      const undoable = change.undoable !== false
      if (undoable) s.undoLocal = []
      s.queue.push(change)
      applyQueuedOps(s, diffs)
      if (undoable) {
        s.undoStack = s.undoStack.slice(0, s.undoPos).concat([s.undoLocal])
        s.undoPos++
        s.redoStack = []
        s.undoLocal = null
      }
    } else if (type === 'undo' || type === 'redo') {
      let ops
      if (type === 'undo') {
        ops = s.undoPos > 0 ? s.undoStack[s.undoPos - 1] : undefined
        if (!ops) throw new RangeError('Cannot undo: there is nothing to be undone')
        const redo = []
        for (const op of ops) {
          if (op.action === 'inc') { redo.push({ action: 'inc', obj: op.obj, key: op.key, value: -op.value }); continue }
          const f = fieldOps(s, op.obj, op.key)
          if (f.length) redo.push(...f)
          else redo.push({ action: 'del', obj: op.obj, key: op.key })
        }
        s.undoPos--
        s.redoStack = s.redoStack.concat([redo])
      } else {
        ops = s.redoStack[s.redoStack.length - 1]
        if (!ops) throw new RangeError('Cannot redo: the last change was not an undo')
        s.undoPos++
        s.redoStack = s.redoStack.slice(0, -1)
      }
      const c = { actor: change.actor, seq: change.seq, deps: change.deps || {} }
      if (change.message !== undefined) c.message = change.message
      c.ops = ops
      s.queue.push(c)
      applyQueuedOps(s, diffs)
    } else {
      throw new RangeError(`Unknown requestType: ${type}`)
    }
    const patch = makePatch(s, diffs)
    patch.actor = change.actor
    patch.seq = change.seq
    return [s, patch]
  },
}

// Clock objects keyed by actor id: the same rule as the GPU drop-in (GpuDocBackend.js newClock),
// so the baseline does not pay V8's per-key hidden-class transitions when every document has its
// own actors (hypermerge mints an actor per document): past 1024 distinct actor ids seen, clocks
// start in dictionary mode
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

function makePatch(s, diffs) {
  const clock = newClock(), deps = newClock()
  for (const [a, q] of s.clock) clock[a] = q
  for (const [a, q] of s.deps) deps[a] = q
  return { clock, deps, canUndo: s.undoPos > 0, canRedo: s.redoStack.length > 0, diffs }
}

// DocBackend (src/DocBackend.ts:46-213) over the restatement, synchronous Queue semantics
class Queue {
  constructor() { this.buf = []; this.sub = null }
  push(x) { if (this.sub) this.sub(x); else this.buf.push(x) }
  subscribe(f) { this.sub = f; const b = this.buf; this.buf = []; b.forEach(f) }
}

class DocBackend {
  constructor(documentId, notify, back) {
    this.id = documentId
    this.actorId = undefined
    this.clock = newClock()
    this.dictClock = CK.dict
    this.back = back
    this.changes = new Map()
    this.ready = new Queue()
    this.notify = notify
    this.minimumClock = undefined
    this.minimumClockSatisfied = false
    this.localChangeQ = new Queue()
    this.remoteChangesQ = new Queue()
    if (back) {
      this.actorId = documentId
      this.ready.subscribe((f) => f())
      this.minimumClockSatisfied = true
      this.subscribeToRemoteChanges()
      this.subscribeToLocalChanges()
      this.notify({ type: 'ReadyMsg', id: this.id, minimumClockSatisfied: true, actorId: this.actorId, history: back.history.length })
    }
  }

  applyRemoteChanges(changes) { this.remoteChangesQ.push(changes) }

  applyLocalChange(change) { this.localChangeQ.push(change) }

  updateClock(changes) {
    if (CK.dict && !this.dictClock) {
      const c = newClock()
      for (const k in this.clock) c[k] = this.clock[k]
      this.clock = c
      this.dictClock = true
    }
    for (const c of changes) {
      if (CK.seen) noteActor(c.actor)
      this.clock[c.actor] = Math.max(this.clock[c.actor] || 0, c.seq)
    }
  }

  init(changes, actorId) {
    const [back, patch] = Backend.applyChanges(Backend.init(), changes)
    this.actorId = this.actorId || actorId
    this.back = back
    this.updateClock(changes)
    this.minimumClockSatisfied = changes.length > 0
    this.ready.subscribe((f) => f())
    this.subscribeToLocalChanges()
    this.subscribeToRemoteChanges()
    this.notify({ type: 'ReadyMsg', id: this.id, minimumClockSatisfied: this.minimumClockSatisfied, actorId: this.actorId,
      patch, history: back.history.length })
  }

  // src/DocBackend.ts:187-205
  subscribeToLocalChanges() {
    this.localChangeQ.subscribe((change) => {
      const [back, patch] = Backend.applyLocalChange(this.back, change)
      this.back = back
      this.updateClock([change])
      this.notify({ type: 'LocalPatchMsg', id: this.id, actorId: this.actorId, minimumClockSatisfied: this.minimumClockSatisfied,
        change, patch, history: back.history.length })
    })
  }

  subscribeToRemoteChanges() {
    this.remoteChangesQ.subscribe((changes) => {
      const [back, patch] = Backend.applyChanges(this.back, changes)
      this.back = back
      this.updateClock(changes)
      this.notify({ type: 'RemotePatchMsg', id: this.id, minimumClockSatisfied: this.minimumClockSatisfied, patch,
        history: back.history.length })
    })
  }
}

// the merged document as plain JS (maps by key, lists in element order; conflicts dropped)
function materialize(s, objId) {
  const obj = s.objs.get(objId || ROOT)
  const val = (ops) => (ops[0].action === 'link' ? materialize(s, ops[0].value) : ops[0].value)
  if (obj.type === 'list' || obj.type === 'text') return obj.elemIds.map((e) => val(obj.keys.get(e)))
  const out = {}
  for (const [k, ops] of obj.keys) if (ops.length) out[k] = val(ops)
  return out
}

module.exports = { Backend, DocBackend, materialize, ROOT }
