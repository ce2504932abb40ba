'use strict'
// Local changes with undo / redo (Backend.applyLocalChange through DocBackend.applyLocalChange,
// src/DocBackend.ts:187-205) on the GPU drop-in and on the JS restatement, side by side:
// seeded documents where a local actor makes undoable (and some non-undoable) changes, undoes,
// redoes, and remote actors' changes arrive in between (with concurrent sets: conflicts).
// Printed per document: every message's type, history, canUndo / canRedo, the local patches'
// actor / seq, each request's thrown error (if any), and the materialized document after every
// step.  argv[2]: engine mode (sync | batched | async), argv[3]: documents.
const path = require('path')
const G = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
const J = require(path.join(__dirname, '..', '..', 'oracle', 'js', 'backend.js'))
const ROOT = '00000000-0000-0000-0000-000000000000'
const mode = process.argv[2] || 'sync'
const nDocs = parseInt(process.argv[3] || '24', 10)
const tick = () => new Promise((r) => setImmediate(r))

function rng(seed) {
  let x = seed >>> 0 || 1
  return () => { x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0; return x / 4294967296 }
}

function canon(v) {
  if (v === null || typeof v !== 'object') return JSON.stringify(v)
  if (Array.isArray(v)) return '[' + v.map(canon).join(',') + ']'
  return '{' + Object.keys(v).sort().map((k) => JSON.stringify(k) + ':' + canon(v[k])).join(',') + '}'
}

function plain(view, uuid) {
  const ov = view.get(uuid)
  if (!ov) return {}
  const val = (e) => (e.link ? plain(view, e.value) : e.value)
  if (ov.type === 'list' || ov.type === 'text') return ov.elems.map(([, e]) => val(e))
  const o = {}
  for (const [k, e] of ov.keys) o[k] = val(e)
  return o
}

// one document's script: steps of ['remote', changes] | ['local', request]
function script(seed) {
  const r = rng(seed)
  const LOCAL = 'mmmm', REMOTES = ['aaaa', 'zzzz']
  const LIST = 'list-' + seed
  const seq = { mmmm: 0, aaaa: 0, zzzz: 0 }
  const heads = {}
  const steps = []
  const elems = []
  let nextElem = 1
  const keys = ['k0', 'k1', 'k2', 'c']
  const mk = (actor, deps, ops) => { seq[actor]++; const c = { actor, seq: seq[actor], deps, ops }; return c }
  // the first change (init): a counter, a list
  const c0 = mk('aaaa', {}, [{ action: 'set', obj: ROOT, key: 'c', value: 10, datatype: 'counter' },
    { action: 'makeList', obj: LIST }, { action: 'link', obj: ROOT, key: 'l', value: LIST }])
  heads.aaaa = 1
  steps.push(['init', [c0]])
  let undos = 0, redos = 0
  for (let s = 0; s < 14; s++) {
    const p = r()
    if (p < 0.25) {
      // a remote change, concurrent with the latest local one half of the time
      const a = REMOTES[Math.floor(r() * 2)]
      // (remote actors have not seen the local actor's changes: theirs are concurrent with it)
      const deps = Object.assign({}, heads)
      delete deps[a]
      delete deps.mmmm
      const c = mk(a, deps, [{ action: 'set', obj: ROOT, key: keys[Math.floor(r() * 3)], value: 'r' + s }])
      heads[a] = c.seq
      steps.push(['remote', [c]])
    } else if (p < 0.7) {
      // a local change over the whole document (deps: every head)
      const ops = []
      const n = 1 + Math.floor(r() * 3)
      for (let k = 0; k < n; k++) {
        const q = r()
        if (q < 0.4) ops.push({ action: 'set', obj: ROOT, key: keys[Math.floor(r() * 3)], value: s * 10 + k })
        else if (q < 0.55) ops.push({ action: 'del', obj: ROOT, key: keys[Math.floor(r() * 3)] })
        else if (q < 0.7) ops.push({ action: 'inc', obj: ROOT, key: 'c', value: 1 + Math.floor(r() * 5) })
        else if (q < 0.85 || !elems.length) {
          const e = nextElem++
          const parent = elems.length && r() < 0.5 ? elems[elems.length - 1] : '_head'
          ops.push({ action: 'ins', obj: LIST, key: parent, elem: e })
          ops.push({ action: 'set', obj: LIST, key: LOCAL + ':' + e, value: 'v' + e })
          elems.push(LOCAL + ':' + e)
        } else {
          const e = elems[Math.floor(r() * elems.length)]
          ops.push(r() < 0.5 ? { action: 'del', obj: LIST, key: e } : { action: 'set', obj: LIST, key: e, value: 'w' + s })
        }
      }
      const req = mk(LOCAL, Object.assign({}, heads, { mmmm: undefined }), ops)
      delete req.deps.mmmm
      req.requestType = 'change'
      if (r() < 0.15) req.undoable = false
      heads.mmmm = req.seq
      steps.push(['local', req])
    } else {
      // undo or redo (sometimes with nothing to undo / redo: the request throws)
      const kind = r() < 0.6 ? 'undo' : 'redo'
      const req = { requestType: kind, actor: LOCAL, seq: seq.mmmm + 1, deps: Object.assign({}, heads) }
      delete req.deps.mmmm
      steps.push(['request', req])
      if (kind === 'undo') undos++; else redos++
    }
  }
  return steps
}

async function run(which) {
  let lastErr = null
  const engine = which === 'gpu' ? new G.GpuEngine({ mode, aStride: 8, onError: (e) => { lastErr = e.message } }) : null
  const out = []
  for (let d = 0; d < nDocs; d++) {
    const msgs = []
    const doc = which === 'gpu' ? new G.DocBackend('doc' + d, (m) => msgs.push(m), undefined, engine)
      : new J.DocBackend('doc' + d, (m) => msgs.push(m))
    const trace = []
    const steps = script(1000 + d)
    let localSeq = 0
    for (const [kind, x] of steps) {
      let err = null
      if (kind === 'init') doc.init(x, 'mmmm')
      else if (kind === 'remote') doc.applyRemoteChanges(x)
      else {
        const req = Object.assign({}, x, { seq: localSeq + 1 })
        if (req.requestType !== 'change') req.deps = x.deps
        lastErr = null
        try { doc.applyLocalChange(req) } catch (e) { err = e.message }
        if (engine) await engine.idle()
        if (!err && lastErr) err = lastErr
        if (!err) localSeq++
      }
      if (engine) await engine.idle()
      const st = which === 'gpu' ? plain(G.materialize(doc.back), ROOT) : J.materialize(doc.back)
      trace.push([kind, err, canon(st)])
    }
    out.push({ trace, msgs: msgs.map((m) => [m.type, m.history, m.patch ? !!m.patch.canUndo : null,
      m.patch ? !!m.patch.canRedo : null, m.patch && m.patch.actor, m.patch && m.patch.seq]) })
  }
  return out
}

(async () => {
  const gpu = await run('gpu')
  const cpu = await run('cpu')
  // (exit once the line is flushed: a pipe takes stdout asynchronously)
  process.stdout.write(JSON.stringify({ gpu, cpu }) + '\n', () => process.exit(0))
})().catch((e) => { console.error(e && e.stack || e); process.exit(1) })
