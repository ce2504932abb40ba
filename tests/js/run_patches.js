'use strict'
// Patch diffs of GpuDocBackend (test driver for tests/test_node_gpu.py): documents are fed in
// chunks (init, then applyRemoteChanges one event-loop turn apart, batched engine); every
// patch's diffs are applied, in the order the patches were computed (ReadyMsg's patch is
// computed at init), by a restatement of Frontend.applyPatch's effect on a document
// (test infrastructure); the result is rendered in hypermerge_amd/render.py's canonical form.
const path = require('path')
const { GpuEngine, DocBackend } = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
const ROOT = '00000000-0000-0000-0000-000000000000'

function applyDiffs(objects, diffs) {
  for (const d of diffs) {
    if (d.action === 'create') { objects.set(d.obj, { type: d.type, keys: new Map(), elems: [] }); continue }
    const o = objects.get(d.obj)
    if (!o) throw new Error(`diff on unknown object ${d.obj}`)
    const e = { value: d.value, link: !!d.link, datatype: d.datatype, conflicts: d.conflicts }
    if (d.type === 'list' || d.type === 'text') {
      if (d.action === 'insert') o.elems.splice(d.index, 0, e)
      else if (d.action === 'set') o.elems[d.index] = e
      else if (d.action === 'remove') o.elems.splice(d.index, 1)
      else throw new Error(`bad list diff ${d.action}`)
    } else if (d.action === 'set') o.keys.set(d.key, e)
    else if (d.action === 'remove') o.keys.delete(d.key)
    else throw new Error(`bad map diff ${d.action}`)
  }
}

function render(objects, uuid, depth) {
  const o = objects.get(uuid)
  if (!o || depth > 64) return { cycle: uuid }
  const val = (v, link) => (link ? render(objects, v, depth + 1) : v)
  const ent = (e) => {
    const r = { value: val(e.value, e.link) }
    if (e.conflicts) r.conflicts = e.conflicts.map((c) => [c.actor, val(c.value, c.link)])
    if (e.datatype) r.datatype = e.datatype
    return r
  }
  if (o.type === 'list' || o.type === 'text') return { [o.type]: o.elems.map(ent) }
  const keys = Array.from(o.keys.keys()).sort()
  return { [o.type === 'table' ? 'table' : 'map']: keys.map((k) => [k, ent(o.keys.get(k))]) }
}

const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const engine = new GpuEngine({ mode: input.mode || 'batched', binary: input.binary !== false })
const tick = () => new Promise((r) => setImmediate(r))
;(async () => {
  const docs = input.docs.map((chunks, i) => {
    const msgs = []
    return { d: new DocBackend('doc' + i, (m) => msgs.push(m), undefined, engine), chunks, msgs }
  })
  const rounds = Math.max(...input.docs.map((c) => c.length))
  for (let r = 0; r < rounds; r++) {
    for (const x of docs) {
      if (r >= x.chunks.length) continue
      if (r === 0) x.d.init(x.chunks[0], 'local')
      else if (x.chunks[r].length) x.d.applyRemoteChanges(x.chunks[r])
    }
    if (engine.mode === 'async') await engine.idle()
    else { await tick(); await tick() }
  }
  const out = docs.map((x) => {
    const objects = new Map([[ROOT, { type: 'map', keys: new Map(), elems: [] }]])
    const ready = x.msgs.filter((m) => m.type === 'ReadyMsg')
    const remote = x.msgs.filter((m) => m.type === 'RemotePatchMsg')
    let nDiffs = 0
    for (const m of ready.concat(remote)) { applyDiffs(objects, m.patch.diffs); nDiffs += m.patch.diffs.length }
    return { state: render(objects, ROOT, 0), nDiffs, nonEmpty: x.msgs.filter((m) => m.patch && m.patch.diffs.length > 0).length,
      incremental: engine.stats().hitPatches + engine.stats().opPatches }
  })
  process.stdout.write(JSON.stringify({ docs: out }) + '\n')
})().catch((e) => { console.error(e); process.exit(1) })
