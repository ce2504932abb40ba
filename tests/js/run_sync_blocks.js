'use strict'
// RepoBackend.syncChanges over the device CursorStore, with raw blocks (test driver for
// tests/test_node_gpu.py): stdin {docs: {docId: [actorIds]}, feeds: {actorId: [JSON block text]},
// present: [{actorId: [0|1 per block]} per sync round]}.  Every document's cursor holds each of
// its actors at INFINITY_SEQ (CursorStore.addActor); each round, syncPlan picks the documents of
// every synced actor and their contiguous ranges [doc.changes[actor], first missing block), and
// the ranges' raw blocks go to DocBackend.applyRemoteBlocks (no Actor.parseBlock on the host).
// Prints {plans: [[docId, actor, lo, end]...] per round, docs: {docId: {history, clock, view}}}.
const path = require('path')
const G = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const engine = new G.GpuEngine({ mode: process.argv[2] || 'async' })
const cursors = new G.CursorStore(engine, 16)
const ROOT = '00000000-0000-0000-0000-000000000000'

function plain(view, uuid) {
  const ov = view.get(uuid)
  if (!ov) return {}
  const val = (e) => (e.link ? plain(view, e.value) : e.value)
  if (ov.type === 'list' || ov.type === 'text') return ov.elems.filter(Boolean).map(([, e]) => val(e))
  const o = {}
  for (const [k, e] of ov.keys) o[k] = val(e)
  return o
}

;(async () => {
  const docs = new Map()
  const upd = {}
  for (const [d, actors] of Object.entries(input.docs)) {
    const doc = new G.DocBackend(d, () => {}, undefined, engine)
    doc.init([], 'local')
    docs.set(d, doc)
    upd[d] = Object.fromEntries(actors.map((a) => [a, Infinity]))
  }
  cursors.updateMany('repo', upd)
  await engine.idle()
  const feeds = {}
  for (const [a, f] of Object.entries(input.feeds)) feeds[a] = f.map((t) => Buffer.from(t))
  const plans = []
  for (const present of input.present) {
    const plan = G.syncPlan(engine, cursors, 'repo', Object.keys(present), docs, present)
    plans.push(plan)
    for (const [d, a, lo, end] of plan) {
      const doc = docs.get(d)
      doc.changes.set(a, end)
      if (end > lo) doc.applyRemoteBlocks(feeds[a].slice(lo, end))
    }
    await engine.idle()
  }
  const out = {}
  for (const [d, doc] of docs) {
    const h = doc.back.getIn(['opSet', 'history'])
    out[d] = { history: h.slice(0, h.size).toArray().map((c) => [c.actor, c.seq]), clock: doc.clock,
      view: plain(G.materialize(doc.back), ROOT), cursor: cursors.get('repo', d),
      entry: cursors.entries('repo', input.docs[d].map((a) => [d, a])) }
  }
  process.stdout.write(JSON.stringify({ plans, docs: out }) + '\n')
})().catch((e) => { console.error(e); process.exit(1) })
