'use strict'
// Feeds documents through GpuDocBackend in batched mode: chunk 0 via init(), the other
// chunks via applyRemoteChanges() one event-loop turn apart (every document that got
// changes in a turn is merged in the same GPU submit).  Prints per document the final
// history (actor, seq order from back.getIn(['opSet','history']).slice().toArray()),
// opSet clock/deps of the last patch, DocBackend.clock and the message types seen.
const path = require('path')
const { GpuEngine, DocBackend, ClockStore } = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))

const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const engine = new GpuEngine({ mode: input.mode || 'batched', aStride: 8 })
const tick = () => new Promise((r) => setImmediate(r))

;(async () => {
  const docs = input.docs.map((chunks, i) => {
    const msgs = []
    const d = new DocBackend('doc' + i, (m) => msgs.push(m), undefined, engine)
    return { d, chunks, msgs }
  })
  const rounds = Math.max(...input.docs.map((c) => c.length))
  // ClockStore.update(self, doc, doc.clock) after every round (src/RepoBackend.ts:343-345):
  // GPU-batched updateDocs vs the scalar host ClockStore (pinned to the reference SQL)
  const gpuStore = new ClockStore(engine), hostStore = new ClockStore(null)
  let gpuPush = 0, hostPush = 0, clockMismatch = 0
  gpuStore.updateQ.subscribe(() => { gpuPush++ })
  hostStore.updateQ.subscribe(() => { hostPush++ })
  for (let r = 0; r < rounds; r++) {
    for (const x of docs) {
      if (r >= x.chunks.length) continue
      if (r === 0) x.d.init(x.chunks[0], 'local')
      else if (x.chunks[r].length) x.d.applyRemoteChanges(x.chunks[r])
    }
    if (engine.mode === 'async') await engine.idle()
    else { await tick(); await tick() }
    const sat = docs.filter((x) => x.d.back && x.d.minimumClockSatisfied).map((x) => x.d)
    const g = gpuStore.updateDocs('self', sat)
    sat.forEach((d, i) => {
      const h = hostStore.update('self', d.id, d.clock)
      if (JSON.stringify(h[2]) !== JSON.stringify(g[i][2])) clockMismatch++
    })
  }
  const out = docs.map((x) => {
    const h = x.d.back.getIn(['opSet', 'history'])
    const last = x.msgs[x.msgs.length - 1]
    return { types: x.msgs.map((m) => m.type), history: h.slice(0, h.size).toArray().map((c) => [c.actor, c.seq]),
      clock: last.patch.clock, deps: last.patch.deps, backendClock: x.d.clock, histLen: last.history }
  })
  process.stdout.write(JSON.stringify({ docs: out, submits: engine.submits, gpuPush, hostPush, clockMismatch }) + '\n')
})().catch((e) => { console.error(e); process.exit(1) })
