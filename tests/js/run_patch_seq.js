'use strict'
// Patch sequences of GpuDocBackend against the JS restatement (test driver for
// tests/test_node_gpu.py): the same documents, fed in the same chunks (init, then
// applyRemoteChanges one event-loop turn apart), through the reference DocBackend API of both
// (oracle/js/backend.js is test infrastructure); every delivered message's patch — clock, deps
// and the diffs in order — is collected per document.  Output: {docs: [{gpu: [patch...],
// cpu: [patch...]}], stats}.
const path = require('path')
const G = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
const C = require(path.join(__dirname, '..', '..', 'oracle', 'js', 'backend.js'))

const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const engine = new G.GpuEngine({ mode: input.mode || 'batched', binary: input.binary !== false })
const tick = () => new Promise((r) => setImmediate(r))
const keep = (m) => (m.patch ? { type: m.type, history: m.history, patch: m.patch } : { type: m.type, history: m.history })

;(async () => {
  const docs = input.docs.map((chunks, i) => {
    const gpu = [], cpu = []
    return {
      g: new G.DocBackend('doc' + i, (m) => gpu.push(keep(m)), undefined, engine),
      c: new C.DocBackend('doc' + i, (m) => cpu.push(keep(m))),
      chunks, gpu, cpu,
    }
  })
  const rounds = Math.max(...input.docs.map((c) => c.length))
  for (let r = 0; r < rounds; r++) {
    for (const x of docs) {
      if (r >= x.chunks.length) continue
      if (r === 0) { x.g.init(x.chunks[0], 'local'); x.c.init(x.chunks[0], 'local') }
      else if (x.chunks[r].length) { x.g.applyRemoteChanges(x.chunks[r]); x.c.applyRemoteChanges(x.chunks[r]) }
    }
    if (engine.mode === 'async') await engine.idle()
    else { await tick(); await tick() }
  }
  const out = docs.map((x) => ({ gpu: x.gpu, cpu: x.cpu }))
  process.stdout.write(JSON.stringify({ docs: out, stats: engine.stats() }) + '\n')
})().catch((e) => { console.error(e); process.exit(1) })
