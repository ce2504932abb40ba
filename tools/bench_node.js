'use strict'
// Node end-to-end rate of the remote-change path through the DocBackend message API:
//   cpu  the JS restatement (oracle/js/backend.js: Automerge 0.12 rules over JS Maps,
//        synchronous Queue semantics) on this one Node thread — BASELINE.md's second baseline
//   gpu  the drop-in (hypermerge_amd/js/GpuDocBackend.js) in batched mode: every document
//        that receives changes in an event-loop turn is merged in one GPU submit
//   gpu_async  the same in async mode (the device wait on the store's host thread)
// Input (file argv[2]): {"docs": [[chunk0 changes], [chunk1], ...] per document}; chunk 0 goes
// through init(), later chunks through applyRemoteChanges(), one round per chunk index.
// Output: one JSON line {mode: {changes, seconds, changes_per_s, patches, digest}}; `digest`
// hashes every document's final DocBackend.clock and history length, so the modes can be
// compared for equality.
const path = require('path')
const fs = require('fs')
const crypto = require('crypto')

const input = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'))
const modes = (process.argv[3] || 'cpu,gpu').split(',')
const patchesOn = process.argv[4] !== 'nopatch'
const tick = () => new Promise((r) => setImmediate(r))
const nChanges = input.docs.reduce((s, chunks) => s + chunks.reduce((t, c) => t + c.length, 0), 0)
const rounds = Math.max(...input.docs.map((c) => c.length))

function digest(docs) {
  const h = crypto.createHash('sha256')
  for (const d of docs) {
    const c = {}
    Object.keys(d.clock).sort().forEach((a) => { c[a] = d.clock[a] })
    h.update(JSON.stringify([d.id, c, d.hist]))
  }
  return h.digest('hex').slice(0, 16)
}

async function runCpu() {
  const { DocBackend } = require(path.join(__dirname, '..', 'oracle', 'js', 'backend.js'))
  let patches = 0
  const docs = input.docs.map((_, i) => new DocBackend('doc' + i, () => { patches++ }))
  const t0 = process.hrtime.bigint()
  for (let r = 0; r < rounds; r++) {
    input.docs.forEach((chunks, i) => {
      if (r >= chunks.length) return
      if (r === 0) docs[i].init(chunks[0], 'local')
      else if (chunks[r].length) docs[i].applyRemoteChanges(chunks[r])
    })
  }
  const s = Number(process.hrtime.bigint() - t0) / 1e9
  return { changes: nChanges, seconds: s, changes_per_s: nChanges / s, patches,
    digest: digest(docs.map((d) => ({ id: d.id, clock: d.clock, hist: d.back.history.length }))) }
}

async function runGpu(mode) {
  const { GpuEngine, DocBackend } = require(path.join(__dirname, '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
  const engine = new GpuEngine({ mode, aStride: 8, patches: patchesOn })
  const settle = async () => { if (mode === 'async') await engine.idle(); else { await tick(); await tick() } }
  // warm the device (engine, store, kernels) outside the timed region
  const w = new DocBackend('warm', () => {}, undefined, engine)
  w.init(input.docs[0][0].slice(0, 1), 'local')
  await settle()
  let patches = 0
  const docs = input.docs.map((_, i) => new DocBackend('doc' + i, () => { patches++ }, undefined, engine))
  const t0 = process.hrtime.bigint()
  for (let r = 0; r < rounds; r++) {
    input.docs.forEach((chunks, i) => {
      if (r >= chunks.length) return
      if (r === 0) docs[i].init(chunks[0], 'local')
      else if (chunks[r].length) docs[i].applyRemoteChanges(chunks[r])
    })
    await settle()
  }
  await engine.idle()
  const s = Number(process.hrtime.bigint() - t0) / 1e9
  const inc = docs.reduce((t, d) => t + (d.back.incrementalPatches || 0), 0)
  return { changes: nChanges, seconds: s, changes_per_s: nChanges / s, patches, submits: engine.submits,
    patch_diffs: patchesOn, incremental_patches: inc, mode, digest: digest(docs.map((d) => ({ id: d.id, clock: d.clock, hist: d.back.histLen }))) }
}

;(async () => {
  const out = {}
  for (const m of modes) out[m] = m === 'cpu' ? await runCpu() : await runGpu(m === 'gpu_async' ? 'async' : 'batched')
  process.stdout.write(JSON.stringify(out) + '\n')
})().catch((e) => { console.error(e); process.exit(1) })
