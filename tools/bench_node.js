'use strict'
// Node end-to-end rate of the remote-change path through the DocBackend message API.  Input
// (file argv[2]): {"docs": [[chunk0 changes], [chunk1], ...] per document}; every change is
// first rendered as the hypercore block the reference stores (Block.pack of a JSON Change
// that brotli does not shrink is the JSON text, src/Block.ts:6-16), outside the timed region.
// Chunk 0 goes through init(), later chunks through applyRemoteChanges(), one round per
// chunk index.  Legs (argv[3], comma separated):
//   cpu         the JS restatement (oracle/js/backend.js: Automerge 0.12 rules over JS Maps,
//               synchronous Queue semantics) handed parsed Change objects — BASELINE.md's
//               second baseline, with Actor.parseBlock done for it outside the timed region
//   cpu_blocks  the same from the blocks: Actor.parseBlock (JSON.parse per block,
//               src/Actor.ts:137-141) inside the timed region, as the reference runs it
//   gpu         the drop-in (hypermerge_amd/js/GpuDocBackend.js) in batched mode handed the
//               raw blocks (the docset parses them natively, multi-threaded)
//   gpu_async   the same in async mode (the round on the docset's host thread)
//   gpu_objects the drop-in in async mode handed parsed Change objects (stringified for the
//               docset), the reference's exact call shape
// Every delivered message's patch is consumed as DocFrontend does (patch.diffs.length,
// src/DocFrontend.ts:167).  Output: one JSON line {leg: {changes, seconds, changes_per_s,
// patches, diffs, digest, state_digest}}; `digest` hashes every document's DocBackend.clock
// and history length, `state_digest` its materialized document (maps by key, lists in order).
const path = require('path')
const fs = require('fs')
const crypto = require('crypto')

const input = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'))
const legs = (process.argv[3] || 'cpu,gpu').split(',')
const patchesOn = process.argv[4] !== 'nopatch'
const tick = () => new Promise((r) => setImmediate(r))
const nChanges = input.docs.reduce((s, chunks) => s + chunks.reduce((t, c) => t + c.length, 0), 0)
const rounds = Math.max(...input.docs.map((c) => c.length))
const blocks = input.docs.map((chunks) => chunks.map((ch) => ch.map((c) => Buffer.from(JSON.stringify(c)))))

function canon(v) {
  if (v === null || typeof v !== 'object') return JSON.stringify(v)
  if (Array.isArray(v)) return '[' + v.map(canon).join(',') + ']'
  return '{' + Object.keys(v).sort().map((k) => JSON.stringify(k) + ':' + canon(v[k])).join(',') + '}'
}

function digest(docs) {
  const h = crypto.createHash('sha256')
  for (const d of docs) h.update(canon([d.id, d.clock, d.hist]))
  return h.digest('hex').slice(0, 16)
}

function stateDigest(states) {
  const h = crypto.createHash('sha256')
  for (const s of states) h.update(canon(s))
  return h.digest('hex').slice(0, 16)
}

async function runCpu(fromBlocks) {
  const { DocBackend, materialize } = require(path.join(__dirname, '..', 'oracle', 'js', 'backend.js'))
  let patches = 0, diffs = 0
  const docs = input.docs.map((_, i) => new DocBackend('doc' + i, (m) => { patches++; if (m.patch) diffs += m.patch.diffs.length }))
  const parsed = fromBlocks ? null : input.docs
  profStart()
  const t0 = process.hrtime.bigint()
  for (let r = 0; r < rounds; r++) {
    input.docs.forEach((chunks, i) => {
      if (r >= chunks.length) return
      const ch = fromBlocks ? blocks[i][r].map((b) => JSON.parse(b.toString())) : parsed[i][r]
      if (r === 0) docs[i].init(ch, 'local')
      else if (ch.length) docs[i].applyRemoteChanges(ch)
    })
  }
  const s = Number(process.hrtime.bigint() - t0) / 1e9
  await profStop()
  return { changes: nChanges, seconds: s, changes_per_s: nChanges / s, patches, diffs,
    digest: digest(docs.map((d) => ({ id: d.id, clock: d.clock, hist: d.back.history.length }))),
    state_digest: stateDigest(docs.map((d) => materialize(d.back))) }
}

function plain(view, uuid) {
  const ov = view.get(uuid)
  if (!ov) return {}
  const val = (e) => (e.link ? plain(view, e.value) : e.value)
  if (ov.type === 'list' || ov.type === 'text') return ov.elems.filter(Boolean).map(([, e]) => val(e))
  const o = {}
  for (const [k, e] of ov.keys) o[k] = val(e)
  return o
}

// HM_NODE_PROF=file: a V8 CPU profile of the timed region (the inspector's profiler, started
// after the device is open: `node --cpu-prof` from process start makes HSA device discovery
// fail under the profiler's signals)
let prof = null
function profStart() {
  if (!process.env.HM_NODE_PROF) return
  const inspector = require('inspector')
  prof = new inspector.Session()
  prof.connect()
  prof.post('Profiler.enable')
  prof.post('Profiler.setSamplingInterval', { interval: 200 })
  prof.post('Profiler.start')
}
function profStop() {
  if (!prof) return Promise.resolve()
  return new Promise((resolve) => prof.post('Profiler.stop', (err, r) => {
    if (!err) fs.writeFileSync(process.env.HM_NODE_PROF, JSON.stringify(r.profile))
    prof.disconnect()
    prof = null
    resolve()
  }))
}

async function runGpu(mode, objects, diffsForm) {
  const G = require(process.env.HM_GPU_JS || path.join(__dirname, '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
  const engine = new G.GpuEngine({ mode, patches: patchesOn, diffs: diffsForm || 'ops' })
  const settle = async () => { if (mode === 'async') await engine.idle(); else { await tick(); await tick() } }
  // warm the device (engine, stores, kernels) outside the timed region
  const w = new G.DocBackend('warm', () => {}, undefined, engine)
  w.init(blocks[0][0].slice(0, 1), 'local')
  await settle()
  let patches = 0, diffs = 0
  const docs = input.docs.map((_, i) => new G.DocBackend('doc' + i, (m) => { patches++; if (m.patch) diffs += m.patch.diffs.length },
    undefined, engine))
  const src = objects ? input.docs : blocks
  const st0 = engine.stats()
  profStart()
  const t0 = process.hrtime.bigint()
  for (let r = 0; r < rounds; r++) {
    src.forEach((chunks, i) => {
      if (r >= chunks.length) return
      if (r === 0) docs[i].init(chunks[0], 'local')
      else if (chunks[r].length) docs[i].applyRemoteChanges(chunks[r])
    })
    await settle()
  }
  await engine.idle()
  const s = Number(process.hrtime.bigint() - t0) / 1e9
  await profStop()
  const st = engine.stats()
  return { changes: nChanges, seconds: s, changes_per_s: nChanges / s, patches, diffs, submits: engine.submits,
    patch_diffs: patchesOn, diffs_form: engine.diffs, op_patches: st.opPatches - st0.opPatches,
    replay_mismatch: st.replayMismatch - st0.replayMismatch,
    hit_register_patches: st.hitPatches - st0.hitPatches, full_patches: st.fullPatches - st0.fullPatches,
    routing: { incremental: st.incremental - st0.incremental, remerged: st.remerged - st0.remerged,
      handed_back: st.handedBack - st0.handedBack },
    mode, input: objects ? 'Change objects' : 'raw blocks',
    digest: digest(docs.map((d) => ({ id: d.id, clock: d.clock, hist: d.back.histLen }))),
    state_digest: stateDigest(docs.map((d) => plain(G.materialize(d.back), '00000000-0000-0000-0000-000000000000'))) }
}

;(async () => {
  const out = {}
  for (const m of legs) {
    let key = m
    for (let i = 2; key in out; i++) key = `${m}#${i}`           // a repeated leg: m#2, m#3, ...
    if (m === 'cpu') out[key] = await runCpu(false)
    else if (m === 'cpu_blocks') out[key] = await runCpu(true)
    else if (m === 'gpu') out[key] = await runGpu('batched', false)
    else if (m === 'gpu_async') out[key] = await runGpu('async', false)
    else if (m === 'gpu_objects') out[key] = await runGpu('async', true)
    else if (m === 'gpu_async_net') out[key] = await runGpu('async', false, 'net')
    else throw new Error(`unknown leg ${m}`)
  }
  process.stdout.write(JSON.stringify(out) + '\n')
})().catch((e) => { console.error(e); process.exit(1) })
