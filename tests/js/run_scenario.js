'use strict'
// Replays the DocBackend scenarios of tests/golden/docbackend_traces.json on the GPU
// DocBackend (hypermerge_amd/js/GpuDocBackend.js) and prints the same trace shape as
// tools/golden/gen_docbackend_traces.js.  argv[2] = 'sync' | 'batched'.
const path = require('path')
const fs = require('fs')
const { GpuEngine, DocBackend } = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))

const mode = process.argv[2] || 'sync'
const gold = JSON.parse(fs.readFileSync(path.join(__dirname, '..', 'golden', 'docbackend_traces.json'), 'utf8'))
const engine = new GpuEngine({ mode, aStride: 8 })
const tick = () => new Promise((r) => setImmediate(r))

async function run(steps) {
  const trace = []
  const docs = {}
  const notify = (m) => trace.push({ msg: m.type, id: m.id, minimumClockSatisfied: m.minimumClockSatisfied,
    history: m.history, actorId: m.actorId, patch: m.patch !== undefined })
  for (const [op, id, a, b] of steps) {
    if (op === 'new') docs[id] = new DocBackend(id, notify, undefined, engine)
    else if (op === 'readyPush') docs[id].ready.push(() => docs[id].applyRemoteChanges(a))
    else if (op === 'remote') docs[id].applyRemoteChanges(a)
    else if (op === 'init') docs[id].init(a, b === null ? undefined : b)
    else if (op === 'minClock') docs[id].updateMinimumClock(a)
    else if (op === 'initActor') docs[id].initActor(a)
    else if (op === 'snapshot') {
      const d = docs[id]
      trace.push({ snapshot: id, clock: Object.assign({}, d.clock), minimumClockSatisfied: d.minimumClockSatisfied,
        actorId: d.actorId })
    }
    if (mode === 'batched') { await tick(); await tick() }
  }
  return trace
}

(async () => {
  const out = {}
  for (const [name, sc] of Object.entries(gold.scenarios)) out[name] = await run(sc.steps)
  out._submits = engine.submits
  process.stdout.write(JSON.stringify(out) + '\n')
})().catch((e) => { console.error(e); process.exit(1) })
