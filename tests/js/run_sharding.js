'use strict'
// GpuEngine over device shards (documents routed by FNV-1a64(docId) % devices) and stride
// classes (a document re-strided to a wider store when a new actor outgrows it), plus the
// node-wide clock exchange (GpuEngine.exchangeClocks).  argv[2] = JSON list of device
// ordinals; stdin = JSON {docId: [change batches]}.  Prints one JSON line:
// {docs: {docId: {view, clock, shard, stride}}, exchanged, restrides, submits}.
const path = require('path')
const G = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))

const devices = JSON.parse(process.argv[2] || '[0]')
const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const engine = new G.GpuEngine({ devices, mode: 'sync', aStride: 8 })
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

const states = new Map()
const ids = Object.keys(input)
const rounds = Math.max(...ids.map((d) => input[d].length))
for (let r = 0; r < rounds; r++) {
  for (const d of ids) {
    if (r >= input[d].length) continue
    if (!states.has(d)) states.set(d, engine.init(d))
    engine.applyChanges(states.get(d), input[d][r])
  }
}
const out = { docs: {}, restrides: engine.restrides, submits: engine.submits }
for (const [d, st] of states) {
  out.docs[d] = { view: plain(G.materialize(st), ROOT), clock: st.backClock, shard: st.shard, stride: st.stride,
    expectShard: Number(G.fnv1a64(d) % BigInt(devices.length)) }
}
out.exchanged = engine.exchangeClocks(Array.from(states.values()))
process.stdout.write(JSON.stringify(out) + '\n')
