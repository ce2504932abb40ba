'use strict'
// Documents opened while an async round is in flight (ADVICE r02: no call may race the
// store's host thread): docsetOpen runs at any time, every other docset call on a busy
// device throws instead of racing; after the round all documents are correct.
const path = require('path')
const G = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const engine = new G.GpuEngine({ mode: 'async' })
const store = new G.ClockStore(engine)

;(async () => {
  const first = input.docs.slice(0, input.docs.length / 2), second = input.docs.slice(input.docs.length / 2)
  const docs = []
  first.forEach((chs, i) => { const d = new G.DocBackend('a' + i, () => {}, undefined, engine); d.init(chs, 'x'); docs.push(d) })
  // let the round start on the host thread, then open and init more documents during it
  await new Promise((r) => setImmediate(r))
  const busyDuring = engine.flushing
  let busyThrow = null
  try { G.addon.docsetClockUpdate(engine.docsets[0], Uint32Array.of(0)) } catch (e) { busyThrow = e.message }
  if (busyDuring && docs.some((d) => d.back)) throw new Error('documents finished before the round')
  second.forEach((chs, i) => { const d = new G.DocBackend('b' + i, () => {}, undefined, engine); d.init(chs, 'x'); docs.push(d) })
  await engine.idle()
  const upd = store.updateDocs('self', docs)
  process.stdout.write(JSON.stringify({ busyDuring, busyThrow, n: docs.length,
    docs: docs.map((d) => ({ clock: d.clock, hist: d.back.histLen, stored: upd.shift()[2] })) }) + '\n')
})().catch((e) => { console.error(e); process.exit(1) })
