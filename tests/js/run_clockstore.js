'use strict'
// Replays tests/golden/clockstore_vectors.json on the JS ClockStore of GpuDocBackend.js.
const path = require('path')
const fs = require('fs')
const { ClockStore } = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
const gold = JSON.parse(fs.readFileSync(path.join(__dirname, '..', 'golden', 'clockstore_vectors.json'), 'utf8'))
const out = {}
for (const [name, c] of Object.entries(gold.cases)) {
  const st = new ClockStore(null)
  let pushed = 0
  st.updateQ.subscribe(() => { pushed++ })
  out[name] = c.ops.map(([kind, a, b, clock]) => {
    if (kind === 'update' || kind === 'set') {
      const before = pushed
      const obj = {}
      for (const [k, v] of clock) obj[k] = v
      const [, , stored] = st[kind](a, b, obj)
      return { stored: Object.entries(stored), pushed: pushed > before }
    }
    if (kind === 'get') return { clock: Object.entries(st.get(a, b)) }
    if (kind === 'repos') return { ids: st.getAllRepoIds().sort() }
    return { ids: st.getAllDocumentIds(a).sort() }
  })
}
process.stdout.write(JSON.stringify(out) + '\n')
