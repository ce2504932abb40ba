'use strict'
// The ClockStore persistence batch (takeBatch) and the key tables' collision check, on the host
// (no GPU): a sequence of update / set calls grouped in rounds; after each round the batch of
// rows the store wrote.  tests/test_node_host.py replays the batches into sqlite3 and compares
// the table with the reference SQL's (tests/golden/clockstore_batches.json).
const path = require('path')
const fs = require('fs')
const G = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'GpuDocBackend.js'))
const input = JSON.parse(fs.readFileSync(0, 'utf8'))
const st = new G.ClockStore(null)
const batches = input.rounds.map((calls) => {
  for (const [kind, repo, doc, clock] of calls) st[kind](repo, doc, Object.fromEntries(clock))
  return st.takeBatch()
})
// a key function that collides (every id of the same length shares a key): an error, not a merge
const kt = new G.KeyTable((s) => BigInt(s.length))
let collision = null
try { kt.key('actorA'); kt.key('actorA'); kt.key('actorB') } catch (e) { collision = e.message }
process.stdout.write(JSON.stringify({ batches, collision, get: input.docs.map(([r, d]) => Object.entries(st.get(r, d))) }) + '\n')
