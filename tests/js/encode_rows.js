'use strict'
// Encodes the document chunks read from stdin ([[changes, ...chunks], ...] per document)
// with hypermerge_amd/js/columnar.js and prints, per chunk, the rows as hex + totals.
const path = require('path')
const C = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'columnar.js'))
const clocks = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'clocks.js'))
const Channel = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'channel.js'))

const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const pool = new C.StringPool()
const out = { docs: [], strings: null, clock: [], channel: [] }
for (const chunks of input.docs) {
  const e = new C.DocEncoder(pool)
  out.docs.push(chunks.map((ch) => {
    const a = e.encode(ch)
    return { changes: a.changes.toString('hex'), deps: a.deps.toString('hex'), ops: a.ops.toString('hex'),
      nActors: a.nActors, nRegs: a.nRegs, nObjs: a.nObjs, flags: a.flags, remap: a.remap ? Array.from(a.remap) : null,
      actors: e.actors.slice() }
  }))
}
out.strings = pool.strings
for (const [a, b] of input.clocks || []) out.clock.push([clocks.cmp(a, b), clocks.union(a, b), clocks.equal(a, b)])
// channel: buffered then subscribed delivery, then synchronous push, unsubscribe + once
const q = new Channel('t')
const seen = []
q.push(1); q.push(2)
q.subscribe((x) => seen.push(x))
q.push(3)
q.unsubscribe()
q.push(4)
q.once((x) => seen.push('once' + x))
q.push(5)
out.channel = [seen, q.length]
process.stdout.write(JSON.stringify(out) + '\n')
