'use strict'
// Feeds documents through the JS restatement's DocBackend (oracle/js/backend.js): chunk 0
// via init(), the rest via applyRemoteChanges(); prints per document the history
// (actor, seq), opSet clock, queued count and the materialized document.
const path = require('path')
const { DocBackend, materialize } = require(path.join(__dirname, '..', '..', 'oracle', 'js', 'backend.js'))

const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const out = input.docs.map((chunks, i) => {
  const msgs = []
  const d = new DocBackend('doc' + i, (m) => msgs.push(m))
  let err = null
  try {
    chunks.forEach((c, r) => (r === 0 ? d.init(c, 'local') : d.applyRemoteChanges(c)))
  } catch (e) { err = e.message }
  const s = d.back
  const clock = {}
  if (s) for (const [a, q] of s.clock) clock[a] = q
  return { err, history: s ? s.history.map((c) => [c.actor, c.seq]) : [], clock, queued: s ? s.queue.length : 0,
    doc: s && !err ? materialize(s) : null, types: msgs.map((m) => m.type) }
})
process.stdout.write(JSON.stringify({ docs: out }) + '\n')
