'use strict'
// Golden message traces of the reference's DocBackend (SURVEY.md §8c, Appendix C
// "DocBackend sequencing"): runs /root/reference/dist/DocBackend.js in THIS container
// (never on the GPU box) and records, per scenario, the notify() messages (type, id,
// minimumClockSatisfied, history, actorId, patch present) and DocBackend.clock /
// minimumClockSatisfied snapshots.  Output: tests/golden/docbackend_traces.json.
//
// DocBackend's dependencies that are absent here are stubbed in a temp dir on NODE_PATH:
//   automerge         — a Backend whose applyChanges asks the CPU restatement (oracle/) for
//                       the merged history size and applied clock of the changes handed so
//                       far, so opSet.history.size follows the restated queue rules;
//                       everything DocBackend itself does (queues, clock quirk, minimum
//                       clock, message order) is the reference's own code;
//   bs58, hypercore-crypto — never called on this path (imported by Keys.js).
// Usage: node tools/golden/gen_docbackend_traces.js > tests/golden/docbackend_traces.json
const fs = require('fs')
const os = require('os')
const path = require('path')

const REF = '/root/reference/dist/DocBackend.js'
const tmp = fs.mkdtempSync(path.join(os.tmpdir(), 'hm-stubs-'))
const stub = (name, src) => {
  fs.mkdirSync(path.join(tmp, name), { recursive: true })
  fs.writeFileSync(path.join(tmp, name, 'index.js'), src)
}
// the queue rules (history sizes, applied clock) come from the CPU restatement of Automerge
// (oracle/oracle.c via tools/golden/oracle_history.py): every applyChanges re-merges the
// changes handed so far (applyChanges is a left fold of addChange)
const ORACLE = path.join(__dirname, 'oracle_history.py')
stub('automerge', `
const { execFileSync } = require('child_process')
function applyChanges(state, changes) {
  const log = state.log.concat(changes)
  const r = JSON.parse(execFileSync('python3', [${JSON.stringify(ORACLE)}], { input: JSON.stringify(log) }).toString())
  if (r.status !== 0) throw new Error('oracle status ' + r.status)
  const st = mk({ log, history: r.history, clock: r.clock })
  return [st, { clock: Object.assign({}, r.clock), deps: {}, diffs: changes.length ? [{}] : [] }]
}
function mk(s) {
  return Object.assign(s, { getIn: (p) => ({ size: s.history }) })
}
module.exports = { Backend: { init: () => mk({ log: [], history: 0, clock: {} }), applyChanges } }
`)
stub('bs58', 'module.exports = { encode: (b) => b.toString("hex"), decode: (s) => Buffer.from(s, "hex") }')
stub('hypercore-crypto', 'module.exports = { keyPair: () => ({}), discoveryKey: (b) => b }')
process.env.NODE_PATH = [tmp, '/usr/share/nodejs', process.env.NODE_PATH || ''].join(path.delimiter)
require('module').Module._initPaths()
const { DocBackend } = require(REF)

const ch = (actor, seq, deps, key) => ({ actor, seq, deps, ops: [{ action: 'set', obj: '00000000-0000-0000-0000-000000000000', key, value: seq }] })

// scenario steps (shared with tests/js/run_scenario.js, which replays them on the GPU backend)
const SCENARIOS = {
  buffered_before_init: [
    ['new', 'D'],
    ['readyPush', 'D', [ch('bbbb', 1, { aaaa: 1 }, 'y')]],
    ['remote', 'D', [ch('bbbb', 2, {}, 'y')]],
    ['init', 'D', [ch('aaaa', 1, {}, 'x'), ch('aaaa', 2, {}, 'x')], 'aaaa'],
    ['snapshot', 'D'],
    ['remote', 'D', [ch('bbbb', 3, { aaaa: 2 }, 'z')]],
    ['snapshot', 'D'],
  ],
  queued_change_clock: [
    ['new', 'D'],
    ['init', 'D', [ch('aaaa', 1, {}, 'x')], 'aaaa'],
    ['remote', 'D', [ch('bbbb', 2, {}, 'y')]],            // bbbb:1 missing -> queued, clock still advances
    ['snapshot', 'D'],
    ['remote', 'D', [ch('bbbb', 1, {}, 'y')]],            // unblocks bbbb:2
    ['snapshot', 'D'],
    ['remote', 'D', [ch('aaaa', 1, {}, 'x')]],            // duplicate: no history change
    ['snapshot', 'D'],
  ],
  empty_init_then_min_clock: [
    ['new', 'D'],
    ['init', 'D', [], 'aaaa'],
    ['snapshot', 'D'],
    ['minClock', 'D', { aaaa: 2, bbbb: 1 }],
    ['snapshot', 'D'],
    ['remote', 'D', [ch('aaaa', 1, {}, 'x')]],
    ['snapshot', 'D'],
    ['minClock', 'D', { cccc: 1 }],                       // unioned while unsatisfied
    ['remote', 'D', [ch('aaaa', 2, {}, 'x'), ch('bbbb', 1, { aaaa: 2 }, 'y')]],
    ['snapshot', 'D'],
    ['remote', 'D', [ch('cccc', 1, {}, 'z')]],
    ['snapshot', 'D'],
    ['minClock', 'D', { dddd: 9 }],                       // no-op once satisfied
    ['snapshot', 'D'],
  ],
  init_actor_and_two_docs: [
    ['new', 'D'],
    ['new', 'E'],
    ['initActor', 'D', 'zzzz'],                           // before init: no message
    ['init', 'E', [ch('cccc', 1, {}, 'k')], 'eeee'],
    ['init', 'D', [ch('aaaa', 1, {}, 'x')], undefined],
    ['initActor', 'D', 'qqqq'],
    ['remote', 'E', [ch('cccc', 2, {}, 'k'), ch('dddd', 1, { cccc: 2 }, 'k')]],
    ['remote', 'D', [ch('aaaa', 3, {}, 'x')]],
    ['snapshot', 'D'],
    ['snapshot', 'E'],
  ],
}

function run(steps) {
  const trace = []
  const docs = {}
  const notify = (m) => trace.push({ msg: m.type, id: m.id, minimumClockSatisfied: m.minimumClockSatisfied,
    history: m.history, actorId: m.actorId, patch: m.patch !== undefined })
  for (const [op, id, a, b] of steps) {
    if (op === 'new') docs[id] = new DocBackend(id, notify)
    else if (op === 'readyPush') docs[id].ready.push(() => docs[id].applyRemoteChanges(a))
    else if (op === 'remote') docs[id].applyRemoteChanges(a)
    else if (op === 'init') docs[id].init(a, b)
    else if (op === 'minClock') docs[id].updateMinimumClock(a)
    else if (op === 'initActor') docs[id].initActor(a)
    else if (op === 'snapshot') {
      const d = docs[id]
      trace.push({ snapshot: id, clock: Object.assign({}, d.clock), minimumClockSatisfied: d.minimumClockSatisfied,
        actorId: d.actorId })
    }
  }
  return trace
}

const out = { generator: 'tools/golden/gen_docbackend_traces.js', reference: 'dist/DocBackend.js', scenarios: {} }
for (const [name, steps] of Object.entries(SCENARIOS)) out.scenarios[name] = { steps, trace: run(steps) }
fs.rmSync ? fs.rmSync(tmp, { recursive: true, force: true }) : null
process.stdout.write(JSON.stringify(out, null, 1) + '\n')
