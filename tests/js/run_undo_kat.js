'use strict'
// Known answers of the JS restatement's local undo / redo (oracle/js/backend.js,
// Backend.applyLocalChange; SURVEY Appendix A.4 [R]): each case prints the materialized
// document and canUndo / canRedo after every request, and the thrown message where one throws.
const path = require('path')
const { Backend, materialize } = require(path.join(__dirname, '..', '..', 'oracle', 'js', 'backend.js'))
const R = '00000000-0000-0000-0000-000000000000'
const out = {}
function run(name, init, reqs) {
  let [s] = Backend.applyChanges(Backend.init(), init)
  const steps = []
  for (const q of reqs) {
    try {
      const [s2, p] = Backend.applyLocalChange(s, q)
      s = s2
      steps.push([materialize(s), p.canUndo, p.canRedo, p.actor, p.seq])
    } catch (e) { steps.push(['throw', e.message]) }
  }
  out[name] = steps
}
const ch = (seq, ops, extra) => Object.assign({ requestType: 'change', actor: 'loc', seq, deps: { rem: 1 }, ops }, extra || {})
const rq = (type, seq) => ({ requestType: type, actor: 'loc', seq, deps: { rem: 1 } })
const base = [{ actor: 'rem', seq: 1, deps: {}, ops: [{ action: 'set', obj: R, key: 'x', value: 1 },
  { action: 'set', obj: R, key: 'n', value: 5, datatype: 'counter' }, { action: 'makeList', obj: 'L' },
  { action: 'link', obj: R, key: 'l', value: 'L' }] }]
run('set_undo_redo', base, [ch(1, [{ action: 'set', obj: R, key: 'x', value: 2 }]), rq('undo', 2), rq('redo', 3), rq('redo', 4)])
run('new_key_undo_is_del', base, [ch(1, [{ action: 'set', obj: R, key: 'y', value: 'a' }]), rq('undo', 2)])
run('inc_undo', base, [ch(1, [{ action: 'inc', obj: R, key: 'n', value: 3 }]), rq('undo', 2), rq('redo', 3)])
run('list_insert_undo', base, [ch(1, [{ action: 'ins', obj: 'L', key: '_head', elem: 1 }, { action: 'set', obj: 'L', key: 'loc:1', value: 'a' }]),
  rq('undo', 2), rq('redo', 3)])
run('not_undoable', base, [ch(1, [{ action: 'set', obj: R, key: 'x', value: 2 }], { undoable: false }), rq('undo', 2)])
run('nothing_to_undo', base, [rq('undo', 1), rq('redo', 1)])
run('two_undos_then_change_clears_redo', base, [ch(1, [{ action: 'set', obj: R, key: 'x', value: 2 }]),
  ch(2, [{ action: 'set', obj: R, key: 'x', value: 3 }]), rq('undo', 3), rq('undo', 4), rq('undo', 5),
  ch(5, [{ action: 'set', obj: R, key: 'z', value: 0 }]), rq('redo', 6)])
run('same_key_twice_in_one_change', base, [ch(1, [{ action: 'set', obj: R, key: 'x', value: 2 }, { action: 'set', obj: R, key: 'x', value: 3 }]),
  rq('undo', 2)])
run('unknown_request_type', base, [{ requestType: 'bogus', actor: 'loc', seq: 1, deps: {} }])
process.stdout.write(JSON.stringify(out) + '\n')
