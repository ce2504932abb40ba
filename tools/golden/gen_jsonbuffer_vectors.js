// Generates tests/golden/jsonbuffer_vectors.json by running the reference's own compiled
// JsonBuffer module (dist/JsonBuffer.js, from src/JsonBuffer.ts) in Node: every block is
// JsonBuffer.bufferify(change) (what Block.pack keeps when brotli does not shrink it,
// src/Block.ts:6-16) and its expected value JsonBuffer.parse(block) (src/Block.ts:23, the '{"'
// branch of unpack); malformed blocks record whether JsonBuffer.parse throws.
// Run in the build container only:  node tools/golden/gen_jsonbuffer_vectors.js /root/reference
// The output is data (inputs + outputs); no reference source is copied.
const path = require('path')
const fs = require('fs')
const ref = process.argv[2] || '/root/reference'
const JB = require(path.join(ref, 'dist', 'JsonBuffer.js'))
const ROOT = '00000000-0000-0000-0000-000000000000'
const L1 = '11111111-2222-4333-8444-555555555555'
const values = [0, -0, 1, -1, 7.5, 0.1 + 0.2, 1e21, -1e-7, 2 ** 53, -(2 ** 53), 2 ** 53 + 2, 1.7976931348623157e308,
  5e-324, 123456789.125, true, false, null, '', 'plain', 'é☃', '😀 surrogate pair', 'quote " and \\ backslash',
  'tab\tnewline\ncontrol\u0001', '  ', 'a'.repeat(300)]
const docs = []
// documents of valid changes: map sets of every value kind, counters, a list, deps, messages
{
  const chs = []
  let seq = { 'actor-b': 0, 'actor-a': 0, 'é-actor': 0 }
  const next = (a) => ++seq[a]
  values.forEach((v, i) => {
    const a = ['actor-b', 'actor-a', 'é-actor'][i % 3]
    const deps = i ? { [['actor-b', 'actor-a', 'é-actor'][(i + 1) % 3]]: Math.max(1, Math.floor(i / 3)) } : {}
    chs.push({ actor: a, seq: next(a), deps: i > 3 ? deps : {}, message: i % 4 === 0 ? `m${i} é` : undefined,
      ops: [{ action: 'set', obj: ROOT, key: `k${i % 5}`, value: v }] })
  })
  docs.push(chs)
  const d2 = [
    { actor: 'w', seq: 1, deps: {}, ops: [{ action: 'makeList', obj: L1 }, { action: 'link', obj: ROOT, key: 'list', value: L1 },
      { action: 'ins', obj: L1, key: '_head', elem: 1 }, { action: 'set', obj: L1, key: 'w:1', value: 'x' },
      { action: 'set', obj: ROOT, key: 'n', value: 3, datatype: 'counter' }] },
    { actor: 'v', seq: 1, deps: { w: 1 }, ops: [{ action: 'inc', obj: ROOT, key: 'n', value: 2.25 },
      { action: 'ins', obj: L1, key: 'w:1', elem: 2 }, { action: 'set', obj: L1, key: 'v:2', value: -0 },
      { action: 'del', obj: L1, key: 'w:1' }] },
    { actor: 'w', seq: 2, deps: { v: 1 }, requestType: 'change', ops: [{ action: 'set', obj: ROOT, key: 'd', value: 1e21, datatype: 'timestamp' }] },
  ]
  docs.push(d2)
}
const out = { source: 'dist/JsonBuffer.js (reference build of src/JsonBuffer.ts)', valid: [], malformed: [] }
for (const chs of docs) {
  out.valid.push(chs.map((c) => {
    const block = JB.bufferify(c)
    return { block: block.toString('base64'), parsed: JSON.stringify(JB.parse(block)) }
  }))
}
// malformed blocks: JsonBuffer.parse throws (Block.unpack's '{"' branch)
const bad = ['{"actor":"a","seq":1', '{"actor":"a","seq":tru}', '{"actor":"a"}x', '{"a":1,}', '{"a":"\\x"}', '{"a":01}',
  '{"a":"unterminated}']
for (const t of bad) {
  let throws = false
  try { JB.parse(Buffer.from(t)) } catch (e) { throws = true }
  out.malformed.push({ block: Buffer.from(t).toString('base64'), throws })
}
// headers Block.unpack rejects (src/Block.ts:20-27 switch on the first two bytes: only '{"' and 'BR'
// are blocks; anything else throws 'fail to unpack blocks - head is ...'): read from the source —
// dist/Block.js requires the native module iltorb, which is not installed, so it is not run
out.bad_header = ['[1,2]', ' {"actor":"a"}', '{ "actor":"a","seq":1,"deps":{},"ops":[]}', 'XY{"a":1}', ''].map((t) => Buffer.from(t).toString('base64'))
fs.writeFileSync(path.join(__dirname, '..', '..', 'tests', 'golden', 'jsonbuffer_vectors.json'), JSON.stringify(out, null, 1) + '\n')
console.log('valid docs', out.valid.length, 'malformed', out.malformed.length, 'bad headers', out.bad_header.length)
