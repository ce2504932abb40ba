'use strict'
// Block round trips for tests/test_node_host.py: every change of the input is packed as a raw
// JSON block and as a 'BR' + brotli(text mode) block (the two forms src/Block.ts:6-16 writes),
// unpacked with columnar.unpackBlock, and both decodings are encoded to columnar rows.
const path = require('path')
const zlib = require('zlib')
const C = require(path.join(__dirname, '..', '..', 'hypermerge_amd', 'js', 'columnar'))

let input = ''
process.stdin.on('data', (d) => { input += d })
process.stdin.on('end', () => {
  const { changes } = JSON.parse(input)
  const raw = changes.map((c) => Buffer.from(JSON.stringify(c)))
  const br = raw.map((b) => Buffer.concat([Buffer.from('BR'), zlib.brotliCompressSync(b, {
    params: { [zlib.constants.BROTLI_PARAM_MODE]: zlib.constants.BROTLI_MODE_TEXT } })]))
  const a = C.unpackBlocks(raw), b = C.unpackBlocks(br.map((x) => new Uint8Array(x)))
  const same = changes.every((c, i) => C.canonical(c) === C.canonical(a[i]) && C.canonical(c) === C.canonical(b[i]))
  const ea = new C.DocEncoder(new C.StringPool()).encode(a), eb = new C.DocEncoder(new C.StringPool()).encode(b)
  const rowsSame = ea.changes.equals(eb.changes) && ea.deps.equals(eb.deps) && ea.ops.equals(eb.ops)
  let err = ''
  try { C.unpackBlock(Buffer.from('xx{}')) } catch (e) { err = e.message }
  process.stdout.write(JSON.stringify({ same, rowsSame, n: changes.length, brBytes: br.reduce((s, x) => s + x.length, 0),
    rawBytes: raw.reduce((s, x) => s + x.length, 0), err }))
})
