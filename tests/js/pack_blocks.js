'use strict'
// Block.pack (src/Block.ts:6-16) for test inputs: stdin = {docs: [[change, ...], ...], brotli:
// 'auto' | 'always' | 'never'}; stdout = {docs: [[base64 block, ...], ...]}.  'auto' keeps raw
// JSON when brotli (text mode, Node's zlib: the iltorb stream format) is larger, as pack does.
const zlib = require('zlib')
const input = JSON.parse(require('fs').readFileSync(0, 'utf8'))
const mode = input.brotli || 'auto'
const pack = (obj) => {
  const source = Buffer.from(JSON.stringify(obj))
  if (mode === 'never') return source
  const body = zlib.brotliCompressSync(source, { params: { [zlib.constants.BROTLI_PARAM_MODE]: zlib.constants.BROTLI_MODE_TEXT } })
  if (mode === 'auto' && source.length < body.length) return source
  return Buffer.concat([Buffer.from('BR'), body])
}
process.stdout.write(JSON.stringify({ docs: input.docs.map((d) => d.map((c) => pack(c).toString('base64'))) }) + '\n')
