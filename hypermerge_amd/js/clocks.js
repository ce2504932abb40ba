'use strict'
// Clock.js — vector-clock algebra with the reference's semantics (src/Clock.ts):
// a missing entry counts as 0 under gte/cmp/equal (src/Clock.ts:13-38); union keeps
// c1's keys then c2's new keys (src/Clock.ts:87-95).  Dense rank-indexed rows are what
// the engine works on; toRow/fromRow convert with a document's actor table.

function gte(a, b) {
  for (const id in a) if (a[id] < (b[id] || 0)) return false
  for (const id in b) if (b[id] > (a[id] || 0)) return false
  return true
}

function cmp(a, b) {
  const ag = gte(a, b), bg = gte(b, a)
  if (ag && bg) return 'EQ'
  if (ag) return 'GT'
  if (bg) return 'LT'
  return 'CONCUR'
}

const equal = (a, b) => cmp(a, b) === 'EQ'

function union(c1, c2) {
  const acc = Object.assign({}, c1)
  for (const id in c2) acc[id] = Math.max(acc[id] || 0, c2[id])
  return acc
}

const CMP_CODES = ['EQ', 'GT', 'LT', 'CONCUR']     // hm_doc_result.min_cmp

function toRow(clock, actors, aStride) {
  const row = new Uint32Array(aStride)
  actors.forEach((a, i) => { if (clock[a]) row[i] = Math.min(clock[a], 0xffffffff) })
  return row
}

function fromRow(buf, offset, actors) {
  const c = {}
  actors.forEach((a, i) => { const v = buf.readUInt32LE(offset + 4 * i); if (v) c[a] = v })
  return c
}

module.exports = { gte, cmp, equal, union, toRow, fromRow, CMP_CODES }
