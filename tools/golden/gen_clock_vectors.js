// Generates tests/golden/clock_vectors.json by running the reference's own
// compiled Clock module (dist/Clock.js, from src/Clock.ts) in Node.
// Run in the build container only:  node tools/golden/gen_clock_vectors.js /root/reference
// The output is data (inputs + outputs); no reference source is copied.
const path = require('path')
const fs = require('fs')
const ref = process.argv[2] || '/root/reference'
const Clock = require(path.join(ref, 'dist', 'Clock.js'))

// deterministic PRNG
let s = 0x5eed1234
const rnd = () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s / 4294967296 }
const ACTORS = ['a', 'b', 'c', 'd', 'e', 'f', 'g', 'h']
function randClock() {
  const c = {}
  const n = Math.floor(rnd() * 5)
  const ids = ACTORS.slice().sort(() => rnd() - 0.5).slice(0, n)
  for (const id of ids) {
    const r = rnd()
    c[id] = r < 0.15 ? 0 : Math.floor(rnd() * 6)   // zero entries on purpose (src/Clock.ts:13-21)
  }
  return c
}
const enc = (v) => (v === Infinity ? 'Infinity' : v)
const encClock = (c) => { const o = {}; for (const k of Object.keys(c)) o[k] = enc(c[k]); return o }
const out = { source: 'dist/Clock.js (reference build of src/Clock.ts)', cases: [] }
// the reference's own unit tests (tests/unit.test.ts)
const unit = [
  [{ a: 100, b: 100, c: 100 }, { a: 101, b: 101, c: 101 }],
  [{ a: 100, b: 100, c: 100 }, { a: 101, b: 100, c: 100 }],
  [{ a: 100, b: 100, c: 100 }, { a: 100, b: 100, c: 100, d: 1 }],
  [{ a: 100, b: 100, c: 100 }, { a: 101, b: 100, c: 100, d: 1 }],
  [{ a: 100, b: 100, c: 100 }, { a: 99, b: 101, c: 100, d: 1 }],
  [{ a: 100, b: 200, c: 300 }, { b: 10, c: 2000, d: 50 }],
  [{ x: 1, y: 0 }, { x: 1 }],
  [{}, { z: 0 }],
]
const pairs = unit.slice()
for (let i = 0; i < 400; i++) pairs.push([randClock(), randClock()])
// Infinity via strs2clock (src/Clock.ts:40-53)
pairs.push([Clock.strs2clock(['a', 'b:3']), { a: 5, b: 3 }])
pairs.push([Clock.strs2clock('a'), { a: 7 }])
for (const [a, b] of pairs) {
  out.cases.push({
    a: encClock(a), b: encClock(b),
    gte: Clock.gte(a, b), cmp: Clock.cmp(a, b), equal: Clock.equal(a, b),
    equivalent: Clock.equivalent(a, b),
    union: encClock(Clock.union(a, b)), union_keys: Object.keys(Clock.union(a, b)),
    intersection: encClock(Clock.intersection(a, b)),
  })
}
out.strs2clock = [['a'], ['a:3', 'b'], ['x:0', 'y:12']].map((x) => ({ in: x, out: encClock(Clock.strs2clock(x)) }))
out.clock2strs = [{ a: Infinity, b: 3 }, { x: 0 }].map((c) => ({ in: encClock(c), out: Clock.clock2strs(c) }))
fs.mkdirSync(path.join(__dirname, '..', '..', 'tests', 'golden'), { recursive: true })
fs.writeFileSync(path.join(__dirname, '..', '..', 'tests', 'golden', 'clock_vectors.json'), JSON.stringify(out, null, 0))
console.log('cases', out.cases.length)
