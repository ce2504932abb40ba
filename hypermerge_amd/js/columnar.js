'use strict'
// columnar.js — the Node host's encoder: decoded Automerge 0.12 `Change` objects
// (what Block.unpack yields, src/Block.ts:18-29, src/Actor.ts:137-141) -> the columnar
// rows of include/hypermerge_amd.h.  Mirror of hypermerge_amd/store.py DocEncoder:
// per document, actor ids keep their JS string order as the rank (a new actor can
// re-rank earlier rows: the engine applies the returned remap on the device); object
// UUIDs, (object, key) / (list, elemId) registers and change contents keep the ids they
// were first given.  Strings never reach the device.

const ROOT_ID = '00000000-0000-0000-0000-000000000000'
const ACTIONS = { makeMap: 0, makeTable: 1, makeList: 2, makeText: 3, ins: 4, set: 5, del: 6, link: 7, inc: 8 }
const DATATYPES = { counter: 1, timestamp: 2 }
const V = { NULL: 0, FALSE: 1, TRUE: 2, INT: 3, FLOAT: 4, STR: 5, OBJ: 6 }
const HEAD = 0xffffffff
const NONE = 0xffffffff
const DOC_HAS_LISTS = 1
const DOC_HAS_COUNTERS = 2
const TWO53 = 9007199254740992

// row sizes (bytes)
const DOC_ROW = 48, CHANGE_ROW = 24, DEP_ROW = 8, OP_ROW = 32, DOC_RESULT = 32, REG_RESULT = 16, SURV_RESULT = 16

class StringPool {
  constructor() { this.index = new Map(); this.strings = [] }
  intern(s) {
    let i = this.index.get(s)
    if (i === undefined) { i = this.strings.length; this.index.set(s, i); this.strings.push(s) }
    return i
  }
}

// Immutable.fromJS(change).equals(other): maps compare order-insensitively, lists in order
function canonical(x) {
  if (x === null || typeof x !== 'object') return JSON.stringify(x)
  if (Array.isArray(x)) return '[' + x.map(canonical).join(',') + ']'
  return '{' + Object.keys(x).sort().map((k) => JSON.stringify(k) + ':' + canonical(x[k])).join(',') + '}'
}

const f64 = new Float64Array(1)
const f64u = new Uint32Array(f64.buffer)

class DocEncoder {
  constructor(pool) {
    this.pool = pool
    this.actors = []                 // rank -> actor id
    this.objs = new Map([[ROOT_ID, 0]])
    this.objList = [ROOT_ID]
    this.regs = new Map()            // `${obj}\u0000${key}` -> reg
    this.regList = []                // reg -> [obj, key]
    this.content = new Map()         // `${actor}\u0000${seq}` -> [[cid, canonical|null, change]]
    this.nContent = 0
    this.flags = 0
    this.journal = null              // content entries replaced since the last snapshot
  }

  obj(u) {
    let i = this.objs.get(u)
    if (i === undefined) { i = this.objList.length; this.objs.set(u, i); this.objList.push(u) }
    return i
  }

  reg(o, key) {
    const k = o + '\u0000' + key
    let i = this.regs.get(k)
    if (i === undefined) { i = this.regList.length; this.regs.set(k, i); this.regList.push([o, key]) }
    return i
  }

  // O(1) snapshot: the tables only grow (actors are replaced, never edited), so a snapshot is
  // their lengths plus a journal of the content entries an encode replaces
  snapshot() {
    this.journal = []
    return [this.actors, this.objList.length, this.regList.length, this.nContent, this.flags, this.journal]
  }

  restore(s) {
    const [actors, nObj, nReg, nContent, flags, journal] = s
    this.actors = actors
    for (let i = nObj; i < this.objList.length; i++) this.objs.delete(this.objList[i])
    this.objList.length = nObj
    for (let i = nReg; i < this.regList.length; i++) this.regs.delete(this.regList[i][0] + '\u0000' + this.regList[i][1])
    this.regList.length = nReg
    for (let i = journal.length - 1; i >= 0; i--) {
      const [k, prev] = journal[i]
      if (prev === undefined) this.content.delete(k); else this.content.set(k, prev)
    }
    journal.length = 0
    this.nContent = nContent
    this.flags = flags
  }

  // content id (Immutable `equals` classes): equal content needs equal (actor, seq), so the
  // canonical form is only built when an (actor, seq) repeats in the document
  contentId(c) {
    const k = c.actor + '\u0000' + c.seq
    const ent = this.content.get(k)
    if (ent === undefined) {
      const cid = this.nContent++
      if (this.journal) this.journal.push([k, undefined])
      this.content.set(k, [[cid, null, c]])
      return cid
    }
    const ck = canonical(c)
    for (const e of ent) {
      if (e[1] === null) e[1] = canonical(e[2])
      if (e[1] === ck) return e[0]
    }
    const cid = this.nContent++
    if (this.journal) this.journal.push([k, ent])
    this.content.set(k, ent.concat([[cid, ck, c]]))
    return cid
  }

  // -> { changes: Buffer, deps: Buffer, ops: Buffer, nActors, nRegs, nObjs, flags, remap: Uint8Array|null }
  encode(changes, extraActors) {
    const known = new Set(this.actors)
    const fresh = new Set()
    const addActor = (a) => { if (!known.has(a)) fresh.add(a) }
    ;(extraActors || []).forEach(addActor)
    for (const c of changes) {
      addActor(c.actor)
      for (const a of Object.keys(c.deps || {})) addActor(a)
    }
    let remap = null
    if (fresh.size) {
      const ranked = this.actors.concat(Array.from(fresh)).sort()   // JS string order (UTF-16 code units)
      const rank = new Map(ranked.map((a, i) => [a, i]))
      if (this.actors.length) {
        const mp = Uint8Array.from(this.actors.map((a) => rank.get(a)))
        if (mp.some((v, i) => v !== i)) remap = mp
      }
      this.actors = ranked
    }
    const rank = new Map(this.actors.map((a, i) => [a, i]))
    let nDeps = 0, nOps = 0
    for (const c of changes) { nDeps += Object.keys(c.deps || {}).length; nOps += (c.ops || []).length }
    const cb = Buffer.alloc(changes.length * CHANGE_ROW)
    const db = Buffer.alloc(nDeps * DEP_ROW)
    const ob = Buffer.alloc(nOps * OP_ROW)
    let di = 0, oi = 0, flags = 0
    changes.forEach((c, ci) => {
      const deps = c.deps || {}
      const depOff = di
      for (const a of Object.keys(deps)) {
        db.writeUInt16LE(rank.get(a), di * DEP_ROW)
        db.writeUInt32LE(deps[a] >>> 0, di * DEP_ROW + 4)
        di++
      }
      const cid = this.contentId(c)
      const opFirst = oi
      for (const op of c.ops || []) {
        const act = ACTIONS[op.action]
        if (act === undefined) throw new Error(`unknown op action ${op.action}`)
        const o = this.obj(op.obj)
        let reg = NONE, parent = NONE, elem = 0, key = 0, vt = V.NULL, lo = 0, hi = 0
        if (act === ACTIONS.ins) {
          elem = op.elem >>> 0
          reg = this.reg(o, `${c.actor}:${op.elem}`)
          parent = op.key === '_head' ? HEAD : this.reg(o, op.key)
        } else if (act >= ACTIONS.set) {
          reg = this.reg(o, op.key)
          key = this.pool.intern(op.key)
          if (act === ACTIONS.link) { vt = V.OBJ; lo = this.obj(op.value) } else if (act !== ACTIONS.del) {
            const v = op.value
            if (v === null || v === undefined) vt = V.NULL
            else if (v === true) vt = V.TRUE
            else if (v === false) vt = V.FALSE
            else if (typeof v === 'number') {
              if (Number.isInteger(v) && Math.abs(v) < TWO53) {
                vt = V.INT
                lo = v >>> 0
                hi = Math.floor(v / 4294967296) >>> 0      // two's complement high word
              } else { vt = V.FLOAT; f64[0] = v; lo = f64u[0]; hi = f64u[1] }
            } else if (typeof v === 'string') { vt = V.STR; lo = this.pool.intern(v) } else {
              throw new Error(`unsupported op value ${JSON.stringify(v)}`)
            }
          }
        }
        const dt = op.datatype ? DATATYPES[op.datatype] : 0
        if (act === ACTIONS.makeList || act === ACTIONS.makeText) flags |= DOC_HAS_LISTS
        if (act === ACTIONS.inc || dt === DATATYPES.counter) flags |= DOC_HAS_COUNTERS
        const b = oi * OP_ROW
        ob.writeUInt32LE(o, b); ob.writeUInt32LE(reg >>> 0, b + 4); ob.writeUInt32LE(parent >>> 0, b + 8)
        ob.writeUInt32LE(elem, b + 12); ob.writeUInt8(act, b + 16); ob.writeUInt8(dt, b + 17); ob.writeUInt8(vt, b + 18)
        ob.writeUInt32LE(key, b + 20); ob.writeUInt32LE(lo, b + 24); ob.writeUInt32LE(hi, b + 28)
        oi++
      }
      const b = ci * CHANGE_ROW
      cb.writeUInt16LE(rank.get(c.actor), b); cb.writeUInt16LE(Object.keys(deps).length, b + 2)
      cb.writeUInt32LE(c.seq >>> 0, b + 4); cb.writeUInt32LE(depOff, b + 8)
      cb.writeUInt32LE(oi - opFirst, b + 12); cb.writeUInt32LE(opFirst, b + 16); cb.writeUInt32LE(cid, b + 20)
    })
    this.flags |= flags
    return { changes: cb, deps: db, ops: ob, nActors: this.actors.length, nRegs: this.regList.length,
      nObjs: this.objList.length, flags, remap }
  }
}

// Block.unpack (src/Block.ts:18-29): a hypercore block is raw JSON (header '{"', blocks
// written before compression was added) or 'BR' + brotli(JSON).  iltorb (the reference's native
// brotli) is not part of this engine; Node's zlib brotli decodes the same stream format.
// JsonBuffer.parse is JSON.parse(buffer.toString()) (src/JsonBuffer.ts:1-4).
const zlib = require('zlib')
function unpackBlock(data) {
  const buf = Buffer.isBuffer(data) ? data : Buffer.from(data.buffer, data.byteOffset, data.byteLength)
  const header = buf.slice(0, 2).toString()
  switch (header) {
    case '{"':
      return JSON.parse(buf.toString())
    case 'BR':
      return JSON.parse(zlib.brotliDecompressSync(buf.slice(2)).toString())
    default:
      throw new Error(`fail to unpack blocks - head is '${header}'`)
  }
}

// Actor.parseBlock over downloaded blocks (src/Actor.ts:120-141): one Change per block
function unpackBlocks(blocks) { return blocks.map(unpackBlock) }

// Concatenate per-document appends into one hm_batch (rows' offsets rebased).
function buildBatch(appends, aStride) {
  const n = appends.length
  let nc = 0, nd = 0, no = 0
  for (const a of appends) { nc += a.changes.length / CHANGE_ROW; nd += a.deps.length / DEP_ROW; no += a.ops.length / OP_ROW }
  const docs = Buffer.alloc(n * DOC_ROW)
  const changes = Buffer.alloc(nc * CHANGE_ROW), deps = Buffer.alloc(nd * DEP_ROW), ops = Buffer.alloc(no * OP_ROW)
  let remap = null
  let c0 = 0, d0 = 0, o0 = 0
  appends.forEach((a, i) => {
    const k = a.changes.length / CHANGE_ROW, kd = a.deps.length / DEP_ROW, ko = a.ops.length / OP_ROW
    const b = i * DOC_ROW
    docs.writeUInt32LE(c0, b); docs.writeUInt32LE(k, b + 4); docs.writeUInt32LE(d0, b + 8); docs.writeUInt32LE(kd, b + 12)
    docs.writeUInt32LE(o0, b + 16); docs.writeUInt32LE(ko, b + 20); docs.writeUInt32LE(0, b + 24)
    docs.writeUInt32LE(a.nRegs, b + 28); docs.writeUInt32LE(a.nObjs, b + 32)
    docs.writeUInt16LE(a.nActors, b + 36); docs.writeUInt16LE(a.flags, b + 38)
    a.changes.copy(changes, c0 * CHANGE_ROW)
    for (let j = 0; j < k; j++) {
      const r = (c0 + j) * CHANGE_ROW
      changes.writeUInt32LE(changes.readUInt32LE(r + 8) + d0, r + 8)
      changes.writeUInt32LE(changes.readUInt32LE(r + 16) + o0, r + 16)
    }
    a.deps.copy(deps, d0 * DEP_ROW)
    a.ops.copy(ops, o0 * OP_ROW)
    if (a.remap) {
      if (!remap) {
        remap = Buffer.alloc(n * aStride)
        for (let r = 0; r < n; r++) for (let x = 0; x < aStride; x++) remap[r * aStride + x] = x
      }
      for (let x = 0; x < a.remap.length; x++) remap[i * aStride + x] = a.remap[x]
    }
    c0 += k; d0 += kd; o0 += ko
  })
  return { docs, changes, deps, ops, remap }
}

function readDocResult(buf, i) {
  const b = i * DOC_RESULT
  return {
    status: buf.readInt32LE(b), errChange: buf.readUInt32LE(b + 4), errOp: buf.readUInt32LE(b + 8),
    histLen: buf.readUInt32LE(b + 12), nQueued: buf.readUInt32LE(b + 16), nSurv: buf.readUInt32LE(b + 20),
    minCmp: buf.readUInt32LE(b + 24),
  }
}

module.exports = {
  ROOT_ID, ACTIONS, DATATYPES, V, HEAD, NONE, DOC_HAS_LISTS, DOC_HAS_COUNTERS,
  DOC_ROW, CHANGE_ROW, DEP_ROW, OP_ROW, DOC_RESULT, REG_RESULT, SURV_RESULT,
  StringPool, DocEncoder, buildBatch, readDocResult, canonical, unpackBlock, unpackBlocks,
}
