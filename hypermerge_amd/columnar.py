"""Columnar batch format (mirror of include/hypermerge_amd.h) and the
JSON ``Change`` -> columnar encoder.

The reference hands Automerge 0.12 a JS array of decoded ``Change`` objects
(``src/DocBackend.ts:172``; decoded by ``Block.unpack``, ``src/Block.ts:18-29``,
from hypercore blocks in ``Actor.parseBlock``, ``src/Actor.ts:137-141``).
Here the same changes become plain integer tables so the merge can run on
the GPU:

* actor id strings -> per-document *rank* in JS (UTF-16 code unit) string
  order, so every Automerge ``sortBy(actor)`` / ``lamportCompare`` actor tie
  break is an integer compare;
* object UUIDs -> per-document object ids (``ROOT`` = 0);
* (object, key) and (list, elemId) -> per-document *register* ids;
* a change's full content -> ``content_id`` (equal ids <=> Immutable
  ``change.equals``), for the duplicate-seq check of ``applyChange``.
"""
from __future__ import annotations

import ctypes
import json
import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

ROOT_ID = "00000000-0000-0000-0000-000000000000"

# enums (hypermerge_amd.h)
MAKE_MAP, MAKE_TABLE, MAKE_LIST, MAKE_TEXT, INS, SET, DEL, LINK, INC = range(9)
ACTIONS = {"makeMap": MAKE_MAP, "makeTable": MAKE_TABLE, "makeList": MAKE_LIST,
           "makeText": MAKE_TEXT, "ins": INS, "set": SET, "del": DEL, "link": LINK, "inc": INC}
ACTION_NAMES = {v: k for k, v in ACTIONS.items()}
DT_NONE, DT_COUNTER, DT_TIMESTAMP = 0, 1, 2
DATATYPES = {None: DT_NONE, "counter": DT_COUNTER, "timestamp": DT_TIMESTAMP}
V_NULL, V_FALSE, V_TRUE, V_INT, V_FLOAT, V_STR, V_OBJ = range(7)
HEAD = 0xFFFFFFFF
NONE = 0xFFFFFFFF
DOC_HAS_LISTS = 1
DOC_HAS_COUNTERS = 2
TWO53 = 2 ** 53

STATUS = {0: "OK", 1: "INCONSISTENT_SEQ", 2: "UNKNOWN_OBJECT", 3: "DUPLICATE_OBJECT",
          4: "DUPLICATE_ELEM", 5: "MISSING_ELEM", 16: "UNSUPPORTED", 32: "INVALID",
          33: "DEVICE", 34: "NOMEM"}

DOC_DT = np.dtype([("change_off", "<u4"), ("n_changes", "<u4"), ("dep_off", "<u4"), ("n_deps", "<u4"),
                   ("op_off", "<u4"), ("n_ops", "<u4"), ("reg_off", "<u4"), ("n_regs", "<u4"),
                   ("n_objs", "<u4"), ("n_actors", "<u2"), ("flags", "<u2"), ("reserved", "<u4", (2,))])
CHANGE_DT = np.dtype([("actor", "<u2"), ("n_deps", "<u2"), ("seq", "<u4"), ("dep_off", "<u4"),
                      ("n_ops", "<u4"), ("op_first", "<u4"), ("content_id", "<u4")])
DEP_DT = np.dtype([("actor", "<u2"), ("pad", "<u2"), ("seq", "<u4")])
OP_DT = np.dtype([("obj", "<u4"), ("reg", "<u4"), ("parent", "<u4"), ("elem", "<u4"),
                  ("action", "u1"), ("datatype", "u1"), ("vtag", "u1"), ("pad", "u1"),
                  ("key", "<u4"), ("value", "<u8")])
DOC_RESULT_DT = np.dtype([("status", "<i4"), ("err_change", "<u4"), ("err_op", "<u4"),
                          ("hist_len", "<u4"), ("n_queued", "<u4"), ("n_surv", "<u4"),
                          ("min_cmp", "<u4"), ("pad", "<u4")])
REG_RESULT_DT = np.dtype([("n_surv", "<u4"), ("surv_off", "<u4"), ("list_index", "<i4"),
                          ("obj", "<u4")])
SURV_RESULT_DT = np.dtype([("op", "<u4"), ("vtag", "<u4"), ("value", "<u8")])
assert DOC_DT.itemsize == 48 and CHANGE_DT.itemsize == 24 and DEP_DT.itemsize == 8
assert OP_DT.itemsize == 32 and DOC_RESULT_DT.itemsize == 32
assert REG_RESULT_DT.itemsize == 16 and SURV_RESULT_DT.itemsize == 16


class CBatch(ctypes.Structure):
    """struct hm_batch"""
    _fields_ = [("n_docs", ctypes.c_uint32), ("n_changes", ctypes.c_uint32),
                ("n_deps", ctypes.c_uint32), ("n_ops", ctypes.c_uint32),
                ("n_regs", ctypes.c_uint32), ("a_stride", ctypes.c_uint32),
                ("max_changes", ctypes.c_uint32), ("max_ops", ctypes.c_uint32),
                ("max_regs", ctypes.c_uint32), ("max_objs", ctypes.c_uint32),
                ("doc_flags", ctypes.c_uint32), ("max_deps", ctypes.c_uint32),
                ("docs", ctypes.c_void_p), ("changes", ctypes.c_void_p),
                ("deps", ctypes.c_void_p), ("ops", ctypes.c_void_p),
                ("min_clock", ctypes.c_void_p)]


class CResults(ctypes.Structure):
    """struct hm_results"""
    _fields_ = [("docs", ctypes.c_void_p), ("clock", ctypes.c_void_p),
                ("back_clock", ctypes.c_void_p), ("heads", ctypes.c_void_p),
                ("hist", ctypes.c_void_p), ("all_deps", ctypes.c_void_p),
                ("regs", ctypes.c_void_p), ("surv", ctypes.c_void_p)]


def js_key(s: str) -> bytes:
    """Sort key giving JS ``<`` order on strings (UTF-16 code units)."""
    return s.encode("utf-16-be", "surrogatepass")


def _norm_json(x: Any) -> Any:
    """Value-equality normal form of a JSON value (JS has one number type)."""
    if isinstance(x, bool) or x is None or isinstance(x, str):
        return x
    if isinstance(x, (int, float)):
        f = float(x)
        if math.isfinite(f) and f == int(f) and abs(f) < TWO53:
            return int(f)
        return f
    if isinstance(x, dict):
        return {k: _norm_json(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm_json(v) for v in x]
    return x


def content_key(change: Dict[str, Any]) -> str:
    """Immutable ``Map.equals`` is order-insensitive for maps, order-sensitive for lists."""
    return json.dumps(_norm_json(change), sort_keys=True, separators=(",", ":"))


@dataclass
class Batch:
    docs: np.ndarray
    changes: np.ndarray
    deps: np.ndarray
    ops: np.ndarray
    a_stride: int
    min_clock: Optional[np.ndarray] = None
    # string tables (host side only; never shipped to the device)
    strings: List[str] = field(default_factory=list)          # string pool (keys + values)
    doc_actors: List[List[str]] = field(default_factory=list)  # rank -> actor id
    doc_objs: List[List[str]] = field(default_factory=list)    # obj id -> uuid
    doc_regs: List[List[Tuple[int, str]]] = field(default_factory=list)  # reg -> (obj, key|elemId)

    @property
    def n_docs(self) -> int:
        return len(self.docs)

    def c_struct(self) -> CBatch:
        for a in (self.docs, self.changes, self.deps, self.ops):
            assert a.flags["C_CONTIGUOUS"]
        mc = None
        if self.min_clock is not None:
            assert self.min_clock.dtype == np.uint32 and self.min_clock.flags["C_CONTIGUOUS"]
            mc = self.min_clock.ctypes.data
        nd = len(self.docs)
        mx = (lambda f: int(self.docs[f].max()) if nd else 0)
        return CBatch(nd, len(self.changes), len(self.deps), len(self.ops),
                      int(self.docs["n_regs"].sum()) if nd else 0, self.a_stride,
                      mx("n_changes"), mx("n_ops"), mx("n_regs"), mx("n_objs"),
                      int(np.bitwise_or.reduce(self.docs["flags"])) if nd else 0, mx("n_deps"),
                      self.docs.ctypes.data, self.changes.ctypes.data, self.deps.ctypes.data,
                      self.ops.ctypes.data, mc)

    def doc_algorithmic_bytes(self, results: Optional["Results"] = None) -> np.ndarray:
        """Per document, SURVEY.md §8(d): Σ_changes(24 + 8·nDeps + 4·A) + Σ_ops 32 + 8·A
        + Σ_segments 16 + Σ_conflicts 16 (A = the batch's per-actor row stride; a segment is
        a register, its winner or element order written once; conflicts = survivors beyond
        each register's winner, so they need ``results.regs``)."""
        A = self.a_stride
        d = self.docs
        b = (d["n_changes"].astype(np.int64) * (24 + 4 * A) + 8 * d["n_deps"].astype(np.int64)
             + 32 * d["n_ops"].astype(np.int64) + 8 * A + 16 * d["n_regs"].astype(np.int64))
        if results is not None and results.regs is not None and len(d):
            live = np.concatenate([[0], np.cumsum(results.regs["n_surv"] > 0, dtype=np.int64)])
            lo = d["reg_off"].astype(np.int64)
            hi = lo + d["n_regs"].astype(np.int64)
            winners = live[hi] - live[lo]
            b += 16 * (results.docs["n_surv"].astype(np.int64) - winners)
        return b

    def algorithmic_bytes(self, results: Optional["Results"] = None) -> int:
        return int(self.doc_algorithmic_bytes(results).sum())

@dataclass
class Results:
    docs: np.ndarray
    clock: np.ndarray
    back_clock: np.ndarray
    heads: np.ndarray
    hist: np.ndarray
    all_deps: np.ndarray
    regs: np.ndarray
    surv: np.ndarray

    @staticmethod
    def alloc(b: Batch) -> "Results":
        S = b.a_stride
        nd, nc, no = len(b.docs), len(b.changes), len(b.ops)
        nr = int(b.docs["n_regs"].sum()) if nd else 0
        return Results(np.zeros(nd, DOC_RESULT_DT), np.zeros(nd * S, np.uint32),
                       np.zeros(nd * S, np.uint32), np.zeros(nd * S, np.uint32),
                       np.zeros(nc, np.int32), np.zeros(nc * S, np.uint32),
                       np.zeros(max(nr, 0), REG_RESULT_DT), np.zeros(no, SURV_RESULT_DT))

    def c_struct(self) -> CResults:
        return CResults(*(a.ctypes.data for a in (self.docs, self.clock, self.back_clock, self.heads,
                                                  self.hist, self.all_deps, self.regs, self.surv)))


def _value(v: Any, strings: Dict[str, int], pool: List[str], objs: Dict[str, int]) -> Tuple[int, int]:
    if v is None:
        return V_NULL, 0
    if v is True:
        return V_TRUE, 0
    if v is False:
        return V_FALSE, 0
    if isinstance(v, (int, float)):
        f = float(v)
        if math.isfinite(f) and f == int(f) and abs(f) < TWO53:
            return V_INT, int(f) & 0xFFFFFFFFFFFFFFFF
        return V_FLOAT, int(np.array([f], "<f8").view("<u8")[0])
    if isinstance(v, str):
        if v not in strings:
            strings[v] = len(pool)
            pool.append(v)
        return V_STR, strings[v]
    raise TypeError(f"unsupported op value {v!r}")


class BatchBuilder:
    """Encodes per-document lists of Automerge 0.12 ``Change`` dicts."""

    def __init__(self) -> None:
        self._docs: List[Tuple] = []
        self._changes: List[Tuple] = []
        self._deps: List[Tuple] = []
        self._ops: List[Tuple] = []
        self._strings: Dict[str, int] = {}
        self._pool: List[str] = []
        self._content: Dict[str, int] = {}
        self._doc_actors: List[List[str]] = []
        self._doc_objs: List[List[str]] = []
        self._doc_regs: List[List[Tuple[int, str]]] = []
        self._reg_off = 0
        self._max_actors = 1

    def _intern(self, s: str) -> int:
        if s not in self._strings:
            self._strings[s] = len(self._pool)
            self._pool.append(s)
        return self._strings[s]

    def add_doc(self, changes: Sequence[Dict[str, Any]], extra_actors: Sequence[str] = ()) -> int:
        actors = set(extra_actors)
        for c in changes:
            actors.add(c["actor"])
            actors.update((c.get("deps") or {}).keys())
        ranked = sorted(actors, key=js_key)
        rank = {a: i for i, a in enumerate(ranked)}
        objs: Dict[str, int] = {ROOT_ID: 0}
        obj_list = [ROOT_ID]
        regs: Dict[Tuple[int, str], int] = {}
        reg_list: List[Tuple[int, str]] = []

        def obj_id(u: str) -> int:
            if u not in objs:
                objs[u] = len(obj_list)
                obj_list.append(u)
            return objs[u]

        def reg_id(o: int, key: str) -> int:
            if (o, key) not in regs:
                regs[(o, key)] = len(reg_list)
                reg_list.append((o, key))
            return regs[(o, key)]

        change_off, op_off, dep_off0 = len(self._changes), len(self._ops), len(self._deps)
        for c in changes:
            a = rank[c["actor"]]
            deps = c.get("deps") or {}
            dep_off = len(self._deps)
            for da, ds in deps.items():
                self._deps.append((rank[da], 0, int(ds)))
            ck = content_key(c)
            if ck not in self._content:
                self._content[ck] = len(self._content)
            op_first = len(self._ops)
            for op in c.get("ops", []):
                act = ACTIONS[op["action"]]
                o = obj_id(op["obj"])
                reg, parent, elem, key = NONE, NONE, 0, NONE
                vt, val = V_NULL, 0
                if act == INS:
                    elem = int(op["elem"])
                    reg = reg_id(o, f"{c['actor']}:{elem}")
                    parent = HEAD if op["key"] == "_head" else reg_id(o, op["key"])
                elif act in (SET, DEL, LINK, INC):
                    reg = reg_id(o, op["key"])
                    key = self._intern(op["key"])
                    if act == LINK:
                        vt, val = V_OBJ, obj_id(op["value"])
                    elif act in (SET, INC):
                        vt, val = _value(op.get("value"), self._strings, self._pool, objs)
                dt = DATATYPES[op.get("datatype")]
                self._ops.append((o, reg, parent, elem, act, dt, vt, 0, key if key != NONE else 0, val))
            self._changes.append((a, len(deps), int(c["seq"]), dep_off, len(self._ops) - op_first,
                                  op_first, self._content[ck]))
        n_regs = len(reg_list)
        has_lists = any(o[4] in (MAKE_LIST, MAKE_TEXT) for o in self._ops[op_off:])
        has_counters = any(o[4] == INC or o[5] == DT_COUNTER for o in self._ops[op_off:])
        self._docs.append((change_off, len(changes), dep_off0, len(self._deps) - dep_off0,
                           op_off, len(self._ops) - op_off, self._reg_off, n_regs, len(obj_list), len(ranked),
                           (DOC_HAS_LISTS if has_lists else 0) | (DOC_HAS_COUNTERS if has_counters else 0),
                           (0, 0)))
        self._reg_off += n_regs
        self._max_actors = max(self._max_actors, len(ranked))
        self._doc_actors.append(ranked)
        self._doc_objs.append(obj_list)
        self._doc_regs.append(reg_list)
        return len(self._docs) - 1

    def build(self, a_stride: Optional[int] = None) -> Batch:
        S = a_stride or self._max_actors
        assert S >= self._max_actors
        return Batch(np.array(self._docs, DOC_DT), np.array(self._changes, CHANGE_DT),
                     np.array(self._deps, DEP_DT) if self._deps else np.zeros(0, DEP_DT),
                     np.array(self._ops, OP_DT) if self._ops else np.zeros(0, OP_DT), S,
                     None, list(self._pool), self._doc_actors, self._doc_objs, self._doc_regs)


def encode(docs: Sequence[Sequence[Dict[str, Any]]], a_stride: Optional[int] = None) -> Batch:
    bb = BatchBuilder()
    for d in docs:
        bb.add_doc(d)
    return bb.build(a_stride)


def decode_doc(b: Batch, d: int) -> List[Dict[str, Any]]:
    """Columnar rows of document d -> Automerge 0.12 ``Change`` dicts (test/bench
    utility: turns synthetic feeds into the JSON the host encoders take).  Names
    are synthesised where the batch carries no string tables: actor ids that sort
    in rank order, object UUIDs, map keys ``k<reg>``, string values ``s<id>``."""
    doc = b.docs[d]
    c0, n = int(doc["change_off"]), int(doc["n_changes"])
    o0, m = int(doc["op_off"]), int(doc["n_ops"])
    d0 = int(doc["dep_off"])
    A = int(doc["n_actors"])
    actors = b.doc_actors[d] if b.doc_actors else [f"actor{r:03d}" for r in range(A)]
    objs = b.doc_objs[d] if b.doc_objs else [ROOT_ID] + [f"{i:08x}-0000-4000-8000-{d:012x}" for i in range(1, int(doc["n_objs"]))]
    ops = b.ops[o0: o0 + m]
    chs = b.changes[c0: c0 + n]
    regkey: Dict[int, str] = {}
    if b.doc_regs:
        for g, (_, k) in enumerate(b.doc_regs[d]):
            regkey[g] = k
    else:
        for ch in chs:                                   # element registers: actor:elem of their ins
            s = int(ch["op_first"]) - o0
            for op in ops[s: s + int(ch["n_ops"])]:
                if op["action"] == INS:
                    regkey.setdefault(int(op["reg"]), f"{actors[int(ch['actor'])]}:{int(op['elem'])}")

    def key_of(reg: int) -> str:
        return regkey.get(reg, f"k{reg}")

    def val(op) -> Any:
        vt, v = int(op["vtag"]), int(op["value"])
        if vt == V_NULL:
            return None
        if vt in (V_FALSE, V_TRUE):
            return vt == V_TRUE
        if vt == V_INT:
            return v - (1 << 64) if v >= (1 << 63) else v
        if vt == V_FLOAT:
            return float(np.array([v], "<u8").view("<f8")[0])
        if vt == V_STR:
            return b.strings[v] if b.strings else f"s{v}"
        return objs[v]

    out = []
    for ch in chs:
        deps = {actors[int(x["actor"])]: int(x["seq"])
                for x in b.deps[int(ch["dep_off"]): int(ch["dep_off"]) + int(ch["n_deps"])]}
        s = int(ch["op_first"]) - o0
        jops = []
        for op in ops[s: s + int(ch["n_ops"])]:
            a = int(op["action"])
            j: Dict[str, Any] = {"action": ACTION_NAMES[a], "obj": objs[int(op["obj"])]}
            if a == INS:
                p = int(op["parent"])
                j["key"] = "_head" if p == HEAD else key_of(p)
                j["elem"] = int(op["elem"])
            elif a in (SET, DEL, LINK, INC):
                j["key"] = key_of(int(op["reg"]))
                if a == LINK:
                    j["value"] = objs[int(op["value"])]
                elif a != DEL:
                    j["value"] = val(op)
                if op["datatype"]:
                    j["datatype"] = {DT_COUNTER: "counter", DT_TIMESTAMP: "timestamp"}[int(op["datatype"])]
            jops.append(j)
        out.append({"actor": actors[int(ch["actor"])], "seq": int(ch["seq"]), "deps": deps, "ops": jops})
    return out
