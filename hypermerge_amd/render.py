"""Canonical materialized state rendered from the
engine's result tables.

Both the HIP engine and the CPU oracle fill the same ``Results`` tables, so
the same renderer turns either into canonical JSON; parity tests compare the
raw tables (bit-exact) *and* the rendered bytes.

Shape: maps are ``{"map": [[key, entry], ...]}`` with keys in JS string
order; lists/text are ``{"list": [entry, ...]}`` in document order, where
``entry = {"value": v, "conflicts": [[actor, v], ...], "datatype": dt}``
(conflicts/datatype omitted when empty).  Linked child objects are rendered
recursively in place of ``v``.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List

import numpy as np

from .columnar import (Batch, Results, js_key, MAKE_LIST, MAKE_TEXT, MAKE_TABLE, SET, LINK,
                       V_NULL, V_FALSE, V_TRUE, V_INT, V_FLOAT, V_STR, V_OBJ, STATUS)

_DT_NAMES = {1: "counter", 2: "timestamp"}


def _scalar(b: Batch, vtag: int, value: int) -> Any:
    if vtag == V_NULL:
        return None
    if vtag == V_FALSE:
        return False
    if vtag == V_TRUE:
        return True
    if vtag == V_INT:
        v = int(value)
        return v - (1 << 64) if v >= (1 << 63) else v
    if vtag == V_FLOAT:
        f = float(np.array([value], "<u8").view("<f8")[0])
        return int(f) if f.is_integer() and abs(f) < 2 ** 53 else f
    if vtag == V_STR:
        return b.strings[int(value)]
    raise ValueError(vtag)


def doc_state(b: Batch, r: Results, d: int) -> Dict[str, Any]:
    doc = b.docs[d]
    ops = b.ops[int(doc["op_off"]): int(doc["op_off"]) + int(doc["n_ops"])]
    changes = b.changes[int(doc["change_off"]): int(doc["change_off"]) + int(doc["n_changes"])]
    actors = b.doc_actors[d]
    regs = r.regs[int(doc["reg_off"]): int(doc["reg_off"]) + int(doc["n_regs"])]
    surv = r.surv[int(doc["op_off"]): int(doc["op_off"]) + int(doc["n_ops"])]
    # op -> issuing change's actor
    op_actor = np.zeros(len(ops), np.int64)
    for ch in changes:
        s = int(ch["op_first"]) - int(doc["op_off"])
        op_actor[s: s + int(ch["n_ops"])] = int(ch["actor"])
    objtype: Dict[int, int] = {0: -1}
    for op in ops:
        if op["action"] <= MAKE_TEXT:
            objtype.setdefault(int(op["obj"]), int(op["action"]))
    by_obj: Dict[int, List[int]] = {}
    for g, rr in enumerate(regs):
        if rr["n_surv"] > 0 and rr["obj"] != 0xFFFFFFFF:
            by_obj.setdefault(int(rr["obj"]), []).append(g)

    def value_of(k: int, vtag: int, value: int, depth: int) -> Any:
        if ops[k]["action"] == LINK or vtag == V_OBJ:
            return render(int(value), depth + 1)
        return _scalar(b, vtag, value)

    def entry(g: int, depth: int) -> Dict[str, Any]:
        rr = regs[g]
        ss = surv[int(rr["surv_off"]): int(rr["surv_off"]) + int(rr["n_surv"])]
        k0 = int(ss[0]["op"])
        e: Dict[str, Any] = {"value": value_of(k0, int(ss[0]["vtag"]), int(ss[0]["value"]), depth)}
        if ops[k0]["datatype"]:
            e["datatype"] = _DT_NAMES[int(ops[k0]["datatype"])]
        if len(ss) > 1:
            e["conflicts"] = [[actors[op_actor[int(s["op"])]],
                               value_of(int(s["op"]), int(s["vtag"]), int(s["value"]), depth)]
                              for s in ss[1:]]
        return e

    def render(o: int, depth: int = 0) -> Any:
        if depth > 64:
            return {"cycle": b.doc_objs[d][o]}
        t = objtype.get(o, -1)
        gs = by_obj.get(o, [])
        if t in (MAKE_LIST, MAKE_TEXT):
            gs = sorted((g for g in gs if regs[g]["list_index"] >= 0), key=lambda g: int(regs[g]["list_index"]))
            return {"text" if t == MAKE_TEXT else "list": [entry(g, depth) for g in gs]}
        keyed = sorted(((b.doc_regs[d][g][1], g) for g in gs), key=lambda kg: js_key(kg[0]))
        return {"table" if t == MAKE_TABLE else "map": [[k, entry(g, depth)] for k, g in keyed]}

    return render(0)


def doc_summary(b: Batch, r: Results, d: int) -> Dict[str, Any]:
    """Canonical per-doc record: state + clocks + deps + history (Appendix A.5)."""
    doc = b.docs[d]
    S = b.a_stride
    actors = b.doc_actors[d]
    A = int(doc["n_actors"])
    dr = r.docs[d]
    c0, n = int(doc["change_off"]), int(doc["n_changes"])
    hist = r.hist[c0: c0 + n]
    order = sorted((int(h), i) for i, h in enumerate(hist) if h >= 0)
    ch = b.changes[c0: c0 + n]
    out: Dict[str, Any] = {"status": STATUS.get(int(dr["status"]), str(int(dr["status"])))}
    if dr["status"] != 0:
        out["error_at"] = [int(dr["err_change"]), int(dr["err_op"])]
        return out

    def clk(a: np.ndarray) -> Dict[str, int]:
        row = a[d * S: d * S + A]
        return {actors[i]: int(row[i]) for i in range(A) if row[i]}

    out.update({
        "clock": clk(r.clock), "backend_clock": clk(r.back_clock), "deps": clk(r.heads),
        "history": [[actors[int(ch[i]["actor"])], int(ch[i]["seq"])] for _, i in order],
        "queued": int(dr["n_queued"]),
        "state": doc_state(b, r, d),
    })
    return out


def canonical_json(b: Batch, r: Results, d: int) -> str:
    return json.dumps(doc_summary(b, r, d), sort_keys=True, separators=(",", ":"))
