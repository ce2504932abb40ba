"""ctypes face of the docset (include/hypermerge_amd.h hm_docset_*, csrc/docset.cpp): the
Node drop-in's host engine — raw hypercore blocks of many documents in, one applyChanges round
each (src/DocBackend.ts:169-185), results + patches + DocBackend.clock out as JSON.

Used by the Python tests; the production caller is the N-API addon (js/hmgpu_node.c)."""
from __future__ import annotations

import ctypes
import sys
import json
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .columnar import DOC_RESULT_DT
from .decode import pack_offsets
from .engine import Engine, lib

NO_PATCHES = 1          # HM_DOCSET_NO_PATCHES
NET_DIFFS = 4           # HM_DOCSET_NET_DIFFS


class _Cfg(ctypes.Structure):
    _fields_ = [("threads", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class _Info(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint32) for f in ("a_stride", "n_changes", "n_ops", "n_actors", "n_objs", "n_regs",
                                               "hist_len", "n_queued")]


def _text(L, t) -> Tuple[str, np.ndarray]:
    n = ctypes.c_size_t()
    p = L.hm_text_data(t, ctypes.byref(n))
    s = ctypes.string_at(p, n.value).decode("utf-8", "surrogatepass") if n.value else ""
    k = ctypes.c_uint32()
    rp = L.hm_text_results(t, ctypes.byref(k))
    res = np.zeros(k.value, DOC_RESULT_DT)
    if k.value:
        ctypes.memmove(res.ctypes.data, rp, k.value * DOC_RESULT_DT.itemsize)
    L.hm_text_free(t)
    return s, res


class DocSet:
    def __init__(self, engine: Engine, threads: int = 0, patches: bool = True, net_diffs: bool = False):
        self._L, self.engine = lib(), engine
        h = ctypes.c_void_p()
        cfg = _Cfg(threads, (0 if patches else NO_PATCHES) | (NET_DIFFS if net_diffs else 0))
        engine._check(self._L.hm_docset_create(engine._h, ctypes.byref(cfg), ctypes.byref(h)), "hm_docset_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.hm_docset_destroy(self._h)
            self._h = None

    def __del__(self):
        # (at interpreter exit finalizers run in any order: the engine may be gone, and the
        # process releases the device anyway)
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    def open(self, n: int = 1) -> int:
        first = ctypes.c_uint32()
        self.engine._check(self._L.hm_docset_open(self._h, n, ctypes.byref(first)), "hm_docset_open")
        return first.value

    def apply(self, docs: Sequence[int], blocks: Sequence[Sequence[bytes]]) -> Tuple[np.ndarray, Dict[str, Any]]:
        """One applyChanges round: docs[i] receives blocks[i] (one JSON Change per block).
        Returns (per-document hm_doc_result rows, {"p": [patch|None], "b": [DocBackend.clock|None]})."""
        data, bo, db = pack_offsets(blocks)
        ids = np.ascontiguousarray(docs, np.uint32)
        t = ctypes.c_void_p()
        self.engine._check(self._L.hm_docset_apply(self._h, data.ctypes.data, bo.ctypes.data, db.ctypes.data,
                                                   ids.ctypes.data, len(ids), ctypes.byref(t)), "hm_docset_apply")
        s, res = _text(self._L, t)
        return res, json.loads(s)

    def info(self, doc: int) -> Dict[str, int]:
        i = _Info()
        self.engine._check(self._L.hm_docset_doc_info(self._h, doc, ctypes.byref(i)), "hm_docset_doc_info")
        return {f: int(getattr(i, f)) for f, _ in _Info._fields_}

    def history_prefix(self, doc: int, n: int) -> List[int]:
        out = np.zeros(max(n, 1), np.uint32)
        k = self._L.hm_docset_history_prefix(self._h, doc, n, out.ctypes.data)
        if k < 0:
            self.engine._check(-k, "hm_docset_history_prefix")
        return [int(x) for x in out[:k]]

    def clock_update(self, docs: Sequence[int]) -> Tuple[np.ndarray, np.ndarray, List[Dict[str, int]]]:
        ids = np.ascontiguousarray(docs, np.uint32)
        w = np.zeros(max(len(ids), 1), np.uint8)
        d = np.zeros(max(len(ids), 1), np.uint8)
        t = ctypes.c_void_p()
        self.engine._check(self._L.hm_docset_clock_update(self._h, len(ids), ids.ctypes.data, w.ctypes.data, d.ctypes.data,
                                                          ctypes.byref(t)), "hm_docset_clock_update")
        s, _ = _text(self._L, t)
        return w[:len(ids)], d[:len(ids)], json.loads(s)

    def view(self, doc: int) -> Dict[str, Any]:
        t = ctypes.c_void_p()
        self.engine._check(self._L.hm_docset_view(self._h, doc, ctypes.byref(t)), "hm_docset_view")
        s, _ = _text(self._L, t)
        return json.loads(s)

    def handles(self, a_stride: int) -> Dict[str, int]:
        """hm_docset_handles: handles opened in the a_stride store and released ones awaiting reuse."""
        o, f = ctypes.c_uint32(), ctypes.c_uint32()
        self.engine._check(self._L.hm_docset_handles(self._h, a_stride, ctypes.byref(o), ctypes.byref(f)),
                           "hm_docset_handles")
        return {"opened": o.value, "free": f.value}

    def routing(self) -> Dict[str, int]:
        """hm_docset_routing: document rounds by store route so far."""
        out = np.zeros(3, np.uint64)
        self.engine._check(self._L.hm_docset_routing(self._h, out.ctypes.data), "hm_docset_routing")
        return {"incremental": int(out[0]), "remerged": int(out[1]), "handed_back": int(out[2])}

    def stats(self) -> Dict[str, int]:
        out = np.zeros(8, np.uint64)
        self.engine._check(self._L.hm_docset_stats(self._h, out.ctypes.data), "hm_docset_stats")
        return {"calls": int(out[0]), "docs": int(out[1]), "moves": int(out[2]), "hit_patches": int(out[3]),
                "full_patches": int(out[4]), "op_patches": int(out[5]), "replay_mismatch": int(out[6])}


# ---- test helpers: the frontend's view of a document rebuilt from patches ----
ROOT = "00000000-0000-0000-0000-000000000000"


def apply_diffs(objects: Dict[str, Dict[str, Any]], diffs: Sequence[Dict[str, Any]]) -> None:
    """Frontend.applyPatch's effect on a document (src/DocFrontend.ts:162-179), restated."""
    for d in diffs:
        if d["action"] == "create":
            objects[d["obj"]] = {"type": d["type"], "keys": {}, "elems": []}
            continue
        o = objects[d["obj"]]
        e = {"value": d.get("value"), "link": bool(d.get("link")), "datatype": d.get("datatype"),
             "conflicts": d.get("conflicts")}
        if d["type"] in ("list", "text"):
            if d["action"] == "insert":
                o["elems"].insert(d["index"], e)
            elif d["action"] == "set":
                o["elems"][d["index"]] = e
            elif d["action"] == "remove":
                del o["elems"][d["index"]]
            else:
                raise ValueError(d)
        elif d["action"] == "set":
            o["keys"][d["key"]] = e
        elif d["action"] == "remove":
            o["keys"].pop(d["key"], None)          # a per-op remove may name an absent key
        else:
            raise ValueError(d)


def render_objects(objects: Dict[str, Dict[str, Any]], uuid: str = ROOT, depth: int = 0) -> Any:
    """The frontend document in hypermerge_amd/render.py's canonical form."""
    from .columnar import js_key
    o = objects.get(uuid)
    if o is None or depth > 64:
        return {"cycle": uuid}

    def val(v, link):
        return render_objects(objects, v, depth + 1) if link else v

    def ent(e):
        r = {"value": val(e["value"], e["link"])}
        if e.get("datatype"):
            r["datatype"] = e["datatype"]
        if e.get("conflicts"):
            r["conflicts"] = [[c["actor"], val(c.get("value"), c.get("link"))] for c in e["conflicts"]]
        return r
    if o["type"] in ("list", "text"):
        return {o["type"]: [ent(e) for e in o["elems"]]}
    keys = sorted(o["keys"], key=js_key)
    return {"table" if o["type"] == "table" else "map": [[k, ent(o["keys"][k])] for k in keys]}


def view_objects(view: Dict[str, Any]) -> Dict[str, Dict[str, Any]]:
    """hm_docset_view's JSON -> the apply_diffs object form."""
    out = {}
    for uuid, ov in view.items():
        conv = lambda e: {"value": e.get("value"), "link": bool(e.get("link")), "datatype": e.get("datatype"),  # noqa: E731
                          "conflicts": e.get("conflicts")}
        out[uuid] = {"type": ov["type"], "keys": {k: conv(e) for k, e in ov["keys"]},
                     "elems": [conv(e) for _, e in ov["elems"]]}
    return out
