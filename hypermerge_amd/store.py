"""Resident document store: Python face of ``hm_store_*`` / ``hm_doc_*`` /
``hm_batch_submit`` / ``hm_batch_wait`` (include/hypermerge_amd.h).

``DocStore`` keeps every open document's Automerge BackendState on the GPU
(the ``DocBackend.back`` of src/DocBackend.ts:50).  ``DocEncoder`` is the
per-document host interner that turns decoded ``Change`` dicts into columnar
rows across successive ``applyChanges`` calls: actor ids keep their JS string
order as the *rank*, so a new actor can re-rank the document's earlier rows
(the engine applies the returned remap on the device); object UUIDs,
``(object, key)`` / ``(list, elemId)`` registers and change contents keep the
ids they were first given.
"""
from __future__ import annotations

import ctypes
import sys
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .columnar import (ACTIONS, CHANGE_DT, DEP_DT, DOC_DT, DOC_RESULT_DT, OP_DT, REG_RESULT_DT,
                       SURV_RESULT_DT, DATATYPES, DOC_HAS_COUNTERS, DOC_HAS_LISTS, DT_COUNTER, HEAD,
                       INC, INS, LINK, MAKE_LIST, MAKE_TEXT, NONE, ROOT_ID, SET, DEL, V_NULL, V_OBJ,
                       Batch, CBatch, Results, _value, content_key, js_key)
from .engine import Engine, EngineError, lib


class StringPool:
    """Store-wide pool of map keys and string values (host only; ids are shipped)."""

    def __init__(self) -> None:
        self.index: Dict[str, int] = {}
        self.strings: List[str] = []

    def intern(self, s: str) -> int:
        i = self.index.get(s)
        if i is None:
            i = self.index[s] = len(self.strings)
            self.strings.append(s)
        return i


@dataclass
class Append:
    """New rows of one document (offsets local to this append) + its totals after it."""
    changes: np.ndarray
    deps: np.ndarray
    ops: np.ndarray
    n_actors: int
    n_regs: int
    n_objs: int
    flags: int
    remap: Optional[np.ndarray]      # old rank -> new rank (None: unchanged)


class DocEncoder:
    """Interner state of one document across applyChanges calls."""

    def __init__(self, pool: StringPool, keep_log: bool = True) -> None:
        self.pool = pool
        self.actors: List[str] = []                  # rank -> actor id
        self.objs: Dict[str, int] = {ROOT_ID: 0}
        self.obj_list: List[str] = [ROOT_ID]
        self.regs: Dict[Tuple[int, str], int] = {}
        self.reg_list: List[Tuple[int, str]] = []
        self.content: Dict[str, int] = {}
        self.flags = 0
        self.keep_log = keep_log
        self.log_changes = np.zeros(0, CHANGE_DT)    # doc-local offsets
        self.log_deps = np.zeros(0, DEP_DT)
        self.log_ops = np.zeros(0, OP_DT)

    # -- interning -----------------------------------------------------------------------------
    def _obj(self, u: str) -> int:
        i = self.objs.get(u)
        if i is None:
            i = self.objs[u] = len(self.obj_list)
            self.obj_list.append(u)
        return i

    def _reg(self, o: int, key: str) -> int:
        i = self.regs.get((o, key))
        if i is None:
            i = self.regs[(o, key)] = len(self.reg_list)
            self.reg_list.append((o, key))
        return i

    def snapshot(self):
        """State to restore if the append is rolled back (a throwing applyChanges)."""
        return (list(self.actors), dict(self.objs), list(self.obj_list), dict(self.regs), list(self.reg_list),
                dict(self.content), self.flags, self.log_changes, self.log_deps, self.log_ops)

    def restore(self, snap) -> None:
        (self.actors, self.objs, self.obj_list, self.regs, self.reg_list, self.content, self.flags,
         self.log_changes, self.log_deps, self.log_ops) = snap

    def encode(self, changes: Sequence[Dict[str, Any]], extra_actors: Sequence[str] = ()) -> Append:
        new_actors = set(extra_actors)
        for c in changes:
            new_actors.add(c["actor"])
            new_actors.update((c.get("deps") or {}).keys())
        new_actors -= set(self.actors)
        remap = None
        if new_actors:
            ranked = sorted(set(self.actors) | new_actors, key=js_key)
            rank = {a: i for i, a in enumerate(ranked)}
            if self.actors:
                mp = np.array([rank[a] for a in self.actors], np.uint8)
                if not np.array_equal(mp, np.arange(len(self.actors), dtype=np.uint8)):
                    remap = mp
            self.actors = ranked
        rank = {a: i for i, a in enumerate(self.actors)}
        ch_rows, dep_rows, op_rows = [], [], []
        flags = 0
        for c in changes:
            deps = c.get("deps") or {}
            dep_off = len(dep_rows)
            for da, ds in deps.items():
                dep_rows.append((rank[da], 0, int(ds)))
            ck = content_key(c)
            cid = self.content.get(ck)
            if cid is None:
                cid = self.content[ck] = len(self.content)
            op_first = len(op_rows)
            for op in c.get("ops", []):
                act = ACTIONS[op["action"]]
                o = self._obj(op["obj"])
                reg, parent, elem, key = NONE, NONE, 0, 0
                vt, val = V_NULL, 0
                if act == INS:
                    elem = int(op["elem"])
                    reg = self._reg(o, f"{c['actor']}:{elem}")
                    parent = HEAD if op["key"] == "_head" else self._reg(o, op["key"])
                elif act in (SET, DEL, LINK, INC):
                    reg = self._reg(o, op["key"])
                    key = self.pool.intern(op["key"])
                    if act == LINK:
                        vt, val = V_OBJ, self._obj(op["value"])
                    elif act in (SET, INC):
                        vt, val = _value(op.get("value"), self.pool.index, self.pool.strings, self.objs)
                dt = DATATYPES[op.get("datatype")]
                if act in (MAKE_LIST, MAKE_TEXT):
                    flags |= DOC_HAS_LISTS
                if act == INC or dt == DT_COUNTER:
                    flags |= DOC_HAS_COUNTERS
                op_rows.append((o, reg, parent, elem, act, dt, vt, 0, key, val))
            ch_rows.append((rank[c["actor"]], len(deps), int(c["seq"]), dep_off, len(op_rows) - op_first,
                            op_first, cid))
        self.flags |= flags
        a = Append(np.array(ch_rows, CHANGE_DT) if ch_rows else np.zeros(0, CHANGE_DT),
                   np.array(dep_rows, DEP_DT) if dep_rows else np.zeros(0, DEP_DT),
                   np.array(op_rows, OP_DT) if op_rows else np.zeros(0, OP_DT),
                   len(self.actors), len(self.reg_list), len(self.obj_list), flags, remap)
        if self.keep_log:
            lc = self.log_changes.copy()
            ld = self.log_deps.copy()
            if remap is not None:
                lc["actor"] = remap[lc["actor"]]
                ld["actor"] = remap[ld["actor"]]
            nc = a.changes.copy()
            nc["dep_off"] += len(ld)
            nc["op_first"] += len(self.log_ops)
            self.log_changes = np.concatenate([lc, nc])
            self.log_deps = np.concatenate([ld, a.deps])
            self.log_ops = np.concatenate([self.log_ops, a.ops])
        return a

    def log_batch(self, a_stride: int) -> Batch:
        """The document's whole log as a one-document batch (oracle / rendering)."""
        doc = np.zeros(1, DOC_DT)
        d = doc[0]
        d["n_changes"], d["n_deps"], d["n_ops"] = len(self.log_changes), len(self.log_deps), len(self.log_ops)
        d["n_regs"], d["n_objs"], d["n_actors"], d["flags"] = len(self.reg_list), len(self.obj_list), \
            len(self.actors), self.flags
        return Batch(doc, self.log_changes.copy(), self.log_deps.copy(), self.log_ops.copy(), a_stride, None,
                     self.pool.strings, [list(self.actors)], [list(self.obj_list)], [list(self.reg_list)])


class _StoreConfig(ctypes.Structure):
    _fields_ = [("a_stride", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class _DocInfo(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint32) for f in ("n_changes", "n_deps", "n_ops", "n_regs", "n_objs", "n_actors",
                                                "hist_len", "n_queued", "n_surv")] + [("status", ctypes.c_int32)]


def _p(a: Optional[np.ndarray]):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


@dataclass
class BatchResult:
    docs: np.ndarray            # DOC_RESULT_DT per batch row
    clock: np.ndarray           # [n, S] opSet.clock
    back_clock: np.ndarray      # [n, S] DocBackend.clock
    heads: np.ndarray           # [n, S] opSet.deps


class DocStore:
    """Device-resident documents of one repo (one GPU)."""

    def __init__(self, engine: Engine, a_stride: int = 8) -> None:
        L = lib()
        self._L, self.engine, self.S = L, engine, a_stride
        h = ctypes.c_void_p()
        engine._check(L.hm_store_create(engine._h, ctypes.byref(_StoreConfig(a_stride, 0)), ctypes.byref(h)),
                      "hm_store_create")
        self._h = h
        self.pool = StringPool()
        self.enc: List[DocEncoder] = []
        self._pending = None

    def close(self) -> None:
        if getattr(self, "_h", None):
            if getattr(self.engine, "_h", None):               # (the store lives on its engine's stream)
                self._L.hm_store_destroy(self._h)
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

    def _check(self, st: int, what: str) -> None:
        self.engine._check(st, what)

    def set_incremental(self, on) -> None:
        """Incremental applyRemoteChanges on the resident state (default on); off = every submit
        re-merges each touched document's whole log; 2 = also small list documents (no cost
        policy).  Results are identical."""
        mode = 2 if on == 2 else int(bool(on))
        self._check(self._L.hm_store_set_incremental(self._h, mode), "hm_store_set_incremental")

    def last_routing(self) -> Dict[str, int]:
        """How the last submit's documents were merged: incremental / re-merged / handed back."""
        out = np.zeros(3, np.uint32)
        self._check(self._L.hm_store_last_routing(self._h, _p(out)), "hm_store_last_routing")
        return {"incremental": int(out[0]), "remerged": int(out[1]), "handed_back": int(out[2])}

    def inc_states(self) -> int:
        """Documents whose resident incremental state a submit can use (hm_store_inc_states)."""
        out = np.zeros(1, np.uint32)
        self._check(self._L.hm_store_inc_states(self._h, _p(out)), "hm_store_inc_states")
        return int(out[0])

    def last_kernel_ms(self) -> Dict[str, float]:
        """Device time of the last submit (HIP events): the incremental kernels and the re-merge."""
        out = np.zeros(2, np.float32)
        self._check(self._L.hm_store_last_kernel_ms(self._h, _p(out)), "hm_store_last_kernel_ms")
        return {"incremental_ms": float(out[0]), "remerge_ms": float(out[1])}

    def open(self) -> int:
        h = ctypes.c_uint32()
        self._check(self._L.hm_doc_open(self._h, ctypes.byref(h)), "hm_doc_open")
        assert h.value == len(self.enc)
        self.enc.append(DocEncoder(self.pool))
        return h.value

    def reset(self, handles) -> None:
        """hm_doc_reset: the handles become empty documents again (their rows are dead space
        until the store compacts)."""
        hs = np.ascontiguousarray(handles, np.uint32)
        self._check(self._L.hm_doc_reset(self._h, _p(hs), len(hs)), "hm_doc_reset")
        for h in hs:
            if h < len(self.enc):
                self.enc[h] = DocEncoder(self.pool)

    # -- applyChanges over many documents -----------------------------------------------------
    def submit(self, items: Sequence[Tuple[int, Sequence[Dict[str, Any]]]],
               extra_actors: Optional[Dict[int, Sequence[str]]] = None) -> int:
        """items: (handle, changes) per document (each handle once)."""
        S = self.S
        appends, snaps = [], []
        for h, changes in items:
            e = self.enc[h]
            snaps.append(e.snapshot())
            a = e.encode(changes, (extra_actors or {}).get(h, ()))
            if a.n_actors > S:
                for (hh, _), sn in zip(items, snaps):
                    self.enc[hh].restore(sn)
                raise EngineError(f"document {h} has {a.n_actors} actors > store a_stride {S}")
            appends.append(a)
        return self._submit_rows([h for h, _ in items], appends, snaps)

    def _submit_rows(self, handles: List[int], appends: List[Append], snaps) -> int:
        S = self.S
        n = len(handles)
        docs = np.zeros(n, DOC_DT)
        chs, dps, ops = [], [], []
        nc = nd = no = 0
        remap = None
        for i, a in enumerate(appends):
            d = docs[i]
            d["change_off"], d["n_changes"], d["dep_off"], d["n_deps"] = nc, len(a.changes), nd, len(a.deps)
            d["op_off"], d["n_ops"] = no, len(a.ops)
            d["n_regs"], d["n_objs"], d["n_actors"], d["flags"] = a.n_regs, a.n_objs, a.n_actors, a.flags
            c = a.changes.copy()
            c["dep_off"] += nd
            c["op_first"] += no
            chs.append(c); dps.append(a.deps); ops.append(a.ops)
            nc += len(a.changes); nd += len(a.deps); no += len(a.ops)
            if a.remap is not None:
                if remap is None:
                    remap = np.tile(np.arange(S, dtype=np.uint8), (n, 1))
                remap[i, :len(a.remap)] = a.remap
        ch = np.concatenate(chs) if chs else np.zeros(0, CHANGE_DT)
        dp = np.concatenate(dps) if dps else np.zeros(0, DEP_DT)
        op = np.concatenate(ops) if ops else np.zeros(0, OP_DT)
        hs = np.array(handles, np.uint32)
        keep = (docs, ch, dp, op, hs, remap)
        cb = CBatch(n, len(ch), len(dp), len(op), int(docs["n_regs"].sum()) if n else 0, S, 0, 0, 0, 0, 0, 0,
                    docs.ctypes.data, ch.ctypes.data, dp.ctypes.data, op.ctypes.data, None)
        bid = ctypes.c_uint64()
        self._check(self._L.hm_batch_submit(self._h, ctypes.byref(cb), _p(hs), _p(remap), ctypes.byref(bid)),
                    "hm_batch_submit")
        self._pending = (bid.value, handles, snaps, keep)
        return bid.value

    def wait(self) -> BatchResult:
        bid, handles, snaps, _ = self._pending
        self._pending = None
        n, S = len(handles), self.S
        r = BatchResult(np.zeros(n, DOC_RESULT_DT), np.zeros((n, S), np.uint32), np.zeros((n, S), np.uint32),
                        np.zeros((n, S), np.uint32))
        self._check(self._L.hm_batch_wait(self._h, ctypes.c_uint64(bid), _p(r.docs), _p(r.clock),
                                          _p(r.back_clock), _p(r.heads)), "hm_batch_wait")
        for i, h in enumerate(handles):          # rolled-back documents: the interner rolls back too
            if r.docs[i]["status"] != 0:
                self.enc[h].restore(snaps[i])
        return r

    def apply(self, items, extra_actors=None) -> BatchResult:
        self.submit(items, extra_actors)
        return self.wait()

    # -- reads -------------------------------------------------------------------------------
    def info(self, h: int) -> Dict[str, int]:
        i = _DocInfo()
        self._check(self._L.hm_doc_info(self._h, h, ctypes.byref(i)), "hm_doc_info")
        return {f: getattr(i, f) for f, _ in _DocInfo._fields_}

    def read(self, h: int) -> Tuple[Batch, Results]:
        """The document's log and merged state as a one-document (Batch, Results); the Batch is
        None for a store fed prebuilt rows (RowStore: no host encoder keeps the log)."""
        inf = self.info(h)
        S = self.S
        b = self.enc[h].log_batch(S) if h < len(self.enc) else None
        r = Results(np.zeros(1, DOC_RESULT_DT), np.zeros(S, np.uint32), np.zeros(S, np.uint32),
                    np.zeros(S, np.uint32), np.zeros(inf["n_changes"], np.int32),
                    np.zeros(inf["n_changes"] * S, np.uint32), np.zeros(inf["n_regs"], REG_RESULT_DT),
                    np.zeros(inf["n_ops"], SURV_RESULT_DT))
        self._check(self._L.hm_doc_read(self._h, h, _p(r.hist), _p(r.all_deps), _p(r.regs), _p(r.surv),
                                        _p(r.clock), _p(r.back_clock), _p(r.heads)), "hm_doc_read")
        d = r.docs[0]
        d["status"], d["hist_len"], d["n_queued"], d["n_surv"] = inf["status"], inf["hist_len"], inf["n_queued"], \
            inf["n_surv"]
        d["err_change"] = d["err_op"] = NONE
        r.surv[inf["n_surv"]:] = 0
        return b, r

    def log(self, h: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        inf = self.info(h)
        c = np.zeros(inf["n_changes"], CHANGE_DT)
        d = np.zeros(inf["n_deps"], DEP_DT)
        o = np.zeros(inf["n_ops"], OP_DT)
        self._check(self._L.hm_doc_log(self._h, h, _p(c), _p(d), _p(o)), "hm_doc_log")
        return c, d, o

    def history_prefix(self, h: int, n: int) -> List[int]:
        out = np.zeros(max(n, 1), np.uint32)
        k = self._L.hm_doc_history_prefix(self._h, h, n, _p(out))
        if k < 0:
            self._check(k, "hm_doc_history_prefix")
        return [int(x) for x in out[:k]]

    def set_min_clock(self, h: int, clock: Dict[str, int]) -> None:
        """minimumClock (actor id -> seq); its actors must already be in the document's actor table."""
        e = self.enc[h]
        row = np.zeros(self.S, np.uint32)
        rank = {a: i for i, a in enumerate(e.actors)}
        for a, s in clock.items():
            row[rank[a]] = min(int(s), 0xFFFFFFFF)
        self._check(self._L.hm_doc_set_min_clock(self._h, h, _p(row)), "hm_doc_set_min_clock")

    def clock_update(self, handles: Sequence[int]):
        """Batched ClockStore.update(self, doc, doc.clock): (written, differs, stored rows)."""
        n = len(handles)
        hs = np.array(handles, np.uint32)
        w = np.zeros(max(n, 1), np.uint8)
        df = np.zeros(max(n, 1), np.uint8)
        st = np.zeros((max(n, 1), self.S), np.uint32)
        self._check(self._L.hm_store_clock_update(self._h, n, _p(hs), _p(w), _p(df), _p(st)),
                    "hm_store_clock_update")
        return w[:n].astype(bool), df[:n].astype(bool), st[:n]


def slice_changes(b: Batch, lo: np.ndarray, hi: np.ndarray, docs: Optional[np.ndarray] = None) -> Batch:
    """For each document d of `docs` (default: all), its changes lo[d] .. hi[d]-1 (document-local
    arrival indices) with their dep and op rows, as a batch with batch-local offsets.  Document
    totals (n_actors / n_regs / n_objs / flags) are kept: the rows' ids are the batch's own."""
    idx = np.arange(b.n_docs) if docs is None else np.asarray(docs, np.int64)
    drow = b.docs[idx].copy()
    lo = np.asarray(lo, np.int64)[idx]
    cnt = np.asarray(hi, np.int64)[idx] - lo
    cnt = np.maximum(cnt, 0)
    tot = int(cnt.sum())
    excl = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(cnt, out=excl[1:])
    ci = np.repeat(drow["change_off"].astype(np.int64) + lo - excl[:-1], cnt) + np.arange(tot)
    ch = b.changes[ci].copy()

    def rows(first, n, table):
        n = n.astype(np.int64)
        off = np.zeros(len(n) + 1, np.int64)
        np.cumsum(n, out=off[1:])
        ri = np.repeat(first.astype(np.int64) - off[:-1], n) + np.arange(int(off[-1]))
        return table[ri].copy(), off
    dp, doff = rows(ch["dep_off"], ch["n_deps"], b.deps)
    op, ooff = rows(ch["op_first"], ch["n_ops"], b.ops)
    ch["dep_off"] = doff[:-1]
    ch["op_first"] = ooff[:-1]
    drow["change_off"] = excl[:-1]
    drow["n_changes"] = cnt
    drow["dep_off"] = doff[excl[:-1]]
    drow["n_deps"] = doff[excl[1:]] - doff[excl[:-1]]
    drow["op_off"] = ooff[excl[:-1]]
    drow["n_ops"] = ooff[excl[1:]] - ooff[excl[:-1]]
    drow["reg_off"] = 0
    return Batch(drow, ch, dp, op, b.a_stride)


class RowStore(DocStore):
    """Resident documents fed with prebuilt columnar rows (no per-document host encoder): actor
    ranks, register and object ids in the rows are the caller's, stable across submits (e.g. a
    synthetic feed, or rows from hm_decode_blocks over a repo-wide interner)."""

    def open_n(self, n: int) -> int:
        first = ctypes.c_uint32()
        self._check(self._L.hm_doc_open_n(self._h, n, ctypes.byref(first)), "hm_doc_open_n")
        return first.value

    def submit_batch(self, b: Batch, handles: np.ndarray) -> int:
        hs = np.ascontiguousarray(handles, np.uint32)
        keep = (b, hs)
        # the store reads the tables and per-document totals only (no launch-size hints)
        cb = CBatch(b.n_docs, len(b.changes), len(b.deps), len(b.ops), 0, b.a_stride, 0, 0, 0, 0, 0, 0,
                    b.docs.ctypes.data, b.changes.ctypes.data, b.deps.ctypes.data, b.ops.ctypes.data, None)
        bid = ctypes.c_uint64()
        self._check(self._L.hm_batch_submit(self._h, ctypes.byref(cb), _p(hs), None, ctypes.byref(bid)),
                    "hm_batch_submit")
        self._pending = (bid.value, len(hs), None, keep)
        return bid.value

    def submit_device(self, n_docs: int, counts, docs, changes, deps, ops, handles) -> int:
        """hm_batch_submit_device: the batch's tables and handles already in HBM (torch tensors or
        device pointers, read in place until wait_device returns); counts = (n_changes, n_deps, n_ops)."""
        ptr = [int(getattr(t, "data_ptr", lambda: t)()) for t in (docs, changes, deps, ops, handles)]
        cb = CBatch(n_docs, int(counts[0]), int(counts[1]), int(counts[2]), 0, self.S, 0, 0, 0, 0, 0, 0,
                    ptr[0], ptr[1], ptr[2], ptr[3], None)
        bid = ctypes.c_uint64()
        self._check(self._L.hm_batch_submit_device(self._h, ctypes.byref(cb), ctypes.c_void_p(ptr[4]), None,
                                                   ctypes.byref(bid)), "hm_batch_submit_device")
        self._pending = (bid.value, n_docs, None, (docs, changes, deps, ops, handles))
        return bid.value

    def wait_device(self, out) -> int:
        """hm_batch_wait_device: the gathered result rows into device memory `out` (a torch tensor of at
        least n * (32 + 12 * a_stride) bytes); returns the number of rows whose status is not OK."""
        bid, n, _, _ = self._pending
        self._pending = None
        nf = ctypes.c_uint32()
        self._check(self._L.hm_batch_wait_device(self._h, ctypes.c_uint64(bid), ctypes.c_void_p(int(out.data_ptr())),
                                                 ctypes.byref(nf)), "hm_batch_wait_device")
        return nf.value

    def wait(self, out: Optional[BatchResult] = None) -> BatchResult:
        """Results of the submitted batch; `out` (arrays of at least the batch's size, e.g. kept
        between rounds by a long-running host) is filled instead of fresh arrays."""
        bid, n, _, _ = self._pending
        self._pending = None
        S = self.S
        if out is not None and len(out.docs) >= n:
            r = BatchResult(out.docs[:n], out.clock[:n], out.back_clock[:n], out.heads[:n])
        else:
            r = BatchResult(np.zeros(n, DOC_RESULT_DT), np.zeros((n, S), np.uint32), np.zeros((n, S), np.uint32),
                            np.zeros((n, S), np.uint32))
        self._check(self._L.hm_batch_wait(self._h, ctypes.c_uint64(bid), _p(r.docs), _p(r.clock),
                                          _p(r.back_clock), _p(r.heads)), "hm_batch_wait")
        return r
