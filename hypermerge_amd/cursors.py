"""CursorStore (src/CursorStore.ts:19-91) over the device table (hm_cursors_*, csrc/cursors.hip),
and the batched syncChanges plan built on it (src/RepoBackend.ts:506-531).

Same API as the reference class: get / update / entry / docsWithActor / addActor, keyed by
(repoId, docId, actorId); updateQ receives the descriptor when the input cursor differs from
the stored one.  Document ids map to dense rows of one device table per repo; actor ids map
to FNV-1a64 keys (the repo-global keys of the clock exchange, hypermerge_amd/exchange.py).
Batched forms (update_many, docs_with_actors, entries) answer many documents / actors in
one launch each."""
from __future__ import annotations

import ctypes
import sys
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from .engine import Engine, lib
from .exchange import KeyTable

INFINITY_SEQ = 9007199254740991            # Number.MAX_SAFE_INTEGER (src/CursorStore.ts:17)
Cursor = Dict[str, float]
Descriptor = Tuple[Cursor, str, str]       # CursorDescriptor = [Cursor, DocId, RepoId]


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


def bounded_seq(seq: float) -> int:
    """Math.max(0, Math.min(seq, INFINITY_SEQ)) (src/CursorStore.ts:89-91)."""
    if not seq > 0:
        return 0
    return INFINITY_SEQ if seq >= INFINITY_SEQ else int(seq)


class _Table:
    def __init__(self, engine: Engine, k: int):
        self._L, self.engine, self.K = lib(), engine, k
        h = ctypes.c_void_p()
        engine._check(self._L.hm_cursors_create(engine._h, k, ctypes.byref(h)), "hm_cursors_create")
        self._h = h
        self.rows: Dict[str, int] = {}
        self.docs: List[str] = []

    def row(self, doc_id: str) -> int:
        r = self.rows.get(doc_id)
        if r is None:
            r = self.rows[doc_id] = len(self.docs)
            self.docs.append(doc_id)
            self.engine._check(self._L.hm_cursors_reserve(self._h, len(self.docs)), "hm_cursors_reserve")
        return r

    def close(self):
        if getattr(self, "_h", None):
            self._L.hm_cursors_destroy(self._h)
            self._h = None


class CursorStore:
    def __init__(self, engine: Engine, max_actors_per_doc: int = 64, hash_fn=None):
        self.engine, self.K = engine, max_actors_per_doc
        self.tables: Dict[str, _Table] = {}
        self.keys = KeyTable(hash_fn)             # a key two actor ids share raises, never merges them
        self.actor_ids: Dict[int, str] = self.keys.ids
        self.updateQ: List[Descriptor] = []

    def close(self):
        for t in self.tables.values():
            t.close()

    def __del__(self):
        # (at interpreter exit finalizers run in any order: the engine may be gone, and the
        # process releases the device anyway)
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    def _t(self, repo_id: str) -> _Table:
        t = self.tables.get(repo_id)
        if t is None:
            t = self.tables[repo_id] = _Table(self.engine, self.K)
        return t

    def _key(self, actor: str) -> int:
        return self.keys.key(actor)

    # -- the reference API --------------------------------------------------------------------
    def get(self, repo_id: str, doc_id: str) -> Cursor:
        return self.get_many(repo_id, [doc_id])[0]

    def update(self, repo_id: str, doc_id: str, cursor: Mapping[str, float]) -> Descriptor:
        return self.update_many(repo_id, {doc_id: cursor})[0]

    def entry(self, repo_id: str, doc_id: str, actor_id: str) -> int:
        return int(self.entries(repo_id, [(doc_id, actor_id)])[0])

    def docsWithActor(self, repo_id: str, actor_id: str, seq: float = 0) -> List[str]:
        # a scan in primary-key order: documentId (BINARY)
        return sorted((d for d, _, _ in self.docs_with_actors(repo_id, {actor_id: seq})), key=lambda d: d.encode("utf-8"))

    def addActor(self, repo_id: str, doc_id: str, actor_id: str, seq: float = INFINITY_SEQ) -> Descriptor:
        return self.update(repo_id, doc_id, {actor_id: bounded_seq(seq)})

    # -- batched forms ---------------------------------------------------------------------------
    def get_many(self, repo_id: str, doc_ids: Sequence[str]) -> List[Cursor]:
        t = self._t(repo_id)
        out: List[Cursor] = []
        rows = [t.rows.get(d) for d in doc_ids]
        have = np.array([r for r in rows if r is not None], np.uint32)
        n = len(have)
        cnt = np.zeros(max(n, 1), np.uint32)
        ak = np.zeros((max(n, 1), self.K), np.uint64)
        sq = np.zeros((max(n, 1), self.K), np.uint64)
        if n:
            self.engine._check(t._L.hm_cursors_get(t._h, n, _p(have), _p(cnt), _p(ak), _p(sq)), "hm_cursors_get")
        j = 0
        for r in rows:
            if r is None:
                out.append({})
                continue
            # `SELECT *` on the WITHOUT ROWID table comes back in primary-key (actorId, BINARY) order
            ent = sorted(((self.actor_ids[int(ak[j, e])], int(sq[j, e])) for e in range(int(cnt[j]))),
                         key=lambda x: x[0].encode("utf-8"))
            out.append(dict(ent))
            j += 1
        return out

    def update_many(self, repo_id: str, cursors: Mapping[str, Mapping[str, float]]) -> List[Descriptor]:
        """CursorStore.update for many documents in one launch; descriptors in input order."""
        t = self._t(repo_id)
        docs = list(cursors)
        rows = np.array([t.row(d) for d in docs], np.uint32)
        off = np.zeros(len(docs) + 1, np.uint32)
        keys: List[int] = []
        seqs: List[float] = []
        for i, d in enumerate(docs):
            for a, s in cursors[d].items():
                keys.append(self._key(a))
                seqs.append(float(s))
            off[i + 1] = len(keys)
        ak = np.array(keys, np.uint64)
        sq = np.array(seqs, np.float64)
        diff = np.zeros(max(len(docs), 1), np.uint8)
        self.engine._check(t._L.hm_cursors_update(t._h, len(docs), _p(rows), _p(off), _p(ak), _p(sq), _p(diff)),
                           "hm_cursors_update")
        stored = self.get_many(repo_id, docs)
        out = []
        for i, d in enumerate(docs):
            desc = (stored[i], d, repo_id)
            if diff[i]:
                self.updateQ.append(desc)
            out.append(desc)
        return out

    def entries(self, repo_id: str, pairs: Sequence[Tuple[str, str]]) -> np.ndarray:
        """CursorStore.entry for many (doc, actor) pairs in one launch."""
        t = self._t(repo_id)
        out = np.zeros(len(pairs), np.uint64)
        idx = [i for i, (d, _) in enumerate(pairs) if d in t.rows]
        if idx:
            rows = np.array([t.rows[pairs[i][0]] for i in idx], np.uint32)
            ak = np.array([self._key(pairs[i][1]) for i in idx], np.uint64)
            got = np.zeros(len(idx), np.uint64)
            self.engine._check(t._L.hm_cursors_entry(t._h, len(idx), _p(rows), _p(ak), _p(got)), "hm_cursors_entry")
            out[idx] = got
        return out

    def docs_with_actors(self, repo_id: str, actors: Mapping[str, float]) -> List[Tuple[str, str, int]]:
        """docsWithActor for many actors in one launch: (docId, actorId, stored seq) per match."""
        t = self._t(repo_id)
        names = list(actors)
        if not names or not t.docs:
            return []
        ak = np.array([self._key(a) for a in names], np.uint64)
        ms = np.array([float(actors[a]) for a in names], np.float64)
        cap = max(16, len(t.docs) * len(names))
        n = ctypes.c_uint32()
        while True:
            r = np.zeros(cap, np.uint32)
            q = np.zeros(cap, np.uint32)
            s = np.zeros(cap, np.uint64)
            st = t._L.hm_cursors_docs_with_actors(t._h, len(names), _p(ak), _p(ms), cap, _p(r), _p(q), _p(s),
                                                   ctypes.byref(n))
            if st == 34 and n.value > cap:                   # HM_ERR_NOMEM: grow and ask again
                cap = n.value
                continue
            self.engine._check(st, "hm_cursors_docs_with_actors")
            break
        k = n.value
        return [(t.docs[int(r[i])], names[int(q[i])], int(s[i])) for i in range(k)]


def sync_plan(engine: Engine, cursors: CursorStore, repo_id: str, actors: Sequence[str],
              doc_changes: Mapping[str, Mapping[str, int]], present: Mapping[str, np.ndarray]
              ) -> List[Tuple[str, str, int, int]]:
    """RepoBackend.syncChanges (src/RepoBackend.ts:506-531) for many synced actors at once:
    for every open document (doc_changes: docId -> DocBackend.changes) whose cursor has the
    actor, the block range [min, end) it receives, min = doc.changes[actor] || 0 and end = the
    first missing block of the actor's feed (present[actor]: downloaded-block flags) at or
    after min, below the cursor entry.  One docsWithActor launch, one contiguity launch
    (hm_sync_ranges_device).  Every (doc, actor) hit is returned: the caller sets
    doc.changes[actor] = end and calls applyRemoteChanges when end > min, as syncChanges does."""
    from .sync import contiguous_ends
    hits = [(d, a, s) for d, a, s in cursors.docs_with_actors(repo_id, {a: 0 for a in actors}) if d in doc_changes]
    if not hits:
        return []
    feeds = list(dict.fromkeys(a for _, a, _ in hits))
    fidx = {a: i for i, a in enumerate(feeds)}
    lo = np.array([int(doc_changes[d].get(a, 0)) for d, a, _ in hits], np.int64)
    hi = np.array([min(int(s), 0xFFFFFFFF) for _, _, s in hits], np.int64)
    hi = np.maximum(hi, lo)
    end = contiguous_ends(engine, [np.asarray(present[a], bool) for a in feeds],
                          np.array([fidx[a] for _, a, _ in hits]), lo.astype(np.uint32),
                          hi.astype(np.uint64), device=engine.device)
    out = [(d, a, int(l), int(e)) for (d, a, _), l, e in zip(hits, lo, end)]
    out.sort(key=lambda x: (x[0], x[1]))
    return out
