"""CursorStore on the device (hm_cursors_*, hypermerge_amd/cursors.py) against the reference's
own SQL run in sqlite3 (schema src/migrations/0001_initial_schema.sql:15-21, statements
src/CursorStore.ts:29-43, boundedSeq :89-91, the updateQ rule :58-61), plus the reference's
tests/CursorStore.test.ts cases and the batched syncChanges plan (src/RepoBackend.ts:506-531)
against a restatement of its loop."""
import math
import sqlite3

import numpy as np
import pytest

from hypermerge_amd.cursors import INFINITY_SEQ, CursorStore, sync_plan

pytestmark = pytest.mark.gpu


class SqlCursors:
    """The reference CursorStore's statements over sqlite3 (test infrastructure)."""

    def __init__(self):
        self.db = sqlite3.connect(":memory:")
        self.db.execute("CREATE TABLE IF NOT EXISTS Cursors (repoId TEXT NOT NULL, documentId TEXT NOT NULL, "
                        "actorId TEXT NOT NULL, seq INTEGER NOT NULL, PRIMARY KEY (repoId, documentId, actorId)) "
                        "WITHOUT ROWID")
        self.updateQ = []

    @staticmethod
    def bounded(s):
        return int(max(0, min(s, INFINITY_SEQ)))

    def get(self, r, d):
        return {a: s for (a, s) in self.db.execute("SELECT actorId, seq FROM Cursors WHERE repoId = ? AND documentId = ?",
                                                   (r, d))}

    def update(self, r, d, cursor):
        for a, s in cursor.items():
            self.db.execute("INSERT INTO Cursors (repoId, documentId, actorId, seq) VALUES (?, ?, ?, ?) "
                            "ON CONFLICT (repoId, documentId, actorId) DO UPDATE SET seq = excluded.seq "
                            "WHERE excluded.seq > seq", (r, d, a, self.bounded(s)))
        stored = self.get(r, d)
        keys = set(cursor) | set(stored)
        if not all(cursor.get(k, 0) == stored.get(k, 0) for k in keys):      # !Clock.equal
            self.updateQ.append((stored, d, r))
        return stored, d, r

    def entry(self, r, d, a):
        row = self.db.execute("SELECT seq FROM Cursors WHERE repoId = ? AND documentId = ? AND actorId = ?",
                              (r, d, a)).fetchone()
        return row[0] if row else 0

    def docs_with_actor(self, r, a, seq=0):
        return [x for (x,) in self.db.execute("SELECT documentId FROM Cursors WHERE repoId = ? AND actorId = ? AND seq >= ?",
                                              (r, a, self.bounded(seq)))]


def test_reference_cursorstore_cases(engine):
    """tests/CursorStore.test.ts:7-36: Infinity clamps to INFINITY_SEQ, zeros are kept; upsert."""
    cs = CursorStore(engine)
    cs.update("repoId", "abc123", {"abc123": math.inf, "def456": 0})
    assert cs.get("repoId", "abc123") == {"abc123": INFINITY_SEQ, "def456": 0}
    cs2 = CursorStore(engine)
    cs2.update("repoId", "abc123", {"abc123": 1, "def456": 0})
    cs2.update("repoId", "abc123", {"abc123": 2, "def456": 0})
    assert cs2.get("repoId", "abc123") == {"abc123": 2, "def456": 0}
    assert cs.entry("repoId", "abc123", "zzz") == 0 and cs.entry("repoId", "nodoc", "abc123") == 0
    assert cs.docsWithActor("repoId", "abc123") == ["abc123"]
    cs.addActor("repoId", "d2", "abc123")
    assert cs.docsWithActor("repoId", "abc123", INFINITY_SEQ) == ["abc123", "d2"]


def test_cursorstore_matches_reference_sql(engine):
    rng = np.random.default_rng(4)
    cs, ref = CursorStore(engine, max_actors_per_doc=32), SqlCursors()
    docs = [f"doc{i:03d}" for i in range(120)]
    actors = [f"actor-{i}" for i in range(24)] + ["é☃", "00"]
    vals = [0, 1, 2, 3, 7, 40, 2.5, -3, math.inf, INFINITY_SEQ, INFINITY_SEQ + 10]
    for rnd in range(12):
        batch = {}
        for d in rng.choice(docs, size=40, replace=False):
            k = int(rng.integers(1, 6))
            batch[str(d)] = {str(a): vals[int(rng.integers(len(vals)))] for a in rng.choice(actors, size=k, replace=False)}
        got = cs.update_many("R", batch)
        want = [ref.update("R", d, c) for d, c in batch.items()]
        assert [g[0] for g in got] == [w[0] for w in want]
        assert [x[1] for x in cs.updateQ] == [x[1] for x in ref.updateQ], rnd
        assert [x[0] for x in cs.updateQ] == [x[0] for x in ref.updateQ]
    for a in actors:
        for s in (0, 3, math.inf):
            assert cs.docsWithActor("R", a, s) == sorted(ref.docs_with_actor("R", a, s), key=lambda x: x.encode()), (a, s)
    pairs = [(str(d), str(a)) for d in docs[:60] for a in actors[:10]]
    assert list(cs.entries("R", pairs)) == [ref.entry("R", d, a) for d, a in pairs]
    assert cs.get_many("R", docs) == [ref.get("R", d) for d in docs]
    assert cs.get("other-repo", docs[0]) == {}


def test_sync_plan_matches_sync_changes_loop(engine):
    """Many actors' feeds sync at once: every open document's [min, end) range equals the
    reference loop `for (i = min; i < max && actor.changes.hasOwnProperty(i); i++)`."""
    rng = np.random.default_rng(9)
    cs = CursorStore(engine)
    actors = [f"a{i}" for i in range(12)]
    present = {a: rng.random(int(rng.integers(0, 300))) < 0.9 for a in actors}
    cursors = {}
    for d in range(200):
        cur = {a: (math.inf if rng.random() < 0.3 else int(rng.integers(0, 320)))
               for a in rng.choice(actors, size=int(rng.integers(1, 5)), replace=False)}
        cursors[f"d{d}"] = cur
    cs.update_many("R", cursors)
    open_docs = {f"d{d}": {a: int(rng.integers(0, 200)) for a in actors if rng.random() < 0.5}
                 for d in range(0, 200, 2)}
    synced = actors[:8]
    got = sync_plan(engine, cs, "R", synced, open_docs, present)
    want = []
    for d, cur in cursors.items():
        if d not in open_docs:
            continue
        for a in synced:
            if a not in cur:
                continue
            mx = min(cur[a], INFINITY_SEQ)
            lo = open_docs[d].get(a, 0)
            i = lo
            while i < mx and i < len(present[a]) and present[a][i]:
                i += 1
            want.append((d, a, lo, i))
    assert got == sorted(want)


def test_cursor_update_is_all_or_nothing(engine):
    """an update that would overflow a row, or that names a row or an actor twice,
    fails with nothing written (the reference's update is one SQLite transaction)."""
    import ctypes
    import numpy as np
    from hypermerge_amd.cursors import CursorStore
    from hypermerge_amd.engine import EngineError
    cs = CursorStore(engine, max_actors_per_doc=3)
    cs.update("r", "d1", {"a": 1, "b": 2})
    cs.update("r", "d2", {"a": 5})
    before = cs.get_many("r", ["d1", "d2"])
    with pytest.raises(EngineError):
        cs.update_many("r", {"d2": {"a": 9}, "d1": {"c": 1, "d": 1, "a": 7}})     # d1 would hold 4 actors
    assert cs.get_many("r", ["d1", "d2"]) == before
    t = cs._t("r")
    rows = np.array([t.rows["d1"], t.rows["d1"]], np.uint32)
    off = np.array([0, 1, 2], np.uint32)
    keys = np.array([cs._key("a"), cs._key("b")], np.uint64)
    seqs = np.array([9.0, 9.0])
    st = t._L.hm_cursors_update(t._h, 2, rows.ctypes.data, off.ctypes.data, keys.ctypes.data, seqs.ctypes.data, None)
    assert st == 32
    rows1 = np.array([t.rows["d1"]], np.uint32)
    off1 = np.array([0, 2], np.uint32)
    keys1 = np.array([cs._key("a"), cs._key("a")], np.uint64)
    st = t._L.hm_cursors_update(t._h, 1, rows1.ctypes.data, off1.ctypes.data, keys1.ctypes.data, seqs.ctypes.data, None)
    assert st == 32
    assert cs.get_many("r", ["d1", "d2"]) == before
    cs.update("r", "d1", {"c": 4})
    assert cs.get("r", "d1") == {"a": 1, "b": 2, "c": 4}


def test_cursorstore_batches_replay_to_reference_tables(engine):
    """Row f3: the Node CursorStore's writes leave as one persistence batch per call (takeBatch:
    ['upsert', repoId, docId, actorId, boundedSeq] per entry handed to update, in order); replayed
    into sqlite3 with the reference's upsert statement (src/CursorStore.ts:31-36) the table after
    every round equals the reference SQL's after the same update calls, and the device rows
    (get) equal it at the end."""
    import json
    import os
    import shutil
    import subprocess
    node = shutil.which("node")
    if node is None:
        pytest.skip("node not installed")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rng = np.random.default_rng(9)
    docs = [f"doc{i:02d}" for i in range(30)]
    actors = [f"actor-{i}" for i in range(12)] + ["é☃", "00"]
    vals = [0, 1, 2, 3, 7, 40, -3, "Infinity", INFINITY_SEQ, INFINITY_SEQ + 10]
    rounds = []
    for _ in range(8):
        r = {}
        for d in rng.choice(docs, size=12, replace=False):
            r[str(d)] = {str(a): vals[int(rng.integers(len(vals)))] for a in rng.choice(actors, size=int(rng.integers(1, 5)), replace=False)}
        rounds.append(r)
    p = subprocess.run([node, os.path.join(root, "tests", "js", "run_cursor_batches.js")],
                       input=json.dumps({"rounds": rounds, "docs": docs}), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(p.stdout)
    ref, db = SqlCursors(), SqlCursors()
    table = "SELECT repoId, documentId, actorId, seq FROM Cursors ORDER BY repoId, documentId, actorId"
    for r, (calls, batch) in enumerate(zip(rounds, got["batches"])):
        for d, c in calls.items():
            ref.update("repo", d, {a: (math.inf if s == "Infinity" else s) for a, s in c.items()})
        assert len(batch) == sum(len(c) for c in calls.values())
        for kind, repo, d, a, s in batch:                 # one transaction per batch
            assert kind == "upsert" and repo == "repo" and 0 <= s <= INFINITY_SEQ
            db.db.execute("INSERT INTO Cursors (repoId, documentId, actorId, seq) VALUES (?, ?, ?, ?) "
                          "ON CONFLICT (repoId, documentId, actorId) DO UPDATE SET seq = excluded.seq "
                          "WHERE excluded.seq > seq", (repo, d, a, s))
        db.db.commit()
        assert db.db.execute(table).fetchall() == ref.db.execute(table).fetchall(), r
    for d, g in zip(docs, got["get"]):
        assert dict(g) == ref.get("repo", d), d
