"""Node host pieces that need no GPU: the JS encoder (hypermerge_amd/js/columnar.js)
must produce the same rows as the Python encoder for the same change sequence (both
feed the same C-ABI), the JS clock helpers must answer like src/Clock.ts (golden
vectors from dist/Clock.js), and the channel must deliver like src/Queue.ts."""
import json
import math
import os
import shutil
import subprocess

import numpy as np
import pytest

from hypermerge_amd import synth
from hypermerge_amd.columnar import ROOT_ID, decode_doc
from hypermerge_amd.store import DocEncoder, StringPool
from kat_cases import CASES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def run_node(payload):
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "encode_rows.js")], input=json.dumps(payload),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    return json.loads(p.stdout)


def test_js_encoder_rows_equal_python_encoder():
    b = synth.generate(synth.config("C5", n_docs=40))
    t = synth.generate(synth.config("C3", n_docs=5, changes_per_actor=30))
    docs = [decode_doc(b, i) for i in range(b.n_docs)] + [decode_doc(t, i) for i in range(t.n_docs)]
    docs += [c[1] for c in CASES]
    rng = np.random.default_rng(5)
    chunked = []
    for chs in docs:
        cuts = sorted(rng.integers(0, len(chs) + 1, size=2))
        chunked.append([chs[:cuts[0]], chs[cuts[0]:cuts[1]], chs[cuts[1]:]])
    got = run_node({"docs": chunked})
    pool = StringPool()
    for chunks, js in zip(chunked, got["docs"]):
        e = DocEncoder(pool, keep_log=False)
        for ch, j in zip(chunks, js):
            a = e.encode(ch)
            cc = a.changes.copy()
            assert cc.tobytes().hex() == j["changes"]
            assert a.deps.tobytes().hex() == j["deps"]
            assert a.ops.tobytes().hex() == j["ops"]
            assert (a.n_actors, a.n_regs, a.n_objs, a.flags) == (j["nActors"], j["nRegs"], j["nObjs"], j["flags"])
            assert (None if a.remap is None else list(a.remap)) == j["remap"]
            assert e.actors == j["actors"]
    assert pool.strings == got["strings"]


def test_js_clock_helpers_match_reference_vectors():
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "clock_vectors.json")))
    cases = [c for c in gold["cases"] if "Infinity" not in json.dumps(c)]
    got = run_node({"docs": [], "clocks": [[c["a"], c["b"]] for c in cases]})
    for c, (cmp, uni, eq) in zip(cases, got["clock"]):
        assert cmp == c["cmp"] and eq == c["equal"]
        assert uni == c["union"]


def test_js_channel_delivery_order():
    got = run_node({"docs": []})
    assert got["channel"] == [[1, 2, 3, "once4"], 1]


def test_js_clockstore_matches_reference_sql():
    """tests/golden/clockstore_vectors.json: the reference's ClockStore SQL executed in
    sqlite3 (tools/golden/gen_clockstore_vectors.py), incl. tests/ClockStore.test.ts."""
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "clockstore_vectors.json")))
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_clockstore.js")], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    for name, c in gold["cases"].items():
        assert got[name] == c["results"], name


def test_block_unpack_raw_and_brotli():
    """Block.unpack (src/Block.ts:18-29): raw '{"' JSON blocks and 'BR' + brotli blocks decode to
    the same Change objects and the same columnar rows; an unknown header throws the
    reference's message."""
    b = synth.generate(synth.config("C5", n_docs=3))
    changes = [c for i in range(b.n_docs) for c in decode_doc(b, i)][:200]
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_blocks.js")], input=json.dumps({"changes": changes}),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    assert got["same"] and got["rowsSame"] and got["n"] == len(changes)
    assert got["err"] == "fail to unpack blocks - head is 'xx'"


def test_js_encoder_snapshot_restore():
    """DocEncoder.snapshot/restore (the rollback of a throwing applyChanges): after restoring,
    re-encoding the same changes gives the same rows, ids and content classes as the first time,
    including a new actor that re-ranks, new objects/registers and a repeated (actor, seq)."""
    script = r"""
const C = require(process.argv[1] + '/hypermerge_amd/js/columnar.js')
const R = '00000000-0000-0000-0000-000000000000'
const ch = (actor, seq, deps, ops) => ({ actor, seq, deps, ops })
const e = new C.DocEncoder(new C.StringPool())
e.encode([ch('mm', 1, {}, [{ action: 'set', obj: R, key: 'x', value: 1 }])])
const B = [ch('aa', 1, {}, [{ action: 'makeMap', obj: 'o1' }, { action: 'link', obj: R, key: 'm', value: 'o1' }]),
           ch('mm', 1, {}, [{ action: 'set', obj: R, key: 'x', value: 2 }]),
           ch('mm', 1, {}, [{ action: 'set', obj: R, key: 'x', value: 1 }])]
const snap = e.snapshot()
const first = e.encode(B)
const t1 = JSON.stringify([e.actors, e.objList, e.regList, e.nContent])
e.restore(snap)
const t0 = JSON.stringify([e.actors, e.objList, e.regList, e.nContent])
const again = e.encode(B)
const t2 = JSON.stringify([e.actors, e.objList, e.regList, e.nContent])
const hex = (a) => [a.changes, a.deps, a.ops].map((b) => b.toString('hex')).join('|')
console.log(JSON.stringify({ same: hex(first) === hex(again), t0, t1, t2, remap: Array.from(first.remap || []),
  cids: [0, 1, 2].map((i) => first.changes.readUInt32LE(i * 24 + 20)) }))
"""
    p = subprocess.run([NODE, "-e", script, ROOT], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    assert got["same"] and got["t1"] == got["t2"]
    assert json.loads(got["t0"]) == [["mm"], [ROOT_ID], [[0, "x"]], 1]
    assert got["remap"] == [1]
    assert got["cids"] == [1, 2, 0]          # aa:1 new, mm:1 with new content new, mm:1 as before = class 0


# the persistence side's own statements (a restatement: one table keyed like the reference's
# Clocks, the upsert-max it runs per entry); the expected tables come from the reference SQL
_CLOCKS = ("CREATE TABLE Clocks (repoId TEXT NOT NULL, documentId TEXT NOT NULL, actorId TEXT NOT NULL, "
           "seq INTEGER NOT NULL, PRIMARY KEY (repoId, documentId, actorId)) WITHOUT ROWID")
_UPSERT = ("INSERT INTO Clocks (repoId, documentId, actorId, seq) VALUES (?, ?, ?, ?) ON CONFLICT (repoId, documentId, "
           "actorId) DO UPDATE SET seq = excluded.seq WHERE excluded.seq > seq")
_DELETE = "DELETE FROM Clocks WHERE repoId = ? AND documentId = ?"


def apply_batch(db, batch):
    """One round's ClockStore.takeBatch() rows in one transaction."""
    with db:
        for row in batch:
            if row[0] == "upsert":
                db.execute(_UPSERT, tuple(row[1:]))
            else:
                db.execute(_DELETE, tuple(row[1:]))


def test_clockstore_batches_replay_to_reference_tables():
    """Row f3: every round's ClockStore writes leave as ONE batch (takeBatch), replayed in one
    sqlite3 transaction; after each round the table equals the reference SQL's after the same
    update / set calls (tests/golden/clockstore_batches.json).  A colliding 64-bit key throws."""
    import sqlite3
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "clockstore_batches.json")))
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_persist.js")],
                       input=json.dumps({"rounds": gold["rounds"], "docs": gold["docs"]}),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    db = sqlite3.connect(":memory:")
    db.execute(_CLOCKS)
    n_rows = 0
    for r, (batch, want) in enumerate(zip(got["batches"], gold["tables"])):
        apply_batch(db, batch)
        n_rows += len(batch)
        table = [list(x) for x in db.execute(
            "SELECT repoId, documentId, actorId, seq FROM Clocks ORDER BY repoId, documentId, actorId").fetchall()]
        assert table == want, r
    assert n_rows < sum(len(c[3]) for rd in gold["rounds"] for c in rd)      # only the rows that changed
    last = {(a, b): [] for a, b in gold["docs"]}
    for rp, d, a, s in gold["tables"][-1]:
        last[(rp, d)].append([a, s])
    for (rp, d), g in zip(gold["docs"], got["get"]):
        assert sorted(g) == sorted(last[(rp, d)]), (rp, d)
    assert got["collision"] and "collision" in got["collision"] and '"actorA"' in got["collision"]
