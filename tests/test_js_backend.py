"""The JS restatement (oracle/js/backend.js, BASELINE.md's second CPU baseline) agrees with the
C restatement (oracle/oracle.c) on generated documents: history order, clocks, queue and the
materialized document, fed in several applyChanges calls through its DocBackend."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc, encode
from hypermerge_amd.render import doc_state
import oracle.oracle as O

from repo_harness import plain

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


@pytest.mark.parametrize("name,n,kw", [("C2", 40, {}), ("C5", 40, {}), ("C3", 4, {"changes_per_actor": 30}),
                                       ("C2", 30, {"arrival": 2, "shuffle_pct": 30})])
def test_js_restatement_matches_oracle(name, n, kw):
    b = synth.generate(synth.config(name, n_docs=n, **kw), threads=2)
    docs = [decode_doc(b, i) for i in range(b.n_docs)]
    rng = np.random.default_rng(2)
    chunks = []
    for chs in docs:
        cuts = sorted(rng.integers(0, len(chs) + 1, size=2))
        chunks.append([chs[:cuts[0]], chs[cuts[0]:cuts[1]], chs[cuts[1]:]])
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_cpu_backend.js")],
                       input=json.dumps({"docs": chunks}), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    js = json.loads(p.stdout.strip().splitlines()[-1])["docs"]
    cold = encode(docs, 8)
    r = O.merge(cold)
    for i, chs in enumerate(docs):
        j = js[i]
        st = int(r.docs["status"][i])
        assert (j["err"] is None) == (st == 0), (i, j["err"], st)
        if st:
            continue
        c0, nc = int(cold.docs["change_off"][i]), int(cold.docs["n_changes"][i])
        pos = r.hist[c0:c0 + nc]
        order = [chs[k] for k in np.argsort(np.where(pos >= 0, pos, 1 << 30), kind="stable")[:int((pos >= 0).sum())]]
        assert j["history"] == [[c["actor"], c["seq"]] for c in order]
        assert j["queued"] == int(r.docs["n_queued"][i])
        S = cold.a_stride
        actors = cold.doc_actors[i]
        clock = {actors[a]: int(v) for a, v in enumerate(r.clock[i * S:(i + 1) * S]) if v}
        assert j["clock"] == clock
        assert j["doc"] == plain(doc_state(cold, r, i)), i


def test_restatement_local_undo_redo_known_answers():
    """Backend.applyLocalChange of the JS restatement (oracle/js/backend.js; SURVEY Appendix A.4
    [R], parity unpinned: Automerge 0.12 is not vendored): undo restores a set field, a new
    key (a del), a counter (the inc's negation) and a list element (removed); redo re-applies;
    `undoable: false` records nothing; a new change clears the redo stack; the throws.  The
    expected answers are hand-checked and kept in tests/golden/undo_kats.json."""
    import json
    import shutil
    import subprocess
    node = shutil.which("node")
    if node is None:
        pytest.skip("node not installed")
    p = subprocess.run([node, os.path.join(ROOT, "tests", "js", "run_undo_kat.js")], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "undo_kats.json")))
    assert got == want
    assert want["set_undo_redo"][1][0]["x"] == 1 and want["set_undo_redo"][1][1:3] == [False, True]
    assert "y" not in want["new_key_undo_is_del"][1][0]
    assert want["inc_undo"][1][0]["n"] == 5 and want["list_insert_undo"][1][0]["l"] == []
    assert want["nothing_to_undo"][0] == ["throw", "Cannot undo: there is nothing to be undone"]
