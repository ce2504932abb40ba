"""Host side of the resident store (no GPU): the incremental interner must produce,
across successive applyChanges calls, exactly the log a one-shot encoding of the
concatenated changes produces (same ranks, registers, objects), so the oracle's
merge of the log equals one cold applyChanges."""
import numpy as np
import pytest

from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc, encode
from hypermerge_amd.render import canonical_json
from hypermerge_amd.store import DocEncoder, StringPool
import oracle.oracle as O

from kat_cases import CASES


def incremental_log(changes, cuts):
    e = DocEncoder(StringPool())
    prev = 0
    remaps = 0
    for c in list(cuts) + [len(changes)]:
        a = e.encode(changes[prev:c])
        remaps += a.remap is not None
        prev = c
    return e, remaps


@pytest.mark.parametrize("name", ["C2", "C5", "C3"])
def test_incremental_log_equals_cold_encoding(name):
    b = synth.generate(synth.config(name, n_docs=60, **({"changes_per_actor": 60} if name == "C3" else {})))
    rng = np.random.default_rng(3)
    for i in range(b.n_docs):
        changes = decode_doc(b, i)
        cuts = sorted(rng.integers(0, len(changes) + 1, size=3))
        e, _ = incremental_log(changes, cuts)
        lb = e.log_batch(8)
        cold = encode([changes], 8)
        for f in ("actor", "n_deps", "seq", "dep_off", "n_ops", "op_first"):
            np.testing.assert_array_equal(lb.changes[f], cold.changes[f], err_msg=f)
        np.testing.assert_array_equal(lb.deps, cold.deps)
        for f in ("obj", "reg", "parent", "elem", "action", "datatype", "vtag", "value"):
            if f == "value":
                strs = cold.ops["vtag"] == 5
                np.testing.assert_array_equal(lb.ops[f][~strs], cold.ops[f][~strs])
            else:
                np.testing.assert_array_equal(lb.ops[f], cold.ops[f], err_msg=f)
        assert canonical_json(lb, O.merge(lb), 0) == canonical_json(cold, O.merge(cold), 0)


@pytest.mark.parametrize("name,changes,expect", CASES, ids=[c[0] for c in CASES])
def test_known_answers_split_in_two_calls(name, changes, expect):
    """applyChanges(applyChanges(init, A), B) == applyChanges(init, A ++ B) on the oracle
    over the incremental log, for every known-answer case and every split point."""
    S = max(8, len({c["actor"] for c in changes} | {a for c in changes for a in c["deps"]}))
    cold = encode([changes], S)
    want = canonical_json(cold, O.merge(cold), 0)
    for cut in range(len(changes) + 1):
        e, _ = incremental_log(changes, [cut])
        lb = e.log_batch(S)
        assert canonical_json(lb, O.merge(lb), 0) == want, (name, cut)


def test_remap_when_a_smaller_actor_arrives():
    from kat_cases import ch, s
    e = DocEncoder(StringPool())
    a1 = e.encode([ch("mmmm", 1, {}, s("x", 1)), ch("zzzz", 1, {}, s("x", 2))])
    assert a1.remap is None and e.actors == ["mmmm", "zzzz"]
    a2 = e.encode([ch("aaaa", 1, {}, s("x", 3))])
    assert list(a2.remap) == [1, 2] and e.actors == ["aaaa", "mmmm", "zzzz"]
    assert list(e.log_changes["actor"]) == [1, 2, 0]
    a3 = e.encode([ch("zzzz", 2, {"aaaa": 1}, s("x", 4))])
    assert a3.remap is None
    snap = e.snapshot()
    e.encode([ch("0000", 1, {}, s("q", 1))])
    e.restore(snap)
    assert e.actors == ["aaaa", "mmmm", "zzzz"] and len(e.log_changes) == 4


def test_feed_bitmaps_pack_lsb_first():
    from hypermerge_amd.sync import pack_feeds
    p = np.zeros(70, bool)
    p[[0, 3, 63, 64, 69]] = True
    w, off = pack_feeds([p, np.ones(3, bool)])
    assert list(off) == [0, 3]
    assert int(w[0]) == (1 | 8 | (1 << 63)) and int(w[1]) == (1 | (1 << 5)) and int(w[2]) == 0
    assert int(w[3]) == 7


def test_slice_changes_rebuilds_each_document_range():
    """store.slice_changes (the bench's / RowStore's row feed): the slices of a batch at any cut
    points concatenate back to each document's rows."""
    from hypermerge_amd.store import slice_changes
    b = synth.generate(synth.config("C5", n_docs=50), threads=2)
    rng = np.random.default_rng(1)
    n = b.docs["n_changes"].astype(np.int64)
    cut = (rng.random(b.n_docs) * (n + 1)).astype(np.int64)
    sel = np.arange(0, b.n_docs, 2)
    p1 = slice_changes(b, np.zeros(b.n_docs, np.int64), cut, sel)
    p2 = slice_changes(b, cut, n, sel)
    def rows(bt, j):
        doc = bt.docs[j]
        c = bt.changes[int(doc["change_off"]): int(doc["change_off"]) + int(doc["n_changes"])]
        dp = bt.deps[int(doc["dep_off"]): int(doc["dep_off"]) + int(doc["n_deps"])]
        op = bt.ops[int(doc["op_off"]): int(doc["op_off"]) + int(doc["n_ops"])]
        # every change's deps / ops are its own, in order
        assert (c["dep_off"][1:] == c["dep_off"][:-1] + c["n_deps"][:-1]).all() if len(c) else True
        assert (c["op_first"][1:] == c["op_first"][:-1] + c["n_ops"][:-1]).all() if len(c) else True
        cf = np.stack([c[f].astype(np.int64) for f in ("actor", "n_deps", "seq", "n_ops", "content_id")], 1)
        return cf, dp, op
    for j, d in enumerate(sel):
        w = rows(b, int(d))
        a, bb = rows(p1, j), rows(p2, j)
        for x, y1, y2 in zip(w, a, bb):
            assert np.concatenate([y1, y2]).tobytes() == x.tobytes()
        for f in ("n_actors", "n_regs", "n_objs"):
            assert p1.docs[f][j] == b.docs[f][d] == p2.docs[f][j]
