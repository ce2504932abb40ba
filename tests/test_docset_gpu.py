"""The docset (hm_docset_*, csrc/docset.cpp): raw JSON blocks of many documents, one
applyChanges round per call (src/DocBackend.ts:169-185, Actor.parseBlock src/Actor.ts:137-141).

Every document is fed in several rounds; after each round its results, opSet clock / deps and
DocBackend.clock, and after the last its history order, merged state (hm_docset_view) and the
document its patches rebuild (a restatement of Frontend.applyPatch) must equal the CPU oracle's
cold merge of the same log.  Errors roll the document back; documents move to wider stores as
actors arrive."""
import json
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _blocks(changes):
    return [json.dumps(c, separators=(",", ":")).encode() for c in changes]


def _oracle(log):
    import oracle.oracle as O
    from hypermerge_amd.columnar import encode
    from hypermerge_amd.render import doc_summary
    b = encode([log])
    return doc_summary(b, O.merge(b), 0)


def _chunks(docs, rng, k=4):
    out = []
    for chs in docs:
        cuts = sorted(rng.integers(0, len(chs) + 1, size=k - 1))
        out.append([chs[:cuts[0]]] + [chs[cuts[i]:cuts[i + 1]] for i in range(k - 2)] + [chs[cuts[-1]:]])
    return out


def _run(ds, chunked, check_each_round=True):
    from hypermerge_amd.docset import apply_diffs, ROOT
    n = len(chunked)
    first = ds.open(n)
    ids = list(range(first, first + n))
    objects = [{ROOT: {"type": "map", "keys": {}, "elems": []}} for _ in range(n)]
    logs = [[] for _ in range(n)]
    last = [None] * n
    for r in range(max(len(c) for c in chunked)):
        sel = [i for i in range(n) if r < len(chunked[i])]
        res, js = ds.apply([ids[i] for i in sel], [_blocks(chunked[i][r]) for i in sel])
        for k, i in enumerate(sel):
            assert res[k]["status"] == 0, (i, r, res[k])
            logs[i] += chunked[i][r]
            apply_diffs(objects[i], js["p"][k]["diffs"])
            last[i] = (res[k], js["p"][k], js["b"][k])
            if check_each_round:
                s = _oracle(logs[i])
                assert int(res[k]["hist_len"]) == len(s["history"]) and int(res[k]["n_queued"]) == s["queued"]
                assert js["p"][k]["clock"] == s["clock"] and js["p"][k]["deps"] == s["deps"], (i, r)
                assert js["b"][k] == s["backend_clock"], (i, r)
    return ids, objects, logs, last


@pytest.mark.parametrize("name,n,net", [("C2", 60, False), ("C4", 80, False), ("C5", 60, False), ("C3", 6, False),
                                        ("C5", 60, True), ("C3", 6, True)])
def test_docset_rounds_equal_oracle(name, n, net):
    """Per-op diffs (default) and net diffs (HM_DOCSET_NET_DIFFS) both rebuild the oracle's
    document round after round; the per-op replay ends on the device's merged registers."""
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc
    from hypermerge_amd.docset import DocSet, render_objects, view_objects
    from hypermerge_amd.engine import Engine
    over = {"changes_per_actor": 30} if name == "C3" else {}
    b = synth.generate(synth.config(name, n_docs=n, **over))
    docs = [decode_doc(b, i) for i in range(b.n_docs)]
    ds = DocSet(Engine(0), net_diffs=net)
    ids, objects, logs, last = _run(ds, _chunks(docs, np.random.default_rng(7)), check_each_round=name != "C3")
    for i, d in enumerate(ids):
        s = _oracle(logs[i])
        assert s["status"] == "OK"
        assert render_objects(objects[i]) == json.loads(json.dumps(s["state"])), i       # patches rebuild it
        assert render_objects(view_objects(ds.view(d))) == json.loads(json.dumps(s["state"])), i
        order = ds.history_prefix(d, 1 << 20)
        assert [[logs[i][k]["actor"], logs[i][k]["seq"]] for k in order] == s["history"], i
        assert last[i][1]["clock"] == s["clock"] and last[i][2] == s["backend_clock"]
    st = ds.stats()
    assert st["calls"] == 4
    if net:
        assert st["hit_patches"] > 0 and st["op_patches"] == 0
    else:
        assert st["op_patches"] > 0 and st["replay_mismatch"] == 0 and st["hit_patches"] == 0


def test_docset_errors_roll_back():
    """A mismatched duplicate (Inconsistent reuse of sequence number) and an undecodable block
    leave the document as it was; the next good round continues from there."""
    from hypermerge_amd.columnar import ROOT_ID as R
    from hypermerge_amd.docset import DocSet
    from hypermerge_amd.engine import Engine
    ds = DocSet(Engine(0))
    d = ds.open(2)
    a, b = "actorA", "actorB"
    c1 = {"actor": a, "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": R, "key": "x", "value": 1}]}
    c2 = {"actor": b, "seq": 1, "deps": {a: 1}, "ops": [{"action": "set", "obj": R, "key": "x", "value": 2}]}
    res, js = ds.apply([d, d + 1], [_blocks([c1]), _blocks([c1])])
    assert (res["status"] == 0).all()
    # the same content with its keys in another order is the same change (a no-op duplicate)
    same = json.dumps({"ops": c1["ops"], "deps": {}, "seq": 1, "actor": a}).encode()
    bad = dict(c1, ops=[{"action": "set", "obj": R, "key": "x", "value": 99}])
    res, js = ds.apply([d, d + 1], [[same] + _blocks([c2]), _blocks([c2, bad])])
    assert res[0]["status"] == 0 and res[1]["status"] == 1
    assert js["p"][1] is None and js["p"][0]["diffs"] == [{"action": "set", "type": "map", "obj": R, "key": "x", "value": 2}]
    assert ds.info(d + 1)["n_changes"] == 1 and ds.info(d + 1)["hist_len"] == 1
    res, js = ds.apply([d + 1], [[b'{"actor": "x", oops'] + _blocks([c2])])
    assert res[0]["status"] == 32 and res[0]["err_change"] == 0
    assert ds.info(d + 1)["n_actors"] == 1
    res, js = ds.apply([d + 1], [_blocks([c2])])
    assert res[0]["status"] == 0 and js["p"][0]["clock"] == {a: 1, b: 1} and js["b"][0] == {a: 1, b: 1}
    assert js["p"][0]["diffs"] == [{"action": "set", "type": "map", "obj": R, "key": "x", "value": 2}]
    assert ds.view(d) == ds.view(d + 1)


@pytest.mark.parametrize("where", ["wait:1", "read"])
def test_docset_failed_call_is_undone_everywhere(where, monkeypatch):
    """A call whose documents live in two store classes fails after the first class's batch was
    applied (wait:1: after the second class's; read: after both, before the patch reads): the
    batches already applied are undone (hm_batch_undo) and every document's host state rolls back,
    so the store and the host agree and the same round applies cleanly afterwards."""
    from hypermerge_amd.columnar import ROOT_ID as R
    from hypermerge_amd.docset import DocSet, render_objects, view_objects
    from hypermerge_amd.engine import Engine, EngineError
    ds = DocSet(Engine(0))
    d = ds.open(2)
    narrow = [{"actor": f"n{i}", "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": R, "key": "k", "value": i}]}
              for i in range(3)]
    wide = [{"actor": f"w{i:02d}", "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": R, "key": f"k{i % 3}", "value": i}]}
            for i in range(12)]                                  # 12 actors: the 16-wide class
    ds.apply([d, d + 1], [_blocks(narrow[:2]), _blocks(wide[:10])])
    info0, view0 = [ds.info(x) for x in (d, d + 1)], [ds.view(x) for x in (d, d + 1)]
    r2 = [narrow[2:] + [{"actor": "n0", "seq": 2, "deps": {"n1": 1, "n2": 1}, "ops": [{"action": "del", "obj": R, "key": "k"}]}],
          wide[10:] + [{"actor": "w00", "seq": 2, "deps": {"w05": 1}, "ops": [{"action": "set", "obj": R, "key": "k1", "value": 7}]}]]
    routed0 = ds.routing()
    monkeypatch.setenv("HM_DOCSET_INJECT_FAIL", where)
    with pytest.raises(EngineError):
        ds.apply([d, d + 1], [_blocks(r2[0]), _blocks(r2[1])])
    monkeypatch.delenv("HM_DOCSET_INJECT_FAIL")
    assert [ds.info(x) for x in (d, d + 1)] == info0
    assert [ds.view(x) for x in (d, d + 1)] == view0
    assert ds.routing() == routed0                            # the undone call's rounds are not counted
    res, js = ds.apply([d, d + 1], [_blocks(r2[0]), _blocks(r2[1])])
    assert (res["status"] == 0).all()
    assert sum(ds.routing().values()) == sum(routed0.values()) + 2
    for k, (x, log) in enumerate(((d, narrow + r2[0][1:]), (d + 1, wide + r2[1][2:]))):
        s = _oracle(log)
        assert js["p"][k]["clock"] == s["clock"] and js["b"][k] == s["backend_clock"]
        assert render_objects(view_objects(ds.view(x))) == json.loads(json.dumps(s["state"]))


def test_docset_failed_call_frees_a_failed_new_documents_handle(monkeypatch):
    """A new document whose own merge throws keeps a fresh (empty) handle; when the call then
    fails as a whole, that handle goes back to the free list and the document must not keep it —
    otherwise a later new document is given the same handle and both share store rows."""
    from hypermerge_amd.columnar import ROOT_ID as R
    from hypermerge_amd.docset import DocSet, render_objects, view_objects
    from hypermerge_amd.engine import Engine, EngineError
    ds = DocSet(Engine(0))
    a = ds.open(3)
    good = [{"actor": "g0", "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": R, "key": "k", "value": 1}]}]
    bad = [{"actor": "b0", "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": "no-such-object", "key": "k", "value": 2}]}]
    monkeypatch.setenv("HM_DOCSET_INJECT_FAIL", "read")
    with pytest.raises(EngineError):
        ds.apply([a, a + 1], [_blocks(good), _blocks(bad)])
    monkeypatch.delenv("HM_DOCSET_INJECT_FAIL")
    assert ds.info(a + 1)["a_stride"] == 0                    # not placed: no handle kept
    h = ds.handles(8)
    assert h["opened"] == h["free"]                           # both fresh handles are free again
    # the failed document, then a fresh one: each gets its own handle
    res, _ = ds.apply([a + 1], [_blocks(bad)])
    assert res["status"][0] != 0
    other = [{"actor": "o0", "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": R, "key": "z", "value": 9}]}]
    res, _ = ds.apply([a, a + 2], [_blocks(good), _blocks(other)])
    assert (res["status"] == 0).all()
    fixed = [{"actor": "b0", "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": R, "key": "q", "value": 3}]}]
    res, _ = ds.apply([a + 1], [_blocks(fixed)])
    assert (res["status"] == 0).all()
    for x, log in ((a, good), (a + 1, fixed), (a + 2, other)):
        assert render_objects(view_objects(ds.view(x))) == json.loads(json.dumps(_oracle(log)["state"])), x
    h = ds.handles(8)
    assert h["opened"] - h["free"] == 3                       # one handle per document


def test_docset_moves_documents_to_wider_stores():
    """Documents whose actors outgrow 8 / 16 / 32 move to the wider store class with their
    whole log; the merged state equals the oracle's, patches included."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_gpu_parity import _float_counter_docs
    from hypermerge_amd.docset import DocSet, render_objects, view_objects
    from hypermerge_amd.engine import Engine
    docs = _float_counter_docs(24, 77, wide=True)
    rng = random.Random(3)
    chunked = []
    for chs in docs:
        cuts = sorted(rng.sample(range(1, len(chs)), min(3, len(chs) - 1))) if len(chs) > 1 else []
        parts, prev = [], 0
        for c in cuts + [len(chs)]:
            parts.append(chs[prev:c])
            prev = c
        chunked.append(parts)
    ds = DocSet(Engine(0))
    ids, objects, logs, last = _run(ds, chunked)
    for i, d in enumerate(ids):
        s = _oracle(logs[i])
        assert render_objects(objects[i]) == json.loads(json.dumps(s["state"])), i
        assert render_objects(view_objects(ds.view(d))) == json.loads(json.dumps(s["state"])), i
        assert ds.info(d)["a_stride"] >= len(s["backend_clock"])
    assert ds.stats()["moves"] > 0 and ds.stats()["replay_mismatch"] == 0


def test_docset_moved_documents_release_their_handles():
    """A document that moves to a wider store releases its old handle (hm_doc_reset): the
    handle is an empty document again and the next documents placed in that store take it
    instead of opening new ones; their rounds (incremental ones included) equal the oracle."""
    from hypermerge_amd.columnar import ROOT_ID as R
    from hypermerge_amd.docset import DocSet, render_objects, view_objects
    from hypermerge_amd.engine import Engine

    def chg(actor, seq, deps, key, value):
        return {"actor": actor, "seq": seq, "deps": deps, "ops": [{"action": "set", "obj": R, "key": key, "value": value}]}
    ds = DocSet(Engine(0))
    a = ds.open(6)
    logs = {}
    first = {a + i: [chg(f"a{i}{j}", 1, {}, f"k{j % 3}", j) for j in range(5)] for i in range(6)}
    ds.apply(list(first), [_blocks(v) for v in first.values()])
    logs.update(first)
    assert ds.handles(8) == {"opened": 6, "free": 0}
    wide = {a + i: [chg(f"w{i}{j:02d}", 1, {}, f"k{j % 4}", 100 + j) for j in range(9)] for i in range(4)}
    res, _ = ds.apply(list(wide), [_blocks(v) for v in wide.values()])
    assert (res["status"] == 0).all()
    for d, v in wide.items():
        logs[d] = logs[d] + v
        assert ds.info(d)["a_stride"] == 16
    assert ds.handles(8) == {"opened": 6, "free": 4} and ds.handles(16)["opened"] == 4
    b = ds.open(3)
    for r in range(3):                                              # placed, then two incremental rounds
        new = {b + i: [chg(f"b{i}", r + 1, {f"b{i}": r} if r else {}, f"k{r}", 10 * i + r)] for i in range(3)}
        res, js = ds.apply(list(new), [_blocks(v) for v in new.values()])
        assert (res["status"] == 0).all()
        for k, (d, v) in enumerate(new.items()):
            logs[d] = logs.get(d, []) + v
            s = _oracle(logs[d])
            assert js["p"][k]["clock"] == s["clock"] and js["b"][k] == s["backend_clock"]
    assert ds.handles(8) == {"opened": 6, "free": 1}
    for d, log in logs.items():
        s = _oracle(log)
        assert render_objects(view_objects(ds.view(d))) == json.loads(json.dumps(s["state"])), d
        assert ds.info(d)["n_changes"] == len(log)


def test_docset_clock_update_matches_reference_sql():
    """ClockStore.update(self, doc, doc.clock) after a round (src/ClockStore.ts:78-91): the
    first update writes, a repeat does not, and the stored clocks are the DocBackend clocks."""
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc
    from hypermerge_amd.docset import DocSet
    from hypermerge_amd.engine import Engine
    b = synth.generate(synth.config("C5", n_docs=30))
    docs = [decode_doc(b, i) for i in range(b.n_docs)]
    ds = DocSet(Engine(0), patches=False)
    first = ds.open(len(docs))
    ids = list(range(first, first + len(docs)))
    res, js = ds.apply(ids, [_blocks(c) for c in docs])
    assert all(p["diffs"] == [] for p in js["p"])
    w, df, stored = ds.clock_update(ids + [ds.open(1)])
    assert w[:-1].all() and not w[-1] and not df.any()
    assert stored[:-1] == js["b"] and stored[-1] == {}
    w, df, stored = ds.clock_update(ids)
    assert not w.any() and not df.any()


def test_docset_rounds_report_their_route():
    """The docset's stores route arriving rounds by the cost rule (store_kernels.h HM_INC_COST):
    after a first load, rounds of 1-2 changes per document go incremental — hm_docset_routing
    counts them — and the patches / state still equal the oracle's; a round as long as the log
    re-merges."""
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc
    from hypermerge_amd.docset import DocSet, render_objects, view_objects
    from hypermerge_amd.engine import Engine
    b = synth.generate(synth.config("C4", n_docs=60))
    docs = [decode_doc(b, i) for i in range(b.n_docs)]
    chunked = []
    for chs in docs:
        parts, k = [chs[:len(chs) - 6]], len(chs) - 6
        while k < len(chs):
            parts.append(chs[k:k + 2])
            k += 2
        chunked.append(parts)
    ds = DocSet(Engine(0))
    ids, objects, logs, last = _run(ds, chunked)
    r = ds.routing()
    assert r["incremental"] >= 2 * len(docs), r             # (the three 2-change rounds, most of them)
    assert r["remerged"] >= len(docs)                        # (the first load)
    for i, d in enumerate(ids[::7]):
        s = _oracle(logs[ids.index(d)])
        assert render_objects(view_objects(ds.view(d))) == json.loads(json.dumps(s["state"]))
