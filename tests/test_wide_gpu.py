"""Documents of more than 64 actors.  The reference mints one actor per writer
(src/RepoBackend.ts:286-293), so a widely shared document outgrows any fixed width; the engine
merges them in the general kernel with per-actor rows up to HM_MAX_STRIDE (256) wide.

Each case is compared with the CPU oracle on the same encoded batch: one batch merge
(hm_merge_host, small documents mixed in), the resident store at strides 128 / 256 over
several applyChanges calls (new actors re-rank the old rows), and the docset, whose documents
move into the 128 / 256 store classes as writers arrive."""
import json
import os
import random
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import oracle.oracle as O                                               # noqa: E402
from hypermerge_amd.columnar import ROOT_ID as R, encode                # noqa: E402

pytestmark = pytest.mark.gpu


def _wide_docs(n_docs, seed, lo, hi):
    """Documents of lo..hi actors: concurrent and causal sets on a few keys (conflicts over
    many actors), counters, a shared list every writer appends to, gossiped deps, and
    shuffled delivery for some (queued changes)."""
    rng = random.Random(seed)
    docs = []
    for _ in range(n_docs):
        na = rng.randint(lo, hi)
        actors = [f"w{rng.randrange(10 ** 6):06d}-{i:03d}" for i in range(na)]
        seqs = {a: 0 for a in actors}
        heard = {a: {} for a in actors}
        chs = []
        first = actors[0]
        seqs[first] = 1
        chs.append({"actor": first, "seq": 1, "deps": {}, "ops": [
            {"action": "makeList", "obj": "LL"}, {"action": "link", "obj": R, "key": "list", "value": "LL"},
            {"action": "set", "obj": R, "key": "n", "value": 0, "datatype": "counter"}]})
        for b in actors:
            heard[b][first] = 1
        elems = {}
        for a in actors[1:] + [rng.choice(actors) for _ in range(na // 2)]:
            seqs[a] += 1
            ops = [{"action": "set", "obj": R, "key": f"k{rng.randrange(4)}", "value": rng.randrange(1000)},
                   {"action": "inc", "obj": R, "key": "n", "value": rng.randint(-3, 9)}]
            if rng.random() < 0.5:
                vis = [e for e, (who, q) in elems.items() if heard[a].get(who, 0) >= q or who == a]
                after = rng.choice(vis) if vis and rng.random() < 0.7 else "_head"
                el = seqs[a] * 1000 + rng.randrange(1000)
                ops += [{"action": "ins", "obj": "LL", "key": after, "elem": el},
                        {"action": "set", "obj": "LL", "key": f"{a}:{el}", "value": a[-3:]}]
                elems[f"{a}:{el}"] = (a, seqs[a])
            deps = {b: q for b, q in heard[a].items() if b != a}
            chs.append({"actor": a, "seq": seqs[a], "deps": deps, "ops": ops})
            for b in actors:
                if b == a or rng.random() < 0.6:
                    heard[b][a] = seqs[a]
        if rng.random() < 0.3:
            rng.shuffle(chs)
        docs.append(chs)
    return docs


@pytest.mark.parametrize("S,lo,hi", [(128, 65, 127), (256, 129, 255)])
def test_wide_batch_equals_oracle(engine, S, lo, hi):
    from test_gpu_parity import assert_same
    docs = _wide_docs(12, S, lo, hi) + _wide_docs(20, S + 1, 2, 8)        # small documents in the same batch
    random.Random(S).shuffle(docs)
    b = encode(docs, a_stride=S)
    # minimumClock rows with entries past actor 64 (DocBackend.updateMinimumClock)
    rng = np.random.default_rng(S)
    mc = np.zeros(b.n_docs * S, np.uint32)
    for d in range(b.n_docs):
        na = int(b.docs["n_actors"][d])
        for a in rng.choice(na, size=min(na, 3), replace=False):
            mc[d * S + a] = int(rng.integers(0, 3))
    b.min_clock = mc
    o = O.merge(b)
    assert (o.docs["status"] == 0).sum() >= len(docs) - 2
    assert assert_same(b, engine.merge(b), o) == 0
    # a minimum clock entry of a small document's row past actor 64: never satisfied
    small = [d for d in range(b.n_docs) if int(b.docs["n_actors"][d]) <= 8 and o.docs["status"][d] == 0]
    mc2 = mc.copy()
    for d in small:
        mc2[d * S + S - 1] = 1
    b.min_clock = mc2
    o2 = O.merge(b)
    assert all(int(o2.docs["min_cmp"][d]) in (2, 3) for d in small)
    assert_same(b, engine.merge(b), o2)


def test_wide_store_rounds_equal_oracle(engine):
    """The resident store at stride 256: documents receive their changes over four calls;
    writers arriving later re-rank the old rows (JS string order); after each call every
    document equals the oracle's cold merge of its log."""
    from test_store_gpu import assert_doc_matches_oracle, split
    from hypermerge_amd.store import DocStore
    docs = _wide_docs(6, 11, 70, 200)
    store = DocStore(engine, a_stride=256)
    hs = [store.open() for _ in docs]
    rng = np.random.default_rng(3)
    parts = [split(d, 4, rng) for d in docs]
    for r in range(4):
        store.apply([(h, parts[i][r]) for i, h in enumerate(hs)])
        for h in hs:
            assert_doc_matches_oracle(store, h)


def test_wide_docset_moves_to_wide_classes():
    """The docset: a document whose writers grow past 64 and 128 moves to the 128 / 256 store
    classes with its log; patches rebuild the oracle's document, clocks equal."""
    from test_docset_gpu import _oracle, _run
    from hypermerge_amd.docset import DocSet, render_objects, view_objects
    from hypermerge_amd.engine import Engine
    docs = _wide_docs(4, 5, 100, 220)
    chunked = []
    for chs in docs:
        k = len(chs)
        chunked.append([chs[: k // 5], chs[k // 5: k // 2], chs[k // 2:]])
    ds = DocSet(Engine(0))
    ids, objects, logs, last = _run(ds, chunked, check_each_round=True)
    for i, d in enumerate(ids):
        s = _oracle(logs[i])
        assert s["status"] == "OK"
        assert render_objects(objects[i]) == json.loads(json.dumps(s["state"])), i
        assert render_objects(view_objects(ds.view(d))) == json.loads(json.dumps(s["state"])), i
        assert ds.info(d)["a_stride"] >= 128
    assert ds.stats()["moves"] > 0


def test_docset_refuses_the_256th_writer():
    """255 writers are the docset's limit (rank 255 is the stores' 'no rank' byte): the call
    that brings the 256th fails for that document only and rolls it back."""
    from hypermerge_amd.docset import DocSet
    from hypermerge_amd.engine import Engine
    ds = DocSet(Engine(0), patches=False)
    d = ds.open(1)
    chs = [{"actor": f"a{i:03d}", "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": R, "key": "x", "value": i}]}
           for i in range(256)]
    blk = lambda cs: [json.dumps(c).encode() for c in cs]                          # noqa: E731
    res, _ = ds.apply([d], [blk(chs[:255])])
    assert res[0]["status"] == 0 and ds.info(d)["n_actors"] == 255
    res, _ = ds.apply([d], [blk(chs[255:])])
    assert res[0]["status"] == 16 and ds.info(d)["n_actors"] == 255
