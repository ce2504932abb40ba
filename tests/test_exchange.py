"""Sharding and the cross-rank clock exchange (hypermerge_amd/exchange.py; C-ABI
hm_clock_* in include/hypermerge_amd.h) with world_size 2 over gloo on CPU — the GPU box
runs the same protocol over RCCL (tests/test_exchange_gpu.py runs the C-ABI itself).

* shards: FNV-1a64(docId) % world partitions the global doc-id stream (disjoint,
  complete), and each shard merges independently (no data-path collective);
* the ranks own *different* documents with *different* actor tables (2..11 actors per
  document, actors shared between documents as a merge/fork shares them); every rank's host
  rebuilds, from the gathered records, exactly the {docId: {actorId: seq}} clocks a
  CursorMessage carries for every document of the node (src/RepoBackend.ts:374-392,
  src/PeerMsg.ts:12-16): the DocBackend.clock of each document (src/DocBackend.ts:135-142);
* the min-clock over replicas (documents held by both ranks at different progress, plus
  documents held by one rank only) equals Clock.intersection (src/Clock.ts:103-113) of the
  holders' clocks.
"""
import os
import random
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from hypermerge_amd import synth
from hypermerge_amd import clock as C
from hypermerge_amd import columnar as col

N_DOCS = 400
B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _b58(rng):
    """A base58 id of 32 random bytes, as hypermerge mints doc and actor ids."""
    n = int.from_bytes(bytes(rng.getrandbits(8) for _ in range(32)), "big")
    s = ""
    while n:
        n, r = divmod(n, 58)
        s = B58[r] + s
    return s


def _world_docs(seed=7, n=48):
    """Documents with ids, actor tables and change feeds (identical on every rank)."""
    rng = random.Random(seed)
    pool = [_b58(rng) for _ in range(40)]                   # actors, some shared across documents
    docs = []
    for _ in range(n):
        doc = _b58(rng)
        actors = rng.sample(pool, rng.randint(2, 11))
        seqs = {a: 0 for a in actors}
        changes = []
        for i in range(rng.randint(3, 30)):
            a = rng.choice(actors)
            seqs[a] += 1
            deps = {b: s for b, s in seqs.items() if b != a and s and rng.random() < 0.5}
            changes.append({"actor": a, "seq": seqs[a], "deps": deps,
                            "ops": [{"action": "set", "obj": col.ROOT_ID, "key": f"k{i % 5}", "value": i}]})
        docs.append((doc, changes))
    return docs


def _doc_clock(changes):
    """DocBackend.updateClock (src/DocBackend.ts:135-142): clock[actor] = max(clock[actor] || 0, seq)."""
    c = {}
    for ch in changes:
        c[ch["actor"]] = max(c.get(ch["actor"], 0), ch["seq"])
    return c


def _engine_rows(owned, keys, X):
    """The dense rows the engine keeps for `owned` documents: encoded columnar batch, the
    CPU restatement's DocBackend.clock (back_clock) per document, actor keys per rank."""
    import oracle.oracle as O
    if not owned:
        return np.zeros(0, X.CLOCK_REC_DT)
    b = col.encode([ch for _, ch in owned], a_stride=16)
    r = O.merge(b)
    S = b.a_stride
    dk = np.array([keys.key(d) for d, _ in owned], np.uint64)
    ak = np.zeros(len(owned) * S, np.uint64)
    for i, actors in enumerate(b.doc_actors):
        for rank_, a in enumerate(actors):
            ak[i * S + rank_] = keys.key(a)
    return X.records_host(dk, ak, r.back_clock.astype(np.uint32))


def _worker(rank, ws, port, out):
    from hypermerge_amd import exchange as X
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        # synthetic shards (bench.py's C4 stream): disjoint, keyed by FNV-1a64 of the doc id
        b = synth.generate(synth.config("C4", n_docs=N_DOCS, shard=rank, n_shards=ws), threads=2)
        gkeys = (b.docs["reserved"][:, 0].astype(np.int64) | (b.docs["reserved"][:, 1].astype(np.int64) << 32))

        world = _world_docs()
        keys = X.KeyTable()
        tr = X.TorchTransport()
        ex = X.ClockExchange(tr, keys)
        owned = [(d, ch) for d, ch in world if X.shard_of(d, ws) == rank]
        own = _engine_rows(owned, keys, X)
        tr.exchange_keys(keys)                    # host id tables (the swarm's feed ids)
        gathered = ex.gather(own)
        clocks = ex.clocks(gathered)

        # replicas: the first 20 documents on both ranks at a different progress, the next 8
        # on one rank only
        rep = []
        for i, (d, ch) in enumerate(world[:28]):
            if i < 20:
                rep.append((d, ch[: max(1, len(ch) * (rank + 1) // 3)]))
            elif i % 2 == rank:
                rep.append((d, ch))
        rown = _engine_rows(rep, keys, X)
        tr.exchange_keys(keys)
        rall = ex.gather(rown)
        mc = ex.min_clock(rall, rown)
        out[rank] = {"keys": gkeys.tolist(), "owned": [d for d, _ in owned], "clocks": clocks, "min": mc,
                     "rep": {d: _doc_clock(ch) for d, ch in rep}, "n_recs": len(gathered)}
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_and_clock_exchange():
    ws = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(ws, port, out), nprocs=ws, join=True)
        out = dict(out)
    # synthetic sharding: disjoint, complete, every key hashes to its shard
    k0, k1 = set(out[0]["keys"]), set(out[1]["keys"])
    assert len(k0) == N_DOCS and len(k1) == N_DOCS and not (k0 & k1)
    for r in (0, 1):
        for g in list(out[r]["keys"])[:50]:
            assert synth.lib().hm_synth_fnv1a64_docid(synth.CONFIGS["C4"].seed, g) % ws == r

    world = _world_docs()
    o0, o1 = set(out[0]["owned"]), set(out[1]["owned"])
    assert o0 and o1 and not (o0 & o1) and o0 | o1 == {d for d, _ in world}
    # the ranks' actor tables differ (documents of different actor sets on each rank)
    acts = [{a for d, ch in world if d in o for a in _doc_clock(ch)} for o in (o0, o1)]
    assert acts[0] != acts[1]
    # every rank rebuilds the CursorMessage clocks of every document of the node, exactly
    expect = {d: _doc_clock(ch) for d, ch in world}
    for r in (0, 1):
        assert out[r]["clocks"] == expect
        assert out[r]["n_recs"] == sum(len(c) for c in expect.values())
    # min-clock = Clock.intersection over the ranks holding each document
    held = [out[0]["rep"], out[1]["rep"]]
    for d in set(held[0]) | set(held[1]):
        cs = [h[d] for h in held if d in h]
        want = cs[0]
        for c in cs[1:]:
            want = C.intersection(want, c)
        for r in (0, 1):
            assert out[r]["min"][d] == want, (d, r)


def test_alignment_and_records_host():
    from hypermerge_amd import exchange as X
    keys = X.KeyTable()
    dk, ak, ck = X.dense_rows([("docA", {"b": 3, "a": 1}), ("docB", {"c": 2})], 4, keys)
    recs = X.records_host(dk, ak, ck)
    assert [(keys[int(r["doc_key"])], keys[int(r["actor_key"])], int(r["seq"])) for r in recs] == \
        [("docA", "a", 1), ("docA", "b", 3), ("docB", "c", 2)]
    # delta records against a stored row: only entries that grew
    base = ck.copy()
    base[0] = 1
    base[1] = 2
    base[4] = 0
    d = X.records_host(dk, ak, ck, base)
    assert [(keys[int(r["actor_key"])], int(r["seq"])) for r in d] == [("b", 3), ("c", 2)]
    other = X.records_host(*X.dense_rows([("docA", {"a": 5, "d": 1})], 4, keys))
    allr = np.concatenate([recs, other])
    pairs, mine = X.align(allr, recs)
    named = [(keys[int(p[0])], keys[int(p[1])]) for p in pairs]
    assert named == sorted(named, key=lambda x: (X.fnv1a64(x[0]), X.fnv1a64(x[1])))
    got = {n: int(v) for n, v in zip(named, mine)}
    assert got[("docA", "a")] == 1 and got[("docA", "b")] == 3 and got[("docA", "d")] == 0
    assert got[("docB", "c")] == 2
    pairs2, mine2 = X.align(allr, other)
    got2 = {(keys[int(p[0])], keys[int(p[1])]): int(v) for p, v in zip(pairs2, mine2)}
    assert got2[("docB", "c")] == X.NOT_HELD and got2[("docA", "b")] == 0 and got2[("docA", "a")] == 5
    # the MIN over the two contributions is Clock.intersection over the holders (docB: one)
    m = np.minimum(mine, mine2)
    inter = {(d, a): int(v) for (d, a), v in zip(named, m) if v not in (0, X.NOT_HELD)}
    assert inter == {("docA", "a"): 1, ("docB", "c"): 2}
    assert C.intersection({"a": 1, "b": 3}, {"a": 5, "d": 1}) == {"a": 1}
    assert X.fnv1a64("") == 0xCBF29CE484222325 and X.fnv1a64("a") == 0xAF63DC4C8601EC8C


def test_align_counts_held_documents_without_records():
    """a rank that holds a document but sends no record for it (an empty clock,
    or delta records) contributes 0, not NOT_HELD, when the held set is given explicitly."""
    from hypermerge_amd.exchange import align, NOT_HELD, CLOCK_REC_DT
    allr = np.zeros(2, CLOCK_REC_DT)
    allr["doc_key"] = [1, 1]
    allr["actor_key"] = [10, 11]
    allr["seq"] = [3, 4]
    own = np.zeros(0, CLOCK_REC_DT)
    _, mine = align(allr, own)
    assert (mine == NOT_HELD).all()
    _, mine = align(allr, own, held=np.array([1], np.uint64))
    assert (mine == 0).all()                 # Clock.intersection with {} drops both entries
    own2 = allr[:1].copy()
    _, mine = align(allr, own2, held=np.array([1, 7], np.uint64))
    assert list(mine) == [3, 0]


def test_key_collisions_fail_loudly():
    """The 64-bit keys stand for id strings; two ids on one key (forced here with a key
    function that collides) raise instead of merging two actors' clocks or cursors — in a
    rank's own table, when tables meet across ranks, and in the dense rows of an exchange."""
    import pytest
    from hypermerge_amd import exchange as X
    weak = lambda s: len(s)                                  # noqa: E731  every id of one length collides
    t = X.KeyTable(weak)
    assert t.key("actorA") == t.key("actorA")
    with pytest.raises(ValueError, match="collision"):
        t.key("actorB")
    other = X.KeyTable(weak)
    other.key("docXY")
    mine = X.KeyTable(weak)
    mine.key("docZW")
    with pytest.raises(ValueError, match="collision"):
        mine.update(other.ids)
    with pytest.raises(ValueError, match="collision"):
        X.dense_rows([("docA", {"ab": 1, "cd": 2})], 4, X.KeyTable(weak))
    # the real key function keeps distinct ids apart
    real = X.KeyTable()
    ids = [f"actor{i}" for i in range(2000)]
    assert len({real.key(a) for a in ids}) == len(ids)
