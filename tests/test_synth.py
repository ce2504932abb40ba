"""Synthetic feeds: deterministic, causally consistent, shard-stable."""
import numpy as np

from hypermerge_amd import synth
import oracle.oracle as O


def test_deterministic():
    a = synth.generate(synth.config("C2", n_docs=50))
    b = synth.generate(synth.config("C2", n_docs=50), threads=1)
    for f in ("docs", "changes", "deps", "ops"):
        assert np.array_equal(getattr(a, f), getattr(b, f))


def test_shards_partition_the_doc_stream():
    from hypermerge_amd.synth import lib
    L = lib()
    ws = 4
    owners = [L.hm_synth_fnv1a64_docid(0xC4, g) % ws for g in range(2000)]
    parts = [synth.generate(synth.config("C4", n_docs=owners.count(r), shard=r, n_shards=ws, doc_base=0))
             for r in range(ws)]
    assert sum(p.n_docs for p in parts) == 2000
    # a document is identical whichever shard generates it
    g0 = owners.index(1)
    one = synth.generate(synth.config("C4", n_docs=1, doc_base=g0))
    d1 = parts[1]
    n = int(d1.docs["n_changes"][0])
    a = d1.changes[:n].copy(); b = one.changes[:n].copy()
    a["dep_off"] -= a["dep_off"][0]; b["dep_off"] -= b["dep_off"][0]
    a["op_first"] -= a["op_first"][0]; b["op_first"] -= b["op_first"][0]
    assert np.array_equal(a, b)


def test_configs_are_causally_complete():
    # every change of the in-order configs is applied (nothing left queued), no errors
    for name, n in (("C1", 1), ("C2", 200), ("C4", 200), ("C3", 3), ("C5", 200)):
        b = synth.generate(synth.config(name, n_docs=n))
        r = O.merge(b)
        assert (r.docs["status"] == 0).all(), name
        assert int(r.docs["n_queued"].sum()) == 0, name


def test_c4_shape():
    b = synth.generate(synth.config("C4", n_docs=100))
    assert (b.docs["n_changes"] == 64).all() and (b.docs["n_actors"] == 8).all()
    per = b.changes["n_ops"]
    assert per.min() >= 1 and per.max() <= 2
