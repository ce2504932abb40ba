"""The general kernel's all-LDS document path (merge_doc_res / l34_res in csrc/merge_large.hip)
and the documents it hands to the general path: each case is built to sit on one side of an
envelope edge of the LDS path, and both engines (small kernel first / general kernel only) must
equal the C oracle bit for bit."""
import numpy as np
import pytest

from hypermerge_amd import synth
from hypermerge_amd.columnar import encode
from oracle import oracle as O
from test_gpu_parity import assert_same
from kat_cases import ch, s, ins, mk, link, A, B, Cc

pytestmark = pytest.mark.gpu


def _long_assign_list(n_changes, actors=(A, B, Cc)):
    """Every change sets the same key: one register with n_changes assigns (the LDS path takes
    assign lists up to 64 per register, longer ones go to the general path)."""
    seqs = {a: 0 for a in actors}
    clock = {}
    changes = []
    for i in range(n_changes):
        a = actors[i % len(actors)]
        seqs[a] += 1
        deps = {k: v for k, v in clock.items() if k != a}
        changes.append(ch(a, seqs[a], deps, s("k", i)))
        if i % 4 != 3:                      # every fourth change stays concurrent with the next
            clock[a] = seqs[a]
    return changes


def _insert_only_text(n_changes, per_change, actor=A):
    """A text whose elements are inserted and never assigned: almost every op is an insert, so
    the Euler tour is as large as the op table (the LDS path checks the tour fits the region its
    per-change tables leave behind)."""
    changes = [ch(actor, 1, {}, mk("makeText", "T"), link("t", "T"))]
    elem, prev = 0, "_head"
    for c in range(n_changes):
        ops = []
        for _ in range(per_change):
            elem += 1
            ops.append(ins("T", prev, elem))
            prev = f"{actor}:{elem}"
        changes.append(ch(actor, c + 2, {}, *ops))
    return changes


@pytest.mark.parametrize("n", [40, 64, 65, 200])
def test_assign_list_length_edges(engine, engine_general, n):
    b = encode([_long_assign_list(n), _long_assign_list(n // 2 + 1)])
    o = O.merge(b)
    assert_same(b, engine.merge(b), o)
    assert_same(b, engine_general.merge(b), o)


@pytest.mark.parametrize("n,per", [(40, 30), (100, 40), (20, 200)])
def test_insert_only_text(engine, engine_general, n, per):
    b = encode([_insert_only_text(n, per)])
    o = O.merge(b)
    assert_same(b, engine.merge(b), o)
    assert_same(b, engine_general.merge(b), o)


@pytest.mark.parametrize("name,n,extra", [
    ("C3", 50, {"actors": 8}),                      # the LDS path's main case
    ("C3", 20, {"actors": 8, "changes_per_actor": 4000}),   # ~7k ops: the layout no longer fits -> general path
    ("C3", 30, {"actors": 3}),
    ("C5", 600, {}),                                # nested objects, deletes, blocked + duplicate changes
    ("C2", 600, {}),                                # counters -> general path
])
def test_text_and_mixed_docs_general_engine(engine_general, name, n, extra):
    b = synth.generate(synth.config(name, n_docs=n, **extra))
    assert_same(b, engine_general.merge(b), O.merge(b, threads=8))


def test_resident_path_repeatable(engine_general):
    """Workgroups reuse the LDS arena and the pool across documents: merging the same batch
    twice gives the same results (nothing depends on what an earlier document left behind)."""
    b = synth.generate(synth.config("C3", n_docs=64))
    g1 = engine_general.merge(b)
    g2 = engine_general.merge(b)
    for f in ("docs", "regs", "surv", "hist", "all_deps", "clock", "heads"):
        np.testing.assert_array_equal(getattr(g1, f), getattr(g2, f))


def _single_actor_chain(n_changes, keys=128):
    """One actor, no listed deps (each change's own predecessor only): more changes than the
    workgroup has threads while the rows still fit the LDS path (the multi-chunk history and
    key-base scans); <= 64 assigns per key, so the LDS path keeps the document."""
    return [ch(A, i + 1, {}, s(f"k{i % keys}", i)) for i in range(n_changes)]


@pytest.mark.parametrize("n", [1000, 1024, 1025, 1150])
def test_more_changes_than_threads(engine, engine_general, n):
    b = encode([_single_actor_chain(n), _single_actor_chain(n // 3)])
    o = O.merge(b)
    assert_same(b, engine.merge(b), o)
    assert_same(b, engine_general.merge(b), o)
