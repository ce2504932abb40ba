"""The general kernel's parallel queue-pass history (merge_large.hip parallel_history),
restated in Python and checked against the oracle's literal applyQueuedOps emulation on
generated arrival orders and the hand-built queue orders (cycles, missing deps, reversed
chains).  The rule: change K applies while arrival t(K) is processed, t(K) = the latest arrival
among K and its ancestors (never: a missing ancestor or a dependency cycle); in pass 1 if
t(K) is K's own arrival, else in pass max(2, pass(D) + [arr(D) > arr(K)]) over its deps D
applied by the same arrival; history = applied changes ordered by (t, pass, arrival).
(Documents with duplicate (actor, seq) copies take the serial emulation; not covered here.)"""
import numpy as np
import pytest

from hypermerge_amd import synth
from hypermerge_amd.columnar import encode
import oracle.oracle as O

from test_gpu_parity import QUEUE_ORDERS


def parallel_history(b, d):
    doc = b.docs[d]
    c0, n, A = int(doc["change_off"]), int(doc["n_changes"]), int(doc["n_actors"])
    ch = b.changes[c0:c0 + n]
    first = {}
    for i in range(n):
        k = (int(ch["actor"][i]), int(ch["seq"][i]))
        if k in first:
            return None                                   # duplicates: serial path
        first[k] = i
    C = np.zeros((n, A), np.int64)
    nev = np.zeros(n, bool)
    deps = []
    for i in range(n):
        a, s = int(ch["actor"][i]), int(ch["seq"][i])
        C[i, a] = s - 1
        nev[i] = s > 1 and (a, s - 1) not in first
        dl = []
        d0, nd = int(ch["dep_off"][i]), int(ch["n_deps"][i])
        for j in range(nd):
            da, ds = int(b.deps["actor"][d0 + j]), int(b.deps["seq"][d0 + j])
            if da == a or ds == 0:
                continue
            nev[i] |= (da, ds) not in first
            C[i, da] = max(C[i, da], ds)
            dl.append(first.get((da, ds)))
        if s > 1:
            dl.append(first.get((a, s - 1)))
        deps.append(dl)
    while True:                                           # closure by pointer jumping
        grew = False
        for i in range(n):
            for a in range(A):
                s = int(C[i, a])
                if not s:
                    continue
                j = first.get((a, s))
                if j is None:
                    grew |= not nev[i]
                    nev[i] = True
                    continue
                m = np.maximum(C[i], C[j])
                if (m != C[i]).any() or (nev[j] and not nev[i]):
                    grew = True
                    C[i] = m
                    nev[i] |= nev[j]
        if not grew:
            break
    bad = {(int(ch["actor"][i]), int(ch["seq"][i])) for i in range(n)
           if nev[i] or C[i, int(ch["actor"][i])] >= int(ch["seq"][i])}

    def pm(a, s):                                         # latest arrival among (a, 1..s); None: never
        v = 0
        for q in range(1, s + 1):
            if (a, q) not in first or (a, q) in bad:
                return None
            v = max(v, first[(a, q)])
        return v
    t = []
    for i in range(n):
        a, s = int(ch["actor"][i]), int(ch["seq"][i])
        tt = None if (a, s) in bad else i
        for x in range(A):
            if tt is not None and C[i, x]:
                v = pm(x, int(C[i, x]))
                tt = None if v is None else max(tt, v)
        t.append(tt)
    ps = [0 if t[i] is None else (1 if t[i] == i else 2) for i in range(n)]
    while True:
        grew = False
        for i in range(n):
            if t[i] is None or t[i] == i:
                continue
            p = max([ps[i]] + [ps[j] + (j > i) for j in deps[i] if j is not None and t[j] == t[i]])
            if p > ps[i]:
                ps[i], grew = p, True
        if not grew:
            break
    hist = [-1] * n
    for h, i in enumerate(sorted((i for i in range(n) if t[i] is not None), key=lambda i: (t[i], ps[i], i))):
        hist[i] = h
    return hist


def check(b):
    r = O.merge(b)
    seen = 0
    for d in range(b.n_docs):
        h = parallel_history(b, d)
        if h is None:
            continue
        c0, n = int(b.docs["change_off"][d]), int(b.docs["n_changes"][d])
        assert h == [int(x) for x in r.hist[c0:c0 + n]], d
        seen += 1
    return seen


@pytest.mark.parametrize("name,n,kw", [
    ("C2", 60, {"arrival": 2, "shuffle_pct": 60, "dup_pct": 0}),
    ("C4", 60, {"arrival": 1}),
    ("C5", 60, {"arrival": 2, "shuffle_pct": 30, "dup_pct": 0}),
    ("C1", 1, {"arrival": 1, "changes_per_actor": 150}),
    ("C3", 4, {"arrival": 2, "shuffle_pct": 50, "dup_pct": 0, "changes_per_actor": 12}),
])
def test_parallel_history_matches_queue_emulation(name, n, kw):
    b = synth.generate(synth.config(name, n_docs=n, **kw), threads=2)
    assert check(b) == b.n_docs


@pytest.mark.parametrize("name,changes", QUEUE_ORDERS, ids=[c[0] for c in QUEUE_ORDERS])
def test_parallel_history_hand_built_orders(name, changes):
    check(encode([changes]))
