"""The CPU restatement (oracle/) against the hand-derived known answers of
tests/kat_cases.py.  Parity for these Automerge 0.12
rules is UNPINNED by reference output (Automerge is not vendored; §8c)."""
import pytest

from hypermerge_amd.columnar import encode
from hypermerge_amd.render import doc_summary
import oracle.oracle as O

from kat_cases import CASES, ENVELOPE_CASES


@pytest.mark.parametrize("name,changes,expect", CASES, ids=[c[0] for c in CASES])
def test_oracle_known_answers(name, changes, expect):
    b = encode([changes])
    r = O.merge(b)
    got = doc_summary(b, r, 0)
    for k, v in expect.items():
        assert got.get(k) == v, (name, k, got)
    if "status" not in expect:
        assert got["status"] == "OK", got


def test_transitive_deps_literal_fold():
    """transitiveDeps reduces the deps map in key order and `.set(actor, seq)`
    overrides the running max: a listed dep that another listed dep already
    dominates LOWERS allDeps.  The oracle keeps that literal behaviour."""
    A, B, C = "aaaa", "bbbb", "cccc"
    from hypermerge_amd.columnar import ROOT_ID as R
    changes = [
        {"actor": A, "seq": 1, "deps": {}, "ops": []},
        {"actor": A, "seq": 2, "deps": {}, "ops": [{"action": "set", "obj": R, "key": "k", "value": "a2"}]},
        {"actor": B, "seq": 1, "deps": {A: 2}, "ops": []},
        {"actor": C, "seq": 1, "deps": {B: 1, A: 1}, "ops": [{"action": "set", "obj": R, "key": "k", "value": "c1"}]},
    ]
    b = encode([changes])
    r = O.merge(b)
    S = b.a_stride
    ad_c1 = list(r.all_deps[3 * S: 3 * S + 3])
    assert ad_c1 == [1, 1, 0]            # {a:1, b:1}: the dominated dep a:1 overrode a:2
    # so A2's set and C1's set are "concurrent" -> both survive (c1 wins by actor)
    got = doc_summary(b, r, 0)
    assert got["state"] == {"map": [["k", {"value": "c1", "conflicts": [[A, "a2"]]}]]}


def test_oracle_insert_after_never_inserted_element():
    """An ins after a never-inserted element is accepted (Automerge 0.12 applyInsert does not
    look the parent up); the element stays hidden, and a set on it throws from getPrevious."""
    changes = [{"actor": "a", "seq": 1, "deps": {}, "ops": [
        {"action": "makeList", "obj": "L"}, {"action": "ins", "obj": "L", "key": "a:7", "elem": 8}]}]
    b = encode([changes])
    assert doc_summary(b, O.merge(b), 0)["status"] == "OK"
    changes.append({"actor": "a", "seq": 2, "deps": {}, "ops": [
        {"action": "set", "obj": "L", "key": "a:8", "value": 1}]})
    b = encode([changes])
    got = doc_summary(b, O.merge(b), 0)
    assert got["status"] == "MISSING_ELEM" and got["error_at"] == [1, 0]


@pytest.mark.parametrize("name,changes,mutate,expect", ENVELOPE_CASES, ids=[c[0] for c in ENVELOPE_CASES])
def test_oracle_envelope_precedence(name, changes, mutate, expect):
    b = encode([changes])
    if mutate:
        mutate(b)
    got = doc_summary(b, O.merge(b), 0)
    for k, v in expect.items():
        assert got.get(k) == v, (name, k, got)


@pytest.mark.parametrize("S", [128, 256])
def test_oracle_wide_rows(S):
    """More than 64 actors (one per writer, src/RepoBackend.ts:286-293): concurrent sets keep
    every writer's value, the highest actor string wins (A.2), clocks span the wide row."""
    from hypermerge_amd.columnar import ROOT_ID as R
    n = S - 1 if S == 256 else 100
    changes = [{"actor": f"w{i:03d}", "seq": 1, "deps": {}, "ops": [{"action": "set", "obj": R, "key": "x", "value": i}]}
               for i in range(n)]
    changes.append({"actor": "w000", "seq": 2, "deps": {f"w{i:03d}": 1 for i in range(n)},
                    "ops": [{"action": "set", "obj": R, "key": "y", "value": "last"}]})
    b = encode([changes], a_stride=S)
    got = doc_summary(b, O.merge(b), 0)
    assert got["status"] == "OK" and len(got["clock"]) == n and got["deps"] == {"w000": 2}
    x = dict(got["state"]["map"])["x"]
    assert x["value"] == n - 1 and len(x["conflicts"]) == n - 1
