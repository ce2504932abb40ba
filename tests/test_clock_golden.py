"""Clock algebra vs golden vectors captured from the reference's dist/Clock.js
(tools/golden/gen_clock_vectors.js; includes tests/unit.test.ts's cases)."""
import json
import math
import os

import numpy as np
import pytest

from hypermerge_amd import clock as C

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "clock_vectors.json")))


def dec(c):
    return {k: (math.inf if v == "Infinity" else v) for k, v in c.items()}


def enc(c):
    return {k: ("Infinity" if v == math.inf else v) for k, v in c.items()}


@pytest.mark.parametrize("case", GOLD["cases"])
def test_clock_ops_match_reference(case):
    a, b = dec(case["a"]), dec(case["b"])
    assert C.gte(a, b) == case["gte"]
    assert C.cmp(a, b) == case["cmp"]
    assert C.equal(a, b) == case["equal"]
    assert C.equivalent(a, b) == case["equivalent"]
    u = C.union(a, b)
    assert enc(u) == case["union"] and list(u) == case["union_keys"]
    assert enc(C.intersection(a, b)) == case["intersection"]


def test_strs2clock_clock2strs():
    for x in GOLD["strs2clock"]:
        assert enc(C.strs2clock(x["in"])) == x["out"]
    for x in GOLD["clock2strs"]:
        assert C.clock2strs(dec(x["in"])) == x["out"]


def test_unit_test_answers():
    # tests/unit.test.ts:4-36
    c1 = {"a": 100, "b": 100, "c": 100}
    c6 = {"a": 99, "b": 101, "c": 100, "d": 1}
    assert C.cmp(c1, c6) == "CONCUR" and C.cmp(c6, c1) == "CONCUR"
    assert C.union({"a": 100, "b": 200, "c": 300}, {"b": 10, "c": 2000, "d": 50}) == {"a": 100, "b": 200, "c": 2000, "d": 50}


def dense_cases():
    """Golden cases as dense rows (no Infinity) for the device clock kernels."""
    rows = [c for c in GOLD["cases"] if "Infinity" not in json.dumps(c)]
    actors = sorted({k for c in rows for k in list(c["a"]) + list(c["b"])})
    rank = {a: i for i, a in enumerate(actors)}
    S = len(actors)
    A = np.array([C.to_dense(c["a"], rank, S) for c in rows], np.uint32)
    B = np.array([C.to_dense(c["b"], rank, S) for c in rows], np.uint32)
    return rows, actors, S, A, B


@pytest.mark.gpu
def test_device_clock_kernels_match_reference(engine):
    import torch
    rows, actors, S, A, B = dense_cases()
    dev = torch.device("cuda", 0)
    ta, tb = torch.from_numpy(A.view(np.int32)).to(dev), torch.from_numpy(B.view(np.int32)).to(dev)
    out8 = torch.zeros(len(rows), dtype=torch.uint8, device=dev)
    outu = torch.zeros_like(ta)
    outi = torch.zeros_like(ta)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        engine.clock_op("cmp", ta.data_ptr(), tb.data_ptr(), out8.data_ptr(), len(rows), S, s.cuda_stream)
        engine.clock_op("union", ta.data_ptr(), tb.data_ptr(), outu.data_ptr(), len(rows), S, s.cuda_stream)
        engine.clock_op("intersection", ta.data_ptr(), tb.data_ptr(), outi.data_ptr(), len(rows), S, s.cuda_stream)
    s.synchronize()
    cmpv, un, it = out8.cpu().numpy(), outu.cpu().numpy().view(np.uint32), outi.cpu().numpy().view(np.uint32)
    for i, c in enumerate(rows):
        assert C.CMP_NAMES[int(cmpv[i])] == c["cmp"], (i, c)
        assert C.from_dense(un[i], actors) == {k: v for k, v in c["union"].items() if v}
        assert C.from_dense(it[i], actors) == c["intersection"]
