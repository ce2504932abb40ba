"""The clock-exchange C-ABI on the device (include/hypermerge_amd.h "Clock exchange"):
hm_clock_records_device against its host form, and the RCCL collectives through a
single-rank communicator (one GPU per box: RCCL refuses two ranks on one device; the
2-rank protocol is tests/test_exchange.py over gloo)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    from hypermerge_amd.engine import Engine
    torch.cuda.set_device(0)
    return Engine(0)


def _rows(n, S, seed):
    rng = np.random.default_rng(seed)
    dk = rng.integers(1, 2 ** 63, size=n, dtype=np.int64).astype(np.uint64)
    ak = rng.integers(1, 2 ** 63, size=n * S, dtype=np.int64).astype(np.uint64)
    nact = rng.integers(0, S + 1, size=n)
    for d in range(n):
        ak[d * S + nact[d]: (d + 1) * S] = 0                 # rank slots past n_actors: no actor
    ck = rng.integers(0, 50, size=n * S).astype(np.uint32)
    ck[ak == 0] = 0
    return dk, ak, ck


@pytest.mark.parametrize("n,S", [(1, 1), (37, 8), (5000, 8), (70000, 4)])
def test_records_device_matches_host(eng, n, S):
    import torch
    from hypermerge_amd import exchange as X
    tr = X.RcclTransport(eng, 1, 0, X.RcclTransport.unique_id(eng))
    try:
        dk, ak, ck = _rows(n, S, n)
        base = (ck // 2).astype(np.uint32)
        dev = torch.device("cuda", 0)
        t = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32)).to(dev)
        for b in (None, base):
            got = tr.records_device(t(dk), t(ak), t(ck), None if b is None else t(b))
            torch.cuda.synchronize()
            g = got.cpu().numpy().view(X.CLOCK_REC_DT)
            want = X.records_host(dk, ak, ck, b)
            assert np.array_equal(g, want)
    finally:
        tr.close()


def test_single_rank_collectives(eng):
    import torch
    from hypermerge_amd import exchange as X
    tr = X.RcclTransport(eng, 1, 0, X.RcclTransport.unique_id(eng))
    try:
        dk, ak, ck = _rows(3000, 8, 11)
        recs = X.records_host(dk, ak, ck)
        allr, counts = tr.gather(recs)
        assert counts == [len(recs)] and np.array_equal(allr, recs)
        empty, c0 = tr.gather(np.zeros(0, X.CLOCK_REC_DT))
        assert c0 == [0] and len(empty) == 0
        seq = np.array([5, 0, X.NOT_HELD, 7], np.uint32)
        assert np.array_equal(tr.min_allreduce(seq), seq)          # one rank: the identity
        # the exchange object end to end at world 1: clocks of every document, min-clock = own
        keys = X.KeyTable()
        docs = [("docA", {"actor1": 3, "actor2": 1}), ("docB", {"actor3": 9})]
        rows = X.dense_rows(docs, 4, keys)
        own = X.records_host(*rows)
        ex = X.ClockExchange(tr, keys)
        g = ex.gather(own)
        assert ex.clocks(g) == dict(docs)
        assert ex.min_clock(g, own) == dict(docs)
    finally:
        tr.close()


def test_local_communicator_host_helpers(eng):
    """hm_comm_create_local + hm_clock_exchange_host / hm_clock_min_host (one process driving
    the node's GPUs, as the Node host's GpuEngine does) at one device."""
    from hypermerge_amd import exchange as X
    L = eng._L
    engines = (ctypes.c_void_p * 1)(eng._h.value)
    comms = (ctypes.c_void_p * 1)()
    eng._check(L.hm_comm_create_local(engines, 1, comms), "hm_comm_create_local")
    try:
        recs = X.records_host(*_rows(200, 8, 3))
        ptrs = (ctypes.c_void_p * 1)(recs.ctypes.data)
        ns = (ctypes.c_uint64 * 1)(len(recs))
        out = np.zeros(len(recs) + 4, X.CLOCK_REC_DT)
        tot = ctypes.c_uint64()
        eng._check(L.hm_clock_exchange_host(comms, 1, ptrs, ns, out.ctypes.data, len(out), ctypes.byref(tot)),
                   "hm_clock_exchange_host")
        assert tot.value == len(recs) and np.array_equal(out[:len(recs)], recs)
        seq = np.array([3, X.NOT_HELD, 0], np.uint32)
        sp = (ctypes.c_void_p * 1)(seq.ctypes.data)
        eng._check(L.hm_clock_min_host(comms, 1, sp, len(seq)), "hm_clock_min_host")
        assert seq.tolist() == [3, X.NOT_HELD, 0]
    finally:
        L.hm_comm_destroy(comms[0])
