"""Sharding and the cross-rank clock exchange (hypermerge_amd/exchange.py) with
world_size 2 over gloo on CPU (the GPU box runs the same code over RCCL).

* shards: FNV-1a64(docId) % world partitions the global doc-id stream (disjoint,
  complete), and each shard merges independently (no data-path collective);
* gather_clock_rows: every rank ends with the union of all ranks' changed clock rows;
* min_clock / union_clock: element-wise MIN / MAX all-reduce == Clock.intersection /
  Clock.union (src/Clock.ts:87-113) of the ranks' clocks.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hypermerge_amd import synth
from hypermerge_amd import clock as C

N_DOCS = 400


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _keys(b):
    return b.docs["reserved"][:, 0].astype(np.int64) | (b.docs["reserved"][:, 1].astype(np.int64) << 32)


def _worker(rank, ws, port, out):
    import oracle.oracle as O
    from hypermerge_amd import exchange as X
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        b = synth.generate(synth.config("C4", n_docs=N_DOCS, shard=rank, n_shards=ws), threads=2)
        r = O.merge(b)
        S = b.a_stride
        keys = torch.from_numpy(_keys(b))
        newc = torch.from_numpy(r.back_clock.view(np.int32).reshape(-1, S).copy())
        rows = X.changed_rows(keys, newc, torch.zeros_like(newc))
        allrows = X.gather_clock_rows(rows)
        # replicas: every rank holds the same 50 documents at a different progress
        rep = synth.generate(synth.config("C4", n_docs=50), threads=2)
        k = 10 + 20 * rank
        sub = rep.changes.copy()
        prog = np.zeros((50, S), np.int64)
        for d in range(50):
            c0 = int(rep.docs["change_off"][d])
            for c in sub[c0: c0 + min(k, int(rep.docs["n_changes"][d]))]:
                prog[d, c["actor"]] = max(prog[d, c["actor"]], int(c["seq"]))
        mn = X.min_clock(torch.from_numpy(prog.copy()))
        mx = X.union_clock(torch.from_numpy(prog.copy()))
        out[rank] = {"keys": _keys(b).tolist(), "rows": allrows.numpy().tolist(), "prog": prog.tolist(),
                     "min": mn.numpy().tolist(), "max": mx.numpy().tolist(), "n_changes": int(r.docs["hist_len"].sum())}
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_and_clock_exchange():
    ws = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(ws, port, out), nprocs=ws, join=True)
        out = dict(out)
    k0, k1 = set(out[0]["keys"]), set(out[1]["keys"])
    assert len(k0) == N_DOCS and len(k1) == N_DOCS and not (k0 & k1)
    for r in (0, 1):                                   # every key hashes to its shard
        for g in list(out[r]["keys"])[:50]:
            assert synth.lib().hm_synth_fnv1a64_docid(synth.CONFIGS["C4"].seed, g) % ws == r
    # gathered rows: identical on both ranks, = union of per-rank rows, one per (doc, actor) entry
    assert out[0]["rows"] == out[1]["rows"]
    keys_in_rows = {row[0] for row in out[0]["rows"]}
    assert keys_in_rows == k0 | k1
    # min/max all-reduce == Clock.intersection / Clock.union of the two ranks' rows
    p0, p1 = np.array(out[0]["prog"]), np.array(out[1]["prog"])
    for d in range(len(p0)):
        a = {str(i): int(v) for i, v in enumerate(p0[d]) if v}
        b = {str(i): int(v) for i, v in enumerate(p1[d]) if v}
        inter, uni = C.intersection(a, b), C.union(a, b)
        assert out[0]["min"][d] == [inter.get(str(i), 0) for i in range(len(p0[d]))]
        assert out[1]["max"][d] == [uni.get(str(i), 0) for i in range(len(p0[d]))]
