"""Seeded synthetic change feeds for the BASELINE.json configs.

The generator is native (csrc/synth.cpp -> _lib/libhmsynth.so); this module
only picks the config and copies its tables into numpy arrays.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, asdict, replace
from typing import Optional

import numpy as np

from .columnar import Batch, DOC_DT, CHANGE_DT, DEP_DT, OP_DT

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_lib", "libhmsynth.so")


class _Cfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("doc_base", ctypes.c_uint64), ("n_docs", ctypes.c_uint32),
                ("shard", ctypes.c_uint32), ("n_shards", ctypes.c_uint32), ("kind", ctypes.c_uint32),
                ("actors", ctypes.c_uint32), ("changes_per_actor", ctypes.c_uint32),
                ("ops_min", ctypes.c_uint32), ("ops_max", ctypes.c_uint32), ("n_keys", ctypes.c_uint32),
                ("counter_pct", ctypes.c_uint32), ("del_pct", ctypes.c_uint32), ("arrival", ctypes.c_uint32),
                ("shuffle_pct", ctypes.c_uint32), ("dup_pct", ctypes.c_uint32), ("alternate", ctypes.c_uint32),
                ("threads", ctypes.c_uint32)]


@dataclass(frozen=True)
class SynthConfig:
    seed: int
    n_docs: int
    kind: int = 0               # 0 flat map, 1 text, 2 nested maps/lists
    actors: int = 4
    changes_per_actor: int = 16  # kind 1: typing ops per doc
    ops_min: int = 1
    ops_max: int = 4
    n_keys: int = 16
    counter_pct: int = 0
    del_pct: int = 0
    arrival: int = 0            # 0 generation order, 1 actor-major (RepoBackend.loadDocument), 2 shuffled
    shuffle_pct: int = 0
    dup_pct: int = 0
    alternate: int = 0
    doc_base: int = 0
    shard: int = 0
    n_shards: int = 1


# SURVEY.md §8(d) "Synthetic inputs"
CONFIGS = {
    # C1: 1 doc, 2 actors alternating, 10k changes, 1 set on key k{i mod 64} (int32)
    "C1": SynthConfig(seed=0xC1, n_docs=1, actors=2, changes_per_actor=5000, n_keys=64, alternate=1),
    # C2: 100k docs x 4 actors x 16 changes, 1-4 ops on 16 keys, 25% counter keys
    "C2": SynthConfig(seed=0xC2, n_docs=100_000, actors=4, changes_per_actor=16, ops_min=1, ops_max=4,
                      n_keys=16, counter_pct=25),
    # C3: 10k text docs x 8 actors, ~2k typing ops/doc, 80% insert / 20% delete
    "C3": SynthConfig(seed=0xC3, n_docs=10_000, kind=1, actors=8, changes_per_actor=2000),
    # C4: 1M docs x 8 actors x 8 changes, 1-2 map sets per change (per GPU shard)
    "C4": SynthConfig(seed=0xC4, n_docs=1_000_000, actors=8, changes_per_actor=8, ops_min=1, ops_max=2,
                      n_keys=16),
    # C5: nested maps/lists, hot keys, 10% deletes, ~20% changes delivered before their deps
    "C5": SynthConfig(seed=0xC5, n_docs=20_000, kind=2, actors=4, changes_per_actor=8, ops_min=1, ops_max=4,
                      n_keys=4, del_pct=10, arrival=2, shuffle_pct=20, dup_pct=3),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
        _lib = ctypes.CDLL(LIB)
        _lib.hm_synth_generate.argtypes = [ctypes.POINTER(_Cfg)]
        _lib.hm_synth_generate.restype = ctypes.c_void_p
        _lib.hm_synth_sizes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        _lib.hm_synth_copy.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 4
        _lib.hm_synth_free.argtypes = [ctypes.c_void_p]
        _lib.hm_synth_fnv1a64_docid.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        _lib.hm_synth_fnv1a64_docid.restype = ctypes.c_uint64
        _lib.hm_synth_blocks.argtypes = [ctypes.c_uint64] + [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 6
        _lib.hm_synth_blocks.restype = ctypes.c_uint64
        _lib.hm_synth_keys.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_void_p]
    return _lib


def generate(cfg: SynthConfig, threads: Optional[int] = None) -> Batch:
    L = lib()
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    c = _Cfg(**{k: v for k, v in asdict(cfg).items()}, threads=threads)
    h = L.hm_synth_generate(ctypes.byref(c))
    try:
        sz = (ctypes.c_uint64 * 6)()
        L.hm_synth_sizes(h, sz)
        nd, nc, ndp, no, nr, S = (int(x) for x in sz)
        docs = np.empty(nd, DOC_DT)
        ch = np.empty(nc, CHANGE_DT)
        dp = np.empty(ndp, DEP_DT)
        op = np.empty(no, OP_DT)
        L.hm_synth_copy(h, docs.ctypes.data, ch.ctypes.data, dp.ctypes.data, op.ctypes.data)
    finally:
        L.hm_synth_free(h)
    return Batch(docs, ch, dp, op, S)


def keys(cfg: SynthConfig, b: Batch):
    """(doc_keys u64[n], actor_keys u64[n*S]): FNV-1a64 of each document's base58 id and of
    its actors' synthetic ids — the repo-global keys of the clock exchange."""
    n, S = b.n_docs, b.a_stride
    dk = np.zeros(n, np.uint64)
    ak = np.zeros(n * S, np.uint64)
    lib().hm_synth_keys(cfg.seed, b.docs.ctypes.data, n, S, dk.ctypes.data, ak.ctypes.data)
    return dk, ak


def blocks(cfg: SynthConfig, b: Batch):
    """The batch's changes as raw-JSON hypercore blocks (one per change, arrival order):
    (data u8, block_off u64[n_changes+1], doc_block u32[n_docs+1]) for hm_decode_blocks.
    Map documents only (flat or nested maps; list ops are not rendered)."""
    L = lib()
    args = (cfg.seed, b.docs.ctypes.data, b.n_docs, b.changes.ctypes.data, b.deps.ctypes.data, b.ops.ctypes.data)
    total = L.hm_synth_blocks(*args, None, None, None)
    data = np.zeros(max(total, 1), np.uint8)
    block_off = np.zeros(len(b.changes) + 1, np.uint64)
    doc_block = np.zeros(b.n_docs + 1, np.uint32)
    L.hm_synth_blocks(*args, data.ctypes.data, block_off.ctypes.data, doc_block.ctypes.data)
    return data, block_off, doc_block


def config(name: str, **overrides) -> SynthConfig:
    return replace(CONFIGS[name], **overrides)
