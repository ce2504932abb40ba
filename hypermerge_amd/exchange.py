"""Cross-GPU clock exchange of the sharded engine (C-ABI in
include/hypermerge_amd.h, "Clock exchange").

Documents shard by ``FNV-1a64(docId) % world``; each rank (one process per GPU) owns its
documents and the merge never communicates.  What crosses GPUs is the ClockStore feed: the
per-document clocks a ``CursorMessage`` carries (``clocks: [{docId, clock: {actorId: seq}}]``,
src/PeerMsg.ts:12-16), which the reference assembles from ``ClockStore.get`` per document
(src/RepoBackend.ts:374-392) and applies with ``ClockStore.update`` + ``updateMinimumClock``
(src/RepoBackend.ts:402,412-418).

Actor *ranks* are per-document and encoder-local, so on the wire every entry is a
repo-global record ``(FNV-1a64(docId), FNV-1a64(actorId), seq)`` (``hm_clock_rec``, 24 B);
each host keeps a :class:`KeyTable` (key -> id string) to turn records back into
``{actorId: seq}`` clocks.

* :meth:`ClockExchange.gather` — every rank's records on every rank, in rank order
  (``hm_clock_count_allgather`` + ``hm_clock_allgather``: exact-size grouped broadcasts).
* :meth:`ClockExchange.min_clock` — ``Clock.intersection`` (src/Clock.ts:103-113) across the
  replicas that hold a document: records are aligned on the gathered (doc, actor) key
  universe (identical on every rank), a rank that does not hold the document contributes
  ``HM_CLOCK_NOT_HELD`` (the MIN identity), one that holds it but lacks the actor 0; one MIN
  all-reduce (``hm_clock_min_allreduce``); 0 / NOT_HELD entries are dropped as intersection does.

Transports: :class:`RcclTransport` (the C-ABI over RCCL, device buffers) on the GPU box;
:class:`TorchTransport` (``torch.distributed``, gloo in the CPU tests) for the same protocol.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

FNV_OFFSET = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3
NOT_HELD = 0xFFFFFFFF
CLOCK_REC_DT = np.dtype([("doc_key", "<u8"), ("actor_key", "<u8"), ("seq", "<u4"), ("flags", "<u4")])
assert CLOCK_REC_DT.itemsize == 24


def fnv1a64(s: str) -> int:
    """FNV-1a 64 over the UTF-8 bytes of an id string (the shard and record key)."""
    h = FNV_OFFSET
    for b in s.encode("utf-8"):
        h = ((h ^ b) * FNV_PRIME) & 0xFFFFFFFFFFFFFFFF
    return h


def shard_of(doc_id: str, world: int) -> int:
    """The rank that owns a document: FNV-1a64(docId) % world."""
    return fnv1a64(doc_id) % world


class KeyTable:
    """key -> id string for the documents and actors a host has seen (a 64-bit key that two
    different ids share is an error, never a silent merge of two actors)."""

    def __init__(self, hash_fn=None) -> None:
        self.ids: Dict[int, str] = {}
        self.hash = hash_fn or fnv1a64

    def key(self, s: str) -> int:
        k = self.hash(s)
        old = self.ids.setdefault(k, s)
        if old != s:
            raise ValueError(f"FNV-1a64 key collision: {old!r} / {s!r}")
        return k

    def update(self, other: Dict[int, str]) -> None:
        for k, s in other.items():
            old = self.ids.setdefault(k, s)
            if old != s:
                raise ValueError(f"FNV-1a64 key collision: {old!r} / {s!r}")

    def __getitem__(self, k: int) -> str:
        return self.ids[k]


def dense_rows(clocks: Sequence[Tuple[str, Dict[str, int]]], a_stride: int, keys: KeyTable):
    """(docId, {actorId: seq}) per document -> the dense rows the engine keeps
    (doc_keys u64[n], actor_keys u64[n*S], clock u32[n*S]); ranks in actor-id string order."""
    n = len(clocks)
    dk = np.zeros(n, np.uint64)
    ak = np.zeros(n * a_stride, np.uint64)
    ck = np.zeros(n * a_stride, np.uint32)
    for i, (doc, clock) in enumerate(clocks):
        dk[i] = keys.key(doc)
        actors = sorted(clock, key=lambda a: a.encode("utf-16-be", "surrogatepass"))
        if len(actors) > a_stride:
            raise ValueError(f"{doc}: {len(actors)} actors > a_stride {a_stride}")
        for r, a in enumerate(actors):
            ak[i * a_stride + r] = keys.key(a)
            ck[i * a_stride + r] = clock[a]
    return dk, ak, ck


def records_host(doc_keys: np.ndarray, actor_keys: np.ndarray, clock: np.ndarray,
                 base: Optional[np.ndarray] = None) -> np.ndarray:
    """Host form of hm_clock_records_device: every entry with actor_key != 0 and clock > base."""
    S = len(actor_keys) // max(len(doc_keys), 1)
    live = (actor_keys != 0) & (clock > (base if base is not None else 0))
    idx = np.nonzero(live)[0]
    out = np.zeros(len(idx), CLOCK_REC_DT)
    out["doc_key"] = doc_keys[idx // S] if S else 0
    out["actor_key"] = actor_keys[idx]
    out["seq"] = clock[idx]
    return out


def clocks_of(recs: np.ndarray, keys: KeyTable) -> Dict[str, Dict[str, int]]:
    """Records -> {docId: {actorId: seq}} (several records of one entry: the max, as
    ClockStore.update's upsert-max keeps, src/ClockStore.ts:37-48,78-91)."""
    out: Dict[str, Dict[str, int]] = {}
    for r in recs:
        c = out.setdefault(keys[int(r["doc_key"])], {})
        a = keys[int(r["actor_key"])]
        c[a] = max(c.get(a, 0), int(r["seq"]))
    return out


class TorchTransport:
    """The exchange protocol over torch.distributed (gloo on CPU, or nccl)."""

    def __init__(self, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.dist, self.torch, self.group = dist, torch, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device or torch.device("cpu")

    def gather(self, recs: np.ndarray) -> Tuple[np.ndarray, List[int]]:
        torch, dist = self.torch, self.dist
        cnt = torch.tensor([len(recs)], dtype=torch.int64, device=self.device)
        cnts = [torch.zeros_like(cnt) for _ in range(self.world)]
        dist.all_gather(cnts, cnt, group=self.group)
        counts = [int(c.item()) for c in cnts]
        kmax = max(counts) if counts else 0
        pad = np.zeros(kmax, CLOCK_REC_DT)
        pad[:len(recs)] = recs
        t = torch.from_numpy(pad.view(np.int64).reshape(-1, 3).copy()).to(self.device)
        parts = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        allr = [p.cpu().numpy().reshape(-1).view(CLOCK_REC_DT)[:k] for p, k in zip(parts, counts)]
        return (np.concatenate(allr) if allr else np.zeros(0, CLOCK_REC_DT)), counts

    def min_allreduce(self, seq: np.ndarray) -> np.ndarray:
        torch, dist = self.torch, self.dist
        t = torch.from_numpy(seq.astype(np.int64)).to(self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return t.cpu().numpy().astype(np.uint32)

    def exchange_keys(self, table: KeyTable) -> None:
        objs: List[Optional[Dict[int, str]]] = [None] * self.world
        self.dist.all_gather_object(objs, dict(table.ids), group=self.group)
        for o in objs:
            table.update(o or {})


class RcclTransport:
    """The exchange protocol through the C-ABI (hm_comm_*, hm_clock_*: RCCL over xGMI) on
    device buffers.  ``unique_id`` = HM_COMM_ID_BYTES from hm_comm_unique_id on rank 0."""

    def __init__(self, engine, world: int, rank: int, unique_id: bytes):
        import torch
        self.torch = torch
        self.eng = engine
        self.L = engine._L
        self.world, self.rank = world, rank
        self.device = torch.device("cuda", torch.cuda.current_device())
        self._h = ctypes.c_void_p()
        idb = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        engine._check(self.L.hm_comm_create(engine._h, world, rank, idb, ctypes.byref(self._h)), "hm_comm_create")
        self.d_counts = torch.zeros(world, dtype=torch.int64, device=self.device)
        self._stream = torch.cuda.Stream(device=self.device)

    def _enter(self, stream):
        """The stream a call runs on.  A NULL stream means the engine's own (non-blocking)
        stream in the C-ABI, so torch's default stream (handle 0) is never passed: without an
        explicit stream the call runs on this transport's stream, ordered after the caller's
        current stream and (``_leave``) before it."""
        if stream is not None:
            return stream
        self._stream.wait_stream(self.torch.cuda.current_stream())
        return self._stream.cuda_stream

    def _leave(self, stream):
        if stream is None:
            self.torch.cuda.current_stream().wait_stream(self._stream)

    @staticmethod
    def unique_id(engine) -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        engine._check(engine._L.hm_comm_unique_id(buf), "hm_comm_unique_id")
        return bytes(buf)

    def close(self) -> None:
        if self._h:
            self.L.hm_comm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def records_device(self, doc_keys, actor_keys, clock, base=None, stream=None):
        """Device rows (torch tensors: int64 [n], int64 [n*S], int32 [n*S]) -> device records
        (uint8 tensor of 24 B records) via hm_clock_records_device."""
        torch = self.torch
        n = doc_keys.numel()
        S = actor_keys.numel() // max(n, 1)
        out = torch.empty(max(n * S, 1) * 24, dtype=torch.uint8, device=self.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
        scr = torch.empty(int(self.L.hm_clock_records_scratch_bytes(n, max(S, 1))) + 16, dtype=torch.uint8,
                          device=self.device)
        st = self._enter(stream)
        self.eng._check(self.L.hm_clock_records_device(
            self.eng._h, doc_keys.data_ptr(), actor_keys.data_ptr(), clock.data_ptr(),
            base.data_ptr() if base is not None else None, n, max(S, 1), out.data_ptr(), cnt.data_ptr(),
            scr.data_ptr(), st), "hm_clock_records_device")
        self._leave(stream)
        if stream is not None:
            torch.cuda.ExternalStream(stream).synchronize()
        k = int(cnt.item())
        return out[: k * 24]

    def gather_device(self, d_recs, stream=None):
        """Every rank's device records, back to back in rank order (device uint8 tensor)."""
        torch = self.torch
        st = self._enter(stream)
        n_local = d_recs.numel() // 24
        self.eng._check(self.L.hm_clock_count_allgather(self._h, n_local, self.d_counts.data_ptr(), st),
                        "hm_clock_count_allgather")           # returns after the counts arrived
        counts = self.d_counts.cpu().numpy().astype(np.uint64)
        total = int(counts.sum())
        out = torch.empty(max(total, 1) * 24, dtype=torch.uint8, device=self.device)
        cbuf = (ctypes.c_uint64 * self.world)(*[int(c) for c in counts])
        self.eng._check(self.L.hm_clock_allgather(self._h, d_recs.data_ptr() if n_local else None, cbuf,
                                                  out.data_ptr(), st), "hm_clock_allgather")
        self._leave(stream)
        return out[: total * 24], [int(c) for c in counts]

    def gather(self, recs: np.ndarray) -> Tuple[np.ndarray, List[int]]:
        torch = self.torch
        d = torch.from_numpy(recs.view(np.uint8).copy()).to(self.device) if len(recs) else \
            torch.empty(0, dtype=torch.uint8, device=self.device)
        out, counts = self.gather_device(d)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(CLOCK_REC_DT).copy(), counts

    def min_allreduce_device(self, d_seq, stream=None) -> None:
        st = self._enter(stream)
        self.eng._check(self.L.hm_clock_min_allreduce(self._h, d_seq.data_ptr(), d_seq.numel(), st),
                        "hm_clock_min_allreduce")
        self._leave(stream)

    def min_allreduce(self, seq: np.ndarray) -> np.ndarray:
        torch = self.torch
        d = torch.from_numpy(seq.astype(np.uint32).view(np.int32).copy()).to(self.device)
        self.min_allreduce_device(d)
        torch.cuda.synchronize()
        return d.cpu().numpy().view(np.uint32).copy()


def align(all_recs: np.ndarray, own: np.ndarray, held: Optional[np.ndarray] = None):
    """The (doc, actor) key universe of the gathered records, sorted (identical on every
    rank), and this rank's contribution to the min-clock over it: its seq for an entry it
    has, 0 for an actor it lacks on a document it holds, NOT_HELD for a document it does
    not hold.  `held` = the doc keys this rank holds; None = the documents `own` has records
    for (right only when `own` carries every held document's full clock row: delta records
    or an empty clock would make a held document look not held)."""
    pairs = np.unique(np.stack([all_recs["doc_key"], all_recs["actor_key"]], axis=1), axis=0) \
        if len(all_recs) else np.zeros((0, 2), np.uint64)
    mine = np.full(len(pairs), NOT_HELD, np.uint32)
    held_keys = own["doc_key"] if held is None else np.asarray(held, np.uint64)
    if len(pairs) and len(held_keys):
        mine[np.isin(pairs[:, 0], held_keys)] = 0
    if len(pairs) and len(own):
        # own entries' positions in the (lexicographically sorted) universe
        keyed = pairs[:, 0].astype(object) * (1 << 64) + pairs[:, 1].astype(object)
        own_k = own["doc_key"].astype(object) * (1 << 64) + own["actor_key"].astype(object)
        for p, s in zip(np.searchsorted(keyed, own_k), own["seq"]):
            mine[p] = max(int(mine[p]), int(s))
    return pairs, mine


class ClockExchange:
    """One rank's side of the node-wide clock exchange (any transport)."""

    def __init__(self, transport, keys: Optional[KeyTable] = None):
        self.t = transport
        self.keys = keys if keys is not None else KeyTable()

    def gather(self, own: np.ndarray) -> np.ndarray:
        """Every rank's records on this rank (rank order)."""
        recs, _ = self.t.gather(own)
        return recs

    def clocks(self, all_recs: np.ndarray) -> Dict[str, Dict[str, int]]:
        return clocks_of(all_recs, self.keys)

    def min_clock(self, all_recs: np.ndarray, own: np.ndarray, held: Optional[np.ndarray] = None) -> Dict[str, Dict[str, int]]:
        """Clock.intersection across the ranks holding each document (`held`: see align)."""
        pairs, mine = align(all_recs, own, held)
        m = self.t.min_allreduce(mine)
        out: Dict[str, Dict[str, int]] = {}
        for (dk, ak), v in zip(pairs, m):
            doc = self.keys[int(dk)]
            c = out.setdefault(doc, {})
            if v != 0 and v != NOT_HELD:
                c[self.keys[int(ak)]] = int(v)
        return out
