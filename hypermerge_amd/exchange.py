"""Cross-GPU clock exchange of the sharded engine.

Documents are independent, so the merge itself never communicates: each rank owns
the documents with ``FNV-1a64(docId) % world == rank``.  What crosses GPUs is clock
bookkeeping, over ``torch.distributed`` (backend "nccl" = RCCL over xGMI on the
GPU box, "gloo" on CPU in the tests):

* ``gather_clock_rows`` — every rank's changed per-document clock rows (the
  ``DocBackend.clock`` entries ClockStore.update would persist, src/ClockStore.ts:78-91,
  src/RepoBackend.ts:343-345) gathered to every rank as fixed-width records
  ``(doc key u64, actor rank, seq)``: one all_gather of counts, one of the rows padded
  to the largest count (one collective per batch, sized for xGMI links, not per doc).
* ``min_clock`` — element-wise MIN all-reduce of dense clock rows: with 0 meaning
  "absent" this is exactly ``Clock.intersection`` (src/Clock.ts:103-113) across ranks,
  the minimum clock every replica has reached (the north star's "ClockStore min-clock").
* ``union_clock`` — element-wise MAX all-reduce = ``Clock.union`` (src/Clock.ts:87-95).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


def changed_rows(doc_keys: torch.Tensor, new_clock: torch.Tensor, old_clock: torch.Tensor) -> torch.Tensor:
    """Records (doc key, actor rank, seq) for every entry where new_clock > old_clock.
    doc_keys: int64 [n]; clocks: int32/uint32-as-int32 [n, S].  Returns int64 [k, 3]."""
    n, S = new_clock.shape
    nc = new_clock.to(torch.int64) & 0xFFFFFFFF
    oc = old_clock.to(torch.int64) & 0xFFFFFFFF
    mask = nc > oc
    idx = mask.nonzero(as_tuple=False)
    return torch.stack([doc_keys[idx[:, 0]], idx[:, 1], nc[idx[:, 0], idx[:, 1]]], dim=1)


def gather_clock_rows(rows: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """All ranks' rows (int64 [k_r, 3]) concatenated in rank order on every rank."""
    ws = dist.get_world_size(group)
    if ws == 1:
        return rows
    cnt = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    cnts = [torch.zeros_like(cnt) for _ in range(ws)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    kmax = max(counts)
    pad = torch.zeros((kmax, 3), dtype=torch.int64, device=rows.device)
    pad[: rows.shape[0]] = rows
    parts = [torch.zeros_like(pad) for _ in range(ws)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:k] for p, k in zip(parts, counts)], dim=0)


def min_clock(rows: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Clock.intersection across ranks of dense rows (0 == absent), in place."""
    if dist.get_world_size(group) > 1:
        dist.all_reduce(rows, op=dist.ReduceOp.MIN, group=group)
    return rows


def union_clock(rows: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Clock.union across ranks of dense rows, in place."""
    if dist.get_world_size(group) > 1:
        dist.all_reduce(rows, op=dist.ReduceOp.MAX, group=group)
    return rows
