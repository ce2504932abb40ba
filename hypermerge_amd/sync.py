"""syncChanges contiguity on the GPU (src/RepoBackend.ts:506-531).

When an actor feed syncs, RepoBackend walks, for every document that has the
actor, the feed's blocks from ``doc.changes[actor]`` up to the cursor and stops
at the first block not downloaded yet (``actor.changes.hasOwnProperty(i)``,
:517-519).  ``contiguous_ends`` answers that for many (document, actor) pairs at
once with hm_sync_ranges_device: each feed's downloaded blocks are a bitmap in
HBM, one lane per pair scans it word by word.
"""
from __future__ import annotations

import ctypes
from typing import Sequence, Tuple

import numpy as np
import torch

from .engine import Engine


def pack_feeds(present: Sequence[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
    """Bitmaps (u64 words) of several feeds concatenated + each feed's first word.
    Every feed gets one spare word so a scan may read past its last block."""
    words, offs, o = [], [], 0
    for p in present:
        p = np.asarray(p, bool)
        n = (len(p) + 63) // 64 + 1
        w = np.zeros(n * 64, bool)
        w[: len(p)] = p
        words.append(np.packbits(w, bitorder="little").view("<u8"))
        offs.append(o)
        o += n
    return (np.concatenate(words) if words else np.zeros(1, np.uint64)), np.array(offs, np.uint64)


def contiguous_ends(engine: Engine, present: Sequence[np.ndarray], feed: np.ndarray, lo: np.ndarray,
                    hi: np.ndarray, device: int = 0) -> np.ndarray:
    """For pair i: first j in [lo[i], hi[i]) with block j of feed[i] missing, else hi[i]."""
    words, offs = pack_feeds(present)
    lens = np.array([len(p) for p in present], np.int64)
    feed = np.asarray(feed, np.int64)
    lo = np.asarray(lo, np.uint32)
    hi = np.minimum(np.asarray(hi, np.uint64), lens[feed].astype(np.uint64) + 64).astype(np.uint32)
    dev = torch.device("cuda", device)
    t_words = torch.from_numpy(words.view(np.int64)).to(dev)
    t_off = torch.from_numpy(offs[feed].view(np.int64)).to(dev)
    t_lo = torch.from_numpy(lo.view(np.int32)).to(dev)
    t_hi = torch.from_numpy(hi.view(np.int32)).to(dev)
    out = torch.zeros(len(lo), dtype=torch.int32, device=dev)
    st = engine._L.hm_sync_ranges_device(engine._h, t_words.data_ptr(), t_off.data_ptr(), t_lo.data_ptr(),
                                         t_hi.data_ptr(), out.data_ptr(), len(lo), None)
    engine._check(st, "hm_sync_ranges_device")
    torch.cuda.synchronize(dev)
    return out.cpu().numpy().view(np.uint32)
