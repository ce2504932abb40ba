"""Blocks -> columnar batch through the native decoder (hm_decode_blocks, csrc/decode.cpp):
Block.unpack + JsonBuffer.parse + Actor.parseBlock (src/Block.ts:18-29, src/JsonBuffer.ts:1-4,
src/Actor.ts:137-141) and the host encoder's rows, multi-threaded over documents."""
from __future__ import annotations

import ctypes
import sys
from typing import List, Sequence, Tuple

import numpy as np

from .columnar import Batch, CBatch, DOC_DT, CHANGE_DT, DEP_DT, OP_DT
from .engine import lib


def pack_offsets(docs: Sequence[Sequence[bytes]]):
    """(data, block_off u64[n_blocks+1], doc_block u32[n_docs+1]) for a list of per-document
    block lists."""
    sizes = [len(b) for d in docs for b in d]
    block_off = np.zeros(len(sizes) + 1, np.uint64)
    np.cumsum(sizes, out=block_off[1:])
    doc_block = np.zeros(len(docs) + 1, np.uint32)
    np.cumsum([len(d) for d in docs], out=doc_block[1:])
    data = np.frombuffer(b"".join(b for d in docs for b in d) or b"\0", np.uint8)
    return data, block_off, doc_block


def decode_packed(data: np.ndarray, block_off: np.ndarray, doc_block: np.ndarray, a_stride: int = 0,
                  threads: int = 16, tables: bool = True) -> Tuple[Batch, np.ndarray]:
    """Decode pre-packed blocks; returns (batch with string/actor tables, per-document status).
    tables=False leaves the per-document actor/object/register name tables out (the rows and
    the string pool are all a merge needs; the names are for rendering)."""
    L = lib()
    n_docs = len(doc_block) - 1
    h = ctypes.c_void_p()
    st = L.hm_decode_blocks(data.ctypes.data, block_off.ctypes.data, doc_block.ctypes.data, n_docs, a_stride,
                            threads, ctypes.byref(h))
    if st:
        raise RuntimeError(f"hm_decode_blocks: {L.hm_status_message(st).decode()}")
    owner = _Decoded(L, h)
    cb = CBatch()
    L.hm_decoded_batch(h, ctypes.byref(cb))

    def take(ptr, n, dt):
        # the decoder's own row buffers, without a copy: they live until the last array over them
        if n == 0:
            return np.zeros(0, dt)
        buf = (ctypes.c_uint8 * (n * dt.itemsize)).from_address(ptr)
        buf._owner = owner
        return np.frombuffer(buf, dt)
    docs = take(cb.docs, cb.n_docs, DOC_DT)
    b = Batch(docs, take(cb.changes, cb.n_changes, CHANGE_DT), take(cb.deps, cb.n_deps, DEP_DT),
              take(cb.ops, cb.n_ops, OP_DT), int(cb.a_stride))
    status = np.ctypeslib.as_array(L.hm_decoded_status(h), shape=(max(n_docs, 1),))[:n_docs].copy()
    ln = ctypes.c_size_t()

    def text(p):
        if not p:
            raise RuntimeError("hm_decoded_*: index out of range")
        return ctypes.string_at(p, ln.value).decode("utf-8", "surrogatepass")
    b.strings = [text(L.hm_decoded_string(h, i, ctypes.byref(ln))) for i in range(L.hm_decoded_n_strings(h))]
    if not tables:
        return b, status
    b.doc_actors = [[text(L.hm_decoded_actor(h, d, r, ctypes.byref(ln))) for r in range(int(docs["n_actors"][d]))]
                    for d in range(n_docs)]
    b.doc_objs = [[text(L.hm_decoded_obj(h, d, o, ctypes.byref(ln))) for o in range(int(docs["n_objs"][d]))]
                  for d in range(n_docs)]
    ob = ctypes.c_uint32()
    b.doc_regs = [[(lambda t: (int(ob.value), t))(text(L.hm_decoded_reg(h, d, g, ctypes.byref(ob), ctypes.byref(ln))))
                   for g in range(int(docs["n_regs"][d]))] for d in range(n_docs)]
    return b, status


class _Decoded:
    """Owns one hm_decoded (its row tables back the batch's arrays)."""

    def __init__(self, L, h):
        self.L, self.h = L, h

    def __del__(self):
        if self.h and not sys.is_finalizing():
            self.L.hm_decoded_free(self.h)
            self.h = None


def decode_blocks(docs: Sequence[Sequence[bytes]], a_stride: int = 0, threads: int = 16):
    return decode_packed(*pack_offsets(docs), a_stride=a_stride, threads=threads)
