"""ctypes binding of the C-ABI in include/hypermerge_amd.h (libhmgpu.so).

This is the Python face of the boundary; the Node face is hypermerge_amd/js
(N-API).  There is no CPU fallback: if the HIP library or a GPU is missing,
``Engine()`` raises.
"""
from __future__ import annotations

import ctypes
import sys
import os
from typing import Optional, Sequence

import numpy as np

from .columnar import Batch, Results, CBatch, CResults

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("HMGPU_LIB") or os.path.join(_HERE, "_lib", "libhmgpu.so")

# every symbol include/hypermerge_amd.h declares
EXPORTS = ("hm_abi_version", "hm_status_message", "hm_engine_create", "hm_engine_destroy",
           "hm_engine_last_error", "hm_merge_host", "hm_scratch_bytes", "hm_merge_device",
           "hm_last_kernel_ms", "hm_last_deferred", "hm_clock_cmp_device", "hm_clock_union_device",
           "hm_clock_intersection_device", "hm_store_create", "hm_store_destroy", "hm_doc_open",
           "hm_batch_submit", "hm_batch_wait", "hm_doc_info", "hm_doc_read", "hm_doc_log",
           "hm_doc_history_prefix", "hm_doc_set_min_clock", "hm_store_clock_update", "hm_sync_ranges_device",
           "hm_comm_unique_id", "hm_comm_create", "hm_comm_destroy", "hm_comm_group_start", "hm_comm_group_end",
           "hm_clock_records_scratch_bytes", "hm_clock_records_device", "hm_clock_count_allgather",
           "hm_clock_allgather", "hm_clock_min_allreduce", "hm_comm_create_local", "hm_clock_exchange_host",
           "hm_clock_min_host", "hm_decode_blocks", "hm_decoded_batch", "hm_decoded_status", "hm_decoded_n_strings",
           "hm_decoded_string", "hm_decoded_actor", "hm_decoded_obj", "hm_decoded_reg", "hm_decoded_free",
           "hm_store_set_incremental", "hm_store_last_routing", "hm_store_last_kernel_ms", "hm_store_inc_states", "hm_debug_async_check", "hm_doc_open_n", "hm_doc_reset", "hm_store_read_regs", "hm_store_read_history",
           "hm_cursors_create", "hm_cursors_destroy", "hm_cursors_reserve", "hm_cursors_update", "hm_cursors_get",
           "hm_cursors_entry", "hm_cursors_docs_with_actors", "hm_docset_create", "hm_docset_destroy",
           "hm_docset_engine", "hm_docset_open", "hm_docset_apply", "hm_text_data", "hm_text_results", "hm_text_free",
           "hm_docset_doc_info", "hm_docset_history_prefix", "hm_docset_clock_update", "hm_docset_view",
           "hm_docset_stats", "hm_docset_routing", "hm_docset_handles", "hm_sync_ranges_host", "hm_batch_submit_device", "hm_batch_wait_device",
           "hm_batch_undo")

_lib = None


class EngineError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise EngineError(f"{LIB} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        # PyTorch-ROCm bundles its own libamdhip64.so.7 (same soname as /opt/rocm's).  Whichever
        # loads first serves the whole process, so let torch's load first: then device pointers
        # and streams from torch tensors are valid in this library's calls.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB)
        L.hm_abi_version.restype = ctypes.c_uint32
        L.hm_status_message.argtypes = [ctypes.c_int]
        L.hm_status_message.restype = ctypes.c_char_p
        L.hm_engine_create.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
        L.hm_engine_destroy.argtypes = [ctypes.c_void_p]
        L.hm_engine_last_error.argtypes = [ctypes.c_void_p]
        L.hm_engine_last_error.restype = ctypes.c_char_p
        L.hm_merge_host.argtypes = [ctypes.c_void_p, ctypes.POINTER(CBatch), ctypes.POINTER(CResults)]
        L.hm_merge_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(CBatch), ctypes.POINTER(CResults),
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.hm_scratch_bytes.argtypes = [ctypes.POINTER(CBatch)]
        L.hm_scratch_bytes.restype = ctypes.c_size_t
        L.hm_last_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        L.hm_last_deferred.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        for f in ("hm_clock_cmp_device", "hm_clock_union_device", "hm_clock_intersection_device"):
            getattr(L, f).argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 3 + [ctypes.c_uint32] * 2 + [ctypes.c_void_p]
        vp, u32 = ctypes.c_void_p, ctypes.c_uint32
        sig = {
            "hm_store_create": [vp, vp, vp], "hm_store_destroy": [vp], "hm_doc_open": [vp, vp],
            "hm_batch_submit": [vp, vp, vp, vp, vp], "hm_batch_wait": [vp, ctypes.c_uint64, vp, vp, vp, vp],
            "hm_batch_submit_device": [vp, vp, vp, vp, vp], "hm_batch_wait_device": [vp, ctypes.c_uint64, vp, vp],
            "hm_batch_undo": [vp, ctypes.c_uint64],
            "hm_doc_info": [vp, u32, vp], "hm_doc_read": [vp, u32] + [vp] * 7, "hm_doc_log": [vp, u32, vp, vp, vp],
            "hm_doc_history_prefix": [vp, u32, u32, vp], "hm_doc_set_min_clock": [vp, u32, vp],
            "hm_store_clock_update": [vp, u32, vp, vp, vp, vp],
            "hm_sync_ranges_device": [vp, vp, vp, vp, vp, vp, u32, vp],
            "hm_comm_unique_id": [vp], "hm_comm_create": [vp, ctypes.c_int, ctypes.c_int, vp, vp],
            "hm_comm_destroy": [vp], "hm_comm_group_start": [], "hm_comm_group_end": [],
            "hm_clock_records_scratch_bytes": [u32, u32],
            "hm_clock_records_device": [vp, vp, vp, vp, vp, u32, u32, vp, vp, vp, vp],
            "hm_clock_count_allgather": [vp, ctypes.c_uint64, vp, vp],
            "hm_clock_allgather": [vp, vp, vp, vp, vp], "hm_clock_min_allreduce": [vp, vp, ctypes.c_uint64, vp],
            "hm_comm_create_local": [vp, ctypes.c_int, vp],
            "hm_clock_exchange_host": [vp, ctypes.c_int, vp, vp, vp, ctypes.c_uint64, vp],
            "hm_clock_min_host": [vp, ctypes.c_int, vp, ctypes.c_uint64],
            "hm_decode_blocks": [vp, vp, vp, u32, u32, ctypes.c_int, vp], "hm_decoded_batch": [vp, vp],
            "hm_decoded_status": [vp], "hm_decoded_n_strings": [vp], "hm_decoded_string": [vp, u32, vp],
            "hm_decoded_actor": [vp, u32, u32, vp], "hm_decoded_free": [vp],
            "hm_decoded_obj": [vp, u32, u32, vp], "hm_decoded_reg": [vp, u32, u32, vp, vp],
            "hm_store_set_incremental": [vp, ctypes.c_int], "hm_store_last_routing": [vp, vp], "hm_store_last_kernel_ms": [vp, vp], "hm_store_inc_states": [vp, vp], "hm_debug_async_check": [vp, ctypes.c_int],
            "hm_doc_open_n": [vp, u32, vp], "hm_doc_reset": [vp, vp, u32], "hm_store_read_regs": [vp, u32, vp, vp, vp, vp, u32, vp],
            "hm_store_read_history": [vp, u32, vp, vp, vp, vp, vp, vp],
            "hm_cursors_create": [vp, u32, vp], "hm_cursors_destroy": [vp], "hm_cursors_reserve": [vp, u32],
            "hm_cursors_update": [vp, u32, vp, vp, vp, vp, vp], "hm_cursors_get": [vp, u32, vp, vp, vp, vp],
            "hm_cursors_entry": [vp, u32, vp, vp, vp],
            "hm_cursors_docs_with_actors": [vp, u32, vp, vp, u32, vp, vp, vp, vp],
            "hm_docset_create": [vp, vp, vp], "hm_docset_destroy": [vp], "hm_docset_engine": [vp],
            "hm_docset_open": [vp, u32, vp], "hm_docset_apply": [vp, vp, vp, vp, vp, u32, vp],
            "hm_text_data": [vp, vp], "hm_text_results": [vp, vp], "hm_text_free": [vp],
            "hm_docset_doc_info": [vp, u32, vp], "hm_docset_history_prefix": [vp, u32, u32, vp],
            "hm_docset_clock_update": [vp, u32, vp, vp, vp, vp], "hm_docset_view": [vp, u32, vp],
            "hm_docset_stats": [vp, vp], "hm_docset_routing": [vp, vp], "hm_docset_handles": [vp, u32, vp, vp], "hm_sync_ranges_host": [vp, vp, vp, vp, vp, vp, u32, u32],
        }
        for f, a in sig.items():
            getattr(L, f).argtypes = a
        L.hm_store_destroy.restype = None
        L.hm_cursors_destroy.restype = None
        L.hm_comm_destroy.restype = None
        L.hm_decoded_status.restype = ctypes.POINTER(ctypes.c_int32)
        L.hm_decoded_n_strings.restype = ctypes.c_uint32
        L.hm_decoded_string.restype = ctypes.c_void_p
        L.hm_decoded_actor.restype = ctypes.c_void_p
        L.hm_decoded_obj.restype = ctypes.c_void_p
        L.hm_decoded_reg.restype = ctypes.c_void_p
        L.hm_decoded_free.restype = None
        L.hm_clock_records_scratch_bytes.restype = ctypes.c_size_t
        L.hm_docset_destroy.restype = None
        L.hm_docset_engine.restype = ctypes.c_void_p
        L.hm_text_data.restype = ctypes.c_void_p
        L.hm_text_results.restype = ctypes.c_void_p
        L.hm_text_free.restype = None
        _lib = L
    return _lib


class _Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("flags", ctypes.c_int)]


GENERAL_ONLY = 1   # HM_CFG_GENERAL_ONLY


class Engine:
    def __init__(self, device: int = 0, flags: int = 0):
        L = lib()
        h = ctypes.c_void_p()
        cfg = _Config(device, flags)
        st = L.hm_engine_create(ctypes.byref(cfg), ctypes.byref(h))
        if st != 0:
            raise EngineError(f"hm_engine_create failed: {L.hm_status_message(st).decode()}")
        self._h = h
        self._L = L
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.hm_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        # (at interpreter exit finalizers run in any order: the engine may be gone, and the
        # process releases the device anyway)
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int, what: str) -> None:
        if st != 0:
            msg = self._L.hm_engine_last_error(self._h).decode()
            raise EngineError(f"{what}: {self._L.hm_status_message(st).decode()} ({msg})")

    def merge(self, batch: Batch, results: Optional[Results] = None) -> Results:
        """Host batch -> GPU merge -> host results (synchronous)."""
        if results is None:
            results = Results.alloc(batch)
        cb, cr = batch.c_struct(), results.c_struct()
        self._check(self._L.hm_merge_host(self._h, ctypes.byref(cb), ctypes.byref(cr)), "hm_merge_host")
        return results

    def merge_device(self, cbatch: CBatch, cresults: CResults, stream: int = 0) -> None:
        """Device-resident merge: every pointer in the structs is a device pointer."""
        self._check(self._L.hm_merge_device(self._h, ctypes.byref(cbatch), ctypes.byref(cresults), None,
                                            ctypes.c_void_p(stream) if stream else None), "hm_merge_device")

    def last_kernel_ms(self) -> Sequence[float]:
        buf = (ctypes.c_float * 4)()
        n = self._L.hm_last_kernel_ms(self._h, buf, 4)
        return [float(buf[i]) for i in range(n)]

    def last_deferred(self, n_docs: int) -> np.ndarray:
        """Launch rows the last launch handed to the general kernel (hand-over order)."""
        out = np.zeros(max(n_docs, 1), np.uint32)
        n = self._L.hm_last_deferred(self._h, out.ctypes.data, len(out))
        if n < 0:
            self._check(-n, "hm_last_deferred")
        return out[:min(n, len(out))].copy()

    def clock_op(self, which: str, a_ptr: int, b_ptr: int, out_ptr: int, n_docs: int, a_stride: int,
                 stream: int = 0) -> None:
        f = {"cmp": self._L.hm_clock_cmp_device, "union": self._L.hm_clock_union_device,
             "intersection": self._L.hm_clock_intersection_device}[which]
        self._check(f(self._h, a_ptr, b_ptr, out_ptr, n_docs, a_stride, stream or None), f"clock_{which}")
