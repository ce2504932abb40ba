"""TEST INFRASTRUCTURE ONLY — ctypes wrapper around oracle/build/liboracle.so,
the CPU restatement of the reference merge path (see oracle/oracle.c for
what it restates and with which provenance).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.oracle_merge.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        _lib.oracle_merge.restype = ctypes.c_int
    return _lib


def merge(batch, results=None, threads: int = 1, doc_range: Optional[tuple] = None):
    """Run the restatement over documents of `batch` into `results`
    (a hypermerge_amd.columnar.Results; allocated when None)."""
    from hypermerge_amd.columnar import Results
    if results is None:
        results = Results.alloc(batch)
    cb, cr = batch.c_struct(), results.c_struct()
    lo, hi = doc_range if doc_range else (0, batch.n_docs)
    L = lib()
    if threads <= 1 or hi - lo < 2:
        L.oracle_merge(ctypes.byref(cb), ctypes.byref(cr), lo, hi)
    else:
        step = (hi - lo + threads - 1) // threads
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda s: L.oracle_merge(ctypes.byref(cb), ctypes.byref(cr), s, min(hi, s + step)),
                        range(lo, hi, step)))
    return results


def sync_end(present, lo: int, hi: int) -> int:
    """RepoBackend.syncChanges' walk (src/RepoBackend.ts:517-519):
    for (i = min; i < max && actor.changes.hasOwnProperty(i); i++) — returns the final i."""
    i = lo
    while i < hi and i < len(present) and present[i]:
        i += 1
    return i
