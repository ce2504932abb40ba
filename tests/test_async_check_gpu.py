"""merge_small_kernel's asynchronous next-row loads (HM_ASYNC_NEXT: inline-asm loads waited for
with a fixed vmcnt that leaves the current document's stores in flight) checked in the check
build (libhmgpu_check.so, HM_ASYNC_CHECK): every document's asynchronously loaded rows are
re-read with counted loads and compared on the device.  Runs the strides and op-row classes that
take the asynchronous path (OPL 1 and 2; actor strides 4, 8, 16, 32 and 64), with outcomes that
pad differently (documents merged OK, documents handed to the general kernel, queued changes),
and requires no difference and results bit-exact with the oracle."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK_LIB = os.path.join(ROOT, "hypermerge_amd", "_lib", "libhmgpu_check.so")

pytestmark = pytest.mark.gpu

SCRIPT = r'''
import ctypes, dataclasses, json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from hypermerge_amd import synth, engine as E
from hypermerge_amd.columnar import decode_doc, encode
import oracle.oracle as O
L = E.lib()
L.hm_debug_async_check.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
eng = E.Engine(0)
out = {}
cnt = (ctypes.c_ulonglong * 2)()
assert L.hm_debug_async_check(cnt, 1) == 1, "not the check build"
# (more documents than the persistent grid holds, so waves load a next document)
cases = [("C2", 4, {}, 40000), ("C2", 8, {"arrival": 2, "shuffle_pct": 30}, 40000), ("C4", 8, {}, 40000),
         ("C4", 8, {"arrival": 1}, 40000), ("C4", 16, {}, 20000), ("C4", 32, {}, 20000), ("C2", 64, {}, 20000),
         ("C5", 8, {}, 40000)]
for name, S, extra, n in cases:
    b = synth.generate(synth.config(name, n_docs=n, **extra))
    if S != b.a_stride:
        b = dataclasses.replace(b, a_stride=S)          # (the tables do not depend on the row stride)
    g = eng.merge(b)
    o = O.merge(b, threads=16)
    same = bool(np.array_equal(g.docs, o.docs)) and all(
        np.array_equal(getattr(g, f), getattr(o, f)) for f in ("clock", "back_clock", "heads", "hist", "all_deps", "regs"))
    assert L.hm_debug_async_check(cnt, 1) == 1
    out[f"{name}/S{S}/{extra}"] = {"same": same, "checked": int(cnt[0]), "bad": int(cnt[1])}
    print(name, S, out[f"{name}/S{S}/{extra}"], file=sys.stderr, flush=True)
print(json.dumps(out))
'''


@pytest.mark.skipif(not os.path.exists(CHECK_LIB), reason="check build not built (hypermerge_amd/build.py)")
def test_async_row_loads_match_counted_loads():
    env = dict(os.environ, HMGPU_LIB=CHECK_LIB)
    p = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(p.stdout.strip().splitlines()[-1])
    checked = 0
    for case, r in got.items():
        assert r["same"], case
        assert r["bad"] == 0, (case, r)
        checked += r["checked"]
    assert checked > 20000, got
