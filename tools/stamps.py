"""Per-phase cycle shares of merge_small_kernel from a diagnostic HM_STAMPS=1 build (dev tool).
Usage: HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so python tools/stamps.py [config] [docs]
Shares only: the stamps' fences forbid overlaps the real kernel has (never quote this build's time)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypermerge_amd import synth
from hypermerge_amd.engine import Engine, lib
NAMES = ["pre-merge", "validate+first-table", "deps/readiness", "history", "ancestor push", "fold+heads+reg-init",
         "K2 op scan", "objects+survivors", "offsets+rank+ties", "lists/counters", "outputs", "stage next", "min_cmp+next-row loads",
         "history: t solve", "history: (pass, pos) solve", "history: check + rank",
         "K3: nodes", "K3: children + siblings", "K3: Euler tour", "K3: positions"]
cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
over = {"arrival": int(sys.argv[3])} if len(sys.argv) > 3 else {}
b = synth.generate(synth.config(cfg, n_docs=n, **over))
e = Engine(0)
L = lib()
L.hm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
buf = (ctypes.c_ulonglong * 20)()
e.merge(b)
L.hm_debug_stamps(buf, 20, 1)
e.merge(b)
L.hm_debug_stamps(buf, 20, 1)
tot = sum(buf)
for i, nm in enumerate(NAMES):
    print(f"{i:2d} {nm:24s} {100.0 * buf[i] / tot:6.2f}%  {buf[i] / n:10.1f} cyc/doc")
