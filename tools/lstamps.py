"""Per-phase cycle shares of merge_large_kernel from a diagnostic HM_STAMPS=1 build (dev tool).
Usage: HMGPU_LIB=hypermerge_amd/_lib/ablate/lib_stamps.so python tools/lstamps.py [config] [docs]
Shares only: each stamp adds a block barrier the real kernel does not have (never quote its time)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypermerge_amd import synth
from hypermerge_amd.engine import Engine, lib
NAMES = ["setup: ranges, table, opchg", "L1 readiness+history", "L2 closure jumping", "L2 literal fold check",
         "L3 survivors loop", "L3 offsets + ranks", "L3 counters", "L4 nodes + siblings",
         "L4 tour jumping", "L4 positions + vis", "outputs", "L3 init + staging", "L3 op scan loop",
         "L3 make-op check", "(L2 closure rounds, count)"]
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
b = synth.generate(synth.config(cfg, n_docs=n))
e = Engine(0)
L = lib()
L.hm_debug_lstamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
buf = (ctypes.c_ulonglong * 15)()
e.merge(b)
L.hm_debug_lstamps(buf, 15, 1)
e.merge(b)
L.hm_debug_lstamps(buf, 15, 1)
tot = sum(buf[:14])
print(f"{cfg}: {b.n_docs} docs, {len(b.changes)} changes, {len(b.ops)} ops; stamped cycles/doc {tot / n:.0f}")
for i, nm in enumerate(NAMES[:14]):
    print(f"{i:2d} {nm:28s} {100.0 * buf[i] / max(tot, 1):6.2f}%  {buf[i] / n:12.1f} cyc/doc")
print(f"14 {NAMES[14]:28s} {buf[14] / n:.2f} per doc (all-LDS path documents)")
