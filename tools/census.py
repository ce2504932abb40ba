"""One C4 (or other config) merge per call of the library named by HMGPU_LIB: the driver of
tools/census.sh, which counts the small kernel's instructions per document under rocprofv3
for each early-exit (HM_ABLATE) build — a dynamic instruction census by phase (dev tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypermerge_amd import synth
from hypermerge_amd.engine import Engine
cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
over = {"arrival": int(sys.argv[3])} if len(sys.argv) > 3 else {}
b = synth.generate(synth.config(cfg, n_docs=n, **over))
e = Engine(0)
for _ in range(2):
    e.merge(b)
print("merged", n, flush=True)
