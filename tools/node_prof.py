"""CPU profile of one Node leg (tools/bench_node.js under the V8 sampling profiler, HM_NODE_PROF):
python tools/node_prof.py <out_dir> [config] [docs] [leg]   (the bench's C2 documents by default)."""
import json
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

out = sys.argv[1]
cfg = sys.argv[2] if len(sys.argv) > 2 else "C2"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
leg = sys.argv[4] if len(sys.argv) > 4 else "gpu_async"
os.makedirs(out, exist_ok=True)
_, docs = bench._node_docs(cfg, n, 16)
here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with tempfile.TemporaryDirectory() as td:
    fn = os.path.join(td, "docs.json")

    def arr(xs):
        return b"[" + b",".join(xs) + b"]"
    with open(fn, "wb") as f:
        f.write(b'{"docs":' + arr([arr([arr(d[:16])] + [arr(d[k:k + 16]) for k in range(16, len(d), 16)]) for d in docs]) + b"}")
    prof = os.path.join(out, f"{cfg}_{leg}.cpuprofile")
    p = subprocess.run(["node", "--max-old-space-size=16384", "--max-semi-space-size=64",
                        os.path.join(here, "tools", "bench_node.js"), fn, leg],
                       env=dict(os.environ, HM_NODE_PROF=prof), capture_output=True, text=True, timeout=600)
    print(p.stdout[-2000:], p.stderr[-2000:])
top = subprocess.run([sys.executable, os.path.join(here, "tools", "cpuprofile_top.py"), prof, "40"],
                     capture_output=True, text=True)
open(os.path.join(out, f"{cfg}_{leg}_top.txt"), "w").write(top.stdout)
print(top.stdout)
