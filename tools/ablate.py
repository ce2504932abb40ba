"""Time alternative builds of the merge library in one GPU session (dev tool).
Usage: python tools/ablate.py lib1.so lib2.so ...   (each timed via bench.py, HMGPU_LIB; ABL_REPS
rounds over the list, alternating; ABL_CONFIG / ABL_DOCS / ABL_ARGS pass through to bench.py)"""
import json
import os
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for rep in range(int(os.environ.get("ABL_REPS", "1"))):
    for so in sys.argv[1:]:
        env = dict(os.environ, HMGPU_LIB=os.path.abspath(so))
        det = os.path.join(tempfile.gettempdir(), f"abl_{os.getpid()}_{os.path.basename(so)}.json")
        out = subprocess.run([sys.executable, os.path.join(R, "bench.py"), "--steps", os.environ.get("ABL_STEPS", "10"),
                              "--warmup", "2", "--no-cpu", "--docs", os.environ.get("ABL_DOCS", "1000000"),
                              "--config", os.environ.get("ABL_CONFIG", "C4"), "--no-traffic", "--no-e2e", "--no-orders",
                              "--no-node", "--no-incremental", "--detail", det] + os.environ.get("ABL_ARGS", "").split(),
                             env=env, capture_output=True, text=True, timeout=600)
        if out.returncode == 0 and os.path.exists(det):
            d = json.load(open(det))
            print(rep, os.path.basename(so), [(k["kernel"][6:11], round(k["ms"], 4)) for k in d["roofline"]["kernels"]],
                  round(d["ms_per_step"], 4), round(d["roofline"]["frac"], 4), d["parity_sample_ok"], flush=True)
        else:
            print(rep, os.path.basename(so), out.stderr[-800:], flush=True)
