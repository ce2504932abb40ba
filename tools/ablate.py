"""Time alternative builds of the merge library in one GPU session (dev tool).
Usage: python tools/ablate.py lib1.so lib2.so ...   (each timed via bench.py, HMGPU_LIB)"""
import os, sys, subprocess, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for so in sys.argv[1:]:
    env = dict(os.environ, HMGPU_LIB=os.path.abspath(so))
    out = subprocess.run([sys.executable, os.path.join(R, "bench.py"), "--steps", "5", "--warmup", "2", "--no-cpu",
                          "--docs", os.environ.get("ABL_DOCS", "1000000"),
                          "--config", os.environ.get("ABL_CONFIG", "C4"), "--no-traffic", "--no-e2e", "--no-orders", "--no-node", "--no-incremental"] + os.environ.get("ABL_ARGS", "").split(), env=env, capture_output=True, text=True,
                         timeout=600)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if line:
        d = json.loads(line[-1])
        print(os.path.basename(so), [(k["kernel"][6:11], round(k["ms"], 4)) for k in d["roofline"]["kernels"]],
              round(d["ms_per_step"], 4), d["parity_sample_ok"], flush=True)
    else:
        print(os.path.basename(so), out.stderr[-800:], flush=True)
