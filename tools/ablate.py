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
    print(os.path.basename(so), (json.loads(line[-1])["roofline"]["kernels"][0]["ms"], json.loads(line[-1])["ms_per_step"], json.loads(line[-1])["parity_sample_ok"]) if line else out.stderr[-800:], flush=True)
