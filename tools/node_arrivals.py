"""The bench's Node live-arrival leg alone (dev): C2 documents loaded with their first `first`
changes through DocBackend.init, then applyRemoteChanges rounds of `chunk` changes, JS restatement
vs the GPU drop-in (async).  Prints the run's JSON (routing included)."""
import argparse
import importlib.util
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=10000)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--first", type=int, default=48)
    ap.add_argument("--chunk", type=int, default=2)
    ap.add_argument("--legs", default="cpu,gpu_async")
    ap.add_argument("--stderr", default=None, help="run node directly, its stderr into this file")
    a = ap.parse_args()
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(HERE, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc
    b = synth.generate(synth.config(a.config, n_docs=a.docs), threads=16)
    if a.stderr:
        # node run here with its stderr (HM_DOCSET_PROFILE phases) kept in a file
        import subprocess
        import tempfile
        docs = [decode_doc(b, i) for i in range(b.n_docs)]
        f0 = a.first
        with tempfile.TemporaryDirectory() as td:
            fn = os.path.join(td, "docs.json")
            with open(fn, "w") as f:
                json.dump({"docs": [[d[:f0]] + [d[k:k + a.chunk] for k in range(f0, len(d), a.chunk)] for d in docs]}, f)
            with open(a.stderr, "w") as ef:
                p = subprocess.run([shutil.which("node"), "--max-old-space-size=16384", "--max-semi-space-size=64",
                                    os.path.join(HERE, "tools", "bench_node.js"), fn, a.legs], stdout=subprocess.PIPE,
                                   stderr=ef, text=True, timeout=900)
        r = json.loads(p.stdout.strip().splitlines()[-1])
    else:
        r = bench._node_run(shutil.which("node"), [decode_doc(b, i) for i in range(b.n_docs)], a.legs.split(","),
                            chunk=a.chunk, first=a.first)
    if "error" not in r and "cpu" in r and "gpu_async" in r:
        r["gpu_async_vs_js"] = r["gpu_async"]["changes_per_s"] / r["cpu"]["changes_per_s"]
    print(json.dumps(r))


if __name__ == "__main__":
    main()
