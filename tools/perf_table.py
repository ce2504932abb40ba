"""Throughput of every BASELINE.json config on one MI355X (BASELINE.md's table): bench.py per
config, kernel (device-resident) and end-to-end (hm_merge_host) merged changes/s, roofline
fraction of merge_small_kernel, and the CPU restatement on 1 and N threads over a sample.
Usage (GPU box): python tools/perf_table.py > gpurun_out/perf_table.md"""
import json
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# config, docs per GPU, CPU sample docs, parity-check docs, timed steps
RUNS = [("C1", 1, 1, 1, 3), ("C2", 100_000, 20_000, 5_000, 10), ("C3", 10_000, 100, 100, 3),
        ("C4", 1_000_000, 200_000, 20_000, 20), ("C5", 100_000, 20_000, 5_000, 10),
        ("C4am", 1_000_000, 100_000, 10_000, 10),       # C4 in loadDocument's actor-major order
        ("C1am", 1, 1, 1, 3)]                           # C1 in loadDocument's actor-major order


def main() -> int:
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    rows = []
    for cfg, docs, cpu_docs, check, steps in RUNS:
        if only and cfg not in only:
            continue
        extra = ["--arrival", "1"] if cfg.endswith("am") else []
        cmd = [sys.executable, os.path.join(R, "bench.py"), "--config", cfg[:2], "--docs", str(docs), "--steps", str(steps),
               "--warmup", "2", "--cpu-sample-docs", str(cpu_docs), "--check-docs", str(check), "--no-traffic"] + extra
        if cfg != "C2":
            cmd.append("--no-node")                     # the Node leg runs its own C2 sample
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
        if p.returncode or not lines:
            print(f"<!-- {cfg} failed: {p.stderr[-400:]} -->", flush=True)
            continue
        d = json.loads(lines[-1])
        rows.append(d)
        print("<!-- " + json.dumps(d) + " -->", flush=True)
    print("| config | workload | merged changes/s (kernel, both kernels) | ms/step | % HBM roofline (algorithmic bytes / step) "
          "| end-to-end changes/s (PCIe incl.) | CPU 1 thread | CPU N threads | parity sample | unsupported docs |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for d in rows:
        c, e, m = d.get("cpu_baseline") or {}, d.get("end_to_end") or {}, d.get("cpu_parallel") or {}
        print(f"| {d['config']['workload'].split(':')[0]} | {d['config']['workload'].split(': ', 1)[1]} | {d['value']:.3e} "
              f"| {d['ms_per_step']:.3f} | {100 * d['roofline']['alg_bytes'] / (d['ms_per_step'] * 1e-3) / 8e12:.1f} % "
              f"| {e.get('value', float('nan')):.3e} "
              f"| {c.get('value', float('nan')):.3e} | {m.get('value', float('nan')):.3e} ({m.get('cores', '?')} threads) "
              f"| {d['parity_sample_ok']} | {d['unsupported_docs']} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
