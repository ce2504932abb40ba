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


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=1_000_000, help="documents per GPU")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--cpu-sample-docs", type=int, default=200_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check-docs", type=int, default=20_000, help="docs checked against the oracle")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes for roofline.traffic")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host->device->host (PCIe-inclusive) leg")
    ap.add_argument("--arrival", type=int, default=None,
                    help="override the config's arrival order (0 generation, 1 actor-major as RepoBackend.loadDocument "
                         "concatenates, 2 shuffled)")
    args = ap.parse_args()

    ws, rank, local = _dist()
    import torch
    import torch.distributed as dist
    if ws > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from hypermerge_amd import synth
    from hypermerge_amd.columnar import CBatch, CResults, Results
    from hypermerge_amd.engine import Engine

    t0 = time.time()
    over = {} if args.arrival is None else {"arrival": args.arrival}
    cfg = synth.config(args.config, n_docs=args.docs, shard=rank, n_shards=ws, **over)
    batch = synth.generate(cfg, threads=min(16, os.cpu_count() or 1))
    gen_s = time.time() - t0

    eng = Engine(local)

    def to_dev(a: np.ndarray) -> torch.Tensor:
        t = torch.from_numpy(a.view(np.uint8).reshape(-1)).to(dev)
        return t

    S = batch.a_stride
    nd, nc, no = batch.n_docs, len(batch.changes), len(batch.ops)
    nr = int(batch.docs["n_regs"].sum())
    d_docs, d_ch, d_dp, d_op = (to_dev(x) for x in (batch.docs, batch.changes, batch.deps, batch.ops))
    u8 = dict(dtype=torch.uint8, device=dev)
    r_docs = torch.zeros(nd * 32, **u8)   # hm_doc_result rows
    r_clock = torch.zeros(nd * S, dtype=torch.int32, device=dev)
    r_bclock = torch.zeros(nd * S, dtype=torch.int32, device=dev)
    r_heads = torch.zeros(nd * S, dtype=torch.int32, device=dev)
    r_hist = torch.zeros(nc, dtype=torch.int32, device=dev)
    r_ad = torch.zeros(nc * S, dtype=torch.int32, device=dev)
    r_regs = torch.zeros(nr * 16, **u8)
    r_surv = torch.zeros(no * 16, **u8)
    hc = batch.c_struct()
    cb = CBatch(hc.n_docs, hc.n_changes, hc.n_deps, hc.n_ops, hc.n_regs, hc.a_stride,
                hc.max_changes, hc.max_ops, hc.max_regs, hc.max_objs, hc.doc_flags, hc.max_deps,
                d_docs.data_ptr(), d_ch.data_ptr(), d_dp.data_ptr(), d_op.data_ptr(), None)
    cr = CResults(r_docs.data_ptr(), r_clock.data_ptr(), r_bclock.data_ptr(), r_heads.data_ptr(),
                  r_hist.data_ptr(), r_ad.data_ptr(), r_regs.data_ptr(), r_surv.data_ptr())
    stream = torch.cuda.Stream(dev)          # a real stream: the C-ABI treats handle 0 as "engine stream"
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    def step():
        eng.merge_device(cb, cr, sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t_start
    ev_ms = ev0.elapsed_time(ev1)
    # per-launch kernel duration: HIP events on the launch stream, one extra timed launch
    klist = []
    for _ in range(max(3, min(args.steps, 10))):
        step()
        klist.append(eng.last_kernel_ms()[0])
    kern_ms = float(np.mean(klist))

    # pull results back once for counting + spot parity
    from hypermerge_amd.columnar import DOC_RESULT_DT
    docs_res = r_docs.cpu().numpy().view(DOC_RESULT_DT)
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
    # every rank's changed DocBackend.clock rows gathered over RCCL (hypermerge_amd/exchange.py)
    xchg = None
    if ws > 1:
        from hypermerge_amd import exchange as X
        keys = torch.from_numpy((batch.docs["reserved"][:, 0].astype(np.int64)
                                 | (batch.docs["reserved"][:, 1].astype(np.int64) << 32))).to(dev)
        newc = r_bclock.view(nd, S)
        zero = torch.zeros_like(newc)
        times = []
        for it in range(4):
            torch.cuda.synchronize(dev)
            dist.barrier()
            t = time.perf_counter()
            rows = X.changed_rows(keys, newc, zero)
            allrows = X.gather_clock_rows(rows)
            torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t)
        xchg = {"clock_rows_gathered": int(allrows.shape[0]), "ms": 1000.0 * float(np.median(times[1:])),
                "collective": "all_gather (RCCL)"}

    value = applied_all * args.steps / wall_max
    ms_per_step = wall_max * 1000.0 / args.steps
    # roofline of the dominant kernel (merge_small_kernel): algorithmic bytes per launch
    full = Results(docs_res, None, None, None, None, None, None, None)
    alg_bytes = batch.algorithmic_bytes(full)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9

    # spot parity against the oracle on a sample (checker only; not timed)
    parity = None
    cpu = cpu_mt = None
    if rank == 0 and ws == 1 and not args.no_cpu:          # CPU legs: rank 0 at N=1 only
        import oracle.oracle as O
        from hypermerge_amd.columnar import Batch
        k = min(args.check_docs, nd)
        sub = _subbatch(batch, k)
        g = eng.merge(sub)
        o = O.merge(sub, threads=min(16, os.cpu_count() or 1))
        parity = bool(_same(sub, g, o))
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
                  "sample": f"same sample, documents split over {nth} threads, {dt:.2f}s"}

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
    traffic = None
    if rank == 0 and ws == 1 and not args.no_traffic:
        traffic = _pmc_traffic(args)

    if rank == 0:
        line = {
            "metric": "merged changes/sec (1M docs×8 actors) at 1/2/4/8 GPUs + % HBM roofline",
            "value": value, "unit": "changes/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u32", "data": "synthetic (seeded gossip feeds, hypermerge_amd/csrc/synth.cpp)",
            "config": {"workload": f"{args.config}: {nd} docs/GPU x {batch.docs['n_actors'].max()} actors x "
                                   f"{nc / max(nd, 1):.0f} changes/doc, {WORKLOAD_KIND.get(args.config, '')}"
                                   + ("" if args.arrival is None else f", arrival order {ARRIVAL[args.arrival]}"), "docs_per_gpu": nd,
                       "changes_per_gpu": nc, "ops_per_gpu": no, "parallelism": f"doc-shard{ws}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic["bytes"] if traffic else None,
                         "kernel": "merge_small_kernel", "kernel_ms": kern_ms, "alg_bytes": alg_bytes,
                         "traffic_detail": traffic},
            "cpu_baseline": cpu, "cpu_parallel": cpu_mt, "end_to_end": e2e,
            "parity_sample_ok": parity, "unsupported_docs": unsupported, "error_docs": errors,
            "gen_s": round(gen_s, 2), "event_ms_per_step": ev_ms / args.steps,
            "clock_exchange": xchg,
        }
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.destroy_process_group()
    return 0


def _pmc_traffic(args):
    """HBM bytes per launch of merge_small_kernel, from two rocprofv3 PMC passes over a short
    run of this same workload (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one pass's
    TCC counters).  Corrected as /opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes: on gfx950
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
               "--no-traffic", "--no-e2e", "--docs", str(args.docs), "--config", args.config] + ([] if args.arrival is None else ["--arrival", str(args.arrival)])
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
                    if "merge_small_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                        got.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not got:
            return None
        vals[ctr] = sum(got) / len(got)
    rd = vals["FETCH_SIZE"] * 1024 * 2
    wr = vals["WRITE_SIZE"] * 1024
    return {"bytes": rd + wr, "read_bytes": rd, "write_bytes": wr, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
            "(separate passes), FETCH_SIZE x2 per MI355X_MICROARCH.md §HBM"}


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
