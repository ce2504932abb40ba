"""Per-phase timing of bench.py's resident_incremental leg, round by round (the same rounds:
every document resident with all but its last `tail` changes, then rounds of 1-2 new changes
per document until the logs are exhausted).  HM_STORE_PROFILE=1 makes hm_batch_submit /
hm_batch_wait print their phases on stderr; run under `rocprofv3 --kernel-trace --stats`
for the kernels."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--incremental", type=int, default=1)
    ap.add_argument("--tail", type=int, default=4)
    ap.add_argument("--device", type=int, default=0, help="1: new rows already in HBM (submit_device)")
    ap.add_argument("--config", default="C4")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from hypermerge_amd import synth
    from hypermerge_amd.engine import Engine, lib
    from hypermerge_amd.store import RowStore, slice_changes
    b = synth.generate(synth.config(a.config, n_docs=a.docs), threads=16)
    eng = Engine(0)
    n = b.n_docs
    nch = b.docs["n_changes"].astype(np.int64)
    pos = np.maximum(nch - a.tail, 0)
    st = RowStore(eng, a_stride=b.a_stride)
    st.set_incremental(a.incremental)          # 2: small list documents too (no cost policy)
    h0 = st.open_n(n)
    S = b.a_stride
    dev = torch.device("cuda", 0)
    out = torch.empty(n * (32 + 12 * S), dtype=torch.uint8, device=dev)

    def to_dev(x, hs):
        t = [torch.from_numpy(np.ascontiguousarray(y).view(np.uint8).reshape(-1)).to(dev) for y in
             (x.docs, x.changes, x.deps, x.ops, np.ascontiguousarray(hs, np.uint32))]
        return (len(x.changes), len(x.deps), len(x.ops)), t
    t = time.perf_counter()
    cnt, tt = to_dev(slice_changes(b, np.zeros(n, np.int64), pos), np.arange(h0, h0 + n))
    st.submit_device(n, cnt, *tt)
    st.wait_device(out)
    del tt
    print(f"initial {time.perf_counter() - t:.3f}s inc_states {st.inc_states()}", flush=True)
    rng = np.random.default_rng(5)
    os.environ["HM_STORE_PROFILE"] = "1"
    # diagnostic builds (-DHM_META_STAMPS=1, via HMGPU_LIB): inc_meta_kernel's per-phase wave time
    # over the rounds below
    import ctypes
    L = lib()
    stamps = np.zeros(8, np.uint64)
    meta = getattr(L, "hm_debug_meta_stamps", None)
    if meta is not None:
        meta.argtypes = [ctypes.c_void_p, ctypes.c_int]
        meta.restype = ctypes.c_int
        meta(stamps.ctypes.data, 1)
    r = 0
    while (pos < nch).any():
        hi = np.minimum(pos + rng.integers(1, 3, n), nch)
        sel = np.nonzero(hi > pos)[0]
        sub = slice_changes(b, pos, hi, sel)
        if a.device:
            cnt, tt = to_dev(sub, sel + h0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.submit_device(len(sel), cnt, *tt)
            t1 = time.perf_counter()
            st.wait_device(out)
            t2 = time.perf_counter()
        else:
            t0 = time.perf_counter()
            st.submit_batch(sub, (sel + h0).astype(np.uint32))
            t1 = time.perf_counter()
            st.wait()
            t2 = time.perf_counter()
        print(f"round {r}: {len(sel)} docs {len(sub.changes)} changes submit {1e3 * (t1 - t0):.2f} ms "
              f"wait {1e3 * (t2 - t1):.2f} ms routing {st.last_routing()} inc_states {st.inc_states()}", flush=True, file=sys.stderr)
        pos = np.maximum(pos, hi)
        r += 1
    if meta is not None and meta(stamps.ctypes.data, 0) == 1:
        names = ["changes+keys", "survivors", "op scan", "list pass 0", "list pass 1", "hole check"]
        tot = float(stamps[:6].sum()) or 1.0
        for k, nm in enumerate(names):
            print(f"inc_meta {nm:14s} {int(stamps[k]):>14d} ticks {100 * stamps[k] / tot:5.1f}%", flush=True)


if __name__ == "__main__":
    main()
