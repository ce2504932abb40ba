"""Per-phase timing of the resident store's applyRemoteChanges rounds (bench.py's
resident_incremental leg): HM_STORE_PROFILE=1 makes hm_batch_submit / hm_batch_wait print
their phases; run under `rocprofv3 --kernel-trace --stats` for the kernels."""
import argparse
import os
import time

import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--incremental", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from hypermerge_amd import synth
    from hypermerge_amd.engine import Engine
    from hypermerge_amd.store import RowStore, slice_changes
    b = synth.generate(synth.config("C4", n_docs=a.docs))
    eng = Engine(0)
    n = b.n_docs
    nch = b.docs["n_changes"].astype(np.int64)
    pos = np.maximum(nch - 2 * a.rounds, 0)
    st = RowStore(eng, a_stride=b.a_stride)
    st.set_incremental(bool(a.incremental))
    h0 = st.open_n(n)
    t = time.perf_counter()
    st.submit_batch(slice_changes(b, np.zeros(n, np.int64), pos), np.arange(h0, h0 + n))
    st.wait()
    print(f"initial {time.perf_counter() - t:.3f}s", flush=True)
    rng = np.random.default_rng(5)
    os.environ["HM_STORE_PROFILE"] = "1"
    for r in range(a.rounds):
        hi = np.minimum(pos + rng.integers(1, 3, n), nch)
        sel = np.nonzero(hi > pos)[0]
        sub = slice_changes(b, pos, hi, sel)
        t0 = time.perf_counter()
        st.submit_batch(sub, sel + h0)
        t1 = time.perf_counter()
        st.wait()
        t2 = time.perf_counter()
        print(f"round {r}: {len(sel)} docs {len(sub.changes)} changes submit {1e3 * (t1 - t0):.2f} ms "
              f"wait {1e3 * (t2 - t1):.2f} ms routing {st.last_routing()}", flush=True)
        pos = np.maximum(pos, hi)


if __name__ == "__main__":
    main()
