"""Quick GPU-vs-oracle parity probe (dev tool): python tools/gpu_check.py"""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from hypermerge_amd import synth
from hypermerge_amd.engine import Engine
import oracle.oracle as O

def compare(b, g, o, name):
    S = b.a_stride
    gs, os_ = g.docs["status"], o.docs["status"]
    unsup = gs == 16
    okdocs = (~unsup) & (os_ == 0)
    bad = []
    if not np.array_equal(gs[~unsup], os_[~unsup]): bad.append("status")
    errd = (~unsup) & (os_ != 0)
    for f in ("err_change", "err_op"):
        if not np.array_equal(g.docs[f][errd], o.docs[f][errd]): bad.append(f)
    for f in ("hist_len", "n_queued", "n_surv", "min_cmp"):
        if not np.array_equal(g.docs[f][okdocs], o.docs[f][okdocs]): bad.append(f)
    dm = np.repeat(okdocs, S)
    for f in ("clock", "back_clock", "heads"):
        if not np.array_equal(getattr(g, f)[dm], getattr(o, f)[dm]): bad.append(f)
    cm = np.repeat(okdocs, b.docs["n_changes"])
    if not np.array_equal(g.hist[cm], o.hist[cm]): bad.append("hist")
    if not np.array_equal(g.all_deps[np.repeat(cm, S)], o.all_deps[np.repeat(cm, S)]): bad.append("all_deps")
    rm = np.repeat(okdocs, b.docs["n_regs"])
    if not np.array_equal(g.regs[rm], o.regs[rm]): bad.append("regs")
    # survivors: valid prefix per doc
    sm = np.zeros(len(b.ops), bool)
    for d in np.nonzero(okdocs)[0]:
        s0 = int(b.docs["op_off"][d]); sm[s0:s0 + int(o.docs["n_surv"][d])] = True
    if not np.array_equal(g.surv[sm], o.surv[sm]): bad.append("surv")
    print(f"{name}: docs={b.n_docs} unsupported={int(unsup.sum())} oracle_err={int((os_!=0).sum())} "
          f"mismatch={bad or 'none'}", flush=True)
    return not bad

e = Engine(0)
allok = True
for name, n, extra in [("C4", 20000, {}), ("C2", 20000, {}), ("C5", 5000, {}),
                       ("C4", 3000, {"arrival": 1}), ("C2", 3000, {"arrival": 2, "shuffle_pct": 30, "dup_pct": 5}),
                       ("C1", 1, {})]:
    b = synth.generate(synth.config(name, n_docs=n, **extra))
    t = time.time(); g = e.merge(b); tg = time.time() - t
    o = O.merge(b, threads=8)
    allok &= compare(b, g, o, f"{name}{extra}")
    print("  kernel ms", e.last_kernel_ms(), "host-call s %.3f" % tg)
sys.exit(0 if allok else 1)
