"""Dev tool: the C5 incremental-parity scenario, incremental store vs re-merge store, stopping
at the first document whose registers differ; prints that round's changes for it and both
register tables (to locate a list-path bug)."""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc
from hypermerge_amd.engine import Engine
from hypermerge_amd.store import DocStore
from test_store_gpu import split

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
b = synth.generate(synth.config("C5", n_docs=n))
docs = [decode_doc(b, i) for i in range(b.n_docs)]
rng = np.random.default_rng(7)
eng = Engine(0)
A, B = DocStore(eng, a_stride=8), DocStore(eng, a_stride=8)
B.set_incremental(False)
ha = [A.open() for _ in docs]
hb = [B.open() for _ in docs]
parts = [split(c, 5, rng) for c in docs]
for rd in range(5):
    sel = [i for i in range(len(docs)) if rd == 0 or parts[i][rd]]
    watch = os.environ.get("DBG_DOC")
    if watch is not None:
        os.environ["HM_INC_DEBUG_HANDLE"] = str(ha[int(watch)])
        print(f"=== round {rd} (store A)", file=sys.stderr, flush=True)
    A.apply([(ha[i], parts[i][rd]) for i in sel])
    os.environ.pop("HM_INC_DEBUG_HANDLE", None)
    print("round", rd, A.last_routing(), flush=True)
    B.apply([(hb[i], parts[i][rd]) for i in sel])
    for i in sel:
        _, ga = A.read(ha[i])
        _, gb = B.read(hb[i])
        if not np.array_equal(ga.regs, gb.regs):
            print("doc", i, "round", rd)
            print("objects:", A.enc[ha[i]].objects if hasattr(A.enc[ha[i]], "objects") else None)
            for c in parts[i][rd]:
                print(" change", json.dumps(c))
            bad = np.nonzero(ga.regs != gb.regs)[0]
            print(" regs differ at", bad.tolist())
            print(" inc   ", [tuple(int(x) for x in r) for r in ga.regs])
            print(" remrg ", [tuple(int(x) for x in r) for r in gb.regs])
            if rd:
                print(" previous rounds' changes:")
                for r0 in range(rd):
                    for c in parts[i][r0]:
                        print("  ", r0, json.dumps(c))
            sys.exit(0)
print("no difference")
