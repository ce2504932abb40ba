"""CPU model of the small kernel's set-parallel queue passes (dev tool): checks the pass-at-a-time
algorithm (applied-ness per key, duplicate copies) against the oracle's history on C5 documents."""
import sys, numpy as np
sys.path.insert(0, "/root/repo")
from hypermerge_amd import synth
import oracle.oracle as O
b = synth.generate(synth.config("C5", n_docs=4000, arrival=1, dup_pct=0) if len(sys.argv) > 1 else synth.config("C5", n_docs=4000))
o = O.merge(b)
bad = 0
for d in range(b.n_docs):
    doc = b.docs[d]
    n = int(doc["n_changes"]); c0 = int(doc["change_off"])
    if n > 64 or doc["n_actors"] > 8: continue
    ch = b.changes[c0:c0+n]
    # first arrival per (a, s)
    first = {}
    for i in range(n):
        k = (int(ch[i]["actor"]), int(ch[i]["seq"]))
        first.setdefault(k, i)
    key = [first[(int(ch[i]["actor"]), int(ch[i]["seq"]))] for i in range(n)]
    dup = [key[i] != i for i in range(n)]
    # content check: skip docs with mismatched dups
    if any(dup[i] and ch[i]["content_id"] != ch[key[i]]["content_id"] for i in range(n)): continue
    dall = []; never = []
    for i in range(n):
        a, s = int(ch[i]["actor"]), int(ch[i]["seq"])
        m = 0; nv = False
        deps = b.deps[int(ch[i]["dep_off"]): int(ch[i]["dep_off"]) + int(ch[i]["n_deps"])]
        for dp in deps:
            da, ds = int(dp["actor"]), int(dp["seq"])
            if da == a or ds == 0: continue
            if (da, ds) in first: m |= 1 << first[(da, ds)]
            else: nv = True
        if s > 1:
            if (a, s - 1) in first: m |= 1 << first[(a, s - 1)]
            else: nv = True
        dall.append(m); never.append(nv)
    hist = [-1] * n; H = 0; applied = 0; queue = 0
    for i in range(n):
        queue |= 1 << i
        P = (1 << i) if (not never[i] and (dall[i] & ~applied) == 0) else 0
        while P:
            ap = 0; keys = 0
            for q in range(n):
                if not (P >> q) & 1: continue
                if not ((applied | keys) >> key[q]) & 1:
                    ap |= 1 << q; keys |= 1 << key[q]
            for q in range(n):
                if (P >> q) & 1:
                    hist[q] = H + bin(ap & ((1 << q) - 1)).count("1") if (ap >> q) & 1 else -2
            H += bin(ap).count("1"); applied |= keys; queue &= ~P
            np_ = 0
            while True:
                nx = 0
                for q in range(n):
                    if not (queue >> q) & 1 or never[q]: continue
                    kb = 0
                    for l in range(q):
                        if (np_ >> l) & 1: kb |= 1 << key[l]
                    if (dall[q] & ~applied & ~kb) == 0: nx |= 1 << q
                if nx == np_: break
                np_ = nx
            P = np_
    want = list(o.hist[c0:c0+n])
    if hist != want:
        bad += 1
        if bad <= 2:
            print("doc", d, "n", n)
            print(" got ", hist)
            print(" want", want)
            print(" dup ", [i for i in range(n) if dup[i]])
print("bad docs", bad)
