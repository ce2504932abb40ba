"""Top self-time functions of a V8 .cpuprofile (node --cpu-prof)."""
import collections
import json
import sys

p = json.load(open(sys.argv[1]))
nodes = {n["id"]: n for n in p["nodes"]}
self_t = collections.Counter()
dt = p.get("timeDeltas", [])
for sid, d in zip(p.get("samples", []), dt):
    n = nodes[sid]["callFrame"]
    self_t[(n["functionName"] or "(anon)", n["url"].split("/")[-1], n["lineNumber"])] += d
tot = sum(self_t.values())
for (f, u, l), t in self_t.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 30):
    print(f"{100 * t / tot:5.1f}% {t / 1e3:8.1f} ms  {f} {u}:{l}")
