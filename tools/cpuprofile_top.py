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

# callers of the native frames among the top entries (a ":-1" frame is a builtin or an addon
# function: its caller names it)
parent = {}
for n in p["nodes"]:
    for c in n.get("children", []):
        parent[c] = n["id"]
by_caller = collections.Counter()
for sid, d in zip(p.get("samples", []), dt):
    n = nodes[sid]["callFrame"]
    if n["url"] or n["functionName"].startswith("("):
        continue
    q = nodes.get(parent.get(sid))
    cf = q["callFrame"] if q else {"functionName": "-", "url": "", "lineNumber": -1}
    by_caller[(n["functionName"], cf["functionName"] or "(anon)", cf["url"].split("/")[-1], cf["lineNumber"])] += d
if by_caller:
    print("native frames by caller:")
    for (f, cfn, u, l), t in by_caller.most_common(12):
        print(f"{100 * t / tot:5.1f}% {t / 1e3:8.1f} ms  {f} <- {cfn} {u}:{l}")
