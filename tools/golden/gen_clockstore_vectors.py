"""Golden vectors for ClockStore (SURVEY.md §8c, Appendix C "ClockStore"), generated
in THIS container by executing the reference's own SQL in Python's sqlite3 3.37
(better-sqlite3 is absent; the statements are read at generation time from
/root/reference/dist/ClockStore.js and the schema from
/root/reference/src/migrations/0001_initial_schema.sql — nothing is copied).

The JS glue around the SQL (src/ClockStore.ts:54-112) is restated here:
  update: for [actor, seq] of Object.entries(clock): INSERT ... ON CONFLICT DO UPDATE
          SET seq=excluded.seq WHERE excluded.seq > seq; stored = get();
          push updateQ iff !Clock.equal(clock, stored)   (zero == missing)
  set:    DELETE rows of (repo, doc), then update
  get:    rows of SELECT * ... reduced into {actorId: seq} in row order
Output: tests/golden/clockstore_vectors.json
Usage:  python tools/golden/gen_clockstore_vectors.py > tests/golden/clockstore_vectors.json
"""
import json
import random
import re
import sqlite3

REF = "/root/reference"
js = open(f"{REF}/dist/ClockStore.js").read()
schema = open(f"{REF}/src/migrations/0001_initial_schema.sql").read()


def sql_of(field):
    m = re.search(r"this\.%s = this\.db\s*\.prepare\((['`])(.*?)\1\)" % field, js, re.S)
    return m.group(2)


SQL_GET, SQL_INSERT, SQL_DELETE = sql_of("preparedGet"), sql_of("preparedInsert"), sql_of("preparedDelete")
SQL_REPOS, SQL_DOCS = sql_of("preparedAllRepoIds"), sql_of("preparedAllDocumentIds")


def gte(a, b):
    return all(v >= (b.get(k) or 0) for k, v in a.items()) and all(v <= (a.get(k) or 0) for k, v in b.items())


def equal(a, b):
    return gte(a, b) and gte(b, a)


class Store:
    def __init__(self):
        self.db = sqlite3.connect(":memory:")
        self.db.executescript(schema)

    def get(self, repo, doc):
        return [[r[2], r[3]] for r in self.db.execute(SQL_GET, (repo, doc)).fetchall()]

    def update(self, repo, doc, clock):
        with self.db:
            for a, s in clock:
                self.db.execute(SQL_INSERT, (repo, doc, a, s))
        stored = self.get(repo, doc)
        return stored, not equal(dict(clock), dict(stored))

    def set(self, repo, doc, clock):
        with self.db:
            self.db.execute(SQL_DELETE, (repo, doc))
        return self.update(repo, doc, clock)


def run(ops):
    st = Store()
    out = []
    for op in ops:
        kind = op[0]
        if kind in ("update", "set"):
            stored, pushed = getattr(st, kind)(op[1], op[2], op[3])
            out.append({"stored": stored, "pushed": pushed})
        elif kind == "get":
            out.append({"clock": st.get(op[1], op[2])})
        elif kind == "repos":
            out.append({"ids": sorted(r[0] for r in st.db.execute(SQL_REPOS))})
        elif kind == "docs":
            out.append({"ids": sorted(r[0] for r in st.db.execute(SQL_DOCS, (op[1],)))})
    return out


R, R2, D, D2 = "repoId", "repoId2", "abc123", "ghi789"
c1 = [["abc123", 1], ["def456", 0]]
CASES = {
    # tests/ClockStore.test.ts:7-129
    "read_and_write": [("update", R, D, c1), ("get", R, D)],
    "upsert": [("update", R, D, c1), ("update", R, D, [["abc123", 2], ["def456", 0]]), ("get", R, D)],
    "set": [("set", R, D, c1), ("set", R, D, [["abc123", 2]]), ("get", R, D)],
    "get_multiple": [("update", R, D, c1), ("update", R, D2, [["ghi789", 2], ["jkl012", 0]]), ("get", R, D), ("get", R, D2)],
    "multiple_repos_get": [("update", R, D, c1), ("update", R, D2, [["ghi789", 2], ["jkl012", 0]]),
                           ("update", R2, D, [["abc123", 1], ["def456", 1]]), ("get", R2, D), ("get", R, D), ("get", R, D2)],
    "multiple_repos_update": [("update", R, D, c1), ("update", R2, D, [["abc123", 1], ["def456", 1]]),
                              ("update", R, D, [["abc123", 2], ["def456", 0]]), ("get", R, D), ("get", R2, D),
                              ("repos",), ("docs", R)],
    # Appendix C extras: a decreasing seq is a no-op; updateQ is pushed when the store held more
    "decreasing_seq_noop": [("update", R, D, [["a", 5]]), ("update", R, D, [["a", 3]]), ("get", R, D)],
    "push_rule": [("update", R, D, [["a", 2], ["b", 1]]), ("update", R, D, [["a", 2]]), ("update", R, D, [["a", 3], ["b", 1]]),
                  ("update", R, D, [["b", 0]]), ("update", R, D, [])],
}

rng = random.Random(0xC10C)
rand_ops = []
actors = ["aa", "bb", "Cc", "dd", "ée"]
for _ in range(400):
    k = rng.random()
    repo, doc = rng.choice([R, R2, "peer3"]), rng.choice(["d0", "d1", "d2", "d3"])
    if k < 0.75:
        clock = [[a, rng.randint(0, 6)] for a in rng.sample(actors, rng.randint(0, 4))]
        rand_ops.append(("update", repo, doc, clock))
    elif k < 0.85:
        clock = [[a, rng.randint(0, 6)] for a in rng.sample(actors, rng.randint(0, 3))]
        rand_ops.append(("set", repo, doc, clock))
    else:
        rand_ops.append(("get", repo, doc))
CASES["random_sequence"] = rand_ops

out = {"generator": "tools/golden/gen_clockstore_vectors.py", "sqlite": sqlite3.sqlite_version,
       "cases": {name: {"ops": [list(o) for o in ops], "results": run(ops)} for name, ops in CASES.items()}}
print(json.dumps(out, ensure_ascii=False))
