"""Golden rounds for the ClockStore persistence batch,
generated in THIS container by executing the reference's own ClockStore SQL in Python's sqlite3
(the statements are read at generation time from /root/reference/dist/ClockStore.js and the
schema from /root/reference/src/migrations/0001_initial_schema.sql — nothing is copied).

Seeded rounds of ClockStore.update / set calls (the JS glue of src/ClockStore.ts:54-112 restated
as in gen_clockstore_vectors.py); after every round the whole Clocks table in primary-key order.
tests/test_node_host.py hands the same rounds to the JS ClockStore, replays each round's
takeBatch() rows in one sqlite3 transaction and compares the table with these.
Usage:  python tools/golden/gen_clockstore_batches.py > tests/golden/clockstore_batches.json
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


SQL_INSERT, SQL_DELETE = sql_of("preparedInsert"), sql_of("preparedDelete")
db = sqlite3.connect(":memory:")
db.executescript(schema)
rng = random.Random(0xBA7C)
actors = ["aa", "bb", "Cc", "dd", "ée", "ff"]
rounds, tables = [], []
for r in range(40):
    calls = []
    for _ in range(rng.randint(1, 12)):
        repo, doc = rng.choice(["self", "peerA", "peerB"]), rng.choice(["d0", "d1", "d2", "d3", "d4"])
        kind = "set" if rng.random() < 0.1 else "update"
        clock = [[a, rng.randint(0, 9)] for a in rng.sample(actors, rng.randint(0, 5))]
        calls.append([kind, repo, doc, clock])
        with db:
            if kind == "set":
                db.execute(SQL_DELETE, (repo, doc))
            for a, s in clock:
                db.execute(SQL_INSERT, (repo, doc, a, s))
    rounds.append(calls)
    tables.append([list(x) for x in db.execute(
        "SELECT repoId, documentId, actorId, seq FROM Clocks ORDER BY repoId, documentId, actorId").fetchall()])
docs = sorted({(c[1], c[2]) for rd in rounds for c in rd})
print(json.dumps({"generator": "tools/golden/gen_clockstore_batches.py", "sqlite": sqlite3.sqlite_version,
                  "rounds": rounds, "tables": tables, "docs": [list(d) for d in docs]}, ensure_ascii=False))
