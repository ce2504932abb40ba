"""Replays tests/golden/repo_scenarios.json — the reference tests' document-level
expectations (tests/repo.test.ts, tests/multiple-repos.test.ts) — over a restatement of
the RepoBackend / DocBackend host logic, with the merge done by a pluggable backend (the
CPU oracle here; the GPU engine replays the same scenarios through the Node drop-in,
tests/js/run_repo_scenarios.js).

Restated host logic (reference file:line):
  DocBackend  constructor / init / applyRemoteChanges / applyLocalChange / updateClock /
              updateMinimumClock / testMinimumClockSatisfied   src/DocBackend.ts:46-213
  RepoBackend create :130-140, open :193-211, merge :213-217, loadDocument :238-257,
              initActorFeed :286-293, documentNotify :313-362, CursorMessage :374-428,
              syncChanges :506-531
  CursorStore update (upsert-max), entry, INFINITY_SEQ           src/CursorStore.ts:17,51-79
  ClockStore  update (upsert-max)                                 src/ClockStore.ts:78-91
  DocFrontend renders iff minimumClockSatisfied && diffs.length  src/DocFrontend.ts:157-167
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional

from hypermerge_amd import clock as C

INF = 9007199254740991


class Doc:
    """DocBackend (src/DocBackend.ts) over a merge backend: `merge(log)` -> (rendered doc,
    history size) of applyChanges(Backend.init(), log) (applyChanges is a left fold)."""

    def __init__(self, repo: "Repo", doc_id: str, back: bool):
        self.repo, self.id = repo, doc_id
        self.clock: Dict[str, int] = {}
        self.changes: Dict[str, int] = {}
        self.min_clock: Optional[Dict[str, int]] = None
        self.satisfied = False
        self.log: List[dict] = []
        self.hist = 0
        self.ready = back
        self.pending: List[Callable[[], None]] = []
        if back:
            self.satisfied = True
            self.repo.notify(self, "ReadyMsg", applied=False)

    def _test(self):
        if self.min_clock is not None:
            self.satisfied = C.cmp(self.clock, self.min_clock) in ("GT", "EQ")

    def update_clock(self, changes):
        for c in changes:
            self.clock[c["actor"]] = max(self.clock.get(c["actor"], 0), c["seq"])
        if not self.satisfied:
            self._test()

    def update_min_clock(self, clock):
        if self.satisfied:
            return
        self.min_clock = C.union(clock, self.min_clock or {})
        self._test()

    def _apply(self, changes) -> bool:
        self.log.extend(changes)
        _, h = self.repo.merge(self.log)
        grew = h > self.hist
        self.hist = h
        return grew

    def init(self, changes):
        self._apply(changes)
        self.update_clock(changes)
        self.satisfied = len(changes) > 0
        self.ready = True
        for f in self.pending:
            f()
        self.pending = []
        self.repo.notify(self, "ReadyMsg", applied=False)

    def apply_remote(self, changes):
        grew = self._apply(changes)
        self.update_clock(changes)
        self.repo.notify(self, "RemotePatchMsg", applied=grew)

    def apply_local(self, change):
        grew = self._apply([change])
        self.update_clock([change])
        self.repo.notify(self, "LocalPatchMsg", applied=grew, change=change)


class Repo:
    def __init__(self, world: "World", rid: str):
        self.world, self.id = world, rid
        self.docs: Dict[str, Doc] = {}
        self.feeds: Dict[str, List[dict]] = {}
        self.cursors: Dict[str, Dict[str, int]] = {}
        self.watched: Dict[str, List[Any]] = {}

    def merge(self, log):
        return self.world.merge(log)

    # CursorStore.update: upsert-max, seq bounded to INFINITY_SEQ
    def cursor_update(self, doc, clock):
        cur = self.cursors.setdefault(doc, {})
        for a, s in clock.items():
            s = min(int(s), INF)
            if s > cur.get(a, -1):
                cur[a] = s

    def notify(self, doc: Doc, kind: str, applied: bool, change=None):
        if kind == "LocalPatchMsg":
            self.feeds.setdefault(change["actor"], []).append(change)       # Actor.writeChange
        if kind in ("RemotePatchMsg", "LocalPatchMsg") and doc.satisfied:
            self.world.clocks_update(self.id, doc.id, doc.clock)          # ClockStore.update
        if doc.id in self.watched and kind != "ReadyMsg" and doc.satisfied and applied:
            self.watched[doc.id].append(self.world.render(doc.log))

    def create(self, doc_id, changes):
        d = Doc(self, doc_id, back=True)
        self.docs[doc_id] = d
        self.cursor_update(doc_id, {doc_id: INF})                        # rootActorId(docId)
        for c in changes:
            d.apply_local(c)

    def open(self, doc_id, actor):
        d = Doc(self, doc_id, back=False)
        self.docs[doc_id] = d
        self.cursor_update(doc_id, {doc_id: INF})
        changes = []
        for a in list(self.cursors[doc_id]):                            # loadDocument
            feed = self.feeds.get(a, [])
            sl = feed[: self.cursors[doc_id][a]]
            d.changes[a] = len(sl)
            changes.extend(sl)
        self.cursor_update(doc_id, {actor: INF})                         # initActorFeed
        d.init(changes)

    def watch(self, doc_id):
        d = self.docs[doc_id]
        self.watched[doc_id] = []
        if d.ready and d.satisfied:
            self.watched[doc_id].append(self.world.render(d.log))

    def sync_changes(self, actor):
        feed = self.feeds.get(actor, [])
        for doc_id, cur in self.cursors.items():
            if actor not in cur or doc_id not in self.docs:
                continue
            d = self.docs[doc_id]

            def run(d=d, cur=cur, doc_id=doc_id):
                mx, lo = cur[actor], d.changes.get(actor, 0)
                i, out = lo, []
                while i < mx and i < len(feed):
                    out.append(feed[i])
                    i += 1
                d.changes[actor] = i
                if out:
                    d.apply_remote(out)
            if d.ready:
                run()
            else:
                d.pending.append(run)

    def merge_clock(self, doc_id, clock):
        self.cursor_update(doc_id, clock)
        for a in clock:
            self.sync_changes(a)

    def change(self, doc_id, change):
        self.docs[doc_id].apply_local(change)

    def cursor_message(self, sender: "Repo", doc_id):
        self.world.clocks_update(sender.id, doc_id, self.world.clocks_get(sender.id, doc_id))
        self.cursor_update(doc_id, sender.cursors.get(doc_id, {}))
        d = self.docs.get(doc_id)
        if d is not None:
            d.update_min_clock(self.world.clocks_get(sender.id, doc_id))
        for a in list(sender.cursors.get(doc_id, {})):
            if a in self.feeds:
                self.sync_changes(a)

    def download(self, sender: "Repo", actor):
        self.feeds[actor] = list(sender.feeds.get(actor, []))
        self.sync_changes(actor)


class World:
    """Repos sharing one ClockStore table keyed (repoId, docId), as each repo's SQLite holds
    its own and its peers' rows (src/ClockStore.ts:78-91, src/RepoBackend.ts:402)."""

    def __init__(self, merge: Callable, render: Callable):
        self.merge, self.render = merge, render
        self.repos: Dict[str, Repo] = {}
        self.clocks: Dict[tuple, Dict[str, int]] = {}

    def repo(self, rid):
        if rid not in self.repos:
            self.repos[rid] = Repo(self, rid)
        return self.repos[rid]

    def clocks_update(self, rid, doc, clock):
        cur = self.clocks.setdefault((rid, doc), {})
        for a, s in clock.items():
            if s > cur.get(a, -1):
                cur[a] = s

    def clocks_get(self, rid, doc):
        return dict(self.clocks.get((rid, doc), {}))

    def run(self, steps, inf):
        for st in steps:
            op = st[0]
            if op == "create":
                self.repo(st[1]).create(st[2], st[3])
            elif op == "open":
                self.repo(st[1]).open(st[2], st[3])
            elif op == "watch":
                self.repo(st[1]).watch(st[2])
            elif op == "merge":
                self.repo(st[1]).merge_clock(st[2], st[3])
            elif op == "change":
                self.repo(st[1]).change(st[2], st[3])
            elif op == "cursor_message":
                self.repo(st[2]).cursor_message(self.repo(st[1]), st[3])
            elif op == "download":
                self.repo(st[2]).download(self.repo(st[1]), st[3])
            elif op == "expect_cursor":
                want = {a: (inf if v == "INF" else v) for a, v in st[3].items()}
                got = self.repo(st[1]).cursors.get(st[2], {})
                assert got == want, (st, got)
            elif op == "expect_clockstore":                 # ClockStore.get(repoId, docId)
                got = self.clocks_get(st[1], st[2])
                assert got == st[3], (st, got)
            elif op == "expect_doc_clock":                  # DocBackend.clock
                got = self.repo(st[1]).docs[st[2]].clock
                assert got == st[3], (st, got)
            else:
                raise ValueError(op)
        return {f"{r.id}/{d}": v for r in self.repos.values() for d, v in r.watched.items()}


def plain(state: Any) -> Any:
    """render.doc_state's canonical form -> the plain JS value a frontend materializes."""
    if isinstance(state, dict) and "map" in state:
        return {k: plain(e["value"]) for k, e in state["map"]}
    if isinstance(state, dict) and ("list" in state or "text" in state):
        return [plain(e["value"]) for e in state.get("list", state.get("text", []))]
    return state


def oracle_backend():
    """(merge, render) over the CPU restatement (test infrastructure)."""
    import oracle.oracle as O
    from hypermerge_amd.columnar import encode
    from hypermerge_amd.render import doc_state

    def merge(log):
        b = encode([log])
        r = O.merge(b)
        assert int(r.docs["status"][0]) == 0, r.docs
        return r, int(r.docs["hist_len"][0])

    def render(log):
        b = encode([log])
        r = O.merge(b)
        return plain(doc_state(b, r, 0))
    return merge, render
