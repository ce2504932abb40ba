"""The Node host side (hypermerge_amd/js: N-API addon + GpuDocBackend.js) on the GPU.

DocBackend message traces must equal the golden traces recorded from the reference's
own dist/DocBackend.js (tools/golden/gen_docbackend_traces.js): message order
(RemotePatchMsg before ReadyMsg for changes buffered before init), the DocBackend.clock
quirk (queued changes advance it), minimumClockSatisfied latching, history sizes.
"""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "docbackend_traces.json")))
NODE = shutil.which("node")

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(NODE is None, reason="node not installed")]


def _strip(t):
    # JSON drops undefined fields; compare on the generator's output form
    return json.loads(json.dumps(t))


@pytest.mark.parametrize("mode", ["sync", "batched"])
def test_docbackend_traces_match_reference(mode):
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_scenario.js"), mode],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout.strip().splitlines()[-1])
    assert got.pop("_submits") > 0
    for name, sc in GOLD["scenarios"].items():
        assert _strip(got[name]) == _strip(sc["trace"]), name


@pytest.mark.parametrize("mode", ["batched", "async"])
def test_batched_feed_matches_oracle(mode):
    """Many documents through GpuDocBackend (batched mode, and async mode: hm_batch_wait on the
    store's host thread, completion through a napi_threadsafe_function): init + 3 remote calls
    each; history order, opSet clock/deps and DocBackend.clock equal the oracle's cold merge."""
    import numpy as np
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc, encode
    from hypermerge_amd.render import doc_summary
    import oracle.oracle as O
    b = synth.generate(synth.config("C5", n_docs=300))
    docs = [decode_doc(b, i) for i in range(b.n_docs)]
    rng = np.random.default_rng(11)
    chunked = []
    for chs in docs:
        cuts = sorted(rng.integers(1, len(chs) + 1, size=3))
        chunked.append([chs[:cuts[0]], chs[cuts[0]:cuts[1]], chs[cuts[1]:cuts[2]], chs[cuts[2]:]])
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_feed.js")], input=json.dumps({"docs": chunked, "mode": mode}),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    assert got["clockMismatch"] == 0 and got["gpuPush"] == got["hostPush"]
    assert got["submits"] <= 4 * 2          # one submit per round (init round + remote rounds), not per document
    cold = encode(docs, 8)
    co = O.merge(cold)
    for i, g in enumerate(got["docs"]):
        s = doc_summary(cold, co, i)
        assert s["status"] == "OK"
        assert g["history"] == s["history"], i
        assert g["histLen"] == len(s["history"])
        assert g["clock"] == s["clock"] and g["deps"] == s["deps"], i
        assert g["backendClock"] == s["backend_clock"], i
        assert g["types"][-1] in ("RemotePatchMsg", "ReadyMsg")


@pytest.mark.parametrize("name,n,mode,binary", [("C5", 200, "batched", True), ("C3", 12, "batched", True),
                                                ("C2", 100, "batched", True), ("C5", 200, "async", True),
                                                ("C4", 300, "async", True), ("C5", 200, "async", False),
                                                ("C3", 12, "batched", False)])
def test_patch_diffs_rebuild_the_merged_document(name, n, mode, binary):
    """Applying every patch's diffs in order (a restatement of Frontend.applyPatch's effect,
    src/DocFrontend.ts:162-179) rebuilds exactly the canonical merged document of the oracle's
    cold merge of the same changes — maps, conflicts, counters, links, lists and text."""
    import numpy as np
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc, encode
    from hypermerge_amd.render import doc_summary
    import oracle.oracle as O
    over = {"changes_per_actor": 40} if name == "C3" else {}
    b = synth.generate(synth.config(name, n_docs=n, **over))
    docs = [decode_doc(b, i) for i in range(b.n_docs)]
    rng = np.random.default_rng(23)
    chunked = []
    for chs in docs:
        cuts = sorted(rng.integers(1, len(chs) + 1, size=3))
        chunked.append([chs[:cuts[0]], chs[cuts[0]:cuts[1]], chs[cuts[1]:cuts[2]], chs[cuts[2]:]])
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_patches.js")],
                       input=json.dumps({"docs": chunked, "mode": mode, "binary": binary}),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)["docs"]
    cold = encode(docs, 8)
    co = O.merge(cold)
    for i, g in enumerate(got):
        s = doc_summary(cold, co, i)
        assert s["status"] == "OK"
        assert g["state"] == json.loads(json.dumps(s["state"])), i
        assert g["nDiffs"] > 0 and g["nonEmpty"] > 0
    if name in ("C2", "C4", "C5"):                 # rounds whose changes all applied patch incrementally
        assert sum(g["incremental"] for g in got) > 0


@pytest.mark.parametrize("name,n,mode,binary,order", [("C5", 150, "batched", True, "arrival"),
                                                      ("C5", 150, "async", False, "shuffled"),
                                                      ("C2", 80, "batched", True, "arrival"),
                                                      ("C3", 10, "batched", True, "arrival"),
                                                      ("C3", 10, "async", True, "shuffled"),
                                                      ("C4", 200, "async", True, "shuffled"),
                                                      # every document with its own actors (as hypermerge mints
                                                      # them): past 1024 distinct ids both sides' clocks switch
                                                      # to V8's dictionary form mid-run
                                                      ("C2", 400, "async", True, "unique")])
def test_patch_diff_sequence_equals_js_restatement(name, n, mode, binary, order):
    """f2 / a12: every RemotePatchMsg / ReadyMsg patch of the GPU
    drop-in — clock, deps and the diffs, one per applied op in application order (create,
    map set/remove with conflicts, list insert/set/remove at the index of that moment) — equals
    the JS restatement's patch for the same documents fed in the same chunks, including rounds
    where queued changes apply later (shuffled arrival).  The device's merged registers equal
    the per-op replay's end state (replayMismatch 0).  Automerge's own diff format is unpinned
    (not vendored); the sequence rule is Appendix A.4's."""
    import numpy as np
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc
    over = {"changes_per_actor": 30} if name == "C3" else {}
    b = synth.generate(synth.config(name, n_docs=n, **over))
    docs = [decode_doc(b, i) for i in range(b.n_docs)]
    rng = np.random.default_rng(29)
    if order == "unique":
        def own(c, i):
            r = dict(c, actor=f"{c['actor']}-{i:05d}")
            r["deps"] = {f"{a}-{i:05d}": q for a, q in c["deps"].items()}
            return r
        docs = [[own(c, i) for c in chs] for i, chs in enumerate(docs)]
    chunked = []
    for chs in docs:
        chs = list(chs)
        if order == "shuffled":
            rng.shuffle(chs)
        cuts = sorted(rng.integers(1, len(chs) + 1, size=3))
        chunked.append([chs[:cuts[0]], chs[cuts[0]:cuts[1]], chs[cuts[1]:cuts[2]], chs[cuts[2]:]])
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_patch_seq.js")],
                       input=json.dumps({"docs": chunked, "mode": mode, "binary": binary}),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(p.stdout)
    assert got["stats"]["replayMismatch"] == 0 and got["stats"]["opPatches"] > 0
    assert got["stats"]["dictClocks"] == (order == "unique")
    n_diffs = 0
    for i, d in enumerate(got["docs"]):
        assert len(d["gpu"]) == len(d["cpu"]), i
        for k, (g, c) in enumerate(zip(d["gpu"], d["cpu"])):
            assert g == c, (i, k)
            n_diffs += len(c.get("patch", {}).get("diffs", []))
    assert n_diffs > 0


def test_materialize_history_prefix():
    """MaterializeMsg (src/RepoBackend.ts:570-579): history.slice(0, n) replayed through
    Backend.applyChanges(Backend.init(), ...) — the reference's tests/repo.test.ts:129-164
    expects foo == 'bar1' for the first 2 entries of foo = bar0, bar1, bar2, bar3."""
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_materialize.js")], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout)
    assert got["materialized"] == {"1": "bar0", "2": "bar1", "3": "bar2", "4": "bar3"}
    assert got["history"] == 4 and got["types"] == ["ReadyMsg", "LocalPatchMsg", "LocalPatchMsg", "LocalPatchMsg"]


def test_repo_scenarios_on_gpu():
    """The reference tests' document-level expectations (tests/golden/repo_scenarios.json:
    repo.test.ts merge / fork, multiple-repos.test.ts share and three-way minimumClock gate)
    replayed through the GPU drop-in DocBackend: every watched document renders exactly the
    documents the reference tests expect."""
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "repo_scenarios.json")))
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_repo_scenarios.js")],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout.strip().splitlines()[-1])
    for name, sc in gold["scenarios"].items():
        for key, want in sc["renders"].items():
            assert got[name][key] == want, (name, key, got[name][key])


@pytest.mark.parametrize("devices", [[0, 0], [0]], ids=["two-shards-one-device", "rccl-one-rank"])
def test_sharded_engine_restride_and_clock_exchange(devices):
    """GpuEngine with device shards (FNV-1a64(docId) % G routing) and stride classes: wide
    documents (9-40 actors) move to wider stores as actors arrive; every document's state
    equals the oracle's, and exchangeClocks returns every document's {actorId: seq} clock
    (RCCL over the devices when they are distinct GPUs)."""
    import random
    import oracle.oracle as O
    from hypermerge_amd.columnar import encode
    from hypermerge_amd.render import doc_state
    from repo_harness import plain
    from test_gpu_parity import _float_counter_docs
    rng = random.Random(5)
    docs = {}
    for i, chs in enumerate(_float_counter_docs(40, 99, wide=True) + _float_counter_docs(40, 98)):
        # causal delivery in 1-4 batches (queued changes would stay queued across batches too)
        cuts = sorted(rng.sample(range(1, len(chs)), min(3, len(chs) - 1))) if len(chs) > 1 else []
        parts, prev = [], 0
        for c in cuts + [len(chs)]:
            parts.append(chs[prev:c])
            prev = c
        docs[f"doc{i:03d}-{rng.randrange(10 ** 9)}"] = parts
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_sharding.js"), json.dumps(devices)],
                       input=json.dumps(docs), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(p.stdout.strip().splitlines()[-1])
    assert got["restrides"] > 0
    shards = set()
    for d, parts in docs.items():
        log = [c for part in parts for c in part]
        b = encode([log])
        o = O.merge(b)
        g = got["docs"][d]
        assert g["shard"] == g["expectShard"]
        shards.add(g["shard"])
        assert g["stride"] >= len(b.doc_actors[0])
        assert g["view"] == plain(doc_state(b, o, 0)), d
        clock = {}
        for c in log:
            clock[c["actor"]] = max(clock.get(c["actor"], 0), c["seq"])
        assert g["clock"] == clock
        assert got["exchanged"][d] == clock
    assert shards == set(range(len(devices)))


def test_raw_blocks_and_device_cursors_sync_equal_oracle():
    """RepoBackend.syncChanges (src/RepoBackend.ts:506-531) on the drop-in: the device
    CursorStore picks the documents of each synced actor, the device contiguity scan stops
    each range at the first block not downloaded, and the ranges' raw blocks go to
    DocBackend.applyRemoteBlocks (parsed natively, Actor.parseBlock src/Actor.ts:137-141).
    The plan equals a host restatement of syncChanges, and every document equals the oracle's
    merge of exactly the blocks it received, in delivery order (two sync rounds: with holes in
    the feeds, then complete)."""
    import numpy as np
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc, encode
    from hypermerge_amd.render import doc_summary
    from repo_harness import plain
    from hypermerge_amd.render import doc_state
    import oracle.oracle as O
    b = synth.generate(synth.config("C5", n_docs=40))
    rng = np.random.default_rng(4)
    docs, feeds = {}, {}
    for i in range(b.n_docs):
        chs = decode_doc(b, i)
        actors = sorted({c["actor"] for c in chs})
        docs[f"doc{i:03d}"] = actors
        for a in actors:                      # an actor feed: its changes in seq order (one per block)
            feeds[a] = [json.dumps(c) for c in sorted((c for c in chs if c["actor"] == a), key=lambda c: c["seq"])]
    holes = {a: [int(rng.random() > 0.15) for _ in f] for a, f in feeds.items()}
    present = [holes, {a: [1] * len(f) for a, f in feeds.items()}]
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_sync_blocks.js"), "async"],
                       input=json.dumps({"docs": docs, "feeds": feeds, "present": present}),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(p.stdout)
    # host restatement of syncChanges: per (doc, actor) from doc.changes[actor] to the first hole
    pos = {(d, a): 0 for d, acts in docs.items() for a in acts}
    delivered = {d: [] for d in docs}
    for rnd, pres in enumerate(present):
        want = []
        for d in sorted(docs, key=lambda x: x.encode()):
            for a in sorted(docs[d], key=lambda x: x.encode()):
                lo = pos[(d, a)]
                end = lo
                while end < len(feeds[a]) and pres[a][end]:
                    end += 1
                want.append([d, a, lo, end])
                pos[(d, a)] = end
                delivered[d] += [json.loads(t) for t in feeds[a][lo:end]]
        assert sorted(got["plans"][rnd]) == sorted(want), rnd
    for d in docs:
        log = delivered[d]
        bb = encode([log])
        o = O.merge(bb)
        s = doc_summary(bb, o, 0)
        g = got["docs"][d]
        assert g["history"] == s["history"], d
        assert g["clock"] == s["backend_clock"], d
        assert g["view"] == plain(doc_state(bb, o, 0)), d
        assert g["cursor"] == {a: 9007199254740991 for a in docs[d]}
        assert g["entry"] == [9007199254740991] * len(docs[d])


def test_documents_open_while_an_async_round_is_in_flight():
    """opening documents while an async round runs on the docset's host thread
    is safe (host state only), every other call on the busy device throws instead of racing, and
    all documents come out as the oracle merges them."""
    from hypermerge_amd import synth
    from hypermerge_amd.columnar import decode_doc, encode
    from hypermerge_amd.render import doc_summary
    import oracle.oracle as O
    b = synth.generate(synth.config("C4", n_docs=4000))
    docs = [decode_doc(b, i) for i in range(b.n_docs)]
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_async_open.js")], input=json.dumps({"docs": docs}),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(p.stdout)
    assert got["busyDuring"] and "busy" in (got["busyThrow"] or "")
    cold = encode(docs, 8)
    o = O.merge(cold)
    assert len(got["docs"]) == len(docs)
    for i, g in enumerate(got["docs"]):
        s = doc_summary(cold, o, i)
        assert g["clock"] == s["backend_clock"] and g["hist"] == len(s["history"]) and g["stored"] == s["backend_clock"], i


@pytest.mark.parametrize("mode", ["sync", "batched", "async"])
def test_local_undo_redo_matches_restatement(mode):
    """applyLocalChange with requestType change / undo / redo (src/DocBackend.ts:187-205,
    Automerge's undo stack, SURVEY Appendix A.4 [R]) through the GPU drop-in and through the JS
    restatement: the same messages, canUndo / canRedo on every patch, the same throws ('Cannot
    undo: there is nothing to be undone', 'Cannot redo: ...') and the same document after every
    step, on seeded documents with counters, lists, deletes and concurrent remote sets."""
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "run_undo.js"), mode, "24"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout.strip().splitlines()[-1])
    assert len(got["gpu"]) == len(got["cpu"]) == 24
    undos = redos = throws = 0
    for d, (g, c) in enumerate(zip(got["gpu"], got["cpu"])):
        assert g["trace"] == c["trace"], d
        assert g["msgs"] == c["msgs"], d
        for kind, err, _ in c["trace"]:
            throws += err is not None
        undos += sum(1 for m in c["msgs"] if m[0] == "LocalPatchMsg" and m[3])
        redos += sum(1 for m in c["msgs"] if m[0] == "LocalPatchMsg" and m[2])
    assert throws > 0 and undos > 0 and redos > 0, (throws, undos, redos)
