"""The native block decoder (hm_decode_blocks, csrc/decode.cpp) against the Node host's own
encoder (hypermerge_amd/js/columnar.js, tests/js/encode_rows.js): the rows of C2-C5 documents,
packed as the reference packs blocks (src/Block.ts:6-16: raw JSON or 'BR' + brotli), are
byte-identical; any thread count gives the same rows; an undecodable block fails only its
document, as Block.unpack / JSON.parse throw for that block (src/Block.ts:26-27)."""
import base64
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from hypermerge_amd import synth
from hypermerge_amd.columnar import decode_doc, encode
from hypermerge_amd.decode import decode_blocks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
needs_node = pytest.mark.skipif(NODE is None, reason="node not installed")


def _node(script, payload):
    p = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", script)], input=json.dumps(payload),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def _docs(name, n, **kw):
    b = synth.generate(synth.config(name, n_docs=n, **kw), threads=2)
    docs = [decode_doc(b, d) for d in range(b.n_docs)]
    # message / request fields ride along (content identity covers them)
    for i, chs in enumerate(docs):
        if chs and i % 3 == 0:
            chs[0]["message"] = f"edit {i} é☃"
            chs[-1]["requestType"] = "change"
    return docs


def _rows_of(b, d):
    doc = b.docs[d]
    c0, n = int(doc["change_off"]), int(doc["n_changes"])
    ch = b.changes[c0: c0 + n].copy()
    ch["dep_off"] -= doc["dep_off"]
    ch["op_first"] -= doc["op_off"]
    dp = b.deps[int(doc["dep_off"]): int(doc["dep_off"]) + int(doc["n_deps"])]
    op = b.ops[int(doc["op_off"]): int(doc["op_off"]) + int(doc["n_ops"])]
    return ch.tobytes().hex(), dp.tobytes().hex(), op.tobytes().hex()


@needs_node
@pytest.mark.parametrize("name,n,kw,mode", [
    ("C2", 60, {}, "auto"), ("C3", 6, {"changes_per_actor": 60}, "always"), ("C4", 80, {}, "never"),
    ("C5", 60, {}, "auto"),
])
def test_rows_identical_to_node_encoder(name, n, kw, mode):
    docs = _docs(name, n, **kw)
    blocks = _node("pack_blocks.js", {"docs": docs, "brotli": mode})
    raw = [[base64.b64decode(x) for x in d] for d in blocks["docs"]]
    if mode == "always":
        assert all(x[:2] == b"BR" for d in raw for x in d)
    b, status = decode_blocks(raw, threads=4)
    assert (status == 0).all()
    js = _node("encode_rows.js", {"docs": [[chs] for chs in docs]})
    assert b.strings == js["strings"]
    for d in range(len(docs)):
        j = js["docs"][d][0]
        assert _rows_of(b, d) == (j["changes"], j["deps"], j["ops"]), (name, d)
        doc = b.docs[d]
        assert (int(doc["n_actors"]), int(doc["n_regs"]), int(doc["n_objs"]), int(doc["flags"])) == \
            (j["nActors"], j["nRegs"], j["nObjs"], j["flags"])
        assert b.doc_actors[d] == j["actors"]
    # the thread count never changes the rows
    b1, _ = decode_blocks(raw, threads=1)
    for f in ("docs", "changes", "deps", "ops"):
        np.testing.assert_array_equal(getattr(b, f), getattr(b1, f))


def test_merge_semantics_equal_python_encoder():
    """Decoded batches merge (oracle) to the same documents as the Python encoder's."""
    import oracle.oracle as O
    from hypermerge_amd.render import canonical_json
    docs = _docs("C5", 40)
    raw = [[json.dumps(c).encode() for c in d] for d in docs]
    b, status = decode_blocks(raw, a_stride=8)
    e = encode(docs, 8)
    rb, re_ = O.merge(b), O.merge(e)
    for d in range(len(docs)):
        assert canonical_json(b, rb, d) == canonical_json(e, re_, d)


def test_undecodable_blocks_fail_their_document_only():
    good = [json.dumps({"actor": "a", "seq": 1, "deps": {}, "ops": [
        {"action": "set", "obj": "00000000-0000-0000-0000-000000000000", "key": "k", "value": 1}]}).encode()]
    bad_header = [b"XX{}"]                                  # 'fail to unpack blocks - head is ...'
    bad_json = [b'{"actor": "a", "seq": 1,']                # JSON.parse throws
    bad_brotli = [b"BR\x00\x01garbage"]
    b, status = decode_blocks([good, bad_header, good, bad_json, bad_brotli, []])
    assert status.tolist() == [0, 32, 0, 32, 32, 0]
    assert b.docs["n_changes"].tolist() == [1, 0, 1, 0, 0, 0]
    # escapes, surrogate pairs and numbers as JSON.parse reads them
    c = {"actor": "éa\U0001F600", "seq": 1, "deps": {}, "ops": [
        {"action": "set", "obj": "00000000-0000-0000-0000-000000000000", "key": "k\n\"q\"", "value": 1e3},
        {"action": "set", "obj": "00000000-0000-0000-0000-000000000000", "key": "f", "value": -0.5},
        {"action": "set", "obj": "00000000-0000-0000-0000-000000000000", "key": "s", "value": "😀x"}]}
    b, status = decode_blocks([[json.dumps(c).encode()], [json.dumps(c, ensure_ascii=False).encode()]])
    assert status.tolist() == [0, 0]
    assert b.doc_actors[0] == [c["actor"]] == b.doc_actors[1]
    e = encode([[c]])
    np.testing.assert_array_equal(b.ops[:3]["value"], e.ops["value"])
    np.testing.assert_array_equal(b.ops[:3]["vtag"], e.ops["vtag"])
    assert b.strings == ["k\n\"q\"", "f", "s", "\U0001F600x"]


@pytest.mark.parametrize("name,kw", [("C1", {"changes_per_actor": 300}), ("C2", {"n_docs": 150}),
                                     ("C4", {"n_docs": 150}), ("C4", {"n_docs": 150, "arrival": 1})])
def test_synth_blocks_decode_to_the_generated_rows(name, kw):
    """hm_synth_blocks renders a generated batch as JSON blocks; decoding them gives back the
    generator's change and dep rows, and the merged documents (oracle) are the same."""
    import oracle.oracle as O
    from hypermerge_amd.decode import decode_packed
    cfg = synth.config(name, **kw)
    b = synth.generate(cfg, threads=2)
    data, bo, db = synth.blocks(cfg, b)
    d, st = decode_packed(data, bo, db, a_stride=b.a_stride, threads=3, tables=False)
    assert (st == 0).all()
    for f in ("actor", "seq", "n_deps", "n_ops"):
        np.testing.assert_array_equal(d.changes[f], b.changes[f], err_msg=f)

    def classes(bt):                                        # content ids as classes: relabel by first appearance
        out = []
        for doc in bt.docs:
            c = bt.changes["content_id"][int(doc["change_off"]): int(doc["change_off"]) + int(doc["n_changes"])]
            first = {}
            out.extend(first.setdefault(int(x), len(first)) for x in c)
        return out
    assert classes(d) == classes(b)
    np.testing.assert_array_equal(d.deps["actor"], b.deps["actor"])
    np.testing.assert_array_equal(d.deps["seq"], b.deps["seq"])
    np.testing.assert_array_equal(d.ops["action"], b.ops["action"])
    ro, rd = O.merge(b), O.merge(d)
    np.testing.assert_array_equal(ro.docs, rd.docs)
    np.testing.assert_array_equal(ro.clock, rd.clock)
    np.testing.assert_array_equal(ro.hist, rd.hist)


def test_tables_independent_of_thread_count_with_failed_documents():
    """Each decoder thread appends its document range into its own tables and a failed document
    rolls its rows and names back: every table is the same at any thread count (more threads
    than documents included), a failed document keeps only the root object, and elemIds of a
    very long actor id (longer than the per-thread name arena's chunk) are intact."""
    root = "00000000-0000-0000-0000-000000000000"
    long_actor = "L" * 70000

    def change(actor, seq, ops, deps=None):
        return json.dumps({"actor": actor, "seq": seq, "deps": deps or {}, "ops": ops}).encode()

    def text_doc(actor, n):
        obj = "11111111-0000-0000-0000-00000000000%d" % (n % 10)
        ops = [{"action": "makeText", "obj": obj},
               {"action": "link", "obj": root, "key": "t", "value": obj}]
        prev = "_head"
        for i in range(1, n + 1):
            ops.append({"action": "ins", "obj": obj, "key": prev, "elem": i})
            ops.append({"action": "set", "obj": obj, "key": f"{actor}:{i}", "value": f"c{i}"})
            prev = f"{actor}:{i}"
        return [change(actor, 1, ops)]

    docs = []
    for d in range(23):
        if d % 5 == 3:                                    # rows appended, then a bad op in the last change
            docs.append(text_doc(f"a{d}", 4) + [change(f"a{d}", 2, [{"action": "bogus", "obj": root}], {f"a{d}": 1})])
        elif d % 7 == 2:
            docs.append([b'{"actor": "x", "seq": 1,'])   # JSON.parse throws
        elif d == 11:
            docs.append(text_doc(long_actor, 3))
        else:
            docs.append(text_doc(f"a{d}", 1 + d % 4) + [change(f"b{d}", 1, [
                {"action": "set", "obj": root, "key": f"k{d}", "value": f"v{d % 3}"}])])
    ref, st = decode_blocks(docs, threads=1)
    bad = [d for d in range(23) if d % 5 == 3 or d % 7 == 2]
    assert [d for d in range(23) if st[d]] == bad
    for d in bad:
        assert int(ref.docs[d]["n_changes"]) == 0 and int(ref.docs[d]["n_regs"]) == 0
        assert ref.doc_objs[d] == [root] and ref.doc_actors[d] == [] and ref.doc_regs[d] == []
    assert ref.doc_actors[11] == [long_actor]
    assert [t for _, t in ref.doc_regs[11]][:3] == ["t", f"{long_actor}:1", f"{long_actor}:2"]
    for threads in (2, 3, 7, 64):
        b, s = decode_blocks(docs, threads=threads)
        np.testing.assert_array_equal(s, st)
        for f in ("docs", "changes", "deps", "ops"):
            np.testing.assert_array_equal(getattr(b, f), getattr(ref, f), err_msg=f"{f} threads={threads}")
        assert b.strings == ref.strings
        assert b.doc_actors == ref.doc_actors and b.doc_objs == ref.doc_objs and b.doc_regs == ref.doc_regs


def test_reference_jsonbuffer_vectors():
    """Blocks written by the reference's own JsonBuffer.bufferify and their JsonBuffer.parse
    values (tests/golden/jsonbuffer_vectors.json, tools/golden/gen_jsonbuffer_vectors.js over
    dist/JsonBuffer.js): the native decoder's rows encode exactly the reference-parsed changes
    (every value kind: -0, 1e21, 2^53 +- 2, denormals, escapes, surrogate pairs, counters,
    timestamps, lists); blocks JsonBuffer.parse throws on, and blocks whose first two bytes are
    neither '{"' nor 'BR' (Block.unpack's switch, src/Block.ts:20-27), fail their document only."""
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "jsonbuffer_vectors.json")))
    raw = [[base64.b64decode(v["block"]) for v in doc] for doc in gold["valid"]]
    parsed = [[json.loads(v["parsed"]) for v in doc] for doc in gold["valid"]]
    b, status = decode_blocks(raw, threads=2)
    assert (status == 0).all(), status
    for d, chs in enumerate(parsed):
        want = decode_doc(encode([chs]), 0)
        assert decode_doc(b, d) == want, d
    bad = [[base64.b64decode(m["block"])] for m in gold["malformed"]]
    bad += [[base64.b64decode(x)] for x in gold["bad_header"]]
    ok_doc = [base64.b64decode(v["block"]) for v in gold["valid"][1]]
    b2, st2 = decode_blocks(bad + [ok_doc], threads=2)
    assert all(m["throws"] for m in gold["malformed"])
    assert (st2[:-1] != 0).all(), st2
    assert st2[-1] == 0 and decode_doc(b2, len(bad)) == decode_doc(encode([parsed[1]]), 0)
