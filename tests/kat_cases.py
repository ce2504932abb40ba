"""Known-answer documents for the Automerge 0.12 rules.

There is no executable Automerge 0.12 here: each expectation
below is derived by hand from the rule it names (Appendix A), so these cases
PIN the oracle's restatement of those rules — they are not reference output.
Each case: (name, changes, expectation dict checked against the canonical
summary of hypermerge_amd.render.doc_summary).
"""
from hypermerge_amd.columnar import ROOT_ID as R


def ch(actor, seq, deps, *ops, **extra):
    c = {"actor": actor, "seq": seq, "deps": deps, "ops": list(ops)}
    c.update(extra)
    return c


def s(key, value, obj=R, **kw):
    o = {"action": "set", "obj": obj, "key": key, "value": value}
    o.update(kw)
    return o


def d(key, obj=R):
    return {"action": "del", "obj": obj, "key": key}


def inc(key, value, obj=R):
    return {"action": "inc", "obj": obj, "key": key, "value": value}


def mk(kind, obj):
    return {"action": kind, "obj": obj}


def link(key, child, obj=R):
    return {"action": "link", "obj": obj, "key": key, "value": child}


def ins(obj, after, elem):
    return {"action": "ins", "obj": obj, "key": after, "elem": elem}


A, B, Cc, D = "aaaa", "bbbb", "cccc", "dddd"

CASES = [
    # A.2: concurrent sets -> winner is the higher actor string, one conflict
    ("concurrent_set", [ch(A, 1, {}, s("x", 1)), ch(B, 1, {}, s("x", 2))],
     {"state": {"map": [["x", {"value": 2, "conflicts": [[A, 1]]}]]},
      "deps": {A: 1, B: 1}, "history": [[A, 1], [B, 1]]}),
    # A.2: causal overwrite -> no conflict
    ("causal_overwrite", [ch(B, 1, {}, s("x", 2)), ch(A, 1, {B: 1}, s("x", 1))],
     {"state": {"map": [["x", {"value": 1}]]}, "deps": {A: 1}}),
    # A.2: set || del -> the set survives
    ("set_concurrent_del", [ch(A, 1, {}, s("x", 1)), ch(B, 1, {}, d("x"))],
     {"state": {"map": [["x", {"value": 1}]]}}),
    # A.2: causal del removes
    ("causal_del", [ch(A, 1, {}, s("x", 1)), ch(B, 1, {A: 1}, d("x"))],
     {"state": {"map": []}}),
    # A.1 consequence: ops of one change are concurrent -> set then del in the same change keeps the set
    ("same_change_set_del", [ch(A, 1, {}, s("x", 1), d("x"))],
     {"state": {"map": [["x", {"value": 1}]]}}),
    # counters: inc after a causally-prior counter set adds; a concurrent inc does not
    ("counter_causal", [ch(A, 1, {}, s("n", 10, datatype="counter")), ch(B, 1, {A: 1}, inc("n", 5)),
                        ch(A, 2, {B: 1}, inc("n", -2))],
     {"state": {"map": [["n", {"value": 13, "datatype": "counter"}]]}}),
    ("counter_concurrent_inc", [ch(A, 1, {}, s("n", 10, datatype="counter")), ch(B, 1, {}, inc("n", 5))],
     {"state": {"map": [["n", {"value": 10, "datatype": "counter"}]]}}),
    ("counter_concurrent_sets", [ch(A, 1, {}, s("n", 1, datatype="counter")), ch(B, 1, {}, s("n", 100, datatype="counter")),
                                 ch(Cc, 1, {A: 1, B: 1}, inc("n", 7))],
     {"state": {"map": [["n", {"value": 107, "datatype": "counter", "conflicts": [[A, 8]]}]]}}),
    # non-integral counters: JS adds doubles, in the order the incs are applied
    # (0.1 + 0.2) + 0.3 = 0.6000000000000001, not 0.1 + (0.2 + 0.3) = 0.6
    ("counter_float_order", [ch(A, 1, {}, s("n", 0.1, datatype="counter")), ch(B, 1, {A: 1}, inc("n", 0.2)),
                             ch(A, 2, {B: 1}, inc("n", 0.3))],
     {"state": {"map": [["n", {"value": (0.1 + 0.2) + 0.3, "datatype": "counter"}]]}}),
    # history order, not arrival order: B1 waits for A2, so 0.3 is applied before 0.2
    ("counter_float_history_order", [ch(B, 1, {A: 2}, inc("n", 0.2)), ch(A, 1, {}, s("n", 0.1, datatype="counter")),
                                     ch(A, 2, {A: 1}, inc("n", 0.3))],
     {"state": {"map": [["n", {"value": (0.1 + 0.3) + 0.2, "datatype": "counter"}]]},
      "history": [[A, 1], [A, 2], [B, 1]]}),
    # integer adds stay exact until the first non-integral operand
    ("counter_int_then_float", [ch(A, 1, {}, s("n", 1, datatype="counter")), ch(A, 2, {}, inc("n", 2)),
                                ch(B, 1, {A: 2}, inc("n", 0.5))],
     {"state": {"map": [["n", {"value": 3.5, "datatype": "counter"}]]}}),
    # a concurrent non-integral inc does not touch the counter
    ("counter_float_concurrent", [ch(A, 1, {}, s("n", 2.5, datatype="counter")), ch(B, 1, {}, inc("n", 0.25)),
                                  ch(A, 2, {A: 1}, inc("n", 1))],
     {"state": {"map": [["n", {"value": 3.5, "datatype": "counter"}]]}}),
    # 40 actors setting one key concurrently: winner = highest actor string, 39 conflicts in
    # actor-descending order (wide documents: no actor limit in the reference)
    ("forty_actors_concurrent", [ch(f"w{i:02d}", 1, {}, s("x", i)) for i in range(40)],
     {"state": {"map": [["x", {"value": 39, "conflicts": [[f"w{i:02d}", i] for i in range(38, -1, -1)]}]]}}),
    # ... and a 40-actor causal chain: each actor overwrites the previous one's value
    ("forty_actors_chain", [ch(f"w{i:02d}", 1, ({f"w{i - 1:02d}": 1} if i else {}), s("x", i)) for i in range(40)],
     {"state": {"map": [["x", {"value": 39}]]}, "deps": {"w39": 1}}),
    # ties: one change setting a key twice -> "append, then reverse" after every assign
    ("tie_two_sets", [ch(A, 1, {}, s("x", "first"), s("x", "second"))],
     {"state": {"map": [["x", {"value": "second", "conflicts": [[A, "first"]]}]]}}),
    ("tie_three_sets", [ch(A, 1, {}, s("x", 1), s("x", 2), s("x", 3))],
     {"state": {"map": [["x", {"value": 3, "conflicts": [[A, 1], [A, 2]]}]]}}),
    # a later concurrent assign by a lower actor flips the tie group again
    ("tie_flipped_by_concurrent", [ch(B, 1, {}, s("x", "b1"), s("x", "b2")), ch(A, 1, {}, s("x", "a"))],
     {"state": {"map": [["x", {"value": "b1", "conflicts": [[B, "b2"], [A, "a"]]}]]}}),
    # A.1 pass order: [C1(dep B1), B1(dep A1), D1(dep A1), A1] -> A1, B1, D1, C1
    # (a pass does not restart after an application: C1 waits for the next pass)
    ("blocked_pass_order", [ch(Cc, 1, {B: 1}, s("x", "X")), ch(B, 1, {A: 1}, s("y", "B1")),
                            ch(D, 1, {A: 1}, s("z", "Y")), ch(A, 1, {}, s("w", "A1"))],
     {"history": [[A, 1], [B, 1], [D, 1], [Cc, 1]], "queued": 0}),
    ("blocked_pass_order2", [ch(Cc, 1, {B: 1}, s("x", 1)), ch(B, 1, {A: 1}, s("y", 2)),
                             ch(A, 2, {}, s("v", 3)), ch(Cc, 2, {A: 1}, s("z", 4)), ch(A, 1, {}, s("w", 5))],
     {"history": [[A, 1], [B, 1], [A, 2], [Cc, 1], [Cc, 2]]}),
    # DocBackend.clock includes queued changes (src/DocBackend.ts:135-142); opSet.clock does not
    ("queued_clock_quirk", [ch(A, 1, {}, s("x", 1)), ch(B, 2, {}, s("y", 2))],
     {"clock": {A: 1}, "backend_clock": {A: 1, B: 2}, "queued": 1, "history": [[A, 1]]}),
    # duplicates are no-ops, mismatched duplicates throw
    ("duplicate_noop", [ch(A, 1, {}, s("x", 1)), ch(A, 1, {}, s("x", 1)), ch(A, 2, {}, s("x", 2))],
     {"history": [[A, 1], [A, 2]], "state": {"map": [["x", {"value": 2}]]}}),
    ("duplicate_mismatch", [ch(A, 1, {}, s("x", 1)), ch(A, 1, {}, s("x", 999))],
     {"status": "INCONSISTENT_SEQ", "error_at": [1, 0xFFFFFFFF]}),
    # deps heads
    ("heads", [ch(A, 1, {}, s("x", 1)), ch(B, 1, {}, s("y", 1)), ch(Cc, 1, {A: 1, B: 1}, s("z", 1)),
               ch(A, 2, {}, s("x", 2))],
     {"deps": {A: 2, Cc: 1}, "clock": {A: 2, B: 1, Cc: 1}}),
    # nested objects via makeMap + link
    ("nested_map", [ch(A, 1, {}, mk("makeMap", "m1"), link("child", "m1"), s("k", "v", obj="m1"))],
     {"state": {"map": [["child", {"value": {"map": [["k", {"value": "v"}]]}}]]}}),
    ("link_vs_set", [ch(A, 1, {}, mk("makeMap", "m1"), link("k", "m1")), ch(B, 1, {}, s("k", 5))],
     {"state": {"map": [["k", {"value": 5, "conflicts": [[A, {"map": []}]]}]]}}),
    # errors abort the document's applyChanges
    ("unknown_object", [ch(A, 1, {}, s("x", 1, obj="nope"))], {"status": "UNKNOWN_OBJECT", "error_at": [0, 0]}),
    ("duplicate_object", [ch(A, 1, {}, mk("makeMap", "m1"), mk("makeMap", "m1"))],
     {"status": "DUPLICATE_OBJECT", "error_at": [0, 1]}),
    # A.3 RGA: concurrent inserts after _head with equal elem -> higher actor first
    ("rga_concurrent_head", [ch(A, 1, {}, mk("makeList", "L"), link("l", "L")),
                             ch(A, 2, {}, ins("L", "_head", 1), s(f"{A}:1", "a", obj="L")),
                             ch(B, 1, {A: 1}, ins("L", "_head", 1), s(f"{B}:1", "b", obj="L"))],
     {"state": {"map": [["l", {"value": {"list": [{"value": "b"}, {"value": "a"}]}}]]}}),
    # typing chain
    ("rga_typing", [ch(A, 1, {}, mk("makeText", "T"), link("t", "T"),
                        ins("T", "_head", 1), s(f"{A}:1", "h", obj="T"),
                        ins("T", f"{A}:1", 2), s(f"{A}:2", "i", obj="T"),
                        ins("T", f"{A}:2", 3), s(f"{A}:3", "!", obj="T"))],
     {"state": {"map": [["t", {"value": {"text": [{"value": "h"}, {"value": "i"}, {"value": "!"}]}}]]}}),
    # higher elem sorts first among siblings; deletes hide; a concurrent set revives
    ("rga_delete_revive", [ch(A, 1, {}, mk("makeList", "L"), link("l", "L"),
                               ins("L", "_head", 1), s(f"{A}:1", "x", obj="L"),
                               ins("L", "_head", 2), s(f"{A}:2", "y", obj="L")),
                           ch(A, 2, {}, d(f"{A}:1", obj="L")),
                           ch(B, 1, {A: 1}, s(f"{A}:1", "X", obj="L"))],
     {"state": {"map": [["l", {"value": {"list": [{"value": "y"}, {"value": "X"}]}}]]}}),
    ("rga_duplicate_elem", [ch(A, 1, {}, mk("makeList", "L"), ins("L", "_head", 1), ins("L", "_head", 1))],
     {"status": "DUPLICATE_ELEM", "error_at": [0, 2]}),
    ("rga_missing_elem", [ch(A, 1, {}, mk("makeList", "L"), s(f"{A}:9", "q", obj="L"))],
     {"status": "MISSING_ELEM", "error_at": [0, 1]}),
    # A.3: applyInsert does not look the parent up -- an insert after an element not inserted
    # yet waits in the parent's _following; once the parent arrives, its subtree is in order
    ("rga_insert_before_parent", [ch(A, 1, {}, mk("makeList", "L"), link("l", "L"),
                                     ins("L", f"{A}:1", 2), ins("L", "_head", 1),
                                     s(f"{A}:1", "a", obj="L"), s(f"{A}:2", "b", obj="L"))],
     {"state": {"map": [["l", {"value": {"list": [{"value": "a"}, {"value": "b"}]}}]]}}),
    # ... across changes: B's element arrives after A's insert that names it
    ("rga_parent_from_later_change", [ch(A, 1, {}, mk("makeList", "L"), link("l", "L"), ins("L", f"{B}:1", 1)),
                                      ch(B, 1, {A: 1}, ins("L", "_head", 1), s(f"{B}:1", "x", obj="L"),
                                         s(f"{A}:1", "y", obj="L"))],
     {"state": {"map": [["l", {"value": {"list": [{"value": "x"}, {"value": "y"}]}}]]}}),
    # a set on an element whose chain is incomplete: getPrevious climbs to the missing parent
    ("rga_set_under_missing_parent", [ch(A, 1, {}, mk("makeList", "L"), ins("L", "zzzz:9", 1),
                                         ins("L", f"{A}:1", 2), s(f"{A}:2", "q", obj="L"))],
     {"status": "MISSING_ELEM", "error_at": [0, 3]}),
    # ... the grandparent arrives in a later change, after the set: still a throw
    ("rga_set_before_grandparent", [ch(A, 1, {}, mk("makeList", "L"), ins("L", f"{B}:1", 1),
                                       ins("L", f"{A}:1", 2)),
                                    ch(A, 2, {}, s(f"{A}:2", "q", obj="L")),
                                    ch(B, 1, {A: 2}, ins("L", "_head", 1))],
     {"status": "MISSING_ELEM", "error_at": [1, 0]}),
    # elements never attached to '_head' (a missing parent, or a cycle of inserts) stay hidden;
    # a delete on one is a no-op
    ("rga_detached_elements_hidden", [ch(A, 1, {}, mk("makeList", "L"), link("l", "L"),
                                         ins("L", "zzzz:9", 1), ins("L", f"{A}:3", 2), ins("L", f"{A}:2", 3),
                                         ins("L", "_head", 4), s(f"{A}:4", "v", obj="L"), d(f"{A}:1", obj="L"))],
     {"state": {"map": [["l", {"value": {"list": [{"value": "v"}]}}]]}}),
]


# ---------------------------------------------------------------------------
# Engine-envelope precedence (not Automerge rules; DESIGN.md "Envelope").
# Inserts after elements not yet inserted are Automerge rules now (CASES above);
# these pin that they no longer leave the envelope, and that a set on an
# element of a cycle of inserts (where the reference's getPrevious never
# returns) does.  Malformed rows (ids outside the doc's tables, gaps/overlaps in
# the change->op/dep layout) put the whole document outside, whatever would
# throw first.
# Each case: (name, changes, mutate(batch) or None, expected summary subset).
# ---------------------------------------------------------------------------
def _orphan_reg_in_queued(b):
    # the queued change's op names a register past the doc's table
    b.ops["reg"][len(b.ops) - 1] = int(b.docs["n_regs"][0]) + 5


def _op_gap(b):
    b.changes["n_ops"][0] = 0          # op 0 belongs to no change


def _op_overlap(b):
    b.changes["op_first"][1] = b.changes["op_first"][0]


ENVELOPE_CASES = [
    ("orphan_insert_after_error",
     [ch(A, 1, {}, mk("makeList", "L"), ins("L", "_head", 1), mk("makeMap", "M")),
      ch(A, 2, {}, mk("makeMap", "M")),
      ch(A, 3, {}, ins("L", "zzzz:99", 5))],
     None, {"status": "DUPLICATE_OBJECT", "error_at": [1, 0]}),
    ("orphan_insert_before_error",
     [ch(A, 1, {}, mk("makeList", "L"), ins("L", "zzzz:99", 1)),
      ch(A, 2, {}, mk("makeMap", "M"), mk("makeMap", "M"))],
     None, {"status": "DUPLICATE_OBJECT", "error_at": [1, 1]}),
    ("orphan_insert_then_error_same_change",
     [ch(A, 1, {}, mk("makeList", "L"), ins("L", "zzzz:5", 1), mk("makeList", "L"))],
     None, {"status": "DUPLICATE_OBJECT", "error_at": [0, 2]}),
    ("duplicate_elem_outranks_orphan_on_same_op",
     [ch(A, 1, {}, mk("makeList", "L"), ins("L", "_head", 1)),
      ch(A, 2, {}, ins("L", "zzzz:9", 1))],
     None, {"status": "DUPLICATE_ELEM", "error_at": [1, 0]}),
    ("orphan_insert_ok",
     [ch(A, 1, {}, mk("makeList", "L"), link("l", "L"), ins("L", "zzzz:99", 1), ins("L", "_head", 2),
         s(f"{A}:2", 7, obj="L"))],
     None, {"status": "OK", "state": {"map": [["l", {"value": {"list": [{"value": 7}]}}]]}}),
    ("set_on_insert_cycle",
     [ch(A, 1, {}, mk("makeList", "L"), ins("L", f"{A}:2", 1), ins("L", f"{A}:1", 2),
         s(f"{A}:1", "q", obj="L"))],
     None, {"status": "UNSUPPORTED"}),
    ("malformed_register_in_queued_change",
     [ch(A, 1, {}, s("x", 1)), ch(B, 2, {}, s("y", 2))],
     _orphan_reg_in_queued, {"status": "UNSUPPORTED"}),
    ("malformed_op_gap",
     [ch(A, 1, {}, s("x", 1)), ch(A, 2, {}, s("y", 2))],
     _op_gap, {"status": "UNSUPPORTED"}),
    ("malformed_op_overlap",
     [ch(A, 1, {}, s("x", 1)), ch(A, 2, {}, s("y", 2))],
     _op_overlap, {"status": "UNSUPPORTED"}),
]
