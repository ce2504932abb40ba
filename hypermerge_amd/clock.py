"""Vector-clock algebra with the reference's exact semantics (src/Clock.ts).

Clocks are ``{actorId: seq}`` dicts; a missing entry counts as 0, so
``{x: 0}`` equals ``{}`` under gte/cmp/equal (src/Clock.ts:13-21), while
``equivalent`` compares entries literally (src/Clock.ts:78-85).  ``union``
keeps key order "c1's keys, then c2's new keys" like the JS object spread.

``to_dense``/``from_dense`` move clocks to the engine's dense per-document
rows (``a_stride`` wide, actor *rank* order, 0 == absent), which is what the
GPU clock kernels (hm_clock_*_device) operate on.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Sequence, Union

Clock = Dict[str, float]
INF = math.inf


def gte(a: Clock, b: Clock) -> bool:
    """src/Clock.ts:13-21"""
    for k, v in a.items():
        if v < (b.get(k) or 0):
            return False
    for k, v in b.items():
        if v > (a.get(k) or 0):
            return False
    return True


def cmp(a: Clock, b: Clock) -> str:
    """src/Clock.ts:27-38 -> 'EQ' | 'GT' | 'LT' | 'CONCUR'"""
    ag, bg = gte(a, b), gte(b, a)
    if ag and bg:
        return "EQ"
    if ag:
        return "GT"
    if bg:
        return "LT"
    return "CONCUR"


def equal(a: Clock, b: Clock) -> bool:
    """src/Clock.ts:23-25"""
    return cmp(a, b) == "EQ"


def equivalent(a: Clock, b: Clock) -> bool:
    """src/Clock.ts:78-85: literal entry comparison (undefined != 0)"""
    for k in set(a) | set(b):
        if a.get(k) != b.get(k):
            return False
    return True


def union(c1: Clock, c2: Clock) -> Clock:
    """src/Clock.ts:87-95: elementwise max, c1 key order then new c2 keys"""
    acc = dict(c1)
    for k, v in c2.items():
        acc[k] = max(acc.get(k) or 0, v)
    return acc


def add_to(acc: Clock, clock: Clock) -> None:
    """src/Clock.ts:97-101"""
    for k, v in clock.items():
        acc[k] = max(acc.get(k) or 0, v)


def intersection(c1: Clock, c2: Clock) -> Clock:
    """src/Clock.ts:103-113: elementwise min over both key sets, zeros dropped"""
    out: Clock = {}
    keys: List[str] = list(dict.fromkeys(list(c1) + list(c2)))
    for k in keys:
        v = min(c1.get(k) or 0, c2.get(k) or 0)
        if v > 0:
            out[k] = v
    return out


def strs2clock(inp: Union[str, Sequence[str]]) -> Clock:
    """src/Clock.ts:40-53"""
    if isinstance(inp, str):
        return {inp: INF}
    out: Clock = {}
    for s in inp:
        parts = s.split(":")
        ident, mx = parts[0], (parts[1] if len(parts) > 1 else "")
        out[ident] = _parse_int(mx) if mx else INF
    return out


def _parse_int(s: str) -> float:
    # JS parseInt: leading integer prefix, NaN if none
    i, sign = 0, 1
    s = s.strip()
    if s[:1] in "+-":
        sign = -1 if s[0] == "-" else 1
        i = 1
    j = i
    while j < len(s) and s[j].isdigit():
        j += 1
    return sign * int(s[i:j]) if j > i else math.nan


def clock2strs(clock: Clock) -> List[str]:
    """src/Clock.ts:55-66"""
    out = []
    for k, v in clock.items():
        out.append(k if v == INF else f"{k}:{_num(v)}")
    return out


def _num(v: float) -> str:
    return str(int(v)) if float(v).is_integer() else repr(v)


def actors(clock: Clock) -> List[str]:
    """src/Clock.ts:9-11"""
    return list(clock.keys())


CMP_CODES = {"EQ": 0, "GT": 1, "LT": 2, "CONCUR": 3}
CMP_NAMES = {v: k for k, v in CMP_CODES.items()}


def to_dense(clock: Clock, ranks: Dict[str, int], a_stride: int, sentinel: int = 0xFFFFFFFF) -> List[int]:
    """Dense row in actor-rank order; Infinity maps to the u32 sentinel."""
    row = [0] * a_stride
    for k, v in clock.items():
        row[ranks[k]] = sentinel if v == INF else int(v)
    return row


def from_dense(row: Iterable[int], actors_by_rank: Sequence[str], sentinel: int = 0xFFFFFFFF) -> Clock:
    out: Clock = {}
    for r, v in enumerate(row):
        if r < len(actors_by_rank) and v:
            out[actors_by_rank[r]] = INF if v == sentinel else int(v)
    return out
