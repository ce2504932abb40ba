"""syncChanges contiguity on the GPU vs the reference walk (oracle.sync_end,
src/RepoBackend.ts:513-522): holes, empty and inverted ranges, cursors past the
feed's end (INFINITY_SEQ-like), word boundaries."""
import numpy as np
import pytest

from hypermerge_amd.sync import contiguous_ends, pack_feeds
import oracle.oracle as O

pytestmark = pytest.mark.gpu


def test_contiguous_ends_match_reference_walk(engine):
    rng = np.random.default_rng(9)
    feeds = []
    for f in range(300):
        n = int(rng.integers(0, 700))
        p = rng.random(n) < rng.choice([0.9, 0.99, 1.0])
        feeds.append(p)
    feeds.append(np.ones(128, bool))          # exact word multiple, all present
    feeds.append(np.zeros(0, bool))
    pairs = []
    for _ in range(20000):
        f = int(rng.integers(0, len(feeds)))
        n = len(feeds[f])
        lo = int(rng.integers(0, n + 2))
        hi = int(rng.choice([rng.integers(0, n + 70), 2 ** 31 - 1, n, lo]))
        pairs.append((f, lo, hi))
    for f in range(len(feeds)):
        pairs.append((f, 0, 2 ** 31 - 1))
        pairs.append((f, 63, 130))
    feed = np.array([p[0] for p in pairs]); lo = np.array([p[1] for p in pairs]); hi = np.array([p[2] for p in pairs])
    got = contiguous_ends(engine, feeds, feed, lo, hi)
    want = np.array([O.sync_end(feeds[f], l, h) for f, l, h in pairs])
    np.testing.assert_array_equal(got, want)
