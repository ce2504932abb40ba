"""The reference tests' document-level expectations (tests/golden/repo_scenarios.json:
tests/repo.test.ts merge / fork, tests/multiple-repos.test.ts two-repo share and the
three-way minimumClock gate) replayed over the restated RepoBackend / DocBackend host logic
with the CPU restatement of Automerge as the merge — pinning the oracle against expected
documents the reference's own tests hold.  The GPU drop-in replays the same scenarios
(tests/test_node_gpu.py::test_repo_scenarios_on_gpu)."""
import json
import os

import pytest

from repo_harness import World, oracle_backend

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "repo_scenarios.json")))


@pytest.mark.parametrize("name", sorted(GOLD["scenarios"]))
def test_reference_scenarios_on_oracle(name):
    sc = GOLD["scenarios"][name]
    merge, render = oracle_backend()
    got = World(merge, render).run(sc["steps"], GOLD["INF"])
    for key, want in sc["renders"].items():
        assert got[key] == want, (name, key, got[key])
