"""bench.py --gpus N: the single-node launcher (rank environments, failure handling, device
count check).  Children are stubbed: no process touches a GPU here."""
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class _Proc:
    def __init__(self, code, polls=1):
        self.code, self.polls, self.terminated = code, polls, False

    def poll(self):
        if self.terminated:
            return -15
        self.polls -= 1
        return self.code if self.polls <= 0 else None

    def terminate(self):
        self.terminated = True


def test_ranks_get_the_launcher_environment():
    b = _bench()
    seen = []

    def popen(cmd, env):
        seen.append((cmd, env))
        return _Proc(0)

    rc = b.launch_ranks(4, ["--gpus", "4", "--steps", "3"], visible=8, popen=popen, port=29511)
    assert rc == 0
    assert len(seen) == 4
    for r, (cmd, env) in enumerate(seen):
        assert cmd[0] == sys.executable and cmd[1].endswith("bench.py")
        assert cmd[2:] == ["--gpus", "4", "--steps", "3"]
        assert env["RANK"] == str(r) and env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == "4" and env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29511"


def test_a_failed_rank_fails_the_launch_and_stops_the_others():
    b = _bench()
    procs = [_Proc(0, polls=50), _Proc(3, polls=2), _Proc(0, polls=50)]
    it = iter(procs)
    rc = b.launch_ranks(3, [], visible=3, popen=lambda cmd, env: next(it), port=1)
    assert rc == 3
    assert procs[0].terminated and procs[2].terminated


def test_too_few_devices_starts_nothing():
    b = _bench()
    started = []
    rc = b.launch_ranks(2, [], visible=1, popen=lambda cmd, env: started.append(1), port=1)
    assert rc != 0 and not started


def test_gpus_2_without_two_devices_exits_nonzero():
    """The real script on this (GPU-less) container: --gpus 2 must refuse, not print n_gpus 1."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert "visible GPUs" in p.stderr
    assert '"n_gpus"' not in p.stdout


def test_gpus_disagreeing_with_world_size_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr
