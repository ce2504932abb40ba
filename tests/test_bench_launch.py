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


def test_visible_gpus_reads_env_then_kfd_topology(tmp_path):
    b = _bench()
    assert b.visible_gpus({"HIP_VISIBLE_DEVICES": "0,3"}, sysfs=str(tmp_path)) == 2
    assert b.visible_gpus({"ROCR_VISIBLE_DEVICES": ""}, sysfs=str(tmp_path)) == 0
    for i, simds in enumerate([0, 1024, 1024, 0, 1024]):      # CPU nodes report simd_count 0
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 64\nsimd_count {simds}\nmax_waves_per_simd 8\n")
    assert b.visible_gpus({}, sysfs=str(tmp_path)) == 3
    assert b.visible_gpus({}, sysfs=str(tmp_path / "missing")) == 0


def test_the_launcher_parent_never_imports_torch():
    """--gpus N without a launcher counts devices from the KFD topology before `import torch`."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    code = ("import runpy, sys; sys.argv = ['bench.py', '--gpus', '2']\n"
            "try:\n    runpy.run_path(%r, run_name='__main__')\nexcept SystemExit:\n    pass\n"
            "print('TORCH' if 'torch' in sys.modules else 'NOTORCH')" % os.path.join(ROOT, "bench.py"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert p.stdout.strip().endswith("NOTORCH"), p.stdout + p.stderr


def test_compact_line_from_the_round5_record():
    """The driver parses the last line of the bench's output: the round-5 record (21 KB as one
    line) must compact below 4 KB with the headline, roofline and CPU baseline intact."""
    import json
    b = _bench()
    full = json.load(open(os.path.join(ROOT, "profiles", "r05", "final4", "bench_line.json")))
    full["detail_file"] = "gpurun_out/bench_detail.json"
    s = b.dump_line(full)
    assert len(s) < 2048 and "\n" not in s
    line = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "config", "dtype",
              "roofline", "cpu_baseline", "cpu_parallel", "parity_sample_ok", "clock_exchange", "legs"):
        assert k in line, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert line["roofline"][k] is not None, k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert line["cpu_baseline"][k] is not None, k
    assert abs(line["value"] - full["value"]) / full["value"] < 1e-5
    assert abs(line["roofline"]["frac"] - full["roofline"]["frac"]) < 1e-5
    assert set(line["legs"]) >= {"end_to_end", "from_blocks", "resident_c4", "resident_c3", "resident_c5",
                                 "node", "actor_major"}
    assert line["legs"]["node"]["C2"]["vs_js"] > 1
    assert line["legs"]["resident_c4"]["speedup"] > 1
    # an oversized record still prints a parseable line below the cap
    full["legs_padding"] = "x" * 10
    big = dict(full, resident_incremental=dict(full["resident_incremental"], value=1.0))
    assert len(b.dump_line(big)) < 4096


def test_failed_side_legs_keep_the_headline():
    """A side leg that raises (a Node timeout, a missing tool) is reported as an error in the
    line, and the headline, roofline and the other legs still print."""
    import json
    b = _bench()
    full = json.load(open(os.path.join(ROOT, "profiles", "r05", "final4", "bench_line.json")))
    err = b._side("node legs", lambda: (_ for _ in ()).throw(TimeoutError("node ran 900 s")))
    assert err == {"error": "TimeoutError: node ran 900 s"}
    full["node_docbackend"] = err
    full["resident_incremental_text"] = {"error": "RuntimeError: x"}
    full["from_blocks"] = {"error": "OSError: y"}
    full["arrival_orders"] = {"actor_major": {"error": "MemoryError: z"}}
    line = json.loads(b.dump_line(full))
    assert abs(line["value"] - full["value"]) / full["value"] < 1e-5 and line["roofline"]["frac"] is not None
    assert line["legs"]["node"]["error"].startswith("TimeoutError")
    assert line["legs"]["resident_c3"] == {"error": "RuntimeError: x"}
    assert line["legs"]["from_blocks"] == {"error": "OSError: y"}
    assert line["legs"]["actor_major"] == {"error": "MemoryError: z"}
    assert line["legs"]["resident_c4"]["speedup"] > 1
