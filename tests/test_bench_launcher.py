"""CPU tests of bench.py's rank plumbing: --gpus N without a launcher spawns N ranks with the
environment torch.distributed.run would give them, a launcher's WORLD_SIZE must equal --gpus, and one failing rank
makes the whole command fail.  The ranks here run bench.py's --launcher-selftest, which touches no GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_resolve_world():
    assert bench.resolve_world(None, {}) == ("single", 1)
    assert bench.resolve_world(1, {}) == ("single", 1)
    assert bench.resolve_world(4, {}) == ("spawn", 4)
    assert bench.resolve_world(None, {"WORLD_SIZE": "8"}) == ("rank", 8)
    assert bench.resolve_world(8, {"WORLD_SIZE": "8"}) == ("rank", 8)
    assert bench.resolve_world(1, {"WORLD_SIZE": "1"}) == ("single", 1)
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {"WORLD_SIZE": "2"})  # a launcher's world must match --gpus
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})


def test_rank_envs():
    envs = bench.rank_envs(3, 29511, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["PATH"] == "/bin"


def _run(tmp_path, args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["NFFT4GP_BENCH_SELFTEST_DIR"] = str(tmp_path)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_spawn_two_ranks(tmp_path):
    r = _run(tmp_path, ["--gpus", "2", "--launcher-selftest", "--steps", "7"])
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])  # rank 0's line only
    assert line == {"selftest": True, "world": 2}
    recs = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(2)]
    assert [x["RANK"] for x in recs] == ["0", "1"]
    assert recs[0]["MASTER_PORT"] == recs[1]["MASTER_PORT"]
    for x in recs:
        assert x["WORLD_SIZE"] == "2" and x["MASTER_ADDR"] == "127.0.0.1"
        assert x["argv"] == ["--gpus", "2", "--launcher-selftest", "--steps", "7"]


def test_failing_rank_fails_the_command(tmp_path):
    r = _run(tmp_path, ["--gpus", "3", "--launcher-selftest", "--launcher-selftest-fail-rank", "1"])
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr


def test_launcher_world_mismatch_is_refused(tmp_path):
    r = _run(tmp_path, ["--gpus", "4", "--launcher-selftest"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "must agree" in r.stderr
