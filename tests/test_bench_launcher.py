"""bench.py's rank launcher on the CPU (no GPU): ``--gpus N`` outside torchrun starts N rank processes with
torchrun's environment before anything imports libmvtv, and fails when a rank fails (ending its peers)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_launcher_gives_each_rank_torchrun_env():
    r = _run("--gpus", "4", "--dry-run")
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(int(x["env"]["RANK"]) for x in lines) == [0, 1, 2, 3]
    for x in lines:
        e = x["env"]
        assert e["LOCAL_RANK"] == e["RANK"] and e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1"
        assert not x["mv_imported"] and x["mode"] == "auto"
    assert len({x["env"]["MASTER_PORT"] for x in lines}) == 1


def test_launcher_fails_when_a_rank_fails_and_ends_the_others():
    t0 = time.time()
    r = _run("--gpus", "3", "--dry-run", "--dry-run-fail-rank", "2")
    assert r.returncode == 3
    assert "ending the others" in r.stderr
    assert time.time() - t0 < 50   # the healthy ranks (sleeping 60 s) were ended, not waited for


def test_one_gpu_runs_in_process():
    r = _run("--gpus", "1", "--dry-run")
    assert r.returncode == 0
    x = json.loads(r.stdout.strip().splitlines()[-1])
    assert x["env"]["RANK"] is None and x["env"]["WORLD_SIZE"] is None
