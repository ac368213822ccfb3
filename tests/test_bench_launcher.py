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


_AGREE = r"""
import os, sys, time
sys.path.insert(0, {root!r})
import bench
D = bench.Dist("gloo")
if D.rank == 1 and {stall}:
    time.sleep(8)            # a peer stuck elsewhere (e.g. inside an RCCL collective) never joins
    print("peer", flush=True)
else:
    t0 = time.time()
    r = D.allreduce_within([float(D.rank + 1)], 3.0)
    print("agreed" if r is not None else "none", r, round(time.time() - t0, 1), flush=True)
"""


def _two_ranks(stall):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", _AGREE.format(root=ROOT, stall=stall)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT))
    return [p.communicate(timeout=120)[0].strip().splitlines()[-1] for p in procs]   # (after gloo's banner)


def test_bounded_agreement_after_a_slab_failure():
    """bench.py's N > 1 fallback: the agreement after a failed slab run gives up after its bound when a peer never
    joins (then the failing rank prints what it has and exits non-zero), and agrees when every rank joins."""
    out = _two_ranks(stall=True)
    assert out[0].startswith("none") and float(out[0].split()[-1]) < 7.0
    out = _two_ranks(stall=False)
    assert out[0].startswith("agreed") and "[2.0]" in out[0]


def test_cpu_baseline_cores_follow_affinity_and_cgroup_quota(monkeypatch):
    """cpu_baseline's threads: the affinity mask capped by cgroup v2 cpu.max (the GPU box grants 16 of 256)."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(bench, "_cgroup_cpu_max", lambda: "1600000 100000")
    assert bench._usable_cores() == 16
    monkeypatch.setattr(bench, "_cgroup_cpu_max", lambda: "max 100000")
    assert bench._usable_cores() == 256
    monkeypatch.setattr(bench, "_cgroup_cpu_max", lambda: None)
    assert bench._usable_cores() == 256
    monkeypatch.setattr(bench, "_cgroup_cpu_max", lambda: "50000 100000")   # half a CPU: at least one thread
    assert bench._usable_cores() == 1
