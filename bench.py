"""Benchmark: ADMM iterations/s on a 512^3 fp64 mesh (BASELINE.json metric), HIP path on MI355X.

One step = one ADMM iteration of the reference's variant-B admm_update
(rcpp-code/MultivarTV/src/solvers.cpp:110-133) on the synthetic 3D towers
problem of SURVEY §8d: lattice data with mesh == data (O = I), lambda = 1,
rho0 = lambda/5, u0 = 0, theta0 = mean(y), fixed-iteration mode (the stopping
test is evaluated but not acted on), PCG theta-solves warm-started at
rtol 1e-10. Inputs are resident in HBM before timing starts.

Other BASELINE configs: ``--dims 2 --size 1024`` (config 2), ``--dims 3 --size 256`` (config 3),
``--dims 4 --size 128`` (config 5 on one GPU) and ``--mode cv`` (config 4's work item: a CV fold's
warm-started lambda chunk on 2048^2 with a 0/1 fold mask W, so the theta-solve is Jacobi-PCG).

Multi-GPU (one process per GPU; ``--gpus N`` starts the N rank processes itself when it is not run
under torchrun). At N > 1 the headline is the metric's own definition: ONE 512^3 mesh
slab-decomposed over the N GPUs (``scaling: strong``; the whole loop inside libmvtv with RCCL on the
solver stream). Before it every rank also fits its own independent 512^3 mesh (noise seed + rank, the
embarrassingly parallel sharding of the north star); that aggregate is reported beside the headline as
``independent_fits`` (``scaling: weak``). One RCCL per process: torch.distributed runs on gloo (host
barriers, max-over-ranks time, the 128-byte RCCL id; torch's own RCCL is never initialised) and every
device collective goes through libmvtv's communicator (``rccl_ranks`` = its size; ROCm's librccl on
libmvtv's HIP runtime).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

mv = None                  # multivartv_amd, imported by _import_mv() (after the rank launcher)
SEED = towers = None
HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _import_mv():
    """libmvtv is loaded before anything that brings its own HIP runtime; never in the launcher process."""
    global mv, SEED, towers
    import multivartv_amd
    from multivartv_amd import synth
    mv, SEED, towers = multivartv_amd, synth.SEED, synth.towers


def _spawn_ranks(n, argv, dry_run=False):
    """``--gpus N`` (N > 1) outside torchrun: start N rank processes of this script, one per GPU, with the
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* environment torchrun would give them. This process imports
    nothing that touches HIP. Rank 0 inherits stdout (the one JSON line); the other ranks' stdout goes to
    stderr. When a rank fails the others are ended (they would wait for it in a collective) and the launcher
    exits non-zero."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = None if (r == 0 or dry_run) else sys.stderr
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env, stdout=out))
    rc = 0
    while procs:
        time.sleep(0.2)
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                log(f"bench.py launcher: a rank exited with status {code}; ending the others")
                for q in procs:
                    q.send_signal(signal.SIGTERM)
                deadline = time.time() + 30
                for q in procs:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
    return rc


def _dry_run(a):
    """--dry-run (CPU test of the launcher): report the rank plumbing, optionally fail one rank."""
    env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    print(json.dumps({"dry_run": True, "gpus": a.gpus, "mode": a.mode, "env": env,
                      "mv_imported": "multivartv_amd" in sys.modules}), file=OUT, flush=True)
    if a.dry_run_fail_rank >= 0 and int(env["RANK"] or 0) == a.dry_run_fail_rank:
        sys.exit(3)
    if a.dry_run_fail_rank >= 0:
        time.sleep(60)   # a healthy rank waiting for its failed peer: the launcher must end it


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", type=int, default=512, help="mesh points per dimension")
    ap.add_argument("--dims", type=int, default=3)
    ap.add_argument("--lam", type=float, default=1.0)
    ap.add_argument("--pcg-rtol", type=float, default=1e-10)
    ap.add_argument("--solver", choices=["auto", "pcg", "spectral"], default="auto",
                    help="theta-solve: auto = spectral (exact DCT solve) where it applies, else the spectrally "
                         "preconditioned PCG (2-3-5-7 meshes), else Jacobi-PCG; pcg = Jacobi-PCG; "
                         "spectral = the exact solve (--mode cv: the spectrally preconditioned PCG)")
    ap.add_argument("--pcg-steps", type=int, default=10,
                    help="steps of the secondary Jacobi-PCG leg reported beside the main one (0 = skip)")
    ap.add_argument("--mode", choices=["auto", "independent", "slab", "cv"], default="auto",
                    help="auto: N = 1 one fit; N > 1 one mesh slab-decomposed over the GPUs (strong scaling, the "
                         "metric) with the independent fits per GPU (weak scaling) reported beside it. "
                         "independent / slab: only that one")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--mesh", type=str, default="",
                    help="--mode slab: an explicit mesh 'm0,m1,...' instead of size^dims (e.g. 512,512,64: one rank's "
                         "share of 512^3 at 8 GPUs, run at world 1 with MVTV_SLAB_DISTRIBUTED=1)")
    ap.add_argument("--slab-ranks", type=int, default=1,
                    help="--mode slab without torchrun: ranks of an in-process rehearsal on one GPU (1: RCCL, one rank)")
    ap.add_argument("--transport", choices=["auto", "rccl", "ipc"], default="auto",
                    help="slab collectives at N > 1: RCCL (one process per GPU), or ipc (HIP IPC buffers between the "
                         "rank processes, host-synchronous: ranks sharing a GPU); auto = RCCL unless ranks share a "
                         "GPU, and ipc when RCCL has no communicator")
    ap.add_argument("--cpu-planes", type=int, default=0,
                    help="cpu_baseline sample: slowest-dim planes of the mesh (0 = a quarter of them)")
    ap.add_argument("--cpu-full", action="store_true", help="cpu_baseline on the whole mesh (no extrapolation)")
    ap.add_argument("--cv-batch", type=int, default=8,
                    help="--mode cv: work items (fold, lambda chunk) run at once per GPU, one HIP stream each")
    ap.add_argument("--dry-run", action="store_true", help="launcher test: ranks report their env and exit")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    return ap.parse_args()


class Dist:
    """Host-side plumbing of the ranks over torch.distributed on gloo (barriers, max-over-ranks time, the
    RCCL id): no torch RCCL communicator, so the process's one RCCL is libmvtv's."""

    def __init__(self, backend="gloo"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.backend = backend
        # MVTV_DIST_FORCE=1 creates the process group at world size 1 too (rehearsal under torchrun)
        if self.world > 1 or os.environ.get("MVTV_DIST_FORCE") == "1":
            import torch.distributed as dist
            if backend == "nccl":
                import torch
                torch.cuda.set_device(self.local)
            dist.init_process_group(backend)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def allreduce(self, vals, op="max"):
        if not self.dist:
            return list(vals)
        import torch
        t = torch.tensor(list(vals), dtype=torch.float64, device=f"cuda:{torch.cuda.current_device()}"
                         if self.backend == "nccl" else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return t.cpu().tolist()

    def allreduce_within(self, vals, seconds, op="max"):
        """allreduce that gives up after `seconds` (None then): the agreement after a failure, whose peers may be
        stuck in an RCCL collective the failed rank will never join."""
        if not self.dist:
            return list(vals)
        import datetime

        import torch
        t = torch.tensor(list(vals), dtype=torch.float64)
        try:
            w = self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM,
                                     async_op=True)
            if not w.wait(timeout=datetime.timedelta(seconds=seconds)):
                return None
        except Exception:  # noqa: BLE001 (a timed-out or broken group: no agreement)
            return None
        return t.tolist()

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def _edge_blocks_note(tim, dims, N, E):
    """Which blocks of D the fused edge pass streamed: every one, or one per twin group (blocks the S' map gives one
    difference set, with equal weights and state: the same numbers; DESIGN.md §4.2 'Twin blocks')."""
    k = {3: "admm_fused", 4: "admm_fused4"}.get(dims)
    t = tim.get(k) if k else None
    if not t or not t["launches"]:
        return None
    full = 8.0 * ((4.0 if dims == 3 else 5.0) * N + 2.0 * E)
    if t["bytes_per_launch"] >= full * (1 - 1e-12):
        return "all blocks streamed"
    groups = {3: "6 of 7 ({1,2} shares S'={0,2} with {0,2})",
              4: "one per S' group (groups {0,2}, {0,3}, {0,2,3} hold 2, 3 and 2 blocks)"}[dims]
    return (f"twin blocks streamed once: {groups}; the twins' state is filled from their partner when the run "
            f"ends (inside the timed region); bytes_per_launch counts the streamed blocks only")


def load_pmc(name):
    """Per-launch HBM bytes of kernel `name` from the last committed rocprofv3 PMC pass of this code
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py): (bytes, source label) or (None, None)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        meta = d.get("_source", {})
        label = f"profiles/pmc_traffic.json ({meta.get('pass', 'rocprofv3 FETCH_SIZE + WRITE_SIZE')}, {meta.get('date', '?')})"
        return d.get(name), label
    except Exception:
        return None, None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _usable_cores():
    """The CPUs this process can actually use: its affinity mask, capped by the cgroup's CPU-time quota (cpu.max:
    on the GPU box the mask shows all 256 host CPUs while the quota grants 16; 256 OpenMP threads under a 16-CPU
    quota would be throttled, not faster). The baseline's OpenMP threads and scipy.fft workers; os.cpu_count()
    and OMP_NUM_THREADS are reported beside it, not used."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = _cgroup_cpu_max()
    if q:
        quota, _, period = q.partition(" ")
        if quota not in ("", "max") and period:
            n = min(n, max(1, int(float(quota) / float(period))))
    return n


def _cgroup_cpu_max():
    """cgroup v2 cpu.max ('quota period', or 'max period'): a CPU-time cap the affinity mask does not show."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            return f.read().strip()
    except OSError:
        return None


def cpu_baseline(m, lam, pcg_iters, planes, full=False):
    """The CPU oracle on the host cores, one ADMM iteration (variant B) of the same towers problem:
      * spectral (the headline's like-for-like, `value`): oracle/c/mvtv_oracle.c's loop with the exact
        theta-solve by scipy.fft.dctn / idctn, all cores, on the WHOLE mesh up to 2^27 nodes (512^3: ~10 s),
        else on a slab of `planes` of the last dimension with the rate scaled by N_full / N_slab;
      * pcg: the same loop with Jacobi-PCG at the GPU PCG leg's mean iteration count, all cores on the slab
        (or the whole mesh with full=True) and 1 thread on a quarter of that, scaled the same way (labelled)."""
    from oracle import c_oracle
    ncores = _usable_cores()
    deltas = [(1.0 + 2e-4) / v for v in m]
    n_full = float(np.prod(m))

    def timed(sub, fn, threads, **kw):
        y = towers(sub)
        th = np.full(y.size, y.mean())
        u = np.zeros(c_oracle.num_edges(sub))
        c_oracle.set_threads(threads)
        t0 = time.perf_counter()
        fn(sub, y, lam, th, u, lam / 5.0, deltas, fixed_iters=1, **kw)
        return time.perf_counter() - t0, n_full / float(y.size)

    import scipy.fft
    sub_s = list(m) if (full or n_full <= 2.0 ** 27) else list(m[:-1]) + [planes]
    sym = c_oracle.dtd_symbol(sub_s, deltas)                                   # setup, outside the timing
    scipy.fft.dctn(np.zeros([8] * len(m)), type=2, norm="ortho", workers=ncores)   # thread-pool warm-up
    t_spec, sc_spec = timed(sub_s, c_oracle.admm_rcpp_spectral, ncores, workers=ncores, sym=sym)
    del sym
    sub_p = list(m) if full else list(m[:-1]) + [planes]
    t_pcg, sc_pcg = timed(sub_p, c_oracle.admm_rcpp, ncores, pcg_fixed=int(pcg_iters))
    sub1 = sub_p[:-1] + [max(1, sub_p[-1] // 4)]
    t_1, sc_1 = timed(sub1, c_oracle.admm_rcpp, 1, pcg_fixed=int(pcg_iters))
    c_oracle.set_threads(ncores)
    dims = lambda sub: "x".join(map(str, sub))   # noqa: E731
    where_s = "the whole mesh" if sc_spec == 1.0 else f"a {dims(sub_s)} slab, rate scaled by {sc_spec:.0f}"
    return dict(value=1.0 / (t_spec * sc_spec), unit="iters/s", cores=ncores, kind="port",
                cpu_model=_cpu_model(), affinity_cpus=len(os.sched_getaffinity(0)), host_cpus=os.cpu_count(),
                omp_num_threads=os.environ.get("OMP_NUM_THREADS"), cgroup_cpu_max=_cgroup_cpu_max(),
                algorithm="spectral",
                sample=(f"1 ADMM iteration (variant B) of the same towers problem on {where_s}, {ncores} threads: "
                        f"oracle/c/mvtv_oracle.c loop with the exact theta-solve by scipy.fft DCT ({t_spec:.2f} s)"),
                spectral_all_cores=1.0 / (t_spec * sc_spec), spectral_seconds=round(t_spec, 2),
                pcg_all_cores=1.0 / (t_pcg * sc_pcg), pcg_iters=int(pcg_iters), pcg_seconds=round(t_pcg, 2),
                pcg_sample=f"{dims(sub_p)}" + ("" if sc_pcg == 1.0 else f" slab, rate scaled by {sc_pcg:.0f}"),
                pcg_1thread=1.0 / (t_1 * sc_1),
                pcg_1thread_sample=f"{dims(sub1)} slab, {t_1:.1f} s, rate scaled by {sc_1:.0f}")


METRIC = "ADMM iters/sec on 512^3 fp64 mesh; achieved HBM GB/s vs peak at 1/2/4/8 GPUs"


def _roofline(tim):
    """The dominant kernel (by time) of a timing table and its achieved algorithmic GB/s."""
    cand = [k for k in tim if tim[k]["bytes_per_launch"] > 0 and tim[k]["launches"]]
    if not cand:
        return None
    dom = max(cand, key=lambda k: tim[k]["ms"])
    d_avg = tim[dom]["ms"] / tim[dom]["launches"]
    achieved = tim[dom]["bytes_per_launch"] / (d_avg * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
            "bytes_per_launch": tim[dom]["bytes_per_launch"], "avg_launch_ms": round(d_avg, 4)}


def _rccl_comm(D, dev):
    """libmvtv's RCCL communicator over the ranks (the 128-byte id broadcast over gloo)."""
    from multivartv_amd import slab
    return slab.Comm.rccl(dev) if D.dist else slab.Comm.rccl_single(dev)


def _slab_comm(a, D, dev):
    """The slab loop's transport: RCCL (one process per GPU) or the inter-process HIP-IPC group (--transport ipc;
    auto takes it when ranks share a GPU, where RCCL refuses the communicator)."""
    from multivartv_amd import slab
    kind = a.transport
    if kind == "auto":
        shared, = D.allreduce([1.0 if D.world > max(1, mv.device_count()) else 0.0], "max")
        kind = "ipc" if (D.dist and shared) else "rccl"
    return slab.Comm.ipc(dev) if (kind == "ipc" and D.dist) else _rccl_comm(D, dev)


def slab_main(a, D, comm=None):
    """One mesh decomposed over the ranks (the metric at 2/4/8 GPUs): strong scaling.
    Every rank runs the whole ADMM loop inside libmvtv (mvtv_slab_run) with RCCL collectives on its stream.
    World size 1: --slab-ranks R > 1 rehearses an R-rank decomposition on the one GPU with the in-process
    loopback transport; R = 1 runs the slab loop over a one-rank RCCL communicator. Returns rank 0's line."""
    from multivartv_amd import slab
    m = [int(v) for v in a.mesh.split(",")] if a.mesh else [a.size] * a.dims
    lam = a.lam
    deltas = [(1.0 + 2e-4) / v for v in m]
    R = max(1, a.slab_ranks)
    if D.world > 1 or R == 1:
        dev = D.local % max(1, mv.device_count())
        own = comm is None
        if own:
            comm = _slab_comm(a, D, dev)
        b = slab.plane_bounds(m[-1], D.world)
        pl = int(np.prod(m[:-1]))
        y = towers(m, start=int(b[D.rank]) * pl, count=int(b[D.rank + 1] - b[D.rank]) * pl)
        ysum, = D.allreduce([float(y.sum())], "sum")
        S = slab.SlabADMM(m, y, deltas, ysum / float(np.prod(m)), comm, device=dev)
        del y
        if a.warmup > 0:
            S.run(lam, fixed_iters=a.warmup)
        # the value from an event-free region (a rank's ~1 ms iteration at G = 8 runs ~16 launches: per-launch
        # HIP events would cost several %), the per-kernel table from a second region of the same length with them
        D.barrier()
        S.P.timing(False)
        t0 = time.perf_counter()
        st = S.run(lam, fixed_iters=a.steps)   # returns after the stream drained
        t1 = time.perf_counter()
        D.barrier()
        g_elapsed, = D.allreduce([t1 - t0], "max")
        S.P.timing(True)
        t2 = time.perf_counter()
        S.run(lam, fixed_iters=a.steps)
        t3 = time.perf_counter()
        D.barrier()
        tim = S.P.timings()
        S.P.timing(False)
        ev_elapsed, = D.allreduce([t3 - t2], "max")
        nranks = D.world
        rccl_ranks = comm.size if comm.kind == "rccl" else 0
        if comm.kind == "ipc":
            transport = (f"HIP IPC between {D.world} rank processes"
                         + (" on one GPU" if D.world > max(1, mv.device_count()) else "")
                         + ", host-synchronous collectives")
        else:
            transport = "RCCL" if D.world > 1 else "RCCL (one rank)"
        S.close()
        if own:
            comm.close()
    else:
        y = towers(m)
        if a.warmup > 0:
            slab.run_local_group(m, y, deltas, lam, R, fixed_iters=a.warmup)
        t0 = time.perf_counter()
        outs, _ = slab.run_local_group(m, y, deltas, lam, R, fixed_iters=a.steps)
        t1 = time.perf_counter()
        st, tim = outs[0], {}
        transport = f"in-process loopback, {R} ranks on one GPU"
        g_elapsed, nranks, rccl_ranks = t1 - t0, R, 0
        ev_elapsed = None
    per = {k: dict(avg_ms=round(v["ms"] / v["launches"], 4), launches=v["launches"]) for k, v in tim.items()
           if v["launches"]}
    # the line solves cross the ranks (substructured) unless one rank holds the whole lines
    distributed = nranks > 1 or os.environ.get("MVTV_SLAB_DISTRIBUTED", "0") not in ("", "0")
    if D.rank != 0:
        return None
    return {
        "metric": METRIC, "value": round(a.steps / g_elapsed, 4), "unit": "iters/s", "n_gpus": D.world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(g_elapsed / a.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: towers + 0.5 N(0,1) (splitmix64/Box-Muller, seed 0x4D565456), O = I",
        "config": {"workload": f"{len(m)}D {'x'.join(map(str, m))} fp64 mesh-TV ADMM, variant B, lambda={lam}, one mesh "
                               f"slab-decomposed along dim {len(m) - 1} over {nranks} ranks", "mesh": m,
                   "theta_solver": "spectral (local transforms; the last dimension's line solves substructured "
                                   "over the ranks)" if distributed else "spectral (one rank: the whole lines local)",
                   "parallelism": f"slab x{nranks} ({transport}: halo planes, "
                                  f"{'2+2 numbers per line all-to-all, ' if distributed else ''}7-sum all-reduce)"},
        "rccl_ranks": rccl_ranks, "rccl_library": slab.Comm.library() if rccl_ranks else None,
        "transport": transport,
        "roofline": _roofline(tim), "kernels_rank0": per,
        "timing": ("value from an event-free region; kernels_rank0 / roofline from a second region of the same "
                   f"length with per-launch HIP events ({a.steps / ev_elapsed:.2f} it/s with them)")
        if ev_elapsed else "no per-kernel events (in-process ranks)",
        "residuals": {"r_norm": st["r_norm"], "s_norm": st["s_norm"]}, "cpu_baseline": None}


def cv_main(a, D):
    """Config 4's work items (BASELINE.json: 2D 2048^2, 32-lambda CV path batched over 8 GPUs): CV fold paths
    over lambda chunks (rcpp…/solvers.cpp:340-353 -> mbs_path :204-222). Rank r's items are folds
    (r B + i) % 5 over the rank's lambda chunk c = r % 8 (so --cv-batch changes the work per GPU, not its
    mix: the same chunk, the same PCG counts). Work item (fold f, chunk c): the
    lattice minus fold f of kfoldinds (W = O^T O a 0/1 mask, so the theta-solve is the spectrally
    preconditioned PCG, rtol 1e-10, warm-started), lambdas [4c, 4c+4) of create_lambdas' 32-lambda grid
    (lam_max_pinv on the GPU, 1e-4 lambda_max .. lambda_max), steps/4 fixed ADMM iterations at each, theta /
    u / rho carried (one mvtv_path call). Each rank runs --cv-batch items at once, one problem and HIP stream
    per item on its own host thread (the items are independent: no kernel waits for another item's), so the
    short launches of one item's PCG iterations overlap the others'. value = ADMM iterations/s of all items
    of all ranks."""
    import threading
    from multivartv_amd import cv as mcv
    m = [a.size] * a.dims
    y = towers(m)
    fold = mcv.kfoldinds(y.size, 5, seed=0)
    deltas = [(1.0 + 2e-4) / v for v in m]
    B = max(1, a.cv_batch)
    items = [D.rank * B + i for i in range(B)]   # item: fold (item % 5); lambda chunk: the rank's (rank % 8)
    dev = D.local % max(1, mv.device_count())
    probs, ymeans = [], []
    for it in items:
        W = (fold != it % 5).astype(np.float64)
        probs.append(mv.Problem(m, W * y, wdiag=W, deltas=deltas, order=mv.ORDER_CPP, device=dev))
        ymeans.append(float(y[W > 0].mean()))
    del y, fold
    lmax, _ = probs[0].lambda_max()
    grid = np.exp(np.linspace(np.log(lmax * 1e-4), np.log(lmax), 32))[::-1]
    chunks = [grid[(4 * (D.rank % 8) + np.arange(4)) % 32] for _ in items]
    per = max(1, a.steps // 4)
    steps = 4 * per
    solver = {"auto": mv.SOLVER_AUTO, "pcg": mv.SOLVER_PCG, "spectral": mv.SOLVER_PCG_SPECTRAL}[a.solver]
    opts = dict(pcg_rtol=a.pcg_rtol, theta_solver=solver)
    out = [None] * B

    def run_items(fn):
        errs = []

        def work(i):
            try:
                out[i] = fn(i)
            except Exception as e:   # noqa: BLE001 (re-raised below)
                errs.append(e)
        ts = [threading.Thread(target=work, args=(i,)) for i in range(B)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]

    if a.warmup > 0:
        run_items(lambda i: probs[i].path(chunks[i][:1], np.full(probs[i].N, ymeans[i]), chunks[i][0] / 5.0,
                                          want_thetas=False, fixed_iters=a.warmup, **opts))
    # the value: the timed region without per-launch events (this work item's launches are 20-50 us, the
    # event pairs around each would be part of what is timed); then the same region again with them, for
    # the kernels' durations (roofline)
    def timed(events):
        D.barrier()
        for P in probs:
            P.timing(events)
        t0 = time.perf_counter()
        run_items(lambda i: probs[i].path(chunks[i], np.full(probs[i].N, ymeans[i]), chunks[i][0] / 5.0,
                                          want_thetas=False, fixed_iters=per, **opts))
        t1 = time.perf_counter()
        D.barrier()
        tm = [P.timings() for P in probs] if events else None
        for P in probs:
            P.timing(False)
        return t1 - t0, tm
    elapsed, _ = timed(False)
    elapsed_ev, tims = timed(True)
    t0, t1 = 0.0, elapsed_ev
    g_elapsed, = D.allreduce([elapsed], "max")
    stats = [o[2] for o in out]
    kbar = sum(st["pcg_iters"] for sts in stats for st in sts) / (steps * B)
    tim = {k: dict(ms=sum(t[k]["ms"] for t in tims), launches=sum(t[k]["launches"] for t in tims),
                   bytes_per_launch=tims[0][k]["bytes_per_launch"]) for k in tims[0]}
    roof = _roofline(tim)
    N = probs[0].N
    roof["mall_resident"] = 8 * N * 7 < 256 * 2 ** 20
    moved = sum(v["bytes_per_launch"] * v["launches"] for v in tim.values())
    if B > 1:
        # the items' launches overlap, so a launch's duration is shared with other items' kernels: the roofline
        # object is the whole GPU's, the algorithmic bytes of every launch of the event-free region over its time
        per_kernel = dict(roof, note="dominant kernel's launch time while the items run concurrently")
        ach = moved / elapsed / 1e9
        roof = {"bound": "hbm", "kernel": f"all launches of the {B} concurrent items", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None,
                "mall_resident": per_kernel["mall_resident"], "dominant_kernel_concurrent": per_kernel}
    else:
        roof["note"] = "per-launch time of the dominant kernel"
    kern = {k: dict(avg_ms=round(v["ms"] / v["launches"], 4), launches=v["launches"]) for k, v in tim.items()
            if v["launches"]}
    rhos = [float(o[1][-1]) for o in out]
    for P in probs:
        P.close()
    if D.rank != 0:
        return None
    return {
        "metric": METRIC, "value": round(D.world * B * steps / g_elapsed, 4), "unit": "iters/s", "n_gpus": D.world,
        "steps": steps, "warmup": a.warmup, "ms_per_step": round(g_elapsed / steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: 2D towers + 0.5 N(0,1) on the lattice, CV fold masks W (kfoldinds seed 0), O = I on the "
                "training rows",
        "config": {"workload": f"config 4 work items: {a.dims}D {a.size}^{a.dims} CV fold paths over 4-lambda chunks, "
                               f"{B} items per GPU at once (one HIP stream each), 4 lambdas x {per} fixed iterations "
                               f"per item, warm-started, variant B",
                   "mesh": m, "nodes": N, "items_per_gpu": B, "lambda_chunks": [[float(v) for v in c] for c in chunks],
                   "theta_solver": {mv.SOLVER_PCG: "jacobi_pcg", mv.SOLVER_PCG_SPECTRAL: "pcg_spectral"}.get(
                       stats[0][0]["theta_solver"], "?"),
                   "pcg_rtol": a.pcg_rtol, "pcg_iters_mean": round(kbar, 2), "rho_out": rhos,
                   "parallelism": f"(fold, lambda-chunk) work items, {B} concurrent per GPU (x{D.world})"},
        "roofline": roof,
        "aggregate_hbm": {"bytes": moved, "GBps": round(moved / elapsed / 1e9, 1),
                          "frac": round(moved / elapsed / 1e9 / HBM_PEAK_GBPS, 4),
                          "note": "algorithmic bytes of every launch of the rank's items / the rank's wall time"},
        "with_kernel_events": {"ms_per_step": round(elapsed_ev / steps * 1e3, 3),
                               "note": "the same region timed with HIP events around every launch (roofline)"},
        "kernels": kern, "cpu_baseline": None}


def independent_main(a, D, comm=None):
    """Every rank fits its own 512^3 mesh (noise seed + rank): the north star's independent mesh fits,
    weak scaling. The global residual all-reduce goes over libmvtv's RCCL communicator when there is one.
    Returns rank 0's line."""
    m = [a.size] * a.dims
    lam = a.lam
    t_setup = time.perf_counter()
    y = towers(m, seed=SEED + D.rank)
    deltas = [(1.0 + 2e-4) / v for v in m]
    P = mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP, device=D.local % max(1, mv.device_count()))
    P.state_set(np.full(y.size, y.mean()), None, lam / 5.0)
    del y
    log(f"[rank {D.rank}] setup {time.perf_counter() - t_setup:.1f}s: N={P.N} E={P.E} blocks={P.nb}")

    solver = {"auto": mv.SOLVER_AUTO, "pcg": mv.SOLVER_PCG, "spectral": mv.SOLVER_SPECTRAL}[a.solver]
    opts = dict(fixed_iters=a.warmup, pcg_rtol=a.pcg_rtol, theta_solver=solver)
    if a.warmup > 0:
        P.run(lam, **opts)
    # Meshes up to 2^24 nodes run 0.07-0.9 ms iterations, where the per-launch timing events cost 7-30 % (1024^2:
    # 14.1k against 10.1k ADMM it/s, profiles/r04/v1_launch_gap; 256^3: 1166-1174 against 1086-1113): the value comes
    # from an event-free timed region and the per-kernel table from a second region of the same length right after
    # it. Round 6: every mesh (the 512^3 headline's events cost ~1 %; MVTV_BENCH_EVENTS_IN_VALUE=1: one region
    # with the events in it for meshes above 2^24 nodes, the round-5 timing)
    event_free = P.N <= (1 << 24) or os.environ.get("MVTV_BENCH_EVENTS_IN_VALUE", "0") in ("", "0")
    D.barrier()
    P.timing(not event_free)
    t0 = time.perf_counter()
    st = P.run(lam, fixed_iters=a.steps, pcg_rtol=a.pcg_rtol, theta_solver=solver)   # returns after the stream drained
    t1 = time.perf_counter()
    D.barrier()
    elapsed = t1 - t0
    if event_free:
        P.timing(True)
        P.run(lam, fixed_iters=a.steps, pcg_rtol=a.pcg_rtol, theta_solver=solver)
    tim = P.timings()
    P.timing(False)
    used = "spectral" if st["theta_solver"] == mv.SOLVER_SPECTRAL else "pcg"
    kbar = st["pcg_iters"] / max(1, a.steps)
    moved = sum(v["bytes_per_launch"] * v["launches"] for v in tim.values()) / max(1, a.steps)

    # secondary leg: the north star's Jacobi-PCG theta-solve on the same state (reported, not the value)
    pcg_leg = None
    if used == "spectral" and a.pcg_steps > 0:
        P.run(lam, fixed_iters=1, pcg_rtol=a.pcg_rtol, theta_solver=mv.SOLVER_PCG)   # warm the PCG poll schedule
        D.barrier()
        P.timing(True)
        tp0 = time.perf_counter()
        sp = P.run(lam, fixed_iters=a.pcg_steps, pcg_rtol=a.pcg_rtol, theta_solver=mv.SOLVER_PCG)
        tp1 = time.perf_counter()
        D.barrier()
        tp = P.timings()
        P.timing(False)
        g_tp, = D.allreduce([tp1 - tp0], "max")
        fk = tp["pcg_fused3d"] if tp["pcg_fused3d"]["launches"] else tp["pcg_apply_A"]
        pk_ms = fk["ms"] / max(1, fk["launches"])
        pcg_leg = {"value": round(D.world * a.pcg_steps / g_tp, 4), "steps": a.pcg_steps,
                   "pcg_iters_mean": round(sp["pcg_iters"] / a.pcg_steps, 2),
                   "kernel": "pcg_fused3d" if tp["pcg_fused3d"]["launches"] else "pcg_apply_A",
                   "kernel_avg_ms": round(pk_ms, 4),
                   "kernel_GBps": round(fk["bytes_per_launch"] / (pk_ms * 1e-3) / 1e9, 1) if fk["launches"] else None}
    g_elapsed, = D.allreduce([elapsed], "max")
    # global residual all-reduce over the independent fits (RCCL over xGMI through libmvtv's communicator)
    red = [st["r_norm"] ** 2, st["s_norm"] ** 2, float(st["pcg_unconverged"]), kbar]
    if comm is not None:
        red = comm.allreduce_host(red).tolist()
        red_via = f"RCCL ({comm.size} ranks, libmvtv communicator)"
    else:
        red = D.allreduce(red, "sum")
        red_via = "host" if D.world == 1 else "gloo"
    r2, s2, n_unconv, kbar_all = red
    kbar_all /= D.world

    roof = _roofline(tim)
    dom = roof["kernel"]
    per = {}
    for k, v in tim.items():
        if v["launches"]:
            avg = v["ms"] / v["launches"]
            per[k] = dict(avg_ms=round(avg, 4), launches=v["launches"], share=round(v["ms"] / (elapsed * 1e3), 4),
                          GBps=round(v["bytes_per_launch"] / (avg * 1e-3) / 1e9, 1) if v["bytes_per_launch"] else None)
    N, E = P.N, P.E
    iter_gbps = moved * a.steps / elapsed / 1e9                  # algorithmic bytes of every kernel launched
    pmc, pmc_src = load_pmc(dom) if (a.dims, a.size) == (3, 512) else (None, None)
    roof.update(traffic=pmc, traffic_source=pmc_src,
                timing=("HIP events in a second timed region of the same length (event-free value region)"
                        if event_free else "HIP events inside the timed region"),
                # a mesh whose working set fits the 256 MiB Infinity Cache is served partly on-die:
                # its "HBM" fraction is an upper bound, not an HBM measurement (SURVEY §7 hard part 7)
                mall_resident=8 * N * 6 < 256 * 2 ** 20)

    cpu = None
    if D.world == 1 and not a.no_cpu:
        planes = a.cpu_planes or max(4, m[-1] // 4)
        try:
            k_cpu = pcg_leg["pcg_iters_mean"] if pcg_leg else kbar   # the oracle's PCG leg runs the GPU's mean count
            cpu = cpu_baseline(m, lam, max(1, round(k_cpu)), planes, full=a.cpu_full)
            # like for like: spectral GPU value / spectral CPU; Jacobi-PCG leg / the same PCG on the CPU
            cpu["gpu_over_cpu_spectral"] = round(D.world * a.steps / g_elapsed / cpu["spectral_all_cores"], 1)
            if pcg_leg:
                cpu["gpu_pcg_leg_over_cpu_pcg"] = round(pcg_leg["value"] / cpu["pcg_all_cores"], 1)
        except Exception as e:  # the baseline is reported, never required
            log(f"cpu_baseline failed: {e}")
    P.close()
    if D.rank != 0:
        return None
    value = D.world * a.steps / g_elapsed
    return {
        "metric": METRIC, "value": round(value, 4), "unit": "iters/s", "n_gpus": D.world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(g_elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        # one fit of the metric's mesh at N = 1; at N > 1 the line is that same mesh slab-decomposed (total work
        # fixed), so the N = 1 line is the strong-scaling curve's first point
        "scaling": "strong" if D.world == 1 else "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: 3D towers + 0.5 N(0,1) (splitmix64/Box-Muller, seed 0x4D565456 + rank), O = I",
        "config": {"workload": f"{a.dims}D {a.size}^{a.dims} fp64 mesh-TV ADMM, variant B (rcpp admm_update), "
                               f"lambda={lam}, fixed-iteration mode",
                   "theta_solver": used,
                   "mesh": m, "nodes": N, "edges": E, "pcg_rtol": a.pcg_rtol, "pcg_iters_mean": round(kbar_all, 2),
                   "edge_blocks": _edge_blocks_note(tim, a.dims, N, E),
                   "parallelism": (f"independent mesh fits, one per GPU (gloo barrier / max-time, residual "
                                   f"all-reduce over {red_via})") if D.world > 1 else "single GPU"},
        "roofline": roof,
        "iteration_hbm": {"bytes_per_iter": moved, "GBps": round(iter_gbps, 1),
                          "frac": round(iter_gbps / HBM_PEAK_GBPS, 4),
                          "survey_bytes_per_iter": 8.0 * (5 * E + 8 * N + 10 * kbar * N)},
        "pcg_leg": pcg_leg,
        "kernels": per,
        "residuals": {"r_norm": float(np.sqrt(r2)), "s_norm": float(np.sqrt(s2)), "pcg_unconverged": int(n_unconv)},
        "cpu_baseline": cpu,
    }


def main():
    a = parse()
    if a.dry_run:
        return _dry_run(a)
    _import_mv()
    if mv.device_count() < 1:
        raise SystemExit("bench.py: no HIP device")
    D = Dist("gloo")
    line = None
    if a.mode == "cv":
        if a.size == 512 and a.dims == 3:   # config 4's shape unless given
            a.dims, a.size = 2, 2048
        line = cv_main(a, D)
    elif a.mode == "slab":
        line = slab_main(a, D)
    elif a.mode == "independent" or D.world == 1:
        comm = _rccl_comm(D, D.local % mv.device_count()) if D.world > 1 else None
        line = independent_main(a, D, comm)
        if comm is not None:
            comm.close()
    else:
        # N > 1: the metric is one mesh over all GPUs (slab, strong); the independent fits (weak) beside it.
        # A failure of the RCCL communicator or of the slab run (the same on every rank: the ranks agree on it
        # over gloo) still leaves the independent fits' line, labelled with the error.
        comm, err = None, None
        dev = D.local % mv.device_count()
        try:
            comm = _slab_comm(a, D, dev)
        except Exception as e:  # noqa: BLE001 (reported in the line)
            err = f"communicator: {e!r}"
        failed, = D.allreduce([1.0 if comm is None else 0.0], "max")
        if failed and comm is not None:
            comm.close()
            comm = None
        if failed and a.transport == "auto":
            # RCCL refused on some rank: the same slab loop over the HIP IPC group of the node's processes
            from multivartv_amd import slab
            try:
                comm = slab.Comm.ipc(dev)
                err = None
            except Exception as e:  # noqa: BLE001
                err = f"{err}; ipc communicator: {e!r}"
            failed, = D.allreduce([1.0 if comm is None else 0.0], "max")
            if failed and comm is not None:
                comm.close()
                comm = None
            if comm is not None:
                log(f"rank {D.rank}: RCCL communicator failed, slab loop over the ipc transport")
        ind = independent_main(a, D, comm)
        line = None
        if comm is not None:
            try:
                line = slab_main(a, D, comm)
                ok = 1.0
            except Exception as e:  # noqa: BLE001
                err, ok = f"slab run: {e!r}", 0.0
            if ok:
                failed, = D.allreduce([0.0], "max")
            else:
                # a failure that is not every rank's (one rank errs mid-loop) leaves the peers inside an RCCL
                # collective or a stream sync, where a gloo agreement would wait ~30 min: bounded wait, then rank 0
                # prints what it has and this process exits non-zero, so the launcher ends the stuck peers
                agreed = D.allreduce_within([1.0], 120.0, "max")
                if agreed is None:
                    log(f"rank {D.rank}: {err}; peers did not reach the agreement, exiting")
                    if ind is not None:
                        ind["slab_error"] = err
                        ind["config"]["note"] = ("the one-mesh slab run failed on this rank (slab_error); this line "
                                                 "is the independent fits, one mesh per GPU (weak scaling)")
                        print(json.dumps(ind), file=OUT, flush=True)
                    sys.stderr.flush()
                    os._exit(3)
                failed = agreed[0]
            comm.close()
            if failed:
                line = None
                err = err or "slab run failed on another rank"
        if line is not None:
            line["independent_fits"] = {k: ind[k] for k in ("value", "unit", "ms_per_step", "scaling", "roofline",
                                                            "residuals")}
            line["independent_fits"]["workload"] = (f"one {a.size}^{a.dims} fit per GPU (noise seed + rank), "
                                                   f"{D.world} GPUs")
        elif ind is not None:   # rank 0: the slab line could not be produced
            line = ind
            line["slab_error"] = err or "unknown"
            line["config"]["note"] = ("the one-mesh slab run failed (slab_error); this line is the independent "
                                      "fits, one mesh per GPU (weak scaling)")
    if line is not None:
        print(json.dumps(line), file=OUT, flush=True)
    D.close()


# The stream of the one JSON line: fd 1 as the process started (main() below points fd 1 at stderr, so
# what libraries print to stdout, e.g. RCCL's version banner when a communicator is created, cannot land
# beside the line).
OUT = sys.stdout


def _json_stdout():
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


if __name__ == "__main__":
    _a = parse()
    if _a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(_a.gpus, sys.argv[1:], dry_run=_a.dry_run))
    OUT = _json_stdout()
    main()
