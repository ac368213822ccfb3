"""Benchmark: ADMM iterations/s on a 512^3 fp64 mesh (BASELINE.json metric), HIP path on MI355X.

One step = one ADMM iteration of the reference's variant-B admm_update
(rcpp-code/MultivarTV/src/solvers.cpp:110-133) on the synthetic 3D towers
problem of SURVEY §8d: lattice data with mesh == data (O = I), lambda = 1,
rho0 = lambda/5, u0 = 0, theta0 = mean(y), fixed-iteration mode (the stopping
test is evaluated but not acted on), PCG theta-solves warm-started at
rtol 1e-10. Inputs are resident in HBM before timing starts.

Multi-GPU (torchrun, one process per GPU): every rank fits its own independent
512^3 mesh (noise seed + rank) — the embarrassingly parallel "independent mesh
fits" sharding of the north star — so value = total iterations/s of all ranks
and scaling is weak. torch.distributed (RCCL by default, MVTV_DIST_BACKEND=gloo
for host scalars) provides the barriers, the max-over-ranks time and the final
global residual all-reduce.
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

import multivartv_amd as mv  # noqa: E402  (load libmvtv before anything that brings its own HIP runtime)
from multivartv_amd.synth import SEED, towers  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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
                    help="theta-solve: auto = spectral (exact DCT solve) where it applies, else Jacobi-PCG")
    ap.add_argument("--pcg-steps", type=int, default=10,
                    help="steps of the secondary Jacobi-PCG leg reported beside the main one (0 = skip)")
    ap.add_argument("--mode", choices=["independent", "slab"], default="independent",
                    help="N > 1: independent fits per GPU (weak scaling, default) or one mesh slab-decomposed "
                         "over the GPUs (strong scaling; RCCL halo exchange + all-to-all transposes)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-planes", type=int, default=0,
                    help="cpu_baseline sample: slowest-dim planes of the mesh (0 = auto)")
    return ap.parse_args()


class Dist:
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

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def load_pmc(name):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get(name)
    except Exception:
        return None


def cpu_baseline(m, lam, pcg_iters, planes):
    """Oracle (C, OpenMP) on a bounded slab of the same workload, scaled to full-mesh iterations/s."""
    from oracle import c_oracle
    sub = list(m[:-1]) + [planes]
    y = towers(sub)
    N = y.size
    E = c_oracle.num_edges(sub)
    th = np.full(N, y.mean())
    u = np.zeros(E)
    deltas = [(1.0 + 2e-4) / v for v in m]
    t0 = time.perf_counter()
    st = c_oracle.admm_rcpp(sub, y, lam, th, u, lam / 5.0, deltas, fixed_iters=1, pcg_fixed=int(pcg_iters))
    dt = time.perf_counter() - t0
    scale = float(np.prod(m)) / float(N)
    return dict(value=1.0 / (dt * scale), unit="iters/s", cores=c_oracle.threads(), kind="port",
                sample=(f"1 ADMM iteration (variant B, {int(pcg_iters)} PCG iterations = GPU mean) on a "
                        f"{'x'.join(map(str, sub))} slab of the same towers problem ({dt:.1f} s), "
                        f"scaled by N_full/N_slab = {scale:.0f}; oracle/c/mvtv_oracle.c, OpenMP"),
                seconds=dt, pcg_iters=st["pcg_iters"])


def slab_main(a):
    """One 3-D mesh decomposed over the ranks: strong scaling."""
    from multivartv_amd import slab
    # MVTV_SLAB_BACKEND=gloo rehearses the decomposition with host-staged exchanges (several ranks may
    # then share one GPU); the default is RCCL with device-resident exchange buffers
    D = Dist(os.environ.get("MVTV_SLAB_BACKEND", "nccl"))
    dev = D.local % max(1, mv.device_count())
    m = [a.size] * a.dims
    lam = a.lam
    b = slab.plane_bounds(m[-1], D.world)
    pl = int(np.prod(m[:-1]))
    y = towers(m, start=int(b[D.rank]) * pl, count=int(b[D.rank + 1] - b[D.rank]) * pl)
    ysum, = D.allreduce([float(y.sum())], "sum")
    deltas = [(1.0 + 2e-4) / v for v in m]
    S = slab.SlabADMM(m, y, deltas, ysum / float(np.prod(m)), device=dev)
    del y
    if a.warmup > 0:
        S.run(lam, fixed_iters=a.warmup)
    D.barrier()
    S.P.timing(True)
    t0 = time.perf_counter()
    st = S.run(lam, fixed_iters=a.steps)
    t1 = time.perf_counter()
    D.barrier()
    tim = S.P.timings()
    S.P.timing(False)
    g_elapsed, = D.allreduce([t1 - t0], "max")
    per = {k: dict(avg_ms=round(v["ms"] / v["launches"], 4), launches=v["launches"]) for k, v in tim.items() if v["launches"]}
    dom = max((k for k in tim if tim[k]["bytes_per_launch"] > 0 and tim[k]["launches"]), key=lambda k: tim[k]["ms"])
    d_avg = tim[dom]["ms"] / tim[dom]["launches"]
    achieved = tim[dom]["bytes_per_launch"] / (d_avg * 1e-3) / 1e9
    S.close()
    if D.rank == 0:
        print(json.dumps({
            "metric": "ADMM iters/sec on 512^3 fp64 mesh; achieved HBM GB/s vs peak at 1/2/4/8 GPUs",
            "value": round(a.steps / g_elapsed, 4), "unit": "iters/s", "n_gpus": D.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(g_elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: 3D towers + 0.5 N(0,1) (splitmix64/Box-Muller, seed 0x4D565456), O = I",
            "config": {"workload": f"{a.dims}D {a.size}^{a.dims} fp64 mesh-TV ADMM, variant B, lambda={lam}, one mesh "
                                   f"slab-decomposed along dim {a.dims - 1}", "mesh": m, "theta_solver": "spectral",
                       "parallelism": f"slab x{D.world} ({'RCCL' if D.backend == 'nccl' else D.backend} halo planes, "
                                      f"all-to-all transposes, 6-sum all-reduce)"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None},
            "kernels_rank0": per, "residuals": {"r_norm": st["r_norm"], "s_norm": st["s_norm"]},
            "cpu_baseline": None}), flush=True)
    D.close()


def main():
    a = parse()
    if a.mode == "slab" and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return slab_main(a)
    # the independent fits share nothing but the barrier, the max time and the final residual
    # all-reduce: RCCL (device scalars) by default, MVTV_DIST_BACKEND=gloo for host scalars
    D = Dist(os.environ.get("MVTV_DIST_BACKEND", "nccl"))
    if mv.device_count() < 1:
        raise SystemExit("bench.py: no HIP device")
    m = [a.size] * a.dims
    lam = a.lam
    t_setup = time.perf_counter()
    y = towers(m, seed=SEED + D.rank)
    deltas = [(1.0 + 2e-4) / v for v in m]
    P = mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP, device=D.local % max(1, mv.device_count()))
    P.state_set(np.full(y.size, y.mean()), None, lam / 5.0)
    ymean = float(y.mean())
    del y
    log(f"[rank {D.rank}] setup {time.perf_counter() - t_setup:.1f}s: N={P.N} E={P.E} blocks={P.nb}")

    solver = {"auto": mv.SOLVER_AUTO, "pcg": mv.SOLVER_PCG, "spectral": mv.SOLVER_SPECTRAL}[a.solver]
    opts = dict(fixed_iters=a.warmup, pcg_rtol=a.pcg_rtol, theta_solver=solver)
    if a.warmup > 0:
        P.run(lam, **opts)
    D.barrier()
    P.timing(True)
    t0 = time.perf_counter()
    st = P.run(lam, fixed_iters=a.steps, pcg_rtol=a.pcg_rtol, theta_solver=solver)   # returns after the stream drained
    t1 = time.perf_counter()
    D.barrier()
    elapsed = t1 - t0
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
    # global residual all-reduce over the independent fits
    r2, s2, n_unconv = D.allreduce([st["r_norm"] ** 2, st["s_norm"] ** 2, float(st["pcg_unconverged"])], "sum")
    kbar_all, = D.allreduce([kbar], "sum")
    kbar_all /= D.world

    # dominant kernel (by time in the timed region) and its achieved HBM rate
    dom = max((k for k in tim if tim[k]["bytes_per_launch"] > 0), key=lambda k: tim[k]["ms"])
    per = {}
    for k, v in tim.items():
        if v["launches"]:
            avg = v["ms"] / v["launches"]
            per[k] = dict(avg_ms=round(avg, 4), launches=v["launches"], share=round(v["ms"] / (elapsed * 1e3), 4),
                          GBps=round(v["bytes_per_launch"] / (avg * 1e-3) / 1e9, 1) if v["bytes_per_launch"] else None)
    d_avg_ms = tim[dom]["ms"] / tim[dom]["launches"]
    achieved = tim[dom]["bytes_per_launch"] / (d_avg_ms * 1e-3) / 1e9
    N, E = P.N, P.E
    iter_gbps = moved * a.steps / elapsed / 1e9                  # algorithmic bytes of every kernel launched
    pmc = load_pmc(dom)

    cpu = None
    if D.world == 1 and not a.no_cpu:
        planes = a.cpu_planes or max(4, m[-1] // 8)
        try:
            k_cpu = pcg_leg["pcg_iters_mean"] if pcg_leg else kbar   # the oracle's theta-solve is PCG
            cpu = cpu_baseline(m, lam, max(1, round(k_cpu)), planes)
        except Exception as e:  # the baseline is reported, never required
            log(f"cpu_baseline failed: {e}")
    P.close()

    if D.rank == 0:
        value = D.world * a.steps / g_elapsed
        out = {
            "metric": "ADMM iters/sec on 512^3 fp64 mesh; achieved HBM GB/s vs peak at 1/2/4/8 GPUs",
            "value": round(value, 4),
            "unit": "iters/s",
            "n_gpus": D.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(g_elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: 3D towers + 0.5 N(0,1) (splitmix64/Box-Muller, seed 0x4D565456 + rank), O = I",
            "config": {"workload": f"{a.dims}D {a.size}^{a.dims} fp64 mesh-TV ADMM, variant B (rcpp admm_update), "
                                   f"lambda={lam}, fixed-iteration mode",
                       "theta_solver": used,
                       "mesh": m, "nodes": N, "edges": E, "pcg_rtol": a.pcg_rtol, "pcg_iters_mean": round(kbar_all, 2),
                       "parallelism": (f"independent mesh fits, one per GPU ({'RCCL' if D.backend == 'nccl' else D.backend} "
                                       f"barrier / max-time / residual all-reduce)") if D.world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": pmc, "bytes_per_launch": tim[dom]["bytes_per_launch"],
                         "avg_launch_ms": round(d_avg_ms, 4)},
            "iteration_hbm": {"bytes_per_iter": moved, "GBps": round(iter_gbps, 1),
                              "frac": round(iter_gbps / HBM_PEAK_GBPS, 4),
                              "survey_bytes_per_iter": 8.0 * (5 * E + 8 * N + 10 * kbar * N)},
            "pcg_leg": pcg_leg,
            "kernels": per,
            "residuals": {"r_norm": float(np.sqrt(r2)), "s_norm": float(np.sqrt(s2)),
                          "pcg_unconverged": int(n_unconv)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    D.close()


if __name__ == "__main__":
    main()
