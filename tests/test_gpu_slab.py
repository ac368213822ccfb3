"""Slab-decomposed single mesh (csrc/mvtv_slab.cpp, multivartv_amd/slab.py).

The last dimension's line solves are substructured over the ranks (k_tris phase 1, the interface systems
k_tris_iface, phase 3) with the collectives on their own stream: these cases cover blocks of 1 (4 x 4 x 8
over 4 ranks: 2 planes each) to 32 planes per rank, 2-D to 4-D, and the event hand-offs between the streams.

The decomposition changes where planes live and the summation order of the 7 global sums, so the
iteration count and rho must match the one-GPU run exactly and theta to 1e-11 relative. Several ranks
share the one GPU of the test box through the in-process loopback transport (every rank's mvtv_slab_run
on its own host thread, exchanges as device copies); RCCL runs at world size 1 (its self transfers),
since RCCL refuses two ranks on one device."""
import os
import socket

import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")
from multivartv_amd import slab  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402

pytestmark = pytest.mark.gpu


def _reference(m, lam, fixed):
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        th, _, rho, st = P.admm(lam, np.full(y.size, y.mean()), u=np.zeros(P.E), rho=lam / 5, fixed_iters=fixed,
                                return_u=True)
    return y, deltas, th, rho, st


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


@pytest.mark.parametrize("m,lam,world", [([16, 16, 16], 1.0, 1), ([16, 16, 16], 1.0, 2), ([32, 32, 32], 0.5, 4),
                                         ([64, 32], 0.5, 2), ([8, 8, 8, 8], 1.0, 4), ([16, 16, 16, 16], 1.0, 2),
                                         ([4, 4, 8], 1.0, 4), ([64, 64, 64], 1.0, 4), ([32, 32, 32, 8], 1.0, 2)],
                         ids=["3d_16_w1", "3d_16_w2", "3d_32_w4", "2d_64x32_w2", "4d_8_w4", "4d_16_w2",
                              "3d_4x4x8_w4_small_planes", "3d_64_w4", "4d_32x32x32x8_w2"])
@pytest.mark.parametrize("fixed", [7, 0])
def test_local_group_matches_one_gpu(m, lam, world, fixed):
    y, deltas, th, rho, st = _reference(m, lam, fixed)
    out, theta = slab.run_local_group(m, y, deltas, lam, world, fixed_iters=fixed)
    for o in out:
        assert o["iters"] == st["iters"] and o["rho"] == rho
    assert out[0]["r_norm"] == pytest.approx(st["r_norm"], rel=1e-9)
    assert out[0]["s_norm"] == pytest.approx(st["s_norm"], rel=1e-9)
    assert _rel(theta, th) <= 1e-11


def test_loopback_failing_rank_does_not_hang_its_peers():
    """A rank whose loop fails (here: a plane range that is not the communicator's even split) makes its
    peers fail too instead of waiting for its transfers (LocalHub abort, csrc/mvtv_slab.cpp)."""
    import threading
    m, lam = [8, 8, 8], 1.0
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    comms = slab.Comm.local_group(2)
    ranks = [slab.SlabADMM(m, y[r * 256:(r + 1) * 256], deltas, float(y.mean()), comms[r]) for r in range(2)]
    errs = [None, None]
    ranks[1].P.close()   # rank 1's handle is gone: its mvtv_slab_run fails at once
    ranks[1].P._h = None

    def work(r):
        try:
            ranks[r].run(lam, fixed_iters=3)
        except Exception as e:   # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in ts)
    assert errs[0] is not None and errs[1] is not None
    ranks[0].close()
    for c in comms:
        c.close()


def test_uneven_infeasible_line_split_fails_on_every_rank():
    """m_global = 133 over 2 ranks: 66 and 67 planes. Only the 67-plane block (prime, > 64) has no split into the
    line solves' segments; the ranks' layout agreement carries that flag, so BOTH fail with MVTV_BAD_ARG before the
    first collective (over RCCL the 66-plane rank would otherwise wait in the coefficient all-to-all forever)."""
    import threading
    m, lam = [8, 8, 133], 1.0
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    comms = slab.Comm.local_group(2)
    b = slab.plane_bounds(m[-1], 2)
    assert [b[1] - b[0], b[2] - b[1]] == [66, 67]
    ranks = [slab.SlabADMM(m, y[b[r] * 64:b[r + 1] * 64], deltas, float(y.mean()), comms[r]) for r in range(2)]
    errs = [None, None]

    def work(r):
        try:
            ranks[r].run(lam, fixed_iters=2)
        except Exception as e:   # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in ts)
    for e in errs:
        assert isinstance(e, mv.MvtvError) and "line solves" in str(e), e
    for r in ranks:
        r.close()
    for c in comms:
        c.close()


@pytest.mark.parametrize("m,world", [([60, 60, 45], 3), ([24, 24, 37], 2), ([48, 48, 130], 4), ([40, 100], 4),
                                     ([62, 62, 40], 2), ([24, 24, 37], 1)],
                         ids=["3d_60x60x45_w3_mixed_radix", "3d_24x24x37_w2_prime_last", "3d_48x48x130_w4",
                              "2d_40x100_w4", "3d_62x62x40_w2_bluestein_lead", "3d_24x24x37_w1_bluestein_last"])
def test_slab_any_last_dimension_vs_c_oracle(m, world):
    """The last dimension's line solves are substructured over the ranks, so it may have any length (37 is
    prime; 45, 130 not powers of two) and the leading dims any 2-3-5-7 length (k_dctg passes): 12 fixed
    iterations against the C oracle's loop with the exact scipy.fft solve, rho exact, theta 1e-9."""
    from oracle import c_oracle
    lam, fixed = 0.7, 12
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    th = np.full(y.size, y.mean())
    u = np.zeros(c_oracle.num_edges(m))
    ref = c_oracle.admm_rcpp_spectral(m, y, lam, th, u, lam / 5.0, deltas, fixed_iters=fixed)
    out, theta = slab.run_local_group(m, y, deltas, lam, world, fixed_iters=fixed)
    assert all(o["iters"] == fixed and o["rho"] == ref["rho"] for o in out)
    assert _rel(theta, th) <= 1e-9
    assert out[0]["r_norm"] == pytest.approx(ref["r_norm"], rel=1e-8)


def test_slab_one_rank_needs_a_spectral_last_dimension():
    """One rank solves the last dimension locally: any length up to 4096 (Bluestein past 2-3-5-7), not above."""
    y = towers([4, 4, 4099])
    comm = slab.Comm.local_group(1)[0]
    S = slab.SlabADMM([4, 4, 4099], y, [(1.0 + 2e-4) / v for v in (4, 4, 4099)], y.mean(), comm)
    with pytest.raises(mv.MvtvError):
        S.run(1.0, fixed_iters=2)
    S.close()
    comm.close()


def test_slab_4d_16_four_ranks_vs_c_oracle():
    """Config 5's decomposition (4-D, dim 3 split, 4 planes per rank) against the C oracle rather than
    the one-GPU HIP path: 20 fixed iterations of variant B from theta0 = mean y, u0 = 0."""
    from oracle import c_oracle
    m, lam, world, fixed = [16, 16, 16, 16], 1.0, 4, 20
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    th = np.full(y.size, y.mean())
    u = np.zeros(c_oracle.num_edges(m))
    ref = c_oracle.admm_rcpp(m, y, lam, th, u, lam / 5.0, deltas, fixed_iters=fixed, pcg_rtol=1e-13)
    out, theta = slab.run_local_group(m, y, deltas, lam, world, fixed_iters=fixed)
    assert all(o["iters"] == fixed and o["rho"] == ref["rho"] for o in out)
    assert _rel(theta, th) <= 1e-9


def _fold_mask(m, seed=3, keep=0.8):
    """A CV fold's W: 1 on the training nodes, 0 on the held-out ones (config 4's work items)."""
    return (np.random.default_rng(seed).random(int(np.prod(m))) < keep).astype(np.float64)


@pytest.mark.parametrize("m,world", [([32, 32, 32], 1), ([32, 32, 32], 2), ([32, 32, 32], 4), ([64, 48], 2),
                                     ([8, 8, 8, 16], 4), ([4, 4, 8], 4)],
                         ids=["3d_32_w1", "3d_32_w2", "3d_32_w4", "2d_64x48_w2", "4d_8x8x8x16_w4",
                              "3d_4x4x8_w4_small_planes"])
@pytest.mark.parametrize("fixed", [10, 0])
def test_slab_weighted_fold_matches_one_gpu(m, world, fixed):
    """W != I (a CV fold mask): the theta-solve is PCG with the spectral preconditioner of mean(W) I + rho
    D^T D, its operator applied on the owned planes after a halo of the search direction, the preconditioner
    the distributed direct solve, every dot product one all-reduce. Against the one-GPU PCG-spectral solve
    at pcg_rtol 1e-13: iterations and rho exact, theta 1e-8 relative (the PCG stops at different iterates
    when the sums are ordered differently)."""
    lam = 0.6
    y = towers(m)
    w = _fold_mask(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    t0 = float(y[w > 0].mean())
    with mv.Problem(m, w * y, wdiag=w, deltas=deltas, order=mv.ORDER_CPP) as P:
        th, _, rho, st = P.admm(lam, np.full(y.size, t0), u=np.zeros(P.E), rho=lam / 5, fixed_iters=fixed,
                                return_u=True, theta_solver=mv.SOLVER_PCG_SPECTRAL, pcg_rtol=1e-13)
    out, theta = slab.run_local_group(m, y, deltas, lam, world, w=w, theta0=t0, fixed_iters=fixed, pcg_rtol=1e-13)
    for o in out:
        assert o["iters"] == st["iters"] and o["rho"] == rho
        assert o["theta_solver"] == mv.SOLVER_PCG_SPECTRAL and o["pcg_iters"] > 0
    assert _rel(theta, th) <= 1e-9


def test_slab_weighted_counts_vs_c_oracle():
    """Scattered counts W in {0..3} (the diagonally scaled preconditioner: std W >= 0.1 of the operator's
    mean diagonal at small rho), 2 ranks, 15 fixed iterations against the C oracle's Jacobi-PCG loop."""
    from oracle import c_oracle
    m, lam, world, fixed = [16, 16, 24], 0.05, 2, 15
    y = towers(m)
    w = np.random.default_rng(11).integers(0, 4, int(np.prod(m))).astype(np.float64)
    deltas = [(1.0 + 2e-4) / v for v in m]
    t0 = float((w * y).sum() / w.sum())
    th = np.full(y.size, t0)
    u = np.zeros(c_oracle.num_edges(m))
    ref = c_oracle.admm_rcpp(m, w * y, lam, th, u, lam / 5.0, deltas, W=w, fixed_iters=fixed, pcg_rtol=1e-13)
    out, theta = slab.run_local_group(m, y, deltas, lam, world, w=w, theta0=t0, fixed_iters=fixed, pcg_rtol=1e-13)
    assert all(o["iters"] == fixed and o["rho"] == ref["rho"] for o in out)
    assert _rel(theta, th) <= 1e-9


@pytest.mark.parametrize("fixed", [7, 0])
def test_rccl_single_rank(fixed):
    """The RCCL transport at world size 1 (self transfers as device copies, RCCL communicator live):
    the same loop as one GPU."""
    m, lam = [32, 32, 32], 1.0
    y, deltas, th, rho, st = _reference(m, lam, fixed)
    comm = slab.Comm.rccl_single(0)
    S = slab.SlabADMM(m, y, deltas, y.mean(), comm, device=0)
    o = S.run(lam, fixed_iters=fixed)
    assert o["iters"] == st["iters"] and o["rho"] == rho
    assert _rel(S.theta_owned(), th) <= 1e-11
    S.close()
    comm.close()


@pytest.mark.parametrize("transport", ["rccl", "loopback"])
@pytest.mark.parametrize("m", [[32, 32, 32], [16, 16, 16, 16]], ids=["3d_32", "4d_16"])
def test_distributed_path_at_one_rank(transport, m, monkeypatch):
    """MVTV_SLAB_DISTRIBUTED=1 at world size 1: the G-rank loop (substructured line solves with their
    all-to-alls, the collectives' stream and its events, the all-reduce) on one GPU; over RCCL every
    ncclSend / ncclRecv / ncclAllReduce call the multi-GPU runs make, to the rank itself. Converged run:
    iterations and rho exact against the one-GPU path, theta 1e-11."""
    monkeypatch.setenv("MVTV_SLAB_DISTRIBUTED", "1")
    lam = 1.0
    y, deltas, th, rho, st = _reference(m, lam, 0)
    comm = slab.Comm.rccl_single(0) if transport == "rccl" else slab.Comm.local_group(1)[0]
    S = slab.SlabADMM(m, y, deltas, y.mean(), comm, device=0)
    o = S.run(lam, fixed_iters=0)
    assert o["iters"] == st["iters"] and o["rho"] == rho
    assert _rel(S.theta_owned(), th) <= 1e-11
    S.close()
    comm.close()


def _rccl_rank_main(port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    m, lam = [16, 16, 16], 1.0
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    comm = slab.Comm.rccl(0)
    S = slab.SlabADMM(m, y, deltas, y.mean(), comm, device=0)
    o = S.run(lam, fixed_iters=0)
    q.put((o["iters"], o["rho"], S.theta_owned()))
    S.close()
    comm.close()
    dist.destroy_process_group()


def test_rccl_id_through_torch_distributed():
    """Comm.rccl: the unique id travels through torch.distributed (nccl backend, world size 1)."""
    import torch.multiprocessing as mp
    y, deltas, th, rho, st = _reference([16, 16, 16], 1.0, 0)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank_main, args=(port, q))
    p.start()
    r = q.get(timeout=100)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert r[0] == st["iters"] and r[1] == rho
    assert _rel(r[2], th) <= 1e-11
