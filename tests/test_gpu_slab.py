"""Slab-decomposed single mesh (multivartv_amd/slab.py) against the one-GPU solver.

The decomposition changes only where planes live and the summation order of the 7 global sums,
so iteration counts and rho must match the one-GPU run exactly and theta to 1e-11 relative.
Several ranks share the one GPU of the test box through host-staged gloo transport; the RCCL
device transport differs only in where the exchange buffers live."""
import os
import socket

import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")
from multivartv_amd import slab  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402

pytestmark = pytest.mark.gpu

CASES = [([16, 16, 16], 1.0), ([64, 32], 0.5), ([8, 8, 8, 8], 1.0)]


def _reference(m, lam, fixed):
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        th, _, rho, st = P.admm(lam, np.full(y.size, y.mean()), u=np.zeros(P.E), rho=lam / 5, fixed_iters=fixed,
                                return_u=True)
    return y, deltas, th, rho, st


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


@pytest.mark.parametrize("m,lam", CASES)
@pytest.mark.parametrize("fixed", [7, 0])
def test_single_rank_slab_matches(m, lam, fixed):
    y, deltas, th, rho, st = _reference(m, lam, fixed)
    S = slab.SlabADMM(m, y, deltas, y.mean(), group=False, device=0)
    out = S.run(lam, fixed_iters=fixed)
    assert out["iters"] == st["iters"] and out["rho"] == rho
    assert _rel(S.theta_owned(), th) <= 1e-11
    S.close()


def _rank_main(rank, world, port, m, lam, fixed, q, backend="gloo"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        import torch
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    b = slab.plane_bounds(m[-1], world)
    pl = int(np.prod(m[:-1]))
    S = slab.SlabADMM(m, y[b[rank] * pl:b[rank + 1] * pl], deltas, y.mean(), device=0)
    out = S.run(lam, fixed_iters=fixed)
    q.put((rank, out["iters"], out["rho"], S.theta_owned()))
    S.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("m,lam,world", [([16, 16, 16], 1.0, 2), ([8, 8, 8, 8], 1.0, 4), ([64, 32], 0.5, 2)])
def test_multi_rank_slab_matches(m, lam, world):
    import torch.multiprocessing as mp
    fixed = 0
    y, deltas, th, rho, st = _reference(m, lam, fixed)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, m, lam, fixed, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=100) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[1] == st["iters"] and r[2] == rho
    assert _rel(np.concatenate([r[3] for r in res]), th) <= 1e-11


@pytest.mark.parametrize("fixed", [7, 0])
def test_rccl_transport_single_rank(fixed):
    """The "nccl" (RCCL) transport: exchange buffers are device tensors and the all-to-all
    transposes run through RCCL. One rank on the box's one GPU (RCCL refuses two ranks on one
    device), so this covers the device-buffer path and RCCL's self all-to-all, not xGMI."""
    import torch.multiprocessing as mp
    m, lam = [16, 16, 16], 1.0
    y, deltas, th, rho, st = _reference(m, lam, fixed)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_main, args=(0, 1, port, m, lam, fixed, q, "nccl"))
    p.start()
    r = q.get(timeout=100)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert r[1] == st["iters"] and r[2] == rho
    assert _rel(r[3], th) <= 1e-11


def test_slab_4d_16_four_ranks_vs_c_oracle():
    """Config 5's decomposition (4-D, dim 3 split, 4 planes per rank) against the C oracle rather
    than the one-GPU HIP path: 20 fixed iterations of variant B from theta0 = mean y, u0 = 0."""
    import torch.multiprocessing as mp
    from oracle import c_oracle
    m, lam, world, fixed = [16, 16, 16, 16], 1.0, 4, 20
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    th = np.full(y.size, y.mean())
    u = np.zeros(c_oracle.num_edges(m))
    ref = c_oracle.admm_rcpp(m, y, lam, th, u, lam / 5.0, deltas, fixed_iters=fixed, pcg_rtol=1e-13)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, m, lam, fixed, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=100) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[1] == fixed and r[2] == ref["rho"]
    assert _rel(np.concatenate([r[3] for r in res]), th) <= 1e-9
