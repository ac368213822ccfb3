"""The slab loop (mvtv_slab_run) across rank PROCESSES on one GPU, over the inter-process transport
(mvtv_comm_create_ipc: device copies out of the peer's IPC-mapped buffers, shared-memory rendezvous), against the
one-GPU run of the same mesh (rcpp-code/MultivarTV/src/solvers.cpp:110-133 decomposed):
iterations and rho exact, theta to 1e-11 of max|theta| (only the order of the global sums differs), the norms
to 1e-9. Shapes: the metric's 512^3 over 2 processes (256 planes each), config 5's 128^4 over 4 (32 planes of
dim 3 each), world 8 as the driver's 8-GPU runs use it (a 3-D and a 4-D mesh, 8 and 4 planes per rank), a weighted CV fold (the distributed PCG-spectral solve: one all-reduce per dot product) and a
tolerance-mode run to convergence over 3. A rank whose loop fails ends its peers' waits with an error.

The children are started with multiprocessing's spawn (a fresh interpreter each) and use gloo only to hand over
the rendezvous segment's name; the reference theta goes to them through a file."""
import ctypes as C
import os
import socket
import sys

import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")
from multivartv_amd.synth import towers  # noqa: E402

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fold_mask(m):
    return (np.arange(int(np.prod(m))) % 5 != 2).astype(np.float64)


def _say(rank, msg):
    print(f"[ipc rank {rank}] {msg}", file=sys.stderr, flush=True)


def _rank_main(rank, world, port, q, m, lam, iters, ref_path, weighted, fail_rank, t0):
    import faulthandler
    faulthandler.dump_traceback_later(100, exit=False)   # a stuck rank shows where it is
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _say(rank, f"up, mesh {m}")
    try:
        from multivartv_amd import _lib, slab
        deltas = [(1.0 + 2e-4) / v for v in m]
        b = slab.plane_bounds(m[-1], world)
        pl = int(np.prod(m[:-1]))
        own = slice(int(b[rank]) * pl, int(b[rank + 1]) * pl)
        y = towers(m, start=own.start, count=own.stop - own.start)   # this rank's planes only
        w = _fold_mask(m)[own] if weighted else None
        oty = y if w is None else w * y
        comm = slab.Comm.ipc(0)
        _say(rank, "ipc group created")
        S = slab.SlabADMM(m, oty, deltas, t0, comm, device=0, w_owned=w)
        del y, oty
        _say(rank, "slab problem created")
        if rank == fail_rank:   # variant A is refused before any collective: the rank aborts the group
            o = _lib.default_opts(_lib.VARIANT_CPP)
            st = _lib.AdmmStats()
            s = _lib.lib().mvtv_slab_run(S.P._h, comm._h, C.byref(o), lam, t0, lam / 5.0, C.byref(st))
            q.put((rank, {"status": int(s)}, None, None))
        else:
            kw = dict(pcg_rtol=1e-13) if weighted else {}
            try:
                st = S.run(lam, fixed_iters=iters, **kw)
            except Exception as e:  # noqa: BLE001
                q.put((rank, None, None, repr(e)))
                return
            _say(rank, f"run done: {st['iters']} iterations")
            th = S.theta_owned()
            ref = np.load(ref_path, mmap_mode="r")[own]
            q.put((rank, st, float(np.max(np.abs(th - ref))), None))
        S.close()
        comm.close()
    except Exception as e:  # noqa: BLE001 (reported to the parent)
        q.put((rank, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


def _run_group(world, m, lam, iters, ref_path, t0, weighted=False, fail_rank=-1, env=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env = dict(env or {})
    env.setdefault("MVTV_IPC_TIMEOUT", "60")   # a transport wait that never ends fails the test instead
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        procs = [ctx.Process(target=_rank_main, args=(r, world, port, q, m, lam, iters, ref_path, weighted, fail_rank, t0))
                 for r in range(world)]
        for p in procs:
            p.start()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _one_gpu(m, lam, iters, weighted=False):
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    w = _fold_mask(m) if weighted else None
    kw = dict(theta_solver=mv.SOLVER_PCG_SPECTRAL, pcg_rtol=1e-13) if weighted else {}
    t0 = float(y.mean()) if w is None else float(y[w > 0].mean())
    with mv.Problem(m, y if w is None else w * y, wdiag=w, deltas=deltas, order=mv.ORDER_CPP) as P:
        P.state_set(np.full(y.size, t0), None, lam / 5.0)
        st = P.run(lam, fixed_iters=iters, **kw)
        th, _, rho = P.state_get(want_u=False)
    return th, rho, st, t0


def test_slab_processes_weighted_fold(tmp_path):
    """W != I: the distributed PCG-spectral theta-solve (a halo of the search direction and an all-reduce per dot
    product, every one across processes) against the one-GPU PCG-spectral run; iterations and rho exact."""
    m, world, iters, lam = [32, 32, 40], 2, 8, 0.6
    th, rho, st, t0 = _one_gpu(m, lam, iters, weighted=True)
    ref = tmp_path / "theta.npy"
    np.save(ref, th)
    res = _run_group(world, m, lam, iters, str(ref), t0, weighted=True)
    for rank, o, err, exc in res:
        assert exc is None, (rank, exc)
        assert o["iters"] == iters and o["rho"] == rho
        assert o["pcg_iters"] > 0
        assert err <= 1e-9 * float(np.max(np.abs(th))), (rank, err)


def test_failing_rank_ends_its_peers(tmp_path):
    """Rank 1's loop is refused (variant A) before its first collective: it marks the group aborted and rank 0's
    first wait fails with an error instead of hanging (and well before the timeout)."""
    m = [32, 32, 16]
    ref = tmp_path / "theta.npy"
    np.save(ref, np.zeros(int(np.prod(m))))
    res = _run_group(2, m, 1.0, 3, str(ref), 0.0, fail_rank=1)
    from multivartv_amd import _lib
    assert res[1][1]["status"] == _lib.MVTV_BAD_ARG
    assert res[0][3] is not None and "aborted" in res[0][3]


@pytest.mark.parametrize("m,world,iters", [([48, 48, 40], 3, 6), ([80, 80, 33], 2, 0), ([128, 128, 128, 128], 4, 2),
                                           ([512, 512, 512], 2, 2), ([96, 96, 64], 8, 5), ([32, 32, 32, 32], 8, 3)],
                         ids=["3d_3proc", "tolerance_2proc", "config5_128_4d_4proc", "metric_512cubed_2proc",
                              "3d_8proc", "4d_8proc"])
def test_slab_processes_match_one_gpu(tmp_path, m, world, iters):
    lam = 1.0 if iters else 0.4
    th, rho, st, t0 = _one_gpu(m, lam, iters)
    ref = tmp_path / "theta.npy"
    np.save(ref, th)
    scale = float(np.max(np.abs(th)))
    del th
    res = _run_group(world, m, lam, iters, str(ref), t0)
    for rank, o, err, exc in res:
        assert exc is None, (rank, exc)
        assert o["iters"] == st["iters"] and o["rho"] == rho, (rank, o["iters"], st["iters"])
        assert o["r_norm"] == pytest.approx(st["r_norm"], rel=1e-9)
        assert o["s_norm"] == pytest.approx(st["s_norm"], rel=1e-9)
        assert err <= 1e-11 * scale, (rank, err / scale)
