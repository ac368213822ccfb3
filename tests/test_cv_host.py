"""CV / lambda-path driver host logic (multivartv_amd/cv.py) on the CPU: fold labels, mesh layout,
and the multi-rank distribution of whole paths over torch.distributed (gloo, world size 2)."""
import os
import socket

import numpy as np
import pytest

from multivartv_amd import cv
from oracle import mvtv_oracle as O


def test_kfoldinds_balanced_and_seeded():
    f = cv.kfoldinds(103, 5, seed=7)
    counts = np.bincount(f, minlength=5)
    assert sorted(counts.tolist()) == [20, 20, 21, 21, 21]       # i % k labels (rcpp…/utils.cpp:370-371)
    assert np.array_equal(f, cv.kfoldinds(103, 5, seed=7))
    assert not np.array_equal(f, cv.kfoldinds(103, 5, seed=8))


def test_create_mesh_column_major():
    rng = np.random.default_rng(0)
    data = rng.uniform(-1, 2, size=(50, 3))
    mesh = cv.create_mesh(data, [4, 3, 5])
    assert mesh.shape == (60, 3)
    assert np.array_equal(mesh, O.create_mesh_rcpp(data, [4, 3, 5]))
    # dim 0 fastest (vector2tensor, rcpp…/utils.cpp:59-73)
    assert mesh[1, 0] > mesh[0, 0] and mesh[1, 1] == mesh[0, 1]
    assert mesh[4, 1] > mesh[0, 1] and mesh[4, 0] == mesh[0, 0]
    assert mesh[0, 0] == pytest.approx(data[:, 0].min() - 1e-4)


def test_oracle_folds1_refit_follows_stale_cache_matrix():
    """The oracle's mbs_impl (folds = 1) refits as the reference's mbs_fit_optimal does: b with rho_init =
    lambdas[0] / 5 (rcpp…/solvers.cpp:268, :112) but the first solve on crossO + rho crossD with the rho that
    mbs_path carried INTO its last lambda (:213 -> :273 -> use_cache :47 -> :107, :113)."""
    rng = np.random.default_rng(4)
    x = rng.uniform(0, 1, size=(240, 2))
    y = np.where(np.all(x > 0.6, axis=1), 1.0, 0.0) + 0.3 * rng.standard_normal(240)
    m, lams = [10, 8], [2.0, 1.0, 0.5, 0.2, 0.05]
    ref = O.mbs_impl_rcpp(x, y, m, lams, folds=1)
    mesh, deltas = O.create_mesh_rcpp(x, m), O.create_deltas_rcpp(x, m)
    D = O.build_D(m, O.block_table(2, deltas, "cpp"))
    idx = O.nearest_index(x, mesh)
    W, oty = np.bincount(idx, minlength=80).astype(float), np.bincount(idx, weights=y, minlength=80)
    args = (D, oty, W, lams[ref["best"]], np.full(80, y.mean()), np.zeros(D.shape[0]), lams[0] / 5)
    stale = O.admm_rcpp(*args, sigma0=ref["final"][-2].rho)
    fresh = O.admm_rcpp(*args)
    np.testing.assert_array_equal(ref["best_theta"], stale.theta)
    assert stale.iters != fresh.iters


def test_assign_round_robin():
    items = [cv.assign(7, 3, r) for r in range(3)]
    assert items == [[0, 3, 6], [1, 4], [2, 5]]
    assert sorted(sum(items, [])) == list(range(7))


def _fake_runner(nl, log):
    def run(kind, f):
        log.append((kind, f))
        base = 1.0 if kind == "final" else 2.0 + f
        mses = base + np.arange(nl)[::-1] * 0.1 + (0.05 * ((np.arange(nl) - 2) ** 2) if kind != "final" else 0)
        final = None
        if kind == "final":
            final = dict(thetas=[np.full(4, float(i)) for i in range(nl)], fitted=[np.full(20, float(i)) for i in range(nl)],
                         stats=[{}] * nl, model_mses=mses)
        return mses, final
    return run


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []
    data = np.linspace(0, 1, 20).reshape(-1, 1)
    out = cv.mbs_impl(data, data.ravel(), [4], lambdas=[5, 4, 3, 2, 1], folds=3, _runner=_fake_runner(5, log))
    q.put((rank, log, out["cv.mses"].tolist(), out["lambda_minmse_ind"]))
    dist.destroy_process_group()


def test_distributed_paths_match_serial():
    import torch.multiprocessing as mp
    data = np.linspace(0, 1, 20).reshape(-1, 1)
    log = []
    serial = cv.mbs_impl(data, data.ravel(), [4], lambdas=[5, 4, 3, 2, 1], folds=3, group=False,
                         _runner=_fake_runner(5, log))
    assert sorted(log, key=str) == sorted([("final", None), ("fold", 0), ("fold", 1), ("fold", 2)], key=str)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ran = sorted(sum((r[1] for r in res), []), key=str)
    assert ran == sorted(log, key=str)                       # every path exactly once over the ranks
    assert res[0][1][0] == ("final", None)                   # final path on rank 0
    for r in res:
        assert np.allclose(r[2], serial["cv.mses"], rtol=0, atol=0)
        assert r[3] == serial["lambda_minmse_ind"]


def test_tensor_axes_recovers_create_mesh_axes():
    rng = np.random.default_rng(0)
    x = rng.uniform(-1, 3, size=(50, 3))
    m = [4, 5, 6]
    mesh = cv.create_mesh(x, m)
    axes = cv.tensor_axes(mesh, m)
    assert axes is not None
    for j in range(3):
        np.testing.assert_array_equal(axes[j], np.linspace(x[:, j].min() - 1e-4, x[:, j].max() + 1e-4, m[j]))
    assert cv.tensor_axes(mesh[::-1], m) is None            # not column-major
    assert cv.tensor_axes(mesh[:-1], m) is None             # wrong size
    assert cv.tensor_axes(rng.uniform(size=mesh.shape), m) is None
