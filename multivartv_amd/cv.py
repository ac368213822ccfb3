"""Cross-validated lambda path of the released package over the HIP hot path, sharded across GPUs.

Mirrors ``mbs_impl`` and its helpers in rcpp-code/MultivarTV/src/solvers.cpp:
  create_lambdas   :186-200   lambda grid from lam_max_pinv (GPU, ``Problem.lambda_max``)
  mbs_path         :204-222   warm-started path (theta, u, rho carried; resident on the GPU)
  mbs_fit_optimal  :261-274   cold refit at the best lambda (folds == 1), first solve on the
                              matrix mbs_path left in the cache (:213 -> :273 -> :47 -> :107, :113)
  test_mse         :278-288   held-out MSE per lambda
  mbs_impl         :305-376   folds, final path, best model, result list
with create_mesh (rcpp…/utils.cpp:234-254), create_deltas (:256-263) and kfoldinds (:367-376).

Multi-GPU. One process per GPU (torch.distributed, any backend). The
work items are whole paths — the final path on the full data and one path per CV fold — dealt
round-robin over the ranks (the final path on rank 0), each with the reference's exact warm-start
chain, so results do not depend on the number of ranks. The only collective is a sum of the
per-rank fold-MSE columns (n_lambda x folds doubles). ``lambda_path`` is the throughput form
for a single path: contiguous lambda chunks per rank, cold-started at each chunk's head
(theta = mean y, u = 0, rho = lambda_head / 5).

kfoldinds: the reference shuffles with R's RNG through arma::shuffle, which cannot be reproduced
outside R; here the same round-robin labels are permuted by sorting a seeded splitmix64 key per
position, identically in C++ (mvtv::kfoldinds) and Python.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .utils import create_deltas, interp_weights, nearest_index


def create_mesh(data, m, eps: float = 1e-4):
    """rcpp…/utils.cpp:234-254: column-major (dim 0 fastest) tensor mesh, axes linspace(min-EPS, max+EPS, m_j)."""
    data = np.asarray(data, dtype=np.float64).reshape(len(data), -1)
    axes = [np.linspace(data[:, j].min() - eps, data[:, j].max() + eps, int(m[j])) for j in range(data.shape[1])]
    grids = np.meshgrid(*axes, indexing="ij")
    return np.stack([g.reshape(-1, order="F") for g in grids], axis=1)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def kfoldinds(n: int, k: int, seed: int = 0) -> np.ndarray:
    """rcpp…/utils.cpp:367-376: labels i % k, shuffled. The permutation sorts a seeded splitmix64 key
    per position (stable), the same as the C++ host API's mvtv::kfoldinds (csrc/solvers.cpp)."""
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * np.uint64(0xD1B54A32D192ED03)
        key = _splitmix64(base + np.arange(n, dtype=np.uint64))
    perm = np.argsort(key, kind="stable")
    return (perm % k).astype(np.int64)


def create_lambdas(n_lambda: int, problem: "_lib.Problem", lambdas=None) -> np.ndarray:
    """rcpp…/solvers.cpp:186-200: flipud(exp(linspace(log(lmax 1e-4), log(lmax), n)))."""
    if lambdas is not None:
        return np.asarray(lambdas, dtype=np.float64).ravel()
    lmax, _ = problem.lambda_max()
    return np.exp(np.linspace(np.log(lmax * 0.0001), np.log(lmax), int(n_lambda)))[::-1].copy()


def tensor_axes(mesh, m):
    """The sorted axes of a column-major tensor mesh (create_mesh's layout), or None for any other mesh."""
    mesh = np.asarray(mesh, dtype=np.float64)
    if mesh.size != int(np.prod(m)) * len(m):
        return None
    mesh = mesh.reshape(int(np.prod(m)), len(m))
    strides = np.cumprod([1] + list(m[:-1]))
    axes = [mesh[strides[j] * np.arange(m[j]), j] for j in range(len(m))]
    if any(np.any(np.diff(a) <= 0) for a in axes):
        return None
    grids = np.meshgrid(*axes, indexing="ij")
    ok = all(np.array_equal(g.reshape(-1, order="F"), mesh[:, j]) for j, g in enumerate(grids))
    return axes if ok else None


def _cache(mesh, m, deltas, x, yy, device, problem=None, axes=None):
    """create_cache_objects (rcpp…/solvers.cpp:36-44): O from the nearest mesh point -> W, O^T y.

    On a tensor mesh (always, for create_mesh) O, diag(O^T O) and O^T y are built on the GPU
    (Problem.set_scattered); any other mesh is matched on the host."""
    N = int(np.prod(m))
    if axes is not None:
        if problem is None:
            problem = _lib.Problem(m, np.zeros(N), deltas=deltas, order=_lib.ORDER_CPP, weighted=True, device=device)
        return problem, problem.set_scattered(axes, x, yy)
    idx = nearest_index(x, mesh)
    W, oty = interp_weights(idx, N, yy)
    wdiag = None if np.all(W == 1.0) else W
    if problem is None:
        problem = _lib.Problem(m, oty, wdiag=wdiag, deltas=deltas, order=_lib.ORDER_CPP, weighted=True, device=device)
    else:
        problem.set_data(oty, wdiag)   # the same mesh: CV folds re-run create_cache_objects (:347-348)
    return problem, idx


def mbs_path(problem: "_lib.Problem", lambdas, ymean: float, theta0=None, rho0=None):
    """rcpp…/solvers.cpp:204-222 on the resident state (one mvtv_path call): returns (thetas, stats)
    per lambda."""
    lambdas = np.asarray(lambdas, dtype=np.float64)
    th0 = np.full(problem.N, float(ymean)) if theta0 is None else theta0
    r0 = float(lambdas[0]) / 5.0 if rho0 is None else float(rho0)   # u0 = 0 (B)
    thetas, _, stats = problem.path(lambdas, th0, r0)
    return list(thetas), stats


def _dist(group):
    if group is False:
        return None, 1, 0
    try:
        import torch.distributed as dist
    except ImportError:   # torch is optional for single-process use
        return None, 1, 0
    if not dist.is_available() or not dist.is_initialized():
        return None, 1, 0
    return dist, dist.get_world_size(group), dist.get_rank(group)


def _allreduce_sum(dist, group, arr: np.ndarray) -> np.ndarray:
    import torch
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64))
    if dist.get_backend(group) == "nccl":
        import torch.cuda
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.cpu().numpy()


def assign(n_items: int, world: int, rank: int):
    """Work items dealt round-robin: item i (0 = final path, 1.. = folds) runs on rank i % world."""
    return [i for i in range(n_items) if i % world == rank]


def mbs_impl(data, y, m, mesh=None, n_lambda=100, ftrue=None, lambdas=None, folds=1, verbose=False, seed=0,
             device=None, group=None, _runner=None, concurrent=1):
    """rcpp…/solvers.cpp:305-376. Returns the reference's result list as a dict (rank 0; other
    ranks return only 'cv.mses' and 'lambda_minmse_ind').

    ``_runner(kind, fold)`` replaces the GPU path computation (tests of the distribution logic):
    it returns (mse_vector, final_models) exactly as the internal runner does.

    ``concurrent``: work items of this rank run at once, each on its own problem (HIP stream) and host
    thread; the items are independent, so results do not depend on it.
    """
    data = np.asarray(data, dtype=np.float64)
    if data.ndim == 1:
        data = data.reshape(-1, 1)
    y = np.asarray(y, dtype=np.float64).ravel()
    m = [int(v) for v in np.atleast_1d(m)]
    dist, world, rank = _dist(group)
    if device is None:
        import os
        device = int(os.environ.get("LOCAL_RANK", "0")) if world > 1 else 0
    MESH = create_mesh(data, m) if mesh is None else np.asarray(mesh, dtype=np.float64)
    deltas = create_deltas(data, m)
    FTRUE = y if ftrue is None else np.asarray(ftrue, dtype=np.float64).ravel()
    foldinds = kfoldinds(len(y), folds, seed) if folds > 1 else None

    state = {}
    AXES = tensor_axes(MESH, m)

    import threading
    lock = threading.Lock()

    def problem_for(x, yy, own=False):
        """The rank's shared problem (set to this data), or with own=True a new one (concurrent items)."""
        if own:
            return _cache(MESH, m, deltas, x, yy, device, None, AXES)
        with lock:
            P, idx = _cache(MESH, m, deltas, x, yy, device, state.get("P"), AXES)
            state["P"] = P
        return P, idx

    if lambdas is None or _runner is None:
        P, idx_full = problem_for(data, y)
        LAMBDAS = create_lambdas(n_lambda, P, lambdas)
    else:
        LAMBDAS = np.asarray(lambdas, dtype=np.float64).ravel()
    nl = LAMBDAS.size

    own = concurrent > 1

    def runner(kind, f):
        if kind == "final":
            # models' mse: mbs_mse against ftrue (folds == 1) or y (:214, :355); test_mse against y (:330)
            P, idx = problem_for(data, y, own)
            thetas, stats = mbs_path(P, LAMBDAS, y.mean())
            if own:
                P.close()
            fitted = [th[idx] for th in thetas]
            ref = FTRUE if folds == 1 else y
            model_mses = np.array([np.sum((ft - ref) ** 2) / ref.size for ft in fitted])
            test = np.array([np.sum((ft - y) ** 2) / y.size for ft in fitted])
            return test, dict(thetas=thetas, fitted=fitted, stats=stats, model_mses=model_mses)
        tr, te = foldinds != f, foldinds == f
        P, _ = problem_for(data[tr], y[tr], own)
        thetas, _ = mbs_path(P, LAMBDAS, y[tr].mean())
        ti = P.nearest(AXES, data[te]) if AXES is not None else nearest_index(data[te], MESH)
        if own:
            P.close()
        yt = y[te]
        return np.array([np.sum((th[ti] - yt) ** 2) / yt.size for th in thetas]), None

    run = _runner or runner
    n_items = 1 + (folds if folds > 1 else 0)
    mse_mat = np.zeros((nl, max(folds, 1)))
    final = None

    def do_item(item):
        nonlocal final
        if item == 0:
            mses, final = run("final", None)
            if folds == 1:
                mse_mat[:, 0] = mses
        else:
            mse_mat[:, item - 1], _ = run("fold", item - 1)
        if verbose:
            print(f"[rank {rank}] work item {item} done")

    mine = assign(n_items, world, rank)
    if concurrent > 1 and len(mine) > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=min(concurrent, len(mine))) as ex:
            for fut in [ex.submit(do_item, it) for it in mine]:
                fut.result()
    else:
        for item in mine:
            do_item(item)
    if dist is not None and world > 1:
        mse_mat = _allreduce_sum(dist, group, mse_mat)
    cv = mse_mat[:, 0] if folds == 1 else mse_mat.mean(axis=1)
    best = int(np.argmin(cv))
    if rank != 0:
        return {"cv.mses": cv, "lambda_minmse_ind": best + 1}

    thetas, fitted = final["thetas"], final["fitted"]
    if folds == 1 and _runner is None:
        # mbs_fit_optimal (:261-274): cold start at the best lambda with rho_init = lambdas[0] / 5 (:268), but
        # mbs_one takes the cache (:273), whose sp_crosses mbs_path last set to crossO + rho crossD with the
        # rho carried INTO the last lambda (:213); use_cache copies it (:47) and admm_update's first solve
        # uses it (:107, :113), while b is formed with rho_init (:112).
        P, idx = problem_for(data, y)
        st = final["stats"]
        sigma0 = float(st[-2]["rho"]) if len(st) >= 2 else float(LAMBDAS[0]) / 5.0
        th, _, _, _ = P.admm(float(LAMBDAS[best]), np.full(P.N, y.mean()), u=None, rho=float(LAMBDAS[0]) / 5.0,
                             return_u=False, sigma=sigma0)
        best_theta, best_fit = th, th[idx]
    else:
        best_theta, best_fit = thetas[best], fitted[best]
    models = [{"lambda": float(LAMBDAS[i]), "mse": float(final["model_mses"][i]), "theta_hat": thetas[i],
               "fitted": fitted[i]} for i in range(nl)]
    if "P" in state:
        state["P"].close()
    return {"data": data, "fitted": best_fit, "m": m, "mesh": MESH, "theta_hat": best_theta, "y": y,
            "residuals": y - best_fit, "models": models, "lambda_minmse_ind": best + 1, "cv.mses": cv}


def lambda_path(problem: "_lib.Problem", lambdas, ymean: float, group=None):
    """Throughput form of one lambda path over the ranks: rank r takes the
    r-th contiguous chunk of ``lambdas``, warm-started inside the chunk and cold-started at its head.
    Returns (thetas of this rank's chunk, chunk slice, per-lambda ADMM iterations of all ranks)."""
    lambdas = np.asarray(lambdas, dtype=np.float64)
    dist, world, rank = _dist(group)
    bounds = np.linspace(0, lambdas.size, world + 1).round().astype(int)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    thetas, stats = mbs_path(problem, lambdas[lo:hi], ymean) if hi > lo else ([], [])
    iters = np.zeros(lambdas.size)
    iters[lo:hi] = [s["iters"] for s in stats]
    if dist is not None and world > 1:
        iters = _allreduce_sum(dist, group, iters)
    return thetas, slice(lo, hi), iters
