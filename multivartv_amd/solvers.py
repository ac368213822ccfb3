"""The reference's Python solver API (code/solvers.py) on the MI355X hot path.

Same functions, arguments and result dictionaries as code/solvers.py:
``softthresh``, ``mbs_one``, ``mbs_predict``, ``mbs_mse``, ``mbs``. The ADMM loop
(variant C semantics: rho = lambda = tune, threshold lambda/rho, u0 = 1/lambda,
stop at max|theta - theta_old| <= tol) runs in libmvtv.so through the C ABI; there
is no CPU fallback.

``cache``: the reference's cache is a list holding a SuperLU factor and sparse
matrices (code/solvers.py:42-51). Here it is an :class:`MbsCache` (GPU-resident
problem + nearest-mesh index), built by :func:`make_cache` or by ``mbs``.

lambda_max: the reference computes it on the host with SuperLU on the singular matrix
D^T D (code/utils.py:198-209); :func:`lam_max` builds the same sparse D (utils.create_D) and
calls the same library (scipy's SuperLU), so the no-cache ``mbs_one`` and ``mbs`` without
``tuners`` use the reference's own tuning values (setup, not the hot path).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib
from .utils import create_D, interp_weights, lam_max_pinv, mesh_coords, nearest_index


def softthresh(z, lam):
    """code/solvers.py:9-12."""
    z = np.asarray(z, dtype=np.float64)
    return np.sign(z) * np.maximum(np.abs(z) - lam, 0.0)


@dataclass
class MbsCache:
    problem: _lib.Problem
    idx: np.ndarray      # nearest-mesh row of every data point (O)
    mesh: np.ndarray
    ntheta: int
    sigma: float         # the factored matrix is crossO + sigma * crossD (code/solvers.py:37, :130)

    @property
    def rowsD(self):
        return self.problem.E


def make_cache(data, y, m, mesh=None, deltas=None, sigma=1.0, weighted=None, device=0):
    """The reference's cache for mbs_one: O from the nearest mesh point, D = create_D(m, deltas)."""
    data = np.asarray(data, dtype=np.float64)
    if data.ndim == 1:
        data = data.reshape(-1, 1)
    m = [int(v) for v in np.atleast_1d(m)]
    if mesh is None:
        mo = mesh_coords(data, m)
        mesh, deltas = mo["mesh"], mo["deltas"] if deltas is None else deltas
    idx = nearest_index(data, mesh)
    N = int(np.prod(m))
    W, oty = interp_weights(idx, N, y)
    if weighted is None:
        weighted = deltas is not None
    # Python create_D: deltas=None -> all 2^p - 1 blocks unweighted; with deltas the all-ones
    # block is dropped (code/utils.py:138-149)
    P = _lib.Problem(m, oty, wdiag=W, deltas=deltas if deltas is not None else [1.0] * len(m),
                     order=_lib.ORDER_PY, weighted=weighted, device=device)
    return MbsCache(P, idx, np.asarray(mesh), N, float(sigma))


def lam_max(cache: MbsCache, deltas=None):
    """code/utils.py:206-209 (lam_max_pinv) for the cache's mesh and data: max |D splu(D^T D).solve(O^T y)|
    with D = create_D(m, deltas) built on the host exactly as the reference builds it."""
    m = cache.problem.m
    return lam_max_pinv(create_D(m, deltas), cache.problem._oty)


def mbs_one(data, y, m, theta_init=None, mesh=None, tune=1.0, eps=0.01, tol=0.001, cache=None):
    """code/solvers.py:15-78. Returns {'mesh','theta.hat','fitted','data','y','eps','m','counter'}."""
    y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
    if cache is None:
        if mesh is not None:
            # the reference leaves `deltas` unbound on this path (code/solvers.py:24-31)
            raise NameError("name 'deltas' is not defined")
        data = np.asarray(data, dtype=np.float64)
        data = data.reshape(-1, 1) if data.ndim == 1 else data
        deltas = mesh_coords(data, m)["deltas"]
        if len(np.atleast_1d(m)) == 1:
            raise ValueError("blocks must be 2-D")   # create_D(m, deltas) at p = 1 (code/utils.py:145-148)
        cache = make_cache(data, y, m, sigma=tune)
        tune = lam_max(cache, deltas)
        cache.sigma = tune
    ntheta = cache.ntheta
    ym = float(np.mean(y))
    theta0 = np.full(ntheta, ym) if theta_init is None else np.asarray(theta_init, dtype=np.float64).ravel()
    th, _, _, st = cache.problem.admm(float(tune), theta0, variant=_lib.VARIANT_PY, ymean=ym, tol=tol,
                                      sigma=cache.sigma, return_u=False)
    theta = th.reshape(ntheta, 1)
    fitted = theta[cache.idx]
    return {"mesh": cache.mesh, "theta.hat": theta, "fitted": fitted, "data": data, "y": y, "eps": eps, "m": m,
            "counter": 1}


def mbs_predict(mbs_one_object, data):
    """code/solvers.py:80-83."""
    idx = nearest_index(data, mbs_one_object["mesh"])
    return np.asarray(mbs_one_object["theta.hat"]).reshape(-1, 1)[idx]


def mbs_mse(mbs_one_object, y):
    """code/solvers.py:85-89."""
    yhat = np.asarray(mbs_one_object["fitted"]).ravel()
    ytrue = np.asarray(y).ravel()
    return np.sum((yhat - ytrue) ** 2) / ytrue.size


def mbs(data, y, m, ftrue=None, mesh=None, ntune=100, tuners=None, eps=0.01):
    """code/solvers.py:91-141: warm-started path over tuners, best by MSE against ftrue.

    As in the reference, the factored matrix lags the tuning parameter: fit i uses
    crossO + sigma_i crossD with sigma_0 = sigma_1 = lambda_max, sigma_i = tuners[i-2].
    """
    data = np.asarray(data, dtype=np.float64)
    if data.ndim == 1:
        data = data.reshape(-1, 1)
    n = data.shape[0]
    y = np.asarray(y, dtype=np.float64).reshape(n, 1)
    mo = mesh_coords(data, m)
    mesh_, deltas = mo["mesh"], mo["deltas"]
    cache = make_cache(data, y, m, mesh=mesh_ if mesh is None else mesh, deltas=deltas)
    if tuners is None:
        lmax = lam_max(cache, deltas) * float(np.prod(deltas))
        tuners = np.exp(np.linspace(np.log(lmax * 1e-4), np.log(lmax), ntune))[::-1]
        rho = lmax
    else:
        tuners = np.asarray(tuners, dtype=np.float64)
        rho = float(tuners[0])
    ftrue = y if ftrue is None else np.asarray(ftrue, dtype=np.float64)
    fits, mses = [], []
    thetainit = np.full(cache.ntheta, float(np.mean(y)))
    for i, tune in enumerate(tuners):
        cache.sigma = rho
        if i > 0:
            rho = tuners[i - 1]
        fit = mbs_one(data, y, m, mesh=mesh_, tune=tune, eps=eps, theta_init=thetainit, cache=cache)
        fits.append(fit)
        mses.append(mbs_mse(fit, ftrue))
        thetainit = fit["theta.hat"]
    best = int(np.argmin(mses))
    return {"minmse.fits": fits[best], "minmse": mses[best], "minmse.lam": tuners[best]}
