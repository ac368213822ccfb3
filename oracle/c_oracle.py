"""ctypes front of oracle/c/mvtv_oracle.c — CPU ORACLE, TEST INFRASTRUCTURE ONLY.

Used by tests/ (pinned against the SuperLU oracle) and by bench.py's
cpu_baseline leg. Never imported by the multivartv_amd package.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libmvtv_oracle.so")
_L = None
_dp = C.POINTER(C.c_double)


def lib():
    global _L
    if _L is None:
        if not os.path.exists(_PATH):
            raise ImportError(f"{_PATH} not built (make -C oracle)")
        L = C.CDLL(_PATH)
        L.mvtv_oracle_threads.restype = C.c_int
        L.mvtv_oracle_edges.restype = C.c_int64
        L.mvtv_oracle_edges.argtypes = [C.c_int, C.POINTER(C.c_int64), C.c_int, C.c_int]
        L.mvtv_oracle_admm_rcpp.restype = C.c_int
        L.mvtv_oracle_admm_rcpp.argtypes = [C.c_int, C.POINTER(C.c_int64), C.c_int, C.c_int, _dp, _dp, _dp,
                                            C.c_double, _dp, _dp, _dp, C.c_int, C.c_double, C.c_int, C.c_double,
                                            C.c_int, C.c_int, _dp]
        _L = L
    return _L


def threads() -> int:
    return int(lib().mvtv_oracle_threads())


def set_threads(n: int) -> None:
    """omp_set_num_threads for the following oracle calls."""
    L = lib()
    L.mvtv_oracle_set_threads.restype = None
    L.mvtv_oracle_set_threads.argtypes = [C.c_int]
    L.mvtv_oracle_set_threads(int(n))


def num_edges(m, order=0, weighted=1) -> int:
    mm = (C.c_int64 * 4)(*([int(v) for v in m] + [1] * (4 - len(m))))
    return int(lib().mvtv_oracle_edges(len(m), mm, order, weighted))


def admm_rcpp(m, oty, lam, theta, u, rho, deltas, W=None, order=0, weighted=1, fixed_iters=0, tol=1e-4,
              max_counter=3000, pcg_rtol=1e-12, pcg_fixed=0, pcg_maxit=20000):
    """Variant-B ADMM on the CPU (matrix-free D, Jacobi-PCG). theta/u are updated in place."""
    mm = (C.c_int64 * 4)(*([int(v) for v in m] + [1] * (4 - len(m))))
    dl = np.ascontiguousarray(list(deltas) + [1.0] * (4 - len(deltas)), dtype=np.float64)
    oty = np.ascontiguousarray(oty, dtype=np.float64)
    Wp = None if W is None else np.ascontiguousarray(W, dtype=np.float64)
    r = C.c_double(rho)
    stats = np.zeros(8)
    rc = lib().mvtv_oracle_admm_rcpp(len(m), mm, order, weighted, dl.ctypes.data_as(_dp), oty.ctypes.data_as(_dp),
                                     None if Wp is None else Wp.ctypes.data_as(_dp), float(lam),
                                     theta.ctypes.data_as(_dp), u.ctypes.data_as(_dp), C.byref(r), int(fixed_iters),
                                     float(tol), int(max_counter), float(pcg_rtol), int(pcg_fixed), int(pcg_maxit),
                                     stats.ctypes.data_as(_dp))
    if rc != 0:
        raise RuntimeError(f"oracle admm failed ({rc})")
    return dict(rho=r.value, iters=int(stats[0]), r_norm=stats[1], s_norm=stats[2], eps_pri=stats[3],
                eps_dual=stats[4], pcg_iters=int(stats[5]), pcg_relres_max=stats[6])


_SOLVE_FN = C.CFUNCTYPE(C.c_int, C.c_double, _dp, _dp, C.c_void_p)


def _bind_ext():
    L = lib()
    if not hasattr(L, "_ext_bound"):
        L.mvtv_oracle_admm_rcpp_cb.restype = C.c_int
        L.mvtv_oracle_admm_rcpp_cb.argtypes = [C.c_int, C.POINTER(C.c_int64), C.c_int, C.c_int, _dp, _dp, C.c_double,
                                               _dp, _dp, _dp, C.c_int, C.c_double, C.c_int, _dp, _SOLVE_FN, C.c_void_p]
        for name in ("mvtv_oracle_apply_D", "mvtv_oracle_apply_Dt"):
            f = getattr(L, name)
            f.restype = C.c_int
            f.argtypes = [C.c_int, C.POINTER(C.c_int64), C.c_int, C.c_int, _dp, _dp, _dp]
        L._ext_bound = True
    return L


def _geom_args(m, deltas):
    mm = (C.c_int64 * 4)(*([int(v) for v in m] + [1] * (4 - len(m))))
    dl = np.ascontiguousarray(list(deltas) + [1.0] * (4 - len(deltas)), dtype=np.float64)
    return mm, dl


def apply_D(m, theta, deltas, order=0, weighted=1):
    L = _bind_ext()
    mm, dl = _geom_args(m, deltas)
    th = np.ascontiguousarray(theta, dtype=np.float64)
    d = np.empty(num_edges(m, order, weighted))
    if L.mvtv_oracle_apply_D(len(m), mm, order, weighted, dl.ctypes.data_as(_dp), th.ctypes.data_as(_dp),
                             d.ctypes.data_as(_dp)) != 0:
        raise RuntimeError("apply_D")
    return d


def dtd_symbol(m, deltas, order=0, weighted=1):
    """sum_S cS[S] prod_{j in S} 4 sin^2(pi k_j / 2 m_j) on the (k_0, ..., k_{p-1}) grid (Fortran order):
    the eigenvalues of D^T D in the cosine basis (cS[S] = sum of w_b^2 over blocks with S'(b) = S)."""
    from .mvtv_oracle import block_table
    p = len(m)
    blocks = block_table(p, deltas if weighted else None, "cpp" if order == 0 else "py", unit_weights=not weighted)
    cS = {}
    for blk in blocks:
        cS[blk.Sp] = cS.get(blk.Sp, 0.0) + blk.w * blk.w
    lam = [4.0 * np.sin(np.pi * np.arange(mj) / (2.0 * mj)) ** 2 for mj in m]
    out = np.zeros([int(v) for v in m], order="F")
    for S, c in cS.items():
        term = np.full([1] * p, c)
        for j in S:
            shape = [1] * p
            shape[j] = int(m[j])
            term = term * lam[j].reshape(shape)
        out += term
    return out


def admm_rcpp_spectral(m, oty, lam, theta, u, rho, deltas, fixed_iters=0, tol=1e-4, max_counter=3000, workers=-1,
                       sym=None):
    """Variant-B ADMM on the CPU (the C oracle's loop) with the exact theta-solve of the GPU's headline path:
    (I + rho D^T D) theta = b by scipy.fft.dctn / idctn (orthonormal DCT-II, `workers` threads). W = I.
    theta / u are updated in place."""
    import scipy.fft as sfft
    L = _bind_ext()
    shape = [int(v) for v in m]
    N = int(np.prod(shape))
    sym = dtd_symbol(m, deltas) if sym is None else sym

    def solve(sigma, b_ptr, x_ptr, _ctx):
        try:
            b = np.ctypeslib.as_array(b_ptr, shape=(N,)).reshape(shape, order="F")
            x = np.ctypeslib.as_array(x_ptr, shape=(N,)).reshape(shape, order="F")
            t = sfft.dctn(b, type=2, norm="ortho", workers=workers)
            t /= 1.0 + sigma * sym
            x[...] = sfft.idctn(t, type=2, norm="ortho", workers=workers)
            return 0
        except Exception:   # noqa: BLE001 (reported as a failed call)
            return 1

    cb = _SOLVE_FN(solve)
    mm, dl = _geom_args(m, deltas)
    oty = np.ascontiguousarray(oty, dtype=np.float64)
    r = C.c_double(rho)
    stats = np.zeros(8)
    rc = L.mvtv_oracle_admm_rcpp_cb(len(m), mm, 0, 1, dl.ctypes.data_as(_dp), oty.ctypes.data_as(_dp), float(lam),
                                    theta.ctypes.data_as(_dp), u.ctypes.data_as(_dp), C.byref(r), int(fixed_iters),
                                    float(tol), int(max_counter), stats.ctypes.data_as(_dp), cb, None)
    if rc != 0:
        raise RuntimeError(f"oracle spectral admm failed ({rc})")
    return dict(rho=r.value, iters=int(stats[0]), r_norm=stats[1], s_norm=stats[2], eps_pri=stats[3],
                eps_dual=stats[4])
