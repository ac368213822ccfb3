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
