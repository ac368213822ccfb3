"""ctypes binding of libmvtv.so (include/mvtv/mvtv.h).

The library is built in-tree (``multivartv_amd/lib/libmvtv.so``, see
``__graft_entry__.build``). There is no CPU fallback: if the library or a HIP
device is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np

# MVTV_LIB_PATH: load another build of the same library (e.g. a probe build, `make PROBES=1 OUT=...`)
LIB_PATH = os.environ.get("MVTV_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                           "libmvtv.so")

MVTV_OK, MVTV_MAXITER, MVTV_BAD_ARG, MVTV_DIM_MISMATCH = 0, 1, 2, 3
MVTV_HIP_ERROR, MVTV_NO_DEVICE, MVTV_OUT_OF_MEMORY, MVTV_PCG_NOT_CONVERGED = 4, 5, 6, 7
VARIANT_RCPP, VARIANT_CPP, VARIANT_PY = 0, 1, 2
ORDER_CPP, ORDER_PY = 0, 1
KERNELS = ["edge_update", "gather_Dt", "pcg_init", "pcg_apply_A", "pcg_update", "pcg_direction", "reduce", "other",
           "pcg_fused3d", "dct_first", "dct", "admm_fused", "gather4_b", "dct_first_fold",
           "admm_fused4"]
SOLVER_AUTO, SOLVER_PCG, SOLVER_SPECTRAL, SOLVER_PCG_SPECTRAL = 0, 1, 2, 3

_dp = C.POINTER(C.c_double)


class ProblemDesc(C.Structure):
    _fields_ = [("p", C.c_int32), ("m", C.c_int64 * 4), ("block_order", C.c_int32), ("weighted", C.c_int32),
                ("deltas", C.c_double * 4), ("oty", _dp), ("wdiag", _dp), ("device", C.c_int32)]


class AdmmOpts(C.Structure):
    _fields_ = [("variant", C.c_int32), ("tol", C.c_double), ("max_counter", C.c_int32),
                ("fixed_iters", C.c_int32), ("sigma", C.c_double), ("ymean", C.c_double),
                ("pcg_rtol", C.c_double), ("pcg_max_iter", C.c_int32), ("pcg_strict", C.c_int32),
                ("verbose", C.c_int32), ("theta_solver", C.c_int32)]


class AdmmStats(C.Structure):
    _fields_ = [("iters", C.c_int32), ("status", C.c_int32), ("r_norm", C.c_double), ("s_norm", C.c_double),
                ("eps_pri", C.c_double), ("eps_dual", C.c_double), ("rho", C.c_double),
                ("dtheta_max", C.c_double), ("pcg_iters", C.c_int64), ("pcg_iters_max", C.c_int32),
                ("pcg_unconverged", C.c_int32), ("seconds", C.c_double), ("theta_solver", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class MvtvError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"mvtv status {status}: {msg}")
        self.status = status


class DimMismatchError(MvtvError, ValueError):
    pass


class MaxIterError(MvtvError):
    pass


_LIB = None

# name -> (restype, argtypes); mirrors include/mvtv/mvtv.h
SIGNATURES = {
    "mvtv_version": (C.c_char_p, []),
    "mvtv_status_string": (C.c_char_p, [C.c_int32]),
    "mvtv_last_error": (C.c_char_p, []),
    "mvtv_device_count": (C.c_int32, []),
    "mvtv_default_opts": (None, [C.POINTER(AdmmOpts), C.c_int32]),
    "mvtv_problem_create": (C.c_int, [C.POINTER(ProblemDesc), C.POINTER(C.c_void_p)]),
    "mvtv_problem_destroy": (None, [C.c_void_p]),
    "mvtv_problem_nodes": (C.c_int64, [C.c_void_p]),
    "mvtv_problem_edges": (C.c_int64, [C.c_void_p]),
    "mvtv_problem_blocks": (C.c_int32, [C.c_void_p]),
    "mvtv_problem_block_info": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32), _dp]),
    "mvtv_problem_set_data": (C.c_int, [C.c_void_p, _dp, _dp]),
    "mvtv_problem_spectral_ok": (C.c_int32, [C.c_void_p]),
    "mvtv_admm": (C.c_int, [C.c_void_p, C.POINTER(AdmmOpts), C.c_double, _dp, _dp, _dp, C.POINTER(AdmmStats)]),
    "mvtv_state_set": (C.c_int, [C.c_void_p, _dp, _dp, C.c_double]),
    "mvtv_state_get": (C.c_int, [C.c_void_p, _dp, _dp, _dp]),
    "mvtv_admm_run": (C.c_int, [C.c_void_p, C.POINTER(AdmmOpts), C.c_double, C.POINTER(AdmmStats)]),
    "mvtv_path": (C.c_int, [C.c_void_p, C.POINTER(AdmmOpts), _dp, C.c_int32, _dp, C.c_double, _dp, _dp,
                            C.POINTER(AdmmStats)]),
    "mvtv_fitted": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int64, _dp]),
    "mvtv_nearest": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, C.POINTER(C.c_int64)]),
    "mvtv_problem_set_scattered": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp, C.POINTER(C.c_int64)]),
    "mvtv_predict": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, _dp]),
    "mvtv_apply_D": (C.c_int, [C.c_void_p, _dp, _dp]),
    "mvtv_apply_Dt": (C.c_int, [C.c_void_p, _dp, _dp]),
    "mvtv_apply_A": (C.c_int, [C.c_void_p, C.c_double, _dp, _dp]),
    "mvtv_solve": (C.c_int, [C.c_void_p, C.c_double, _dp, _dp, C.c_double, C.c_int32, C.POINTER(C.c_int32), _dp]),
    "mvtv_solve_spectral": (C.c_int, [C.c_void_p, C.c_double, _dp, _dp]),
    "mvtv_lambda_max": (C.c_int, [C.c_void_p, _dp, C.POINTER(C.c_int32)]),
    "mvtv_lambda_max_cpp": (C.c_int, [C.c_void_p, _dp, C.POINTER(C.c_int32)]),
    "mvtv_timing_enable": (C.c_int, [C.c_void_p, C.c_int32]),
    "mvtv_timing_get": (C.c_int, [C.c_void_p, C.c_int32, _dp, C.POINTER(C.c_int64), _dp]),
    "mvtv_kernel_name": (C.c_char_p, [C.c_int32]),
}


def lib():
    """Load libmvtv.so (raises if it was not built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def _check(status):
    if status in (MVTV_OK,):
        return status
    msg = lib().mvtv_last_error().decode()
    if status == MVTV_DIM_MISMATCH:
        raise DimMismatchError(status, msg)
    if status == MVTV_MAXITER:
        raise MaxIterError(status, msg)
    raise MvtvError(status, msg)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _f64(a, n=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).ravel())
    if n is not None and a.size != n:
        raise ValueError(f"expected {n} values, got {a.size}")
    return a


def device_count() -> int:
    return int(lib().mvtv_device_count())


def default_opts(variant=VARIANT_RCPP, **kw) -> AdmmOpts:
    o = AdmmOpts()
    lib().mvtv_default_opts(C.byref(o), variant)
    for k, v in kw.items():
        if v is None:
            continue
        if not hasattr(o, k):
            raise TypeError(f"unknown option {k}")
        setattr(o, k, v)
    return o


class Problem:
    """A mesh-TV problem resident on one GPU (wraps mvtv_problem)."""

    def __init__(self, m, oty, wdiag=None, deltas=None, order=ORDER_CPP, weighted=None, device=0):
        m = [int(v) for v in m]
        p = len(m)
        if not 1 <= p <= 4:
            raise ValueError("p must be 1..4")
        self.m, self.p = m, p
        self.N = int(np.prod(m))
        d = ProblemDesc()
        d.p = p
        for j in range(4):
            d.m[j] = m[j] if j < p else 1
            d.deltas[j] = float(deltas[j]) if (deltas is not None and j < p) else 0.0
        d.block_order = order
        d.weighted = int(deltas is not None) if weighted is None else int(weighted)
        self.deltas = None if deltas is None else [float(v) for v in deltas]
        self.order, self.weighted, self.device = order, bool(d.weighted), device
        self._oty = _f64(oty, self.N)
        self._w = None if wdiag is None else _f64(wdiag, self.N)
        d.oty = _ptr(self._oty)
        d.wdiag = _ptr(self._w)
        d.device = device
        h = C.c_void_p()
        _check(lib().mvtv_problem_create(C.byref(d), C.byref(h)))
        self._h = h
        self.E = int(lib().mvtv_problem_edges(h))
        self.nb = int(lib().mvtv_problem_blocks(h))

    def close(self):
        if getattr(self, "_h", None):
            lib().mvtv_problem_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def block_info(self):
        out = []
        for k in range(self.nb):
            code, sp, w = C.c_int32(), C.c_int32(), C.c_double()
            _check(lib().mvtv_problem_block_info(self._h, k, C.byref(code), C.byref(sp), C.byref(w)))
            out.append((code.value, sp.value, w.value))
        return out

    def set_data(self, oty, wdiag=None):
        self._oty = _f64(oty, self.N)
        self._w = None if wdiag is None else _f64(wdiag, self.N)
        _check(lib().mvtv_problem_set_data(self._h, _ptr(self._oty), _ptr(self._w)))

    # ---- hot path ---------------------------------------------------------------------------
    def admm(self, lam, theta, u=None, rho=None, variant=VARIANT_RCPP, return_u=True, **opts):
        """admm_update drop-in: returns (theta, u, rho, stats)."""
        o = default_opts(variant, **opts)
        th = _f64(theta, self.N).copy()
        uu = None
        if u is not None:
            uu = _f64(u, self.E).copy()
        elif return_u:
            uu = None
        r = C.c_double(lam / 5.0 if rho is None else float(rho))
        st = AdmmStats()
        if u is None and return_u:
            # u0 is the variant default; form it on device, then read it back
            _check(lib().mvtv_state_set(self._h, _ptr(th), None, r.value))
            s = lib().mvtv_admm_run(self._h, C.byref(o), float(lam), C.byref(st))
            if s not in (MVTV_OK, MVTV_MAXITER):
                _check(s)
            uu = np.empty(self.E)
            _check(lib().mvtv_state_get(self._h, _ptr(th), _ptr(uu), C.byref(r)))
        else:
            s = lib().mvtv_admm(self._h, C.byref(o), float(lam), _ptr(th), _ptr(uu), C.byref(r), C.byref(st))
        if s == MVTV_MAXITER and variant == VARIANT_CPP:
            _check(s)
        elif s not in (MVTV_OK, MVTV_MAXITER):
            _check(s)
        return th, uu, r.value, st.as_dict()

    def state_set(self, theta, u=None, rho=0.0):
        self._st_th = _f64(theta, self.N)
        self._st_u = None if u is None else _f64(u, self.E)
        _check(lib().mvtv_state_set(self._h, _ptr(self._st_th), _ptr(self._st_u), float(rho)))

    def state_get(self, want_u=True):
        th = np.empty(self.N)
        uu = np.empty(self.E) if want_u else None
        r = C.c_double()
        _check(lib().mvtv_state_get(self._h, _ptr(th), _ptr(uu), C.byref(r)))
        return th, uu, r.value

    def run(self, lam, variant=VARIANT_RCPP, allow_maxiter=True, **opts):
        o = default_opts(variant, **opts)
        st = AdmmStats()
        s = lib().mvtv_admm_run(self._h, C.byref(o), float(lam), C.byref(st))
        if not (s == MVTV_OK or (s == MVTV_MAXITER and allow_maxiter)):
            _check(s)
        return st.as_dict()

    def path(self, lambdas, theta_init, rho_init, variant=VARIANT_RCPP, want_thetas=True, **opts):
        """mbs_path's warm-started lambda loop in one C call (mvtv_path): (thetas [n x N] or None,
        rhos [n], stats list)."""
        o = default_opts(variant, **opts)
        lam = _f64(lambdas)
        n = lam.size
        th0 = _f64(theta_init, self.N)
        thetas = np.empty((n, self.N)) if want_thetas else None
        rhos = np.empty(n)
        sts = (AdmmStats * max(n, 1))()
        s = lib().mvtv_path(self._h, C.byref(o), _ptr(lam), n, _ptr(th0), float(rho_init),
                            None if thetas is None else thetas.ctypes.data_as(_dp), _ptr(rhos), sts)
        if s not in (MVTV_OK, MVTV_MAXITER):
            _check(s)
        return thetas, rhos, [sts[i].as_dict() for i in range(n)]

    def fitted(self, mesh_index):
        idx = np.ascontiguousarray(np.asarray(mesh_index, dtype=np.int64).ravel())
        out = np.empty(idx.size)
        _check(lib().mvtv_fitted(self._h, idx.ctypes.data_as(C.POINTER(C.c_int64)), idx.size, _ptr(out)))
        return out

    # ---- scattered data (nearest_interp_matrix, create_cache_objects, mbs_predict) -------------
    def _axes_data(self, axes, data):
        axes = [np.asarray(a, dtype=np.float64).ravel() for a in axes]
        if len(axes) != self.p or any(a.size != mj for a, mj in zip(axes, self.m)):
            raise ValueError("axes must hold m_j sorted values per dimension")
        ax = np.ascontiguousarray(np.concatenate(axes))
        d = np.asarray(data, dtype=np.float64)
        d = d.reshape(-1, 1) if d.ndim == 1 else d
        if d.shape[1] != self.p:
            raise ValueError(f"data must be n x {self.p}")
        return ax, np.asfortranarray(d), d.shape[0]

    def nearest(self, axes, data):
        """nearest1 (rcpp…/utils.cpp:280-287) on the GPU: column-major mesh node of each data row."""
        ax, d, n = self._axes_data(axes, data)
        idx = np.empty(n, dtype=np.int64)
        _check(lib().mvtv_nearest(self._h, _ptr(ax), d.ctypes.data_as(_dp), n,
                                  idx.ctypes.data_as(C.POINTER(C.c_int64))))
        return idx

    def set_scattered(self, axes, data, y):
        """create_cache_objects (rcpp…/solvers.cpp:36-44) on the GPU: O^T y and diag(O^T O) become the
        problem's data; returns the mesh node of each data row."""
        ax, d, n = self._axes_data(axes, data)
        yy = _f64(y, n)
        idx = np.empty(n, dtype=np.int64)
        _check(lib().mvtv_problem_set_scattered(self._h, _ptr(ax), d.ctypes.data_as(_dp), n, _ptr(yy),
                                                idx.ctypes.data_as(C.POINTER(C.c_int64))))
        return idx

    def predict(self, axes, data):
        """mbs_predict (rcpp…/solvers.cpp:161-165): O(data) theta of the resident state."""
        ax, d, n = self._axes_data(axes, data)
        out = np.empty(n)
        _check(lib().mvtv_predict(self._h, _ptr(ax), d.ctypes.data_as(_dp), n, _ptr(out)))
        return out

    # ---- operators --------------------------------------------------------------------------
    def apply_D(self, theta):
        th = _f64(theta, self.N)
        out = np.empty(self.E)
        _check(lib().mvtv_apply_D(self._h, _ptr(th), _ptr(out)))
        return out

    def apply_Dt(self, v):
        vv = _f64(v, self.E)
        out = np.empty(self.N)
        _check(lib().mvtv_apply_Dt(self._h, _ptr(vv), _ptr(out)))
        return out

    def apply_A(self, sigma, x):
        xx = _f64(x, self.N)
        out = np.empty(self.N)
        _check(lib().mvtv_apply_A(self._h, float(sigma), _ptr(xx), _ptr(out)))
        return out

    def solve(self, sigma, b, x0=None, rtol=1e-12, max_iter=20000):
        bb = _f64(b, self.N)
        x = np.zeros(self.N) if x0 is None else _f64(x0, self.N).copy()
        it, rr = C.c_int32(), C.c_double()
        _check(lib().mvtv_solve(self._h, float(sigma), _ptr(bb), _ptr(x), float(rtol), int(max_iter),
                                C.byref(it), C.byref(rr)))
        return x, it.value, rr.value

    def lambda_max(self):
        """lam_max_pinv of the released package on the GPU: (lambda_max, CG iterations)."""
        v, it = C.c_double(), C.c_int32()
        _check(lib().mvtv_lambda_max(self._h, C.byref(v), C.byref(it)))
        return v.value, it.value

    def lambda_max_cpp(self):
        """lam_max_pinv of the research code (cpp-code/utils.cpp:354-404) on the GPU: (lambda_max, CG iterations)."""
        v, it = C.c_double(), C.c_int32()
        _check(lib().mvtv_lambda_max_cpp(self._h, C.byref(v), C.byref(it)))
        return v.value, it.value

    def spectral_ok(self) -> bool:
        return bool(lib().mvtv_problem_spectral_ok(self._h))

    def solve_spectral(self, sigma, b):
        bb = _f64(b, self.N)
        x = np.empty(self.N)
        _check(lib().mvtv_solve_spectral(self._h, float(sigma), _ptr(bb), _ptr(x)))
        return x

    # ---- instrumentation --------------------------------------------------------------------
    def timing(self, on=True):
        _check(lib().mvtv_timing_enable(self._h, int(on)))

    def timings(self):
        out = {}
        for k, name in enumerate(KERNELS):
            ms, n, b = C.c_double(), C.c_int64(), C.c_double()
            _check(lib().mvtv_timing_get(self._h, k, C.byref(ms), C.byref(n), C.byref(b)))
            out[name] = dict(ms=ms.value, launches=n.value, bytes_per_launch=b.value)
        return out


def nan():
    return math.nan
