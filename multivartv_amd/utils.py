"""Host-side setup mirroring the reference's code/utils.py (mesh, nearest-mesh map, deltas).

These are O(n p) bookkeeping steps around the hot path; the ADMM loop itself runs in
libmvtv.so. The mesh keeps the reference's row order exactly, including the p >= 3
quirk of np.meshgrid's default 'xy' indexing (code/utils.py:188), so a fit through
this module sees the same theta layout as the reference.
"""
from __future__ import annotations

import numpy as np


def mesh_coords(data, mesh_dims, eps: float = 0.01):
    """code/utils.py:179-193 -> {'mesh': (N, p) array, 'deltas': [delta_j]}."""
    data = np.asarray(data, dtype=np.float64)
    if data.ndim == 1:
        data = data.reshape(-1, 1)
    axes, deltas = [], []
    for j in range(data.shape[1]):
        a = np.linspace(data[:, j].min() - eps, data[:, j].max() + eps, int(mesh_dims[j]))
        axes.append(a)
        deltas.append(np.diff(a)[0])
    grids = np.meshgrid(*axes)
    mesh = np.concatenate([g.reshape(-1, 1) for g in grids], axis=1)
    return {"mesh": mesh, "deltas": deltas}


def _axes_of(mesh):
    """Per-dimension sorted axis values and, per mesh row, its per-dimension axis index."""
    axes, pos = [], []
    for j in range(mesh.shape[1]):
        vals, inv = np.unique(mesh[:, j], return_inverse=True)
        axes.append(vals)
        pos.append(inv)
    return axes, pos


def nearest_index(data, mesh):
    """Row index of the nearest mesh point for every data row (the 1 in row i of O).

    The reference scans all mesh rows (code/utils.py:153-161). For a tensor-product mesh the
    squared distance separates by dimension, so each coordinate is matched on its own axis and
    the resulting multi-index is mapped back to the mesh's row order.
    """
    data = np.asarray(data, dtype=np.float64)
    mesh = np.asarray(mesh, dtype=np.float64)
    if data.ndim == 1:
        data = data.reshape(-1, 1)
    if mesh.ndim == 1:
        mesh = mesh.reshape(-1, 1)
    axes, pos = _axes_of(mesh)
    dims = [len(a) for a in axes]
    if int(np.prod(dims)) != mesh.shape[0]:
        # not a tensor grid: brute force, first minimum (argmin) as the reference
        out = np.empty(len(data), dtype=np.int64)
        for i, x in enumerate(data):
            out[i] = int(np.argmin(np.sum((mesh - x) ** 2, axis=1)))
        return out
    strides = np.cumprod([1] + dims[:-1])
    colmajor = np.zeros(mesh.shape[0], dtype=np.int64)
    for j in range(len(dims)):
        colmajor += pos[j] * strides[j]
    row_of = np.empty(mesh.shape[0], dtype=np.int64)
    row_of[colmajor] = np.arange(mesh.shape[0])
    key = np.zeros(len(data), dtype=np.int64)
    for j, a in enumerate(axes):
        x = data[:, j]
        k = np.clip(np.searchsorted(a, x), 1, len(a) - 1) if len(a) > 1 else np.zeros(len(x), dtype=np.int64)
        if len(a) > 1:
            left = a[k - 1]
            right = a[k]
            k = np.where((x - left) ** 2 <= (right - x) ** 2, k - 1, k)
        key += k * strides[j]
    return row_of[key]


def interp_weights(idx, N, y=None):
    """diag(O^T O) and O^T y from the nearest-mesh index (code/solvers.py:29-35)."""
    idx = np.asarray(idx, dtype=np.int64)
    W = np.bincount(idx, minlength=N).astype(np.float64)
    oty = None if y is None else np.bincount(idx, weights=np.asarray(y, dtype=np.float64).ravel(), minlength=N)
    return W, oty


def create_deltas(data, m, eps: float = 1e-4):
    """rcpp-code/MultivarTV/src/utils.cpp:256-263 (EPS = 1e-4; cpp-code uses 0.01)."""
    data = np.asarray(data, dtype=np.float64).reshape(len(data), -1)
    return [(data[:, j].max() - data[:, j].min() + 2 * eps) / m[j] for j in range(data.shape[1])]


# ---- lambda_max of the Python reference (host setup, scipy's SuperLU as the reference calls it) ----

def _sprime(bits):
    """Effective difference set of a block (mixedpartial differences dim 0 first, code/utils.py:102-129)."""
    S = [j for j, v in enumerate(bits) if v]
    if len(S) <= 1 or S[0] == 0:
        return S
    return sorted(set(S[1:]) | {0})


def create_D(m, deltas=None):
    """code/utils.py:138-149 as a scipy CSR matrix: row blocks b = 1..2^p-1 (MSB = dim 0, fd_binaries
    :63-69), all unweighted when deltas is None; with deltas the all-ones block is dropped and block b
    is scaled by prod_j delta_j^(1-b_j). Block rows enumerate the reduced grid column-major; each
    row is w * sum over T subset of S' of (-1)^|T| theta_{i + e_T}."""
    import scipy.sparse as sp
    m = [int(v) for v in np.atleast_1d(m)]
    p, N = len(m), int(np.prod(m))
    full = (1 << p) - 1
    codes = range(1, full + 1) if deltas is None else range(1, full)
    mats = []
    for b in codes:
        bits = [(b >> (p - 1 - j)) & 1 for j in range(p)]
        w = 1.0
        if deltas is not None:
            for j in range(p):
                if not bits[j]:
                    w *= float(deltas[j])
        S = [j for j in range(p) if bits[j]]
        if len(S) >= 2 and S[0] != 0 and m[0] != m[S[0]]:
            # mixedpartial's product of differently sized difference matrices (code/utils.py:121-128)
            raise ValueError(f"dimension mismatch: block {b} needs m[0] == m[{S[0]}]")
        Sp = _sprime(bits)
        rd = [m[j] - (1 if j in Sp else 0) for j in range(p)]
        R = int(np.prod(rd))
        grids = np.meshgrid(*[np.arange(v, dtype=np.int64) for v in rd], indexing="ij")
        coord = [g.ravel(order="F") for g in grids]
        rows, cols, vals = [], [], []
        for t in range(1 << len(Sp)):
            lin = np.zeros(R, dtype=np.int64)
            stride, sign = 1, 1.0
            for j in range(p):
                q = Sp.index(j) if j in Sp else -1
                shift = 1 if (q >= 0 and (t >> q) & 1) else 0
                if shift:
                    sign = -sign
                lin += (coord[j] + shift) * stride
                stride *= m[j]
            rows.append(np.arange(R, dtype=np.int64))
            cols.append(lin)
            vals.append(np.full(R, sign * w))
        mats.append(sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(R, N)))
    if not mats:
        raise ValueError("blocks must be 2-D")   # scipy.sparse.vstack([]) at p = 1 with deltas (code/utils.py:148)
    return sp.vstack(mats).tocsr()


def lam_max_pinv(D, oty):
    """code/utils.py:198-209: max |D x| with x = splu(D^T D).solve(O^T y). D^T D is singular (the
    constants are its null space); SuperLU returns whatever its pivoting gives on the zero pivot, and
    the reference's lambda grid is that number, so this calls the same library on the same matrix."""
    from scipy.sparse.linalg import splu
    A = (D.T @ D).tocsc()
    x = splu(A).solve(np.asarray(oty, dtype=np.float64).ravel())
    return float(np.max(np.abs(D @ x)))
