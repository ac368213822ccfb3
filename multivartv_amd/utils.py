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
