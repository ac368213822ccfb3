"""Bit-reproducible synthetic inputs for the mesh-TV benchmarks.

The signal is the p-dimensional "towers" function of the reference vignette
(rcpp-code/MultivarTV/vignettes/MultivarTV-intro.Rmd:32-39): 1 where every
coordinate exceeds 0.8, 0.5 where every coordinate is below 0.2, 0 elsewhere.
Noise is sigma * N(0,1) with sigma = 0.5 (vignette :182), drawn from a
counter-based generator (splitmix64 -> Box-Muller) so that any mesh size can be
regenerated identically on any host without storing it.

Lattice data x_j = i_j / (m_j - 1) with mesh == data gives O = I, W = I and
O^T y = y; the mesh is flattened column-major (dim 0 fastest,
cpp-code/utils.cpp:40-52).
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

SEED = 0x4D565456
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser applied to uint64 counters (vectorised, wraps mod 2^64)."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def normal_noise(start: int, count: int, seed: int = SEED) -> np.ndarray:
    """Standard normals for flat indices [start, start+count).

    xi_i = sqrt(-2 ln u1) cos(2 pi u2) with u1, u2 in (0, 1] drawn from
    splitmix64(seed ^ 2i) and splitmix64(seed ^ (2i+1)).
    """
    i = np.arange(start, start + count, dtype=np.uint64)
    s = np.uint64(seed)
    a = splitmix64(s ^ (i << np.uint64(1)))
    b = splitmix64(s ^ ((i << np.uint64(1)) | np.uint64(1)))
    scale = 1.0 / 9007199254740992.0  # 2^-53
    u1 = ((a >> np.uint64(11)).astype(np.float64) + 1.0) * scale
    u2 = ((b >> np.uint64(11)).astype(np.float64) + 1.0) * scale
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def lattice_coords(m) -> list[np.ndarray]:
    """Per-dimension lattice coordinates x_j = i_j / (m_j - 1)."""
    return [np.arange(mj, dtype=np.float64) / max(mj - 1, 1) for mj in m]


def towers(m, sigma: float = 0.5, seed: int = SEED, chunk: int = 1 << 22, threads: int = 0, start: int = 0,
           count: int | None = None) -> np.ndarray:
    """y = towers(x) + sigma * xi on the column-major lattice of shape m (float64, length prod(m)),
    or its flat index range [start, start + count) (a slab of planes of a decomposed mesh).

    Chunks are independent (counter-based noise), so large meshes are generated on a
    thread pool; the result does not depend on ``threads``.
    """
    m = [int(v) for v in m]
    off = int(start)
    n = int(np.prod(m)) - off if count is None else int(count)
    y = np.empty(n, dtype=np.float64)
    coords = lattice_coords(m)
    strides = np.cumprod([1] + m[:-1])

    def work(start):
        cnt = min(chunk, n - start)
        flat = np.arange(off + start, off + start + cnt, dtype=np.int64)
        hi = np.ones(cnt, dtype=bool)
        lo = np.ones(cnt, dtype=bool)
        for j, mj in enumerate(m):
            xj = coords[j][(flat // strides[j]) % mj]
            hi &= xj > 0.8
            lo &= xj < 0.2
        f = np.where(hi, 1.0, np.where(lo, 0.5, 0.0))
        y[start:start + cnt] = f + sigma * normal_noise(off + start, cnt, seed)

    starts = range(0, n, chunk)
    nthreads = threads or min(16, os.cpu_count() or 1)
    if nthreads > 1 and n > chunk:
        with ThreadPoolExecutor(nthreads) as ex:
            list(ex.map(work, starts))
    else:
        for s in starts:
            work(s)
    return y


def towers_scattered(n: int, p: int, sigma: float = 0.5, seed: int = SEED):
    """n scattered points uniform in [0,1]^p (from the same counter stream) and noisy towers values."""
    i = np.arange(n * p, dtype=np.uint64)
    u = (splitmix64(np.uint64(seed ^ 0x5A5A5A5A) ^ i) >> np.uint64(11)).astype(np.float64) / 9007199254740992.0
    data = u.reshape(n, p)
    hi = np.all(data > 0.8, axis=1)
    lo = np.all(data < 0.2, axis=1)
    f = np.where(hi, 1.0, np.where(lo, 0.5, 0.0))
    y = f + sigma * normal_noise(0, n, seed ^ 0x1234)
    return data, y, f
