"""GPU: the fused 3-D Chronopoulos-Gear PCG against SuperLU and against the classic 3-kernel PCG."""
import os

import numpy as np
import pytest

from oracle import mvtv_oracle as O

mv = pytest.importorskip("multivartv_amd")
pytestmark = pytest.mark.gpu

# m0 == m1 (the reference's D construction requires it at p = 3); sizes straddle the 64 x 16
# tile, single and multiple dim-2 chunks, and thin meshes. SuperLU (the oracle) only on small
# meshes: its fill-in on 3-D 27-point matrices makes larger factorisations take minutes.
SHAPES = [[8, 8, 8], [70, 70, 3], [20, 20, 34], [17, 17, 40], [130, 130, 2]]
BIG = [[64, 64, 40], [96, 96, 70], [200, 200, 17]]


@pytest.mark.parametrize("m", SHAPES)
@pytest.mark.parametrize("wdiag", [False, True])
def test_fused_solve_matches_superlu(m, wdiag):
    rng = np.random.default_rng(7)
    N = int(np.prod(m))
    W = rng.integers(0, 4, N).astype(float) if wdiag else None
    deltas = [0.3, 0.2, 0.5]
    D = O.build_D(m, O.block_table(3, deltas, "cpp"))
    P = mv.Problem(m, rng.standard_normal(N), wdiag=W, deltas=deltas)
    b = rng.standard_normal(N)
    sigma = 2.5
    ref = O._solver(np.ones(N) if W is None else W, (D.T @ D).tocsc(), sigma).solve(b)
    x0 = rng.standard_normal(N)
    x, it, rr = P.solve(sigma, b, x0=x0, rtol=1e-13, max_iter=3000)
    assert rr <= 1e-13, (it, rr)
    assert np.max(np.abs(x - ref)) <= 1e-10 * np.max(np.abs(ref))
    P.close()


@pytest.mark.parametrize("m", BIG)
def test_fused_solve_residual_large(m):
    """Larger meshes: the true residual |b - (W + sigma D^T D) x| / |b| from the oracle's sparse D."""
    rng = np.random.default_rng(11)
    N = int(np.prod(m))
    W = rng.integers(0, 4, N).astype(float)
    deltas = [0.3, 0.2, 0.5]
    D = O.build_D(m, O.block_table(3, deltas, "cpp"))
    P = mv.Problem(m, rng.standard_normal(N), wdiag=W, deltas=deltas)
    b = rng.standard_normal(N)
    x, it, rr = P.solve(3.0, b, rtol=1e-12, max_iter=5000)
    true_res = np.linalg.norm(b - O.apply_A(D, W, 3.0, x)) / np.linalg.norm(b)
    assert rr <= 1e-12 and true_res <= 1e-10, (it, rr, true_res)
    P.close()


def test_fused_matches_classic_iterates():
    """Chronopoulos-Gear and classic PCG are the same Krylov method: same iteration counts."""
    m = [48, 48, 40]
    rng = np.random.default_rng(3)
    N = int(np.prod(m))
    b = rng.standard_normal(N)
    out = {}
    for mode in ("fused", "classic"):
        if mode == "classic":
            os.environ["MVTV_PCG"] = "classic"
        try:
            P = mv.Problem(m, b, deltas=[0.02] * 3)
        finally:
            os.environ.pop("MVTV_PCG", None)
        out[mode] = P.solve(6.4, b, rtol=1e-10, max_iter=3000)
        P.close()
    (xf, itf, rf), (xc, itc, rc) = out["fused"], out["classic"]
    assert abs(itf - itc) <= 1
    assert np.max(np.abs(xf - xc)) <= 1e-8 * np.max(np.abs(xc))
