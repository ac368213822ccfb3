"""GPU parity of the scattered-data setup through the C ABI:
nearest1 / nearest_interp_matrix (rcpp-code/MultivarTV/src/utils.cpp:267-304), create_cache_objects'
diag(O^T O) and O^T y (rcpp…/solvers.cpp:36-44) and mbs_predict (:161-165).

The checker is the oracle's brute-force scan over every mesh row (oracle/mvtv_oracle.py
nearest_index, first minimum as arma's index_min) and numpy's bincount (sequential per-node sums in
data order). Bar: mesh indices identical; W and O^T y bit-identical, shown by ADMM runs from the GPU
setup and from the host setup agreeing bit for bit."""
import numpy as np
import pytest

from oracle import mvtv_oracle as O

mv = pytest.importorskip("multivartv_amd")
from multivartv_amd import cv  # noqa: E402

pytestmark = pytest.mark.gpu


def _points(n, p, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(0, 1, size=(n, p)), rng.standard_normal(n)


def _axes(x, m):
    mesh = cv.create_mesh(x, m)
    axes = cv.tensor_axes(mesh, m)
    assert axes is not None
    return mesh, axes


@pytest.mark.parametrize("m,n", [([50], 400), ([12, 9], 500), ([8, 8, 8], 700), ([5, 5, 5, 5], 600)])
def test_nearest_matches_bruteforce(m, n):
    x, _ = _points(n, len(m), seed=sum(m))
    mesh, axes = _axes(x, m)
    # edge cases: points on nodes, on cell midpoints (near-ties), outside the mesh box
    extra = [mesh[3], mesh[-1], 0.5 * (mesh[0] + mesh[1]), mesh[0] - 1.0, mesh[-1] + 1.0]
    x = np.vstack([x, np.array(extra)])
    with mv.Problem(m, np.zeros(int(np.prod(m)))) as P:
        got = P.nearest(axes, x)
    np.testing.assert_array_equal(got, O.nearest_index(x, mesh))


def test_nearest_exact_ties_take_lower_node():
    m = [5, 4]
    axes = [np.arange(5.0), np.arange(4.0)]
    mesh = np.stack([g.reshape(-1, order="F") for g in np.meshgrid(*axes, indexing="ij")], axis=1)
    x = np.array([[0.5, 0.5], [1.5, 2.0], [3.0, 2.5], [3.5, 2.5], [4.0, 3.0]])
    with mv.Problem(m, np.zeros(20)) as P:
        got = P.nearest(axes, x)
    np.testing.assert_array_equal(got, O.nearest_index(x, mesh))
    np.testing.assert_array_equal(got, [0, 11, 13, 13, 19])


@pytest.mark.parametrize("m,n", [([16, 16], 3000), ([8, 8, 8], 300), ([32, 32], 1024)])
def test_set_scattered_bit_identical_to_host_setup(m, n):
    x, y = _points(n, len(m), seed=7 + n)
    mesh, axes = _axes(x, m)
    N = int(np.prod(m))
    idx = O.nearest_index(x, mesh)
    W = np.bincount(idx, minlength=N).astype(float)
    oty = np.bincount(idx, weights=y, minlength=N)
    deltas = O.create_deltas_rcpp(x, m)
    th0 = np.full(N, y.mean())
    with mv.Problem(m, oty, wdiag=W, deltas=deltas, order=mv.ORDER_CPP) as Ph, \
            mv.Problem(m, np.zeros(N), deltas=deltas, order=mv.ORDER_CPP) as Pg:
        got_idx = Pg.set_scattered(axes, x, y)
        np.testing.assert_array_equal(got_idx, idx)
        # W itself: A x with sigma = 0 and x = 1 is W exactly
        np.testing.assert_array_equal(Pg.apply_A(0.0, np.ones(N)), W)
        rh = Ph.admm(0.05, th0, rho=0.01, fixed_iters=6, return_u=False)
        rg = Pg.admm(0.05, th0, rho=0.01, fixed_iters=6, return_u=False)
        np.testing.assert_array_equal(rg[0], rh[0])
        assert rg[2] == rh[2]


def test_one_point_per_node_gives_identity_weights():
    m = [16, 16]
    axes = [np.linspace(0, 1, 16), np.linspace(0, 2, 16)]
    grid = np.stack([g.reshape(-1, order="F") for g in np.meshgrid(*axes, indexing="ij")], axis=1)
    perm = np.random.default_rng(3).permutation(256)
    y = np.random.default_rng(4).standard_normal(256)
    with mv.Problem(m, np.zeros(256)) as P:
        idx = P.set_scattered(axes, grid[perm] + 1e-3, y)
        np.testing.assert_array_equal(idx, perm)
        assert P.spectral_ok()
        th = np.arange(256.0)
        P.state_set(th, None, 1.0)
        np.testing.assert_array_equal(P.apply_A(0.0, th), th)


def test_predict_is_theta_at_nearest_node():
    m = [10, 12]
    x, y = _points(400, 2, seed=11)
    mesh, axes = _axes(x, m)
    xt, _ = _points(77, 2, seed=12)
    with mv.Problem(m, np.zeros(120)) as P:
        P.set_scattered(axes, x, y)
        th = np.random.default_rng(5).standard_normal(120)
        P.state_set(th, None, 1.0)
        np.testing.assert_array_equal(P.predict(axes, xt), th[O.nearest_index(xt, mesh)])
        assert P.predict(axes, np.empty((0, 2))).size == 0


def test_scattered_rejects_bad_axes():
    with mv.Problem([4, 4], np.zeros(16)) as P:
        with pytest.raises(mv.MvtvError):
            P.nearest([np.array([0.0, 2.0, 1.0, 3.0]), np.arange(4.0)], np.zeros((3, 2)))
        with pytest.raises(ValueError):
            P.nearest([np.arange(3.0), np.arange(4.0)], np.zeros((3, 2)))
