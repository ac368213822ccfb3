"""Pin the CPU oracle (oracle/mvtv_oracle.py) against the reference-generated fixtures."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_golden
from oracle import mvtv_oracle as O

DMATS = ["7", "4x5", "5x5", "4x4x4", "4x4x5", "3x3x3x3", "3x3x3x4"]


def _coo(g, key):
    return sp.coo_matrix((g[key + "_v"], (g[key + "_r"], g[key + "_c"])), shape=tuple(g[key + "_shape"])).tocsr()


@pytest.mark.parametrize("tag", DMATS)
def test_D_matches_reference(tag):
    meta, g = load_golden("dmat_" + tag)
    m, dl, p = meta["m"], meta["deltas"], len(meta["m"])
    cases = [("py_none", O.block_table(p, None, "py")),
             ("cpp", O.block_table(p, dl, "cpp")),
             ("cppunit", O.block_table(p, dl, "cpp", unit_weights=True))]
    if p > 1:
        cases.append(("py_w", O.block_table(p, dl, "py")))
    for key, blocks in cases:
        ref = _coo(g, key)
        ours = O.build_D(m, blocks)
        assert ours.shape == ref.shape, key
        assert (ours != ref).nnz == 0, key  # bit-exact
        assert O.num_edges(m, blocks) == ref.shape[0]


def test_dim_mismatch_matches_reference():
    meta, _ = load_golden("dmat_mismatch")
    for case in meta["cases"]:
        m = case["m"]
        blocks = O.block_table(len(m), None, "py")
        if case["raises"]:
            with pytest.raises(O.DimMismatch):
                O.build_D(m, blocks)
        else:
            O.build_D(m, blocks)


def test_reference_unit_pins():
    """The reference's own code/test_utils.py pins, restated."""
    D = O.build_D([3, 3], O.block_table(2, None, "py"))
    assert np.sum(D @ np.tile([1, -1, 1], 3)) == 0.0       # test_utils.py:33-36
    meta, _ = load_golden("py_unit_pins")
    assert meta["t2v_222"] == 26 and meta["v2t_26"] == [2, 2, 2]
    assert list(O.nearest_index(np.array([0.1, 0.9]), np.array([[0], [0.5], [1.0]]))) == meta["nearest"] == [0, 2]
    mesh, deltas = O.mesh_coords_py(np.linspace(0.01, 0.99, 10).reshape(10, 1), [6])
    assert np.round(deltas[0], 2) == meta["mesh_delta"] == 0.2


RCPP = ["rcpp_1d_200", "rcpp_2d_32", "rcpp_2d_24x40", "rcpp_3d_12", "rcpp_3d_8x8x11", "rcpp_4d_5", "rcpp_2d_scat"]


@pytest.mark.parametrize("name", RCPP)
def test_rcpp_fixed_trajectory(name):
    meta, g = load_golden(name)
    m = meta["m"]
    D = O.build_D(m, O.block_table(len(m), meta["deltas"], "cpp"))
    E = D.shape[0]
    res = O.admm_rcpp(D, g["Oty"], g["W"], meta["lam"], g["theta0"], np.zeros(E), meta["rho0"],
                      fixed_iters=20, snapshot_at=(1, 5, 20), record=True)
    scale = np.max(np.abs(g["fixed_theta"]))
    for k in (1, 5, 20):
        assert np.max(np.abs(res.snapshots[k] - g[f"snap{k}"])) <= 1e-11 * scale
    assert np.max(np.abs(res.u - g["fixed_u"])) <= 1e-10 * max(1.0, np.max(np.abs(g["fixed_u"])))
    assert res.rho == float(g["fixed_rho"])
    hist = np.array([[h["r_norm"], h["s_norm"], h["eps_pri"], h["eps_dual"], h["rho"]] for h in res.history])
    np.testing.assert_allclose(hist, g["fixed_hist"], rtol=1e-8, atol=1e-14)


@pytest.mark.parametrize("name", RCPP)
def test_rcpp_converged(name):
    meta, g = load_golden(name)
    m = meta["m"]
    D = O.build_D(m, O.block_table(len(m), meta["deltas"], "cpp"))
    res = O.admm_rcpp(D, g["Oty"], g["W"], meta["lam"], g["theta0"], np.zeros(D.shape[0]), meta["rho0"])
    assert res.iters == meta["iters"]
    assert res.rho == meta["rho"]
    assert np.max(np.abs(res.theta - g["theta"])) <= 1e-10 * np.max(np.abs(g["theta"]))


def test_rcpp_warm_path():
    meta, g = load_golden("rcpp_path_2d_16")
    m = meta["m"]
    D = O.build_D(m, O.block_table(2, meta["deltas"], "cpp"))
    y = g["y"]
    theta, u, rho = np.full(256, y.mean()), np.zeros(D.shape[0]), meta["lams"][0] / 5.0
    for k, lam in enumerate(meta["lams"]):
        res = O.admm_rcpp(D, y, np.ones(256), lam, theta, u, rho)
        theta, u, rho = res.theta, res.u, res.rho
        assert res.iters == int(g[f"iters{k}"])
        assert rho == float(g[f"rho{k}"])
        assert np.max(np.abs(theta - g[f"theta{k}"])) <= 1e-10 * np.max(np.abs(theta))


@pytest.mark.parametrize("name", ["cpp_2d_16", "cpp_3d_8_unit", "cpp_2d_12_frac"])
def test_cpp_variant(name):
    meta, g = load_golden(name)
    m = meta["m"]
    D = O.build_D(m, O.block_table(len(m), meta["deltas"], "cpp", unit_weights=meta["unit"]))
    N = int(np.prod(m))
    res = O.admm_cpp(D, g["y"], np.ones(N), meta["lam"], g["theta0"], meta["ymean"], record=True)
    assert res.iters == meta["iters"]
    assert res.rho == meta["rho"]
    assert np.max(np.abs(res.theta - g["theta"])) <= 1e-11 * np.max(np.abs(g["theta"]))
    hist = np.array([[h["r_norm"], h["s_norm"], h["rho"]] for h in res.history])
    np.testing.assert_allclose(hist, g["hist"], rtol=1e-8, atol=1e-14)


@pytest.mark.parametrize("name", ["py_1d_n1000_m1000_lam2", "py_1d_n1000_m250_lam2", "py_1d_n1000_m1000_lam0.5"])
def test_py_config1(name):
    """Config 1: the reference's own solvers.mbs_one (cache path) on 1D n = 1000."""
    meta, g = load_golden(name)
    mesh, _ = O.mesh_coords_py(g["data"], meta["m"])
    np.testing.assert_array_equal(mesh, g["mesh"])
    idx = O.nearest_index(g["data"], mesh)
    W = np.bincount(idx, minlength=meta["m"][0]).astype(float)
    Oty = np.bincount(idx, weights=g["y"], minlength=meta["m"][0])
    np.testing.assert_array_equal(W, g["W"])
    np.testing.assert_allclose(Oty, g["Oty"], rtol=0, atol=1e-13)
    D = O.build_D(meta["m"], O.block_table(1, None, "py"))
    res = O.admm_py(D, Oty, W, meta["lam"], np.full(meta["m"][0], g["y"].mean()), g["y"].mean())
    assert np.max(np.abs(res.theta - g["theta"])) <= 1e-11 * np.max(np.abs(g["theta"]))
    np.testing.assert_allclose(res.theta[idx], g["fitted"], rtol=0, atol=1e-11)


def test_py_nocache_and_path():
    meta, g = load_golden("py_2d_mbs_one_nocache")
    data, y, m = g["data"], g["y"], meta["m"]
    mesh, deltas = O.mesh_coords_py(data, m)
    np.testing.assert_array_equal(mesh, g["mesh"])
    idx = O.nearest_index(data, mesh)
    N = int(np.prod(m))
    W = np.bincount(idx, minlength=N).astype(float)
    Oty = np.bincount(idx, weights=y, minlength=N)
    D = O.build_D(m, O.block_table(2, deltas, "py"))
    tune = O.lam_max_pinv_py(D, Oty)
    res = O.admm_py(D, Oty, W, tune, np.full(N, y.mean()), y.mean())
    np.testing.assert_allclose(res.theta, g["theta"], rtol=1e-9, atol=1e-12)

    meta, g = load_golden("py_2d_mbs_path")
    thetas, mses, tuners, best = O.mbs_path_py(g["data"], g["y"], meta["m"], ftrue=g["ftrue"], ntune=meta["ntune"])
    assert abs(mses[best] - float(g["minmse"])) <= 1e-10 * float(g["minmse"])
    assert tuners[best] == pytest.approx(float(g["minlam"]), rel=1e-12)
    np.testing.assert_allclose(thetas[best], g["theta"], rtol=1e-9, atol=1e-12)


def test_mesh_coords_3d_quirk():
    meta, g = load_golden("py_mesh_coords_3d")
    mesh, deltas = O.mesh_coords_py(g["data"], meta["m"])
    np.testing.assert_array_equal(mesh, g["mesh"])
    np.testing.assert_array_equal(np.array(deltas), g["deltas"])
