"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the golden fixtures.

Tolerances (fp64): operators D, D^T, A agree with the oracle's sparse products to
1e-13 relative (summation order differs); PCG theta-solves run at rtol 1e-13 and the
spectral solve is exact, so ADMM iterates agree with the SuperLU-driven fixtures to
SURVEY 8(c)'s 1e-9 relative of max|theta| (u to 1e-9 of max(1, max|u|)), the r / s
norms to 1e-9 relative, and iteration counts / final rho must match exactly. The
achieved errors go to $MVTV_PARITY_LOG (conftest.log_parity; table in DESIGN.md 2).
"""
import numpy as np
import pytest

from conftest import load_golden, log_parity
from oracle import mvtv_oracle as O

mv = pytest.importorskip("multivartv_amd")
pytestmark = pytest.mark.gpu

RTOL_OP = 1e-13
RTOL_THETA = 1e-9
RTOL_NORM = 1e-9


def _rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1e-300, np.max(np.abs(b))))


def _relu(a, b):
    """u's error relative to max(1, max|u_ref|) (u is 0 on most edges of a converged fit)."""
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1.0, np.max(np.abs(b))))


SHAPES = [([9], None, "cpp", False), ([7, 5], [0.3, 0.7], "cpp", False), ([6, 6, 6], [0.5, 0.25, 0.125], "cpp", False),
          ([5, 5, 7], [0.2, 0.3, 0.4], "cpp", True), ([4, 4, 4, 5], [0.5, 0.25, 0.125, 0.3], "cpp", False),
          ([6, 5], None, "py", False), ([5, 5, 5], [0.5, 0.25, 0.125], "py", False), ([4, 4, 4, 4], None, "py", False)]


def _problem(m, deltas, order, unit, wdiag=None, seed=0):
    rng = np.random.default_rng(seed)
    N = int(np.prod(m))
    oty = rng.standard_normal(N)
    o = mv.ORDER_CPP if order == "cpp" else mv.ORDER_PY
    weighted = (deltas is not None) and not unit
    P = mv.Problem(m, oty, wdiag=wdiag, deltas=deltas if deltas is not None else [1.0] * len(m), order=o,
                   weighted=weighted)
    D = O.build_D(m, O.block_table(len(m), deltas if weighted else None, order, unit_weights=unit))
    return P, D, oty


@pytest.mark.parametrize("m,deltas,order,unit", SHAPES)
def test_operators(m, deltas, order, unit):
    rng = np.random.default_rng(1)
    N = int(np.prod(m))
    w = rng.uniform(0.0, 3.0, N).round()
    P, D, _ = _problem(m, deltas, order, unit, wdiag=w)
    assert P.E == D.shape[0]
    th = rng.standard_normal(N)
    assert _rel(P.apply_D(th), D @ th) <= RTOL_OP
    v = rng.standard_normal(D.shape[0])
    assert _rel(P.apply_Dt(v), D.T @ v) <= RTOL_OP
    for sigma in (0.0, 0.37, 25.6):
        assert _rel(P.apply_A(sigma, th), O.apply_A(D, w, sigma, th)) <= RTOL_OP
    P.close()


@pytest.mark.parametrize("m,order", [([130, 130, 3], "cpp"), ([65, 65, 65], "py"), ([64, 64, 5], "cpp"),
                                     ([200, 200, 2], "cpp"), ([127, 127, 4], "cpp"), ([70, 70, 70], "py")])
def test_apply_A_3d_multi_run(m, order):
    """the 3-D z-marching operator (k_apply3d) with dim-0 runs past one 64-lane wave: the x +- 1 neighbours
    cross wave boundaries (lanes 0 / 63 load them) and ragged last runs (m_0 = m_1: the S' rule of test_dim_mismatch)."""
    rng = np.random.default_rng(sum(m))
    N = int(np.prod(m))
    w = rng.uniform(0.0, 3.0, N).round()
    P, D, _ = _problem(m, [0.5, 0.25, 0.125], order, False, wdiag=w)
    th = rng.standard_normal(N)
    for sigma in (0.0, 0.37, 25.6):
        assert _rel(P.apply_A(sigma, th), O.apply_A(D, w, sigma, th)) <= RTOL_OP
    P.close()


@pytest.mark.parametrize("m,deltas,order,unit", SHAPES[:6])
def test_pcg_solve(m, deltas, order, unit):
    rng = np.random.default_rng(2)
    N = int(np.prod(m))
    P, D, _ = _problem(m, deltas, order, unit)
    b = rng.standard_normal(N)
    sigma = 3.2
    ref = O._solver(np.ones(N), (D.T @ D).tocsc(), sigma).solve(b)
    x, it, rr = P.solve(sigma, b, rtol=1e-13)
    assert rr <= 1e-13
    assert _rel(x, ref) <= 1e-10
    P.close()


def _jacobi_pcg(D, w, sigma, b, x, k):
    """k iterations of textbook Jacobi-PCG (numpy): the iterates the fused 3-D kernel's single-reduction form
    reproduces up to rounding (rcpp-code/MultivarTV/src/solvers.cpp:113 solves the same system directly)."""
    dinv = 1.0 / (w + sigma * np.asarray((D.T @ D).diagonal()).ravel())
    x = x.copy()
    r = b - O.apply_A(D, w, sigma, x)
    z = dinv * r
    p = z.copy()
    rz = r @ z
    for _ in range(k):
        q = O.apply_A(D, w, sigma, p)
        al = rz / (p @ q)
        x += al * p
        r -= al * q
        z = dinv * r
        rz, rz0 = r @ z, rz
        p = z + (rz / rz0) * p
    return x


@pytest.mark.parametrize("weighted", [False, True])
def test_fused_pcg_stops_after_odd_and_even_iterations(weighted):
    """k_cg3d moves x only in odd iterations (both steps); k_cg_xflush applies the step an even last iteration
    left pending: x after k = 1..6 iterations (rtol unreachable, so max_iter stops the solve) against numpy."""
    rng = np.random.default_rng(5)
    m = [9, 9, 9]
    N = int(np.prod(m))
    w = rng.uniform(0.5, 2.0, N) if weighted else np.ones(N)
    P, D, _ = _problem(m, [0.5, 0.25, 0.125], "cpp", False, wdiag=w if weighted else None)
    b = rng.standard_normal(N)
    x0 = rng.standard_normal(N)
    sigma = 2.7
    for k in range(1, 7):
        x, it, _ = P.solve(sigma, b, x0=x0, rtol=1e-300, max_iter=k)
        assert it == k
        assert _rel(x, _jacobi_pcg(D, w, sigma, b, x0, k)) <= 1e-11, k
    P.close()


def test_dim_mismatch_raises():
    with pytest.raises(mv.DimMismatchError):
        mv.Problem([4, 3, 5], np.zeros(60), deltas=[1, 1, 1])
    mv.Problem([4, 4, 5], np.zeros(80), deltas=[1, 1, 1]).close()


RCPP = ["rcpp_1d_200", "rcpp_2d_32", "rcpp_2d_24x40", "rcpp_3d_12", "rcpp_3d_8x8x11", "rcpp_4d_5", "rcpp_2d_scat"]


def _rcpp_problem(meta, g):
    W = g["W"]
    wdiag = None if np.all(W == 1.0) else W
    return mv.Problem(meta["m"], g["Oty"], wdiag=wdiag, deltas=meta["deltas"], order=mv.ORDER_CPP)


# AUTO = spectral where exact (W = I, every m_j <= 4096: FFT plans for 2-3-5-7 lengths, Bluestein for the rest,
# e.g. the 8 x 8 x 11 fixture), PCG_SPECTRAL for W != I on such meshes
SOLVERS = [mv.SOLVER_PCG, mv.SOLVER_AUTO, mv.SOLVER_PCG_SPECTRAL]


def _skip_unless_pow2(meta, solver):
    if solver == mv.SOLVER_PCG_SPECTRAL and not all(v <= 4096 for v in meta["m"]):
        pytest.skip("the cosine-transform preconditioner needs m_j <= 4096")


@pytest.mark.parametrize("solver", SOLVERS)
@pytest.mark.parametrize("name", RCPP)
def test_rcpp_trajectory(name, solver):
    meta, g = load_golden(name)
    _skip_unless_pow2(meta, solver)
    P = _rcpp_problem(meta, g)
    errs = {}
    for k in (1, 5, 20):
        th, u, rho, st = P.admm(meta["lam"], g["theta0"], u=np.zeros(P.E), rho=meta["rho0"],
                                fixed_iters=k, pcg_rtol=1e-13, theta_solver=solver)
        errs[f"theta{k}"] = _rel(th, g[f"snap{k}"])
        assert st["iters"] == k
    hist = g["fixed_hist"][-1]
    errs["u20"] = _relu(u, g["fixed_u"])
    errs["r_norm"] = abs(st["r_norm"] - hist[0]) / max(abs(hist[0]), 1e-300)
    errs["s_norm"] = abs(st["s_norm"] - hist[1]) / max(abs(hist[1]), 1e-300)
    log_parity(f"trajectory/{name}/{solver}", **errs)
    for k in (1, 5, 20):
        assert errs[f"theta{k}"] <= RTOL_THETA, k
    assert rho == float(g["fixed_rho"])
    assert errs["u20"] <= RTOL_THETA
    assert st["r_norm"] == pytest.approx(hist[0], rel=RTOL_NORM, abs=1e-14)
    assert st["s_norm"] == pytest.approx(hist[1], rel=RTOL_NORM, abs=1e-14)
    assert st["eps_pri"] == pytest.approx(hist[2], rel=1e-10)
    assert st["eps_dual"] == pytest.approx(hist[3], rel=1e-10)
    P.close()


@pytest.mark.parametrize("solver", SOLVERS)
@pytest.mark.parametrize("name", RCPP)
def test_rcpp_converged(name, solver):
    meta, g = load_golden(name)
    _skip_unless_pow2(meta, solver)
    P = _rcpp_problem(meta, g)
    th, u, rho, st = P.admm(meta["lam"], g["theta0"], u=np.zeros(P.E), rho=meta["rho0"], pcg_rtol=1e-13,
                            theta_solver=solver)
    log_parity(f"converged/{name}/{solver}", theta=_rel(th, g["theta"]), u=_relu(u, g["u"]), iters=st["iters"])
    assert st["iters"] == meta["iters"]
    assert rho == meta["rho"]
    assert _rel(th, g["theta"]) <= RTOL_THETA
    assert _relu(u, g["u"]) <= RTOL_THETA
    P.close()


@pytest.mark.parametrize("solver", SOLVERS)
def test_rcpp_warm_path_resident(solver):
    meta, g = load_golden("rcpp_path_2d_16")
    if solver == mv.SOLVER_PCG_SPECTRAL:
        pytest.skip("W = I: the spectral solve is exact there")
    y = g["y"]
    P = mv.Problem(meta["m"], y, deltas=meta["deltas"], order=mv.ORDER_CPP)
    assert P.spectral_ok()
    P.state_set(np.full(256, y.mean()), np.zeros(P.E), meta["lams"][0] / 5.0)
    for k, lam in enumerate(meta["lams"]):
        st = P.run(lam, pcg_rtol=1e-13, theta_solver=solver)
        assert st["theta_solver"] == (mv.SOLVER_PCG if solver == mv.SOLVER_PCG else mv.SOLVER_SPECTRAL)
        th, u, rho = P.state_get()
        log_parity(f"warm_path/{k}/{solver}", theta=_rel(th, g[f"theta{k}"]), u=_relu(u, g[f"u{k}"]))
        assert st["iters"] == int(g[f"iters{k}"])
        assert rho == float(g[f"rho{k}"])
        assert _rel(th, g[f"theta{k}"]) <= RTOL_THETA
        assert _relu(u, g[f"u{k}"]) <= RTOL_THETA
    P.close()


@pytest.mark.parametrize("solver", SOLVERS)
@pytest.mark.parametrize("name", ["cpp_2d_16", "cpp_3d_8_unit", "cpp_2d_12_frac"])
def test_cpp_variant(name, solver):
    meta, g = load_golden(name)
    _skip_unless_pow2(meta, solver)
    P = mv.Problem(meta["m"], g["y"], deltas=meta["deltas"], order=mv.ORDER_CPP, weighted=not meta["unit"])
    th, u, rho, st = P.admm(meta["lam"], g["theta0"], variant=mv.VARIANT_CPP, ymean=meta["ymean"], pcg_rtol=1e-13,
                            theta_solver=solver)
    log_parity(f"cpp/{name}/{solver}", theta=_rel(th, g["theta"]), u=_relu(u, g["u"]))
    assert st["iters"] == meta["iters"]
    assert rho == meta["rho"]
    assert _rel(th, g["theta"]) <= RTOL_THETA
    assert _relu(u, g["u"]) <= RTOL_THETA
    P.close()


@pytest.mark.parametrize("name", ["py_1d_n1000_m1000_lam2", "py_1d_n1000_m250_lam2", "py_1d_n1000_m1000_lam0.5"])
def test_py_config1(name):
    """Config 1: 1D n = 1000 against the reference's own solvers.mbs_one output."""
    meta, g = load_golden(name)
    P = mv.Problem(meta["m"], g["Oty"], wdiag=g["W"], order=mv.ORDER_PY, weighted=False)
    ym = float(g["y"].mean())
    th, _, _, st = P.admm(meta["lam"], np.full(meta["m"][0], ym), variant=mv.VARIANT_PY, ymean=ym,
                          pcg_rtol=1e-13, return_u=False)
    log_parity(f"py/{name}", theta=_rel(th, g["theta"]))
    assert _rel(th, g["theta"]) <= RTOL_THETA
    P.close()
