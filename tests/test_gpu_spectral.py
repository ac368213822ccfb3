"""GPU parity of the spectral theta-solve (mvtv_spectral.hip) through the C ABI.

The spectral solve is a direct method (cosine transforms + diagonal divide), so it is
compared with SciPy's SuperLU factorisation of the same matrix I + sigma D^T D — the
solver the reference calls every ADMM iteration (rcpp-code/MultivarTV/src/solvers.cpp:113)
— at a rounding-level tolerance: max|x - x_ref| <= 1e-12 max|x_ref| (fp64).
At the BASELINE sizes (256^3, 1024^2, 128^4 would not fit SuperLU) the check is the
size-independent residual ||A x - b|| / ||b|| <= 1e-12 with A applied by the stencil kernel.
"""
import numpy as np
import pytest

from oracle import mvtv_oracle as O

mv = pytest.importorskip("multivartv_amd")
pytestmark = pytest.mark.gpu

RTOL_DIRECT = 1e-12


def _cond(P, sigma):
    """cond(I + sigma D^T D) = max mu / min mu; mu = 1 + sigma sum_S cS[S] prod_{j in S} lam_j <= 1 + sigma sum cS 4^|S|."""
    cs = 0.0
    for _, sp, w in P.block_info():
        cs += w * w * 4.0 ** bin(sp).count("1")
    return 1.0 + sigma * cs


def _rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1e-300, np.max(np.abs(b))))


CASES = [([2], None, "cpp", False), ([8], None, "cpp", False), ([1024], None, "py", False),
         ([4096], None, "cpp", False), ([16, 8], [0.3, 0.7], "cpp", False), ([2, 64], [0.5, 0.5], "cpp", False),
         ([32, 32], None, "py", False), ([8, 8, 8], [0.5, 0.25, 0.125], "cpp", False),
         ([16, 16, 16], [0.2, 0.3, 0.4], "cpp", True), ([8, 8, 8], [0.5, 0.25, 0.125], "py", False),
         ([4, 4, 4, 4], [0.5, 0.25, 0.125, 0.3], "cpp", False), ([4, 4, 4, 4], None, "py", False),
         ([8, 8, 8, 8], [0.1, 0.2, 0.3, 0.4], "cpp", False),
         # >= 4096 lines of >= 64 points along the last dim: the tridiagonal last-dimension pass (k_tri)
         # (3-D and 4-D meshes large enough for it are checked by residual and against PCG below)
         ([4096, 64], [0.3, 0.7], "cpp", False), ([4096, 128], None, "py", False),
         # mixed-radix lengths (k_dctg), also powers of two over a general stride
         ([3], None, "cpp", False), ([1000], None, "py", False), ([2187], None, "cpp", False),
         ([12, 8], [0.3, 0.7], "cpp", False), ([24, 40], [0.5, 0.5], "cpp", False), ([63, 10], None, "py", False),
         ([6, 6, 6], [0.5, 0.25, 0.125], "cpp", False), ([10, 10, 10], None, "py", False),
         ([5, 5, 5, 5], [0.1, 0.2, 0.3, 0.4], "cpp", False), ([6, 6, 6, 6], None, "py", False),
         ([7, 7, 7], [0.2, 0.3, 0.4], "cpp", True), ([3, 4096], [0.5, 0.5], "cpp", False),
         # mixed-radix mesh whose last dimension takes the general-length tridiagonal pass (k_trig)
         ([4096, 100], [0.5, 0.5], "cpp", False),
         # ... and on 4-line tiles for the >= 1000 lines of a 2-D mesh (a prime length with a shorter last segment; a
         # mixed-radix one)
         ([1024, 67], [0.5, 0.5], "cpp", False), ([1200, 100], None, "py", False),
         # register-resident mixed-radix passes along dim 0 (k_dctm, m = 500 / 1000; the strided form is checked
         # at 500^3 below: unequal dims are refused at p >= 3, the reference's mixed-partial rule)
         ([500, 6], [0.3, 0.7], "cpp", False), ([1000, 4], None, "py", False),
         # an odd number of lines: k_dctm pairs lines, so these fall back to k_dctg
         ([500, 7], [0.3, 0.7], "cpp", False), ([1000, 3], None, "py", False),
         # lengths with a prime factor >= 11 (Bluestein, k_dctb): FWD / INV along dim 0, MID along a 1-D mesh, a
         # strided MID along the last dimension (few lines; >= 4096 lines of a prime length take k_trig with a
         # shorter last segment: 67 = 4 x 16 + 3),
         # M = 8192 (one line pair in 128 KB of LDS), the R API's default m = floor(sqrt(n)) (31 at n = 1000)
         ([31], None, "cpp", False), ([1009], None, "py", False), ([4093], None, "cpp", False),
         ([37, 37], [0.3, 0.7], "cpp", False), ([22, 13], None, "py", False), ([4096, 67], [0.5, 0.5], "cpp", False),
         ([67, 4096], None, "cpp", False), ([2039, 6], [0.3, 0.7], "cpp", False),
         ([11, 11, 11], [0.2, 0.3, 0.4], "cpp", False), ([8, 8, 11], [0.5, 0.25, 0.125], "cpp", False),
         ([31, 31, 31], None, "py", False), ([11, 11, 11, 11], [0.1, 0.2, 0.3, 0.4], "cpp", False)]


def _problem(m, deltas, order, unit, seed=0):
    rng = np.random.default_rng(seed)
    N = int(np.prod(m))
    o = mv.ORDER_CPP if order == "cpp" else mv.ORDER_PY
    weighted = (deltas is not None) and not unit
    P = mv.Problem(m, rng.standard_normal(N), deltas=deltas if deltas is not None else [1.0] * len(m), order=o,
                   weighted=weighted)
    D = O.build_D(m, O.block_table(len(m), deltas if weighted else None, order, unit_weights=unit))
    return P, D


@pytest.mark.parametrize("m,deltas,order,unit", CASES)
@pytest.mark.parametrize("sigma", [0.05, 3.2, 400.0])
def test_spectral_vs_superlu(m, deltas, order, unit, sigma):
    P, D = _problem(m, deltas, order, unit)
    assert P.spectral_ok()
    N = int(np.prod(m))
    b = np.random.default_rng(3).standard_normal(N)
    ref = O._solver(np.ones(N), (D.T @ D).tocsc(), sigma).solve(b)
    x = P.solve_spectral(sigma, b)
    # both solvers are backward stable: forward error ~ eps * cond(A)
    assert _rel(x, ref) <= max(RTOL_DIRECT, 2e-16 * _cond(P, sigma))
    P.close()


@pytest.mark.parametrize("m", [[256, 256, 256], [1024, 1024], [64, 64, 64, 64], [100, 100, 100], [240, 240, 240],
                               [60, 60, 60, 60], [500, 500, 500], [1000, 1000], [1009, 1009], [251, 251, 251],
                               [2039, 2048]])
def test_spectral_residual_baseline_sizes(m):
    """Config-sized meshes (3D 256^3, 2D 1024^2; 4D at 64^4), mixed-radix ones (k_dctg / k_dctm passes,
    k_trig last dimension) and prime lengths (k_dctb): residual through the stencil operator."""
    p = len(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    N = int(np.prod(m))
    b = np.random.default_rng(5).standard_normal(N)
    with mv.Problem(m, b, deltas=deltas, order=mv.ORDER_CPP) as P:
        for sigma in (0.2, 51.2):
            x = P.solve_spectral(sigma, b)
            r = P.apply_A(sigma, x) - b
            assert np.linalg.norm(r) / np.linalg.norm(b) <= RTOL_DIRECT, (p, sigma)


@pytest.mark.parametrize("m", [[256, 256, 128], [512, 512, 128], [1024, 1024, 128], [256, 256, 300], [512, 512, 135],
                               [256, 256, 48], [96, 96, 400], [128, 128, 37], [256, 256, 101], [64, 64, 1009],
                               [64, 64, 1024], [32, 32, 1024], [128, 128, 512], [64, 64, 64], [48, 48, 256]])
def test_3d_solve_residual_extreme_sigma(m):
    """3-D spectral solves (k_dct8 / k_dctg passes, k_tri along the last dimension) from sigma = 0 (the identity) to a
    dominant coupling (cond ~ 1e7): residual through the stencil operator within the backward-stable bound;
    256 / 512 / 1024-point rows, last-dimension lengths a power of two, 300 = 4 3 5^2 and 135 = 27 5 (k_trig on
    64-line tiles, 20- and 27-row segments), 48 (16-row segments), 400 (25 segments of 16: 32-line tiles), and
    lengths k_trig splits with a shorter last segment: 37 = 3 x 10 + 7, 101 = 6 x 16 + 5 (64-line tiles), the prime
    1009 = 63 x 16 + 1 (a one-row last segment; 16-line tiles, 4096 lines). Round 6 (the factorised line solve,
    k_trir / k_trigr): 1024-point lines on 16-line tiles of 64 segments (64 x 64 x 1024) and on the few-lines 4-line
    tiles (32 x 32 x 1024), the 512-point 32-line tiles (128 x 128 x 512), 64-point lines (64^3: 16-line tiles of 4
    segments) and k_trigr's few-lines tiles over a line stride that is not a power of two (48 x 48 x 256)."""
    p = len(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    N = int(np.prod(m))
    b = np.random.default_rng(7).standard_normal(N)
    with mv.Problem(m, b, deltas=deltas, order=mv.ORDER_CPP) as P:
        for sigma in (0.0, 1e-3, 3.7, 2e5):
            x = P.solve_spectral(sigma, b)
            r = P.apply_A(sigma, x) - b
            # backward stable: residual ~ eps |A| |x| (cond ~ 1e7 at sigma = 2e5)
            assert np.linalg.norm(r) / np.linalg.norm(b) <= max(RTOL_DIRECT, 2e-16 * _cond(P, sigma)), (p, sigma)


def test_spectral_matches_pcg_large():
    """256^3 theta-solve: spectral vs PCG at rtol 1e-13 agree to the PCG tolerance."""
    m = [128, 128, 128]
    N = int(np.prod(m))
    b = np.random.default_rng(6).standard_normal(N)
    deltas = [(1.0 + 2e-4) / v for v in m]
    with mv.Problem(m, b, deltas=deltas, order=mv.ORDER_CPP) as P:
        xs = P.solve_spectral(7.0, b)
        xp, it, rr = P.solve(7.0, b, rtol=1e-13)
        assert rr <= 1e-13
        assert _rel(xs, xp) <= 1e-11


def test_spectral_rejected_when_not_exact():
    rng = np.random.default_rng(0)
    with mv.Problem([4099, 2], rng.standard_normal(8198), deltas=[1, 1]) as P:      # m_0 > 4096
        assert not P.spectral_ok()
        with pytest.raises(mv.MvtvError):
            P.solve_spectral(1.0, np.zeros(8198))
        with pytest.raises(mv.MvtvError):
            P.admm(1.0, np.zeros(8198), u=np.zeros(P.E), rho=0.2, theta_solver=mv.SOLVER_SPECTRAL)
        _, _, _, st = P.admm(1.0, np.zeros(8198), u=np.zeros(P.E), rho=0.2, fixed_iters=2)
        assert st["theta_solver"] == mv.SOLVER_PCG
    with mv.Problem([22, 8], rng.standard_normal(176), deltas=[1, 1]) as P:      # 22 = 2 * 11: Bluestein
        assert P.spectral_ok()
        _, _, _, st = P.admm(1.0, np.zeros(176), u=np.zeros(P.E), rho=0.2, fixed_iters=2)
        assert st["theta_solver"] == mv.SOLVER_SPECTRAL
    with mv.Problem([8, 8], rng.standard_normal(64), wdiag=rng.uniform(0, 2, 64).round(), deltas=[1, 1]) as P:
        assert not P.spectral_ok()                                               # W != I
        _, _, _, st = P.admm(1.0, np.zeros(64), u=np.zeros(P.E), rho=0.2, fixed_iters=2)
        assert st["theta_solver"] == mv.SOLVER_PCG_SPECTRAL                     # AUTO: 2-3-5-7 mesh


def test_spectral_admm_towers_3d():
    """ADMM on the bench's towers problem at 32^3: spectral and PCG runs take the same decisions."""
    from multivartv_amd.synth import towers
    m = [32, 32, 32]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        th0 = np.full(y.size, y.mean())
        ts, us, rs, ss = P.admm(1.0, th0, u=np.zeros(P.E), rho=0.2, theta_solver=mv.SOLVER_SPECTRAL)
        tp, up, rp, sp = P.admm(1.0, th0, u=np.zeros(P.E), rho=0.2, theta_solver=mv.SOLVER_PCG, pcg_rtol=1e-13)
    assert ss["theta_solver"] == mv.SOLVER_SPECTRAL and sp["theta_solver"] == mv.SOLVER_PCG
    assert ss["iters"] == sp["iters"] and rs == rp
    assert _rel(ts, tp) <= 1e-8


@pytest.mark.parametrize("variant", [mv.VARIANT_RCPP, mv.VARIANT_CPP, mv.VARIANT_PY])
def test_async_loop_matches_host_loop(variant, monkeypatch):
    """The device-side ADMM control (k_admm_control, no per-iteration host sync) takes the same
    decisions as the host loop: same iteration count, rho, and theta to the last bit in practice."""
    from multivartv_amd.synth import towers
    m = [16, 16, 16]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    lam = 1.0 if variant == mv.VARIANT_RCPP else 2.0
    out = {}
    for mode in ("async", "sync"):
        if mode == "sync":
            monkeypatch.setenv("MVTV_ADMM_SYNC", "1")
        else:
            monkeypatch.delenv("MVTV_ADMM_SYNC", raising=False)
        with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
            th0 = np.full(y.size, y.mean())
            out[mode] = P.admm(lam, th0, u=np.zeros(P.E) if variant == mv.VARIANT_RCPP else None, rho=lam / 5,
                               variant=variant, ymean=float(y.mean()), return_u=True)
    (ta, ua, ra, sa), (ts, us, rs, ss) = out["async"], out["sync"]
    assert sa["theta_solver"] == mv.SOLVER_SPECTRAL
    assert sa["iters"] == ss["iters"] and ra == rs and sa["status"] == ss["status"]
    assert _rel(ta, ts) <= 1e-12
    assert np.max(np.abs(ua - us)) <= 1e-12 * max(1.0, np.max(np.abs(us)))


@pytest.mark.parametrize("weighted", [True, False])
def test_fused_path_python_block_order(weighted):
    """Python create_D block order (code/utils.py:138-149): 6 blocks when weighted, 7 unweighted;
    the fused 3-D kernel's NB = 6 / 7 instantiations against the SuperLU oracle (10 iterations)."""
    from multivartv_amd.synth import towers
    m = [16, 16, 16]
    y = towers(m, seed=99)
    deltas = [0.3, 0.5, 0.7]
    P = mv.Problem(m, y, deltas=deltas, order=mv.ORDER_PY, weighted=weighted)
    assert P.nb == (6 if weighted else 7)
    th, u, rho, st = P.admm(1.0, np.full(y.size, y.mean()), u=np.zeros(P.E), rho=0.2, fixed_iters=10)
    P.close()
    D = O.build_D(m, O.block_table(3, deltas if weighted else None, "py"))
    ref = O.admm_rcpp(D, y, np.ones(y.size), 1.0, np.full(y.size, y.mean()), np.zeros(D.shape[0]), 0.2,
                      fixed_iters=10)
    assert st["theta_solver"] == mv.SOLVER_SPECTRAL and rho == ref.rho
    assert _rel(th, ref.theta) <= 1e-10
    assert np.max(np.abs(u - ref.u)) <= 1e-10 * max(1.0, np.max(np.abs(ref.u)))


def _scattered_problem(m, n, seed):
    rng = np.random.default_rng(seed)
    p = len(m)
    x = rng.uniform(0, 1, size=(n, p))
    y = np.where(np.all(x > 0.6, axis=1), 1.0, 0.0) + 0.3 * rng.standard_normal(n)
    axes = [np.linspace(-1e-4, 1 + 1e-4, v) for v in m]
    idx = np.zeros(n, dtype=np.int64)
    stride = 1
    for j in range(p):
        idx += np.abs(x[:, j:j + 1] - axes[j][None, :]).argmin(axis=1) * stride
        stride *= m[j]
    N = int(np.prod(m))
    W = np.bincount(idx, minlength=N).astype(float)
    oty = np.bincount(idx, weights=y, minlength=N)
    return W, oty


def _fold_problem(m, k, seed):
    """lattice data with one CV fold held out: W = 1 except zeros on ~1/k of the nodes"""
    from multivartv_amd.synth import towers
    y = towers(m, seed=seed)
    W = (np.random.default_rng(seed).permutation(y.size) % k != 0).astype(float)
    return W, W * y


@pytest.mark.parametrize("case", ["scat_32x32", "scat_16x16x16", "fold_64x64", "fold_16x16x16", "scat_31x31",
                                  "fold_37x37", "scat_11x11x11"])
def test_spectrally_preconditioned_pcg(case):
    """W != I (scattered data, CV folds): PCG preconditioned by S (mean(W) I + sigma D^T D) S (the middle
    factor applied exactly by cosine transforms) reproduces the SuperLU trajectory like Jacobi-PCG."""
    kind, dims = case.split("_")
    m = [int(v) for v in dims.split("x")]
    W, oty = (_scattered_problem(m, 3 * int(np.prod(m)) // 5, seed=len(m)) if kind == "scat"
              else _fold_problem(m, 5, seed=len(m)))
    deltas = [(1.0 + 2e-4) / v for v in m]
    D = O.build_D(m, O.block_table(len(m), deltas, "cpp"))
    th0 = np.full(W.size, oty.sum() / W.sum())
    ref = O.admm_rcpp(D, oty, W, 0.5, th0, np.zeros(D.shape[0]), 0.1, fixed_iters=15)
    out = {}
    with mv.Problem(m, oty, wdiag=W, deltas=deltas, order=mv.ORDER_CPP) as P:
        for solver in (mv.SOLVER_PCG, mv.SOLVER_PCG_SPECTRAL):
            out[solver] = P.admm(0.5, th0, u=np.zeros(P.E), rho=0.1, fixed_iters=15, pcg_rtol=1e-13,
                                 theta_solver=solver)
    for solver, (th, u, rho, st) in out.items():
        assert st["theta_solver"] == solver and rho == ref.rho
        assert _rel(th, ref.theta) <= 1e-9
    print(case, "PCG iterations: Jacobi", out[mv.SOLVER_PCG][3]["pcg_iters"], "spectral",
          out[mv.SOLVER_PCG_SPECTRAL][3]["pcg_iters"])


@pytest.mark.parametrize("variant", [mv.VARIANT_RCPP, mv.VARIANT_CPP, mv.VARIANT_PY])
def test_async_loop_max_counter(variant, monkeypatch):
    """max_counter handling on the device matches the host loop: B stops with MAXITER after
    max_counter - 1 iterations (rcpp…/solvers.cpp:129-132), A reports MAXITER (its throw,
    cpp-code/solvers.cpp:122-124), C stops at max_counter iterations."""
    from multivartv_amd.synth import towers
    m = [16, 16, 16]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    res = {}
    for mode in ("async", "sync"):
        if mode == "sync":
            monkeypatch.setenv("MVTV_ADMM_SYNC", "1")
        else:
            monkeypatch.delenv("MVTV_ADMM_SYNC", raising=False)
        with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
            P.state_set(np.full(y.size, y.mean()), None, 0.2)
            st = P.run(2.0, variant=variant, max_counter=6, tol=1e-12, ymean=float(y.mean()))
            th, _, rho = P.state_get(want_u=False)
        res[mode] = (st, th, rho)
    (sa, ta, ra), (ss, ts, rs) = res["async"], res["sync"]
    assert sa["status"] == ss["status"] == 1          # MVTV_MAXITER
    assert sa["iters"] == ss["iters"] and ra == rs
    assert _rel(ta, ts) <= 1e-12


@pytest.mark.parametrize("m", [[31, 31, 31], [37, 37], [11, 11, 11, 11], [67, 67, 31]],
                         ids=["31^3", "37^2", "11^4", "67x67x31"])
def test_bluestein_admm_vs_c_oracle(m):
    """Prime lengths through the bench's loop (asynchronous control, b formed on load by k_dctb's first pass, the
    fused edge kernels) against the C oracle's variant-B loop with scipy.fft's exact solve (any length):
    rcpp-code/MultivarTV/src/solvers.cpp:110-133, 12 fixed iterations, rho exact, theta / u 1e-10."""
    from multivartv_amd.synth import towers
    from oracle import c_oracle
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    lam, rho0, fixed = 0.8, 0.16, 12
    th0 = np.full(y.size, y.mean())
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        assert P.spectral_ok()
        P.state_set(th0, None, rho0)
        st = P.run(lam, fixed_iters=fixed)
        tg, ug, rg = P.state_get(want_u=True)
    assert st["theta_solver"] == mv.SOLVER_SPECTRAL and st["iters"] == fixed
    th, u = th0.copy(), np.zeros(c_oracle.num_edges(m))
    ref = c_oracle.admm_rcpp_spectral(m, y, lam, th, u, rho0, deltas, fixed_iters=fixed)
    assert rg == ref["rho"]
    assert _rel(tg, th) <= 1e-10
    assert np.max(np.abs(ug - u)) <= 1e-10 * max(1.0, np.max(np.abs(u)))
    assert st["r_norm"] == pytest.approx(ref["r_norm"], rel=1e-9)


@pytest.mark.parametrize("lam,kmax", [(0.5, None), (50.0, 50)], ids=["rho0.1", "rho10"])
def test_r_default_mesh_scattered_fold_takes_spectral_pcg(lam, kmax):
    """The released R API's default mesh for n = 1000 points, m = floor(sqrt(n)) = 31 per dimension
    (rcpp-code/MultivarTV/R/MultivarTV.R:44-48), one CV fold of scattered data (W = training counts, 44 % of the
    nodes empty): AUTO takes PCG with the cosine-transform preconditioner (Bluestein at 31) and matches the SuperLU
    oracle's trajectory (rcpp…/solvers.cpp:113). Iterations per theta-solve: at rho0 = 10 (sigma D^T D comparable
    to W) K-bar < 50; at rho0 = 0.1 the system is W-dominated with weakly coupled empty nodes, where the
    preconditioner still beats Jacobi (K-bar ~ 90 against ~ 145)."""
    m, n = [31, 31], 1000
    rng = np.random.default_rng(17)
    x = rng.uniform(0, 1, size=(n, 2))
    yv = np.where(np.all(x > 0.6, axis=1), 1.0, 0.0) + 0.3 * rng.standard_normal(n)
    train = rng.permutation(n) % 5 != 0
    axes = [np.linspace(0.0, 1.0, v) for v in m]
    idx = np.abs(x[:, :1] - axes[0][None, :]).argmin(axis=1) + 31 * np.abs(x[:, 1:] - axes[1][None, :]).argmin(axis=1)
    W = np.bincount(idx[train], minlength=961).astype(float)
    oty = np.bincount(idx[train], weights=yv[train], minlength=961)
    deltas = [(1.0 + 2e-4) / v for v in m]
    D = O.build_D(m, O.block_table(2, deltas, "cpp"))
    rho0, fixed = lam / 5.0, 20
    th0 = np.full(W.size, oty.sum() / W.sum())
    ref = O.admm_rcpp(D, oty, W, lam, th0, np.zeros(D.shape[0]), rho0, fixed_iters=fixed)
    with mv.Problem(m, oty, wdiag=W, deltas=deltas, order=mv.ORDER_CPP) as P:
        th, u, rho, st = P.admm(lam, th0, u=np.zeros(P.E), rho=rho0, fixed_iters=fixed, pcg_rtol=1e-13)
        _, _, _, sj = P.admm(lam, th0, u=np.zeros(P.E), rho=rho0, fixed_iters=fixed, pcg_rtol=1e-13,
                             theta_solver=mv.SOLVER_PCG)
    assert st["theta_solver"] == mv.SOLVER_PCG_SPECTRAL and rho == ref.rho
    assert _rel(th, ref.theta) <= 1e-9
    kbar, kjac = st["pcg_iters"] / fixed, sj["pcg_iters"] / fixed
    print(f"31 x 31 scattered fold, rho0 {rho0}: K-bar spectral {kbar:.1f}, Jacobi {kjac:.1f}")
    assert kbar < 0.8 * kjac
    if kmax is not None:
        assert kbar < kmax
