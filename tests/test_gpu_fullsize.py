"""BASELINE.json configs at their real shapes, anchored to the CPU oracle where it finishes in seconds.

* metric config, 3-D 512^3, against the C oracle (oracle/c/mvtv_oracle.c's variant-B loop with the exact
  cosine-transform theta-solve by scipy.fft, pinned in tests/test_oracle_c.py): 2 fixed iterations of
  rcpp-code/MultivarTV/src/solvers.cpp:110-133 on the same inputs, the GPU's whole bench path (fused
  k_admm3a at 512^3's tiling, k_dct8 / k_tri, the device-side control) — rho exact, theta and u 1e-10,
  r / s norms 1e-9; and the spectral solve against the Jacobi-PCG (rtol 1e-13) for 3 iterations;
* config 5's tile shapes, 4-D 128 x 128 x 128 x 16, against the same C oracle (k_edge4d / k_gather4a/b on
  128^3 hyperplanes);
* config 5, 4-D 128^4 on one GPU: the same agreement for 2 iterations (one process holds the whole
  128^4 mesh: 15 edge blocks, 32 GB of edge state);
* config 4's work item, 2-D 2048^2 with a 0/1 CV-fold mask W (rcpp…/solvers.cpp:340-353): a
  warm-started lambda chunk (4 lambdas x 3 fixed iterations, theta / u / rho carried,
  rcpp…/solvers.cpp:212-220) against oracle/c/mvtv_oracle.c run on the same inputs, which follows
  the same warm-start chain on the host.

Tolerances: with identical adapt_step decisions theta differs only by the theta-solve's accuracy
(PCG rtol 1e-13 on both sides): |dtheta| <= 1e-9 max|theta|; rho exactly; r and s norms 1e-8 rel.
"""
import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")
from multivartv_amd import cv  # noqa: E402
from multivartv_amd.synth import towers  # noqa: E402

pytestmark = pytest.mark.gpu


def _two_solvers(m, iters):
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    out = {}
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        assert P.spectral_ok()
        th0 = np.full(y.size, y.mean())
        del y
        for solver in (mv.SOLVER_SPECTRAL, mv.SOLVER_PCG):
            P.state_set(th0, None, 0.2)
            st = P.run(1.0, fixed_iters=iters, pcg_rtol=1e-13, theta_solver=solver)
            th, _, rho = P.state_get(want_u=False)
            out[solver] = (th, rho, st)
    (ts, rs, ss), (tp, rp, sp) = out[mv.SOLVER_SPECTRAL], out[mv.SOLVER_PCG]
    assert ss["theta_solver"] == mv.SOLVER_SPECTRAL and sp["theta_solver"] == mv.SOLVER_PCG
    assert ss["iters"] == sp["iters"] == iters
    assert rs == rp
    assert np.max(np.abs(ts - tp)) <= 1e-9 * np.max(np.abs(tp))
    assert ss["r_norm"] == pytest.approx(sp["r_norm"], rel=1e-9)
    assert ss["s_norm"] == pytest.approx(sp["s_norm"], rel=1e-9)
    return ss, sp


def _vs_c_oracle(m, iters):
    """GPU (AUTO = the spectral solve, the bench's path) against the C oracle's spectral loop, same inputs."""
    from oracle import c_oracle
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    lam, rho0 = 1.0, 0.2
    th0 = np.full(y.size, y.mean())
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        P.state_set(th0, None, rho0)
        st = P.run(lam, fixed_iters=iters)
        assert st["theta_solver"] == mv.SOLVER_SPECTRAL and st["iters"] == iters
        tg, ug, rg = P.state_get(want_u=True)
    th, u = th0.copy(), np.zeros(c_oracle.num_edges(m))
    assert u.size == ug.size
    c_oracle.set_threads(min(16, c_oracle.threads()))
    ref = c_oracle.admm_rcpp_spectral(m, y, lam, th, u, rho0, deltas, fixed_iters=iters,
                                      workers=min(16, c_oracle.threads()))
    del y
    assert ref["iters"] == iters and rg == ref["rho"] and st["rho"] == ref["rho"]
    assert np.max(np.abs(tg - th)) <= 1e-10 * np.max(np.abs(th))
    assert np.max(np.abs(ug - u)) <= 1e-10 * np.max(np.abs(u))
    assert st["r_norm"] == pytest.approx(ref["r_norm"], rel=1e-9)
    assert st["s_norm"] == pytest.approx(ref["s_norm"], rel=1e-9)


@pytest.mark.timeout(600)
def test_metric_config_512_cubed_vs_c_oracle():
    _vs_c_oracle([512, 512, 512], 2)


@pytest.mark.timeout(300)
def test_config5_tile_shapes_4d_vs_c_oracle():
    _vs_c_oracle([128, 128, 128, 16], 2)


@pytest.mark.timeout(300)
def test_config3_256_cubed_vs_c_oracle():
    """Config 3 at its own kernel geometry: k_admm3a at 256^3 runs 76 tiles x 10 dim-2 chunks of 26 planes with a
    ragged 22-plane last chunk (mvtv_admm3d.hip f3d_args), which the 64^3 / 128^3 / 512^3 cases never take."""
    _vs_c_oracle([256, 256, 256], 2)


@pytest.mark.timeout(900)
def test_config5_128_4d_vs_c_oracle():
    """Config 5 at its own kernel geometry: k_edge4d marching all 128 w-planes and k_gather4a's 2 z-chunks of 64
    (16 chunks of 8 at 128 x 128 x 128 x 16). One iteration: the C oracle holds ~160 GB of host edge state."""
    _vs_c_oracle([128, 128, 128, 128], 1)


def test_metric_config_512_cubed():
    ss, sp = _two_solvers([512, 512, 512], 3)
    assert sp["pcg_unconverged"] == 0


def test_config5_4d_128_single_gpu():
    ss, sp = _two_solvers([128, 128, 128, 128], 2)
    assert sp["pcg_unconverged"] == 0


@pytest.mark.parametrize("solver", [mv.SOLVER_AUTO, mv.SOLVER_PCG], ids=["auto_pcg_spectral", "jacobi_pcg"])
def test_config4_fold_path_2048_vs_c_oracle(solver):
    from oracle import c_oracle
    m = [2048, 2048]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    fold = cv.kfoldinds(y.size, 5, seed=0)
    W = (fold != 0).astype(np.float64)          # training rows of fold 0: O^T O on the lattice
    oty = W * y                                  # O^T y
    ymean = float(y[W > 0].mean())
    lams = np.array([1.6, 1.2, 0.9, 0.7])
    iters = 3
    with mv.Problem(m, oty, wdiag=W, deltas=deltas, order=mv.ORDER_CPP) as P:
        assert not P.spectral_ok()
        thetas, rhos, stats = P.path(lams, np.full(y.size, ymean), lams[0] / 5.0, fixed_iters=iters,
                                     pcg_rtol=1e-13, theta_solver=solver)
    th = np.full(y.size, ymean)
    u = np.zeros(c_oracle.num_edges(m))
    rho = lams[0] / 5.0
    for k, lam in enumerate(lams):
        st = c_oracle.admm_rcpp(m, oty, lam, th, u, rho, deltas, W=W, fixed_iters=iters, pcg_rtol=1e-13)
        rho = st["rho"]
        want = mv.SOLVER_PCG if solver == mv.SOLVER_PCG else mv.SOLVER_PCG_SPECTRAL
        assert stats[k]["iters"] == iters and stats[k]["theta_solver"] == want
        assert rhos[k] == rho
        assert np.max(np.abs(thetas[k] - th)) <= 1e-9 * np.max(np.abs(th)), k
        assert stats[k]["r_norm"] == pytest.approx(st["r_norm"], rel=1e-9)
        assert stats[k]["s_norm"] == pytest.approx(st["s_norm"], rel=1e-9)


@pytest.mark.parametrize("m", [[160, 160, 8], [256, 256, 4]], ids=["160x160x8", "256x256x4"])
def test_fold_3d_pcg_spectral_multi_run_vs_c_oracle(m):
    """A 3-D CV-fold mask (W != I) on meshes whose dim-0 rows span more than one 128-cell run of the two-cell
    operator (k_apply3d2's W-diagonal, dot-product form inside the spectrally preconditioned PCG, pcgs_solve):
    3 fixed iterations against the C oracle's variant-B loop on the same inputs, rho exact, theta 1e-9."""
    from oracle import c_oracle
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    W = (cv.kfoldinds(y.size, 5, seed=1) != 0).astype(np.float64)
    oty = W * y
    th0 = np.full(y.size, float(y[W > 0].mean()))
    lam, rho0, iters = 0.8, 0.16, 3
    with mv.Problem(m, oty, wdiag=W, deltas=deltas, order=mv.ORDER_CPP) as P:
        th, u, rho, st = P.admm(lam, th0, u=np.zeros(P.E), rho=rho0, fixed_iters=iters, pcg_rtol=1e-13,
                                theta_solver=mv.SOLVER_PCG_SPECTRAL)
    ref_th, ref_u = th0.copy(), np.zeros(c_oracle.num_edges(m))
    ref = c_oracle.admm_rcpp(m, oty, lam, ref_th, ref_u, rho0, deltas, W=W, fixed_iters=iters, pcg_rtol=1e-13)
    assert st["iters"] == iters and st["theta_solver"] == mv.SOLVER_PCG_SPECTRAL
    assert rho == ref["rho"]
    assert np.max(np.abs(th - ref_th)) <= 1e-9 * np.max(np.abs(ref_th))
    assert st["r_norm"] == pytest.approx(ref["r_norm"], rel=1e-8)


def test_metric_512_cubed_eight_rank_decomposition():
    """The metric at 8 GPUs as bench.py runs it (one 512^3 mesh, 64 planes per rank), rehearsed with the
    loopback transport on one GPU: 2 fixed iterations against the one-GPU run, rho exact, theta 1e-11."""
    from multivartv_amd import slab
    m, lam, iters = [512, 512, 512], 1.0, 2
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        P.state_set(np.full(y.size, y.mean()), None, lam / 5.0)
        st = P.run(lam, fixed_iters=iters)
        th, _, rho = P.state_get(want_u=False)
    out, theta = slab.run_local_group(m, y, deltas, lam, 8, fixed_iters=iters)
    assert all(o["iters"] == iters and o["rho"] == rho for o in out)
    assert out[0]["r_norm"] == pytest.approx(st["r_norm"], rel=1e-9)
    assert np.max(np.abs(theta - th)) <= 1e-11 * np.max(np.abs(th))


def test_config5_128_4d_eight_rank_decomposition():
    """Config 5 at its shape: 128^4 slab-decomposed over 8 ranks (16 planes of dim 3 each), the ranks'
    mvtv_slab_run loops on one GPU over the in-process loopback transport, against the one-GPU run:
    2 fixed iterations, rho exact, theta to 1e-11 (only the order of the global sums differs)."""
    from multivartv_amd import slab
    m, lam, iters = [128, 128, 128, 128], 1.0, 2
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        P.state_set(np.full(y.size, y.mean()), None, lam / 5.0)
        st = P.run(lam, fixed_iters=iters)
        th, _, rho = P.state_get(want_u=False)
    out, theta = slab.run_local_group(m, y, deltas, lam, 8, fixed_iters=iters)
    assert all(o["iters"] == iters and o["rho"] == rho for o in out)
    assert out[0]["r_norm"] == pytest.approx(st["r_norm"], rel=1e-9)
    assert np.max(np.abs(theta - th)) <= 1e-11 * np.max(np.abs(th))
