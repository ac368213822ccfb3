"""BASELINE.json configs at (or near) full size, checked through size-independent properties.

SuperLU cannot factor these meshes, so the check is agreement of two independent theta-solvers
on the same ADMM trajectory: the exact spectral solve (default) and the Jacobi-PCG of the north
star at rtol 1e-13. Both follow the reference's variant-B decisions (rcpp…/solvers.cpp:110-133);
with identical decisions theta agrees to the PCG tolerance (asserted at 1e-9 of max|theta|),
the residual norms to 1e-8 relative, and rho exactly.
"""
import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")
from multivartv_amd.synth import towers  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,iters", [([256, 256, 256], 4), ([1024, 1024], 6), ([2048, 2048], 3), ([64, 64, 64, 64], 3)],
                         ids=["3d_256", "2d_1024", "2d_2048", "4d_64"])
def test_spectral_and_pcg_trajectories_agree(m, iters):
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    out = {}
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        assert P.spectral_ok()
        for solver in (mv.SOLVER_SPECTRAL, mv.SOLVER_PCG):
            P.state_set(np.full(y.size, y.mean()), None, 0.2)
            st = P.run(1.0, fixed_iters=iters, pcg_rtol=1e-13, theta_solver=solver)
            th, _, rho = P.state_get(want_u=False)
            out[solver] = (th, rho, st)
    (ts, rs, ss), (tp, rp, sp) = out[mv.SOLVER_SPECTRAL], out[mv.SOLVER_PCG]
    assert ss["theta_solver"] == mv.SOLVER_SPECTRAL and sp["theta_solver"] == mv.SOLVER_PCG
    assert rs == rp
    assert np.max(np.abs(ts - tp)) <= 1e-9 * np.max(np.abs(tp))
    assert ss["r_norm"] == pytest.approx(sp["r_norm"], rel=1e-9)
    assert ss["s_norm"] == pytest.approx(sp["s_norm"], rel=1e-9)

