"""Fused 3-D edge kernel (k_admm3a: 64-column tiles aligned to the edge chunks, 14 owned rows per
tile) on meshes whose dims 0 and 1 leave ragged last tiles (m0 % 64 != 0, m1 % 14 != 0) and on exact
multiples; m2 sets the dim-2 chunking (non-power-of-two meshes take the Jacobi-PCG solve). Each run is
checked against the C oracle (oracle/c/mvtv_oracle.c, variant B of rcpp…/solvers.cpp:96-136,
pinned to the golden fixtures in test_oracle_c.py) over fixed ADMM iterations: rho exactly, theta
and u to 1e-9 of their max (both sides solve to PCG rtol 1e-13, or exactly by DCT on the GPU)."""
import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")
c_oracle = pytest.importorskip("oracle.c_oracle")
from multivartv_amd.synth import towers  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,iters", [([64, 64, 64], 8), ([72, 72, 20], 6), ([100, 100, 30], 5), ([128, 128, 128], 4)],
                         ids=["aligned", "r8", "r36_pcg", "aligned_128"])
def test_fused_ragged_dim0_matches_oracle(m, iters):
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    lam = 1.0
    th0 = np.full(y.size, y.mean())
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        th, u, rho, st = P.admm(lam, th0, u=np.zeros(P.E), rho=lam / 5, fixed_iters=iters, pcg_rtol=1e-13)
        E = P.E
    ref_th = th0.copy()
    ref_u = np.zeros(E)
    rs = c_oracle.admm_rcpp(m, y, lam, ref_th, ref_u, lam / 5, deltas, fixed_iters=iters, pcg_rtol=1e-13)
    assert rho == rs["rho"]
    assert np.max(np.abs(th - ref_th)) <= 1e-9 * np.max(np.abs(ref_th))
    assert np.max(np.abs(u - ref_u)) <= 1e-9 * max(1.0, np.max(np.abs(ref_u)))


@pytest.mark.parametrize("m,lam", [([32, 32, 32], 1.0), ([32, 32, 32], 0.02), ([64, 64, 64], 1.0), ([128, 128, 128], 0.1),
                                   ([128, 96], 1.0), ([1024, 1024], 0.1), ([16, 16, 16, 16], 1.0), ([32, 32, 32, 32], 0.02),
                                   ([500, 24], 1.0), ([500, 40], 0.1)],
                         ids=["m32_lam1", "m32_lam002", "m64_lam1", "m128_lam01", "2d_128x96", "2d_1024", "4d_16_lam1",
                              "4d_32_lam002", "2d_500x24_unfolded", "2d_500x40_unfolded"])
def test_folded_rhs_converged_matches_oracle(m, lam):
    """The asynchronous spectral loop (2-D / 3-D fused kernels, 4-D two-pass gather) on a power-of-two m0 stores the folded s = rho (D^T alpha + D^T u) for the
    next solve's b = oty + s, and after a residual-balancing step that changed rho (7 doublings over these runs)
    forms b = oty + (rho'/rho) s + rho' (c - 1) D^T u. Converged runs against the C oracle's loop with the exact
    DCT solve (rcpp…/solvers.cpp:110-133): iterations and rho exactly, theta to 1e-9. The m0 = 500 cases take the
    unfolded first pass (b = oty + rho' D^T alpha + rho' c D^T u) in k_dctm."""
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    th0 = np.full(y.size, y.mean())
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        th, u, rho, st = P.admm(lam, th0, u=np.zeros(P.E), rho=lam / 5)
        E = P.E
    assert st["theta_solver"] == mv.SOLVER_SPECTRAL
    ref_th = th0.copy()
    ref_u = np.zeros(E)
    rs = c_oracle.admm_rcpp_spectral(m, y, lam, ref_th, ref_u, lam / 5, deltas)
    assert rs["rho"] != lam / 5   # the run adapted rho, so the fix-up path ran
    assert st["iters"] == rs["iters"]
    assert rho == rs["rho"]
    assert np.max(np.abs(th - ref_th)) <= 1e-9 * np.max(np.abs(ref_th))
    assert np.max(np.abs(u - ref_u)) <= 1e-9 * max(1.0, np.max(np.abs(ref_u)))


@pytest.mark.parametrize("m,iters,order,weighted,solver",
                         [([70, 70, 70, 9], 6, "cpp", True, mv.SOLVER_AUTO),
                          ([13, 13, 13, 6], 8, "cpp", True, mv.SOLVER_AUTO),
                          ([128, 128, 128, 3], 3, "cpp", True, mv.SOLVER_AUTO),
                          ([16, 16, 16, 5], 8, "py", True, mv.SOLVER_PCG),
                          ([16, 16, 16, 5], 8, "py", False, mv.SOLVER_PCG),
                          ([24, 24, 24, 4], 6, "cpp", True, mv.SOLVER_PCG)],
                         ids=["ragged_70_zchunks", "bluestein_13_every_plane_a_chunk", "aligned_128",
                              "py_weighted_14_blocks", "py_unweighted_15_blocks", "pcg_sync_loop"])
def test_fused4d_matches_oracle(m, iters, order, weighted, solver):
    """The fused 4-D pass (k_admm4a: edge update + the gather's pass A over one read of the edge state, 64 x 6
    tiles at a fixed w marching z, then k_gather4b) on ragged tiles (m0 % 64, m1 % 6 != 0), z-chunked grids (every
    chunk start recomputes a plane from the old state; 13^3 x 6 makes every plane a chunk), both block orders (15 and
    14 blocks) and the host-synchronous loop of a PCG theta-solve, against the C oracle's variant-B loop
    (rcpp…/solvers.cpp:96-136): rho exactly, theta and u to 1e-9 of their max."""
    y = towers(m)
    o = mv.ORDER_CPP if order == "cpp" else mv.ORDER_PY
    deltas = [(1.0 + 2e-4) / v for v in m]
    lam = 1.0
    th0 = np.full(y.size, y.mean())
    with mv.Problem(m, y, deltas=deltas, order=o, weighted=weighted) as P:
        th, u, rho, st = P.admm(lam, th0, u=np.zeros(P.E), rho=lam / 5, fixed_iters=iters, pcg_rtol=1e-13,
                                theta_solver=solver)
        E = P.E
        tm = None
    ref_th = th0.copy()
    ref_u = np.zeros(E)
    rs = c_oracle.admm_rcpp(m, y, lam, ref_th, ref_u, lam / 5, deltas, order=0 if order == "cpp" else 1,
                            weighted=1 if weighted else 0, fixed_iters=iters, pcg_rtol=1e-13)
    assert st["iters"] == iters and rho == rs["rho"]
    assert np.max(np.abs(th - ref_th)) <= 1e-9 * np.max(np.abs(ref_th))
    assert np.max(np.abs(u - ref_u)) <= 1e-9 * max(1.0, np.max(np.abs(ref_u)))
    del tm


def test_fused4d_kernel_is_the_one_timed():
    """At 4-D the loop's edge work runs in k_admm4a (timing id admm_fused4), not k_edge4d / k_gather4a; its twin
    blocks ({1,2} of S' {0,2}; {1,3}, {2,3} of {0,3}; {1,2,3} of {0,2,3}) are streamed once: 8 (5N + 2 (E - E_twins))."""
    m = [32, 32, 32, 8]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        P.state_set(np.full(y.size, y.mean()), None, 0.2)
        P.timing(True)
        P.run(1.0, fixed_iters=4)
        tm = P.timings()
        N, E = P.N, P.E
    assert tm["admm_fused4"]["launches"] == 4 and tm["edge_update"]["launches"] == 0
    assert tm["gather4_b"]["launches"] == 4 and tm["gather_Dt"]["launches"] == 1   # D^T u0 only
    sp, blen = _blocks(m)
    et = sum(blen[k] for k in range(len(sp)) if sp[k] in sp[:k])
    assert sum(1 for k in range(len(sp)) if sp[k] in sp[:k]) == 4
    assert tm["admm_fused4"]["bytes_per_launch"] == pytest.approx(8.0 * (5 * N + 2 * (E - et)), rel=1e-12)


def _sprime(b, p):
    S = [j for j in range(p) if (b >> (p - 1 - j)) & 1]
    if len(S) <= 1 or 0 in S:
        return tuple(S)
    return tuple(sorted(set(S) - {min(S)} | {0}))


def _blocks(m, order=0, drop_ones=False):
    """(S' per block, block lengths) in the reference's block order (cpp-code/utils.cpp:258-267; Python order
    code/utils.py:138-149, which drops the all-ones block when deltas are given)."""
    p = len(m)
    codes = [(1 << p) - 1] + list(range(1, (1 << p) - 1)) if order == 0 else list(range(1, 1 << p))
    if drop_ones:
        codes = [c for c in codes if c != (1 << p) - 1]
    sp = [_sprime(c, p) for c in codes]
    return sp, [int(np.prod([v - 1 if j in s else v for j, v in enumerate(m)])) for s in sp]


def _twin_blocks(m, order=0):
    """Block indices (canonical, twin) of the pair the S' map gives one difference set (cpp order: {1,2} -> {0,2})."""
    sp, _ = _blocks(m, order)
    for k in range(len(sp)):
        for j in range(k):
            if sp[k] == sp[j]:
                return j, k
    return None


@pytest.mark.parametrize("m", [[40, 40, 24], [12, 12, 12, 6]], ids=["3d", "4d"])
@pytest.mark.parametrize("twin_equal", [True, False], ids=["twin_skipped", "twin_differs"])
def test_twin_block_state_matches_oracle(twin_equal, m):
    """Blocks {0,2} and {1,2} of the reference's D share S' = {0,2} (4-D: three such groups) and, at equal deltas,
    their weight: with equal u they carry the same numbers, so k_admm3a / k_admm4a stream one block per group (and
    fill the others when the run ends). A caller's u whose twin blocks differ keeps them all. Both against the C
    oracle's variant-B loop: rho exactly, theta and u (every block, the twins included) to 1e-9."""
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    lam, iters = 1.0, 5
    th0 = np.full(y.size, y.mean())
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        E = P.E
        rng = np.random.default_rng(7)
        u0 = 0.05 * rng.standard_normal(E)
        _, blen = _blocks(m)
        assert sum(blen) == E
        off = np.concatenate([[0], np.cumsum(blen)])
        sp = _blocks(m)[0]
        twins = [(sp.index(sp[k]), k) for k in range(len(sp)) if sp[k] in sp[:k]]   # (first of the group, twin)
        assert twins and all(blen[c] == blen[k] for c, k in twins)
        for c, k in twins:
            if twin_equal:
                u0[off[k]:off[k + 1]] = u0[off[c]:off[c + 1]]
        th, u, rho, st = P.admm(lam, th0, u=u0.copy(), rho=lam / 5, fixed_iters=iters, pcg_rtol=1e-13)
    ref_th = th0.copy()
    ref_u = u0.copy()
    rs = c_oracle.admm_rcpp(m, y, lam, ref_th, ref_u, lam / 5, deltas, fixed_iters=iters, pcg_rtol=1e-13)
    assert rho == rs["rho"]
    assert np.max(np.abs(th - ref_th)) <= 1e-9 * np.max(np.abs(ref_th))
    assert np.max(np.abs(u - ref_u)) <= 1e-9 * max(1.0, np.max(np.abs(ref_u)))
    if twin_equal:
        for c, k in twins:
            assert np.array_equal(u[off[k]:off[k + 1]], u[off[c]:off[c + 1]])


def test_twin_block_bytes_counted_once():
    """With the twin block skipped, the fused launch's algorithmic bytes are 8 (4N + 2 (E - E_twin))."""
    m = [32, 32, 32]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        P.state_set(np.full(y.size, y.mean()), None, 0.2)
        P.timing(True)
        P.run(1.0, fixed_iters=3)
        tm = P.timings()
        N, E = P.N, P.E
    et = _blocks(m)[1][_twin_blocks(m)[1]]   # the twin block: S' = {0, 2}, 31 x 32 x 31 rows
    assert et == 31 * 32 * 31
    assert tm["admm_fused"]["launches"] == 3
    assert tm["admm_fused"]["bytes_per_launch"] == pytest.approx(8.0 * (4 * N + 2 * (E - et)), rel=1e-12)


def test_twin_block_python_order_matches_oracle():
    """Python block order with deltas (6 blocks at 3-D, the all-ones block dropped): the twin pair is codes 3 and 5;
    an explicit u with equal twins takes the twin kernel. Against the C oracle (order 1, weighted)."""
    m = [36, 36, 20]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    lam, iters = 1.0, 4
    th0 = np.full(y.size, y.mean())
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_PY, weighted=True) as P:
        E = P.E
        sp, blen = _blocks(m, order=1, drop_ones=True)
        assert sum(blen) == E and len(sp) == 6
        off = np.concatenate([[0], np.cumsum(blen)])
        rng = np.random.default_rng(11)
        u0 = 0.05 * rng.standard_normal(E)
        for k in range(len(sp)):
            if sp[k] in sp[:k]:
                c = sp.index(sp[k])
                u0[off[k]:off[k + 1]] = u0[off[c]:off[c + 1]]
        th, u, rho, st = P.admm(lam, th0, u=u0.copy(), rho=lam / 5, fixed_iters=iters, pcg_rtol=1e-13)
    ref_th = th0.copy()
    ref_u = u0.copy()
    rs = c_oracle.admm_rcpp(m, y, lam, ref_th, ref_u, lam / 5, deltas, order=1, weighted=1, fixed_iters=iters,
                            pcg_rtol=1e-13)
    assert rho == rs["rho"]
    assert np.max(np.abs(th - ref_th)) <= 1e-9 * np.max(np.abs(ref_th))
    assert np.max(np.abs(u - ref_u)) <= 1e-9 * max(1.0, np.max(np.abs(ref_u)))


def test_twin_state_carried_across_runs_matches_oracle():
    """Two resident runs in a row (the lambda path's warm start: theta, u and rho carried, rcpp…/solvers.cpp:212-220):
    the first run ends by filling the twin block from its partner, the second resumes from the stored z. Against the
    C oracle called twice on the carried state: rho exactly, theta and u to 1e-9."""
    m = [40, 40, 24]
    y = towers(m)
    deltas = [(1.0 + 2e-4) / v for v in m]
    th0 = np.full(y.size, y.mean())
    lams = (1.0, 0.6)
    with mv.Problem(m, y, deltas=deltas, order=mv.ORDER_CPP) as P:
        E = P.E
        P.state_set(th0, np.zeros(E), lams[0] / 5)
        for lam in lams:
            P.run(lam, fixed_iters=4, pcg_rtol=1e-13)
        th, u, rho = P.state_get()
    ref_th, ref_u, ref_rho = th0.copy(), np.zeros(E), lams[0] / 5
    for lam in lams:
        rs = c_oracle.admm_rcpp(m, y, lam, ref_th, ref_u, ref_rho, deltas, fixed_iters=4, pcg_rtol=1e-13)
        ref_rho = rs["rho"]
    assert rho == ref_rho
    assert np.max(np.abs(th - ref_th)) <= 1e-9 * np.max(np.abs(ref_th))
    assert np.max(np.abs(u - ref_u)) <= 1e-9 * max(1.0, np.max(np.abs(ref_u)))
