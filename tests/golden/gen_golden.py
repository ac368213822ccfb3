"""Generate the golden fixtures in tests/golden/*.npz from the reference itself.

Run here (build container) only: ``python tests/golden/gen_golden.py``. It
imports the reference's Python prototype through ``refload`` (see its header)
and writes small .npz fixtures holding inputs and expected outputs. The
fixtures travel with the repo; the reference never does.

Sources of truth, per fixture family:
  * ``dmat_*``  D matrices built by the reference's own ``code/utils.py``
    (``create_D`` for the Python orders; ``fd_binaries`` + ``binary2diffmat``
    stacked in the C++ order of cpp-code/utils.cpp:245-269).
  * ``py_*``    outputs of the reference's ``code/solvers.py`` (``mbs_one`` cache
    and no-cache paths, ``mbs`` path) — variant C end to end.
  * ``rcpp_*`` / ``cpp_*``  the C++ loops (rcpp…/solvers.cpp:96-136 and
    cpp-code/solvers.cpp:90-130) cannot be compiled here (no Armadillo /
    SuperLU / R); they are restated line by line below, driven by
    the reference-built D and SciPy's SuperLU (the library the R package links).
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import splu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from refload import load_reference  # noqa: E402
from multivartv_amd.synth import towers, towers_scattered  # noqa: E402

ref_utils, ref_solvers = load_reference()


def save(name, meta, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, meta=np.array(json.dumps(meta)), **arrays)
    print(f"wrote {name}.npz  ({os.path.getsize(path)} B)")


def coo(M):
    M = sp.coo_matrix(M)
    order = np.lexsort((M.col, M.row))
    return M.row[order].astype(np.int64), M.col[order].astype(np.int64), M.data[order]


# --------------------------------------------------------------------------- D
def ref_D_cpp(m, deltas, unit=False):
    """C++ create_D order built from the reference's own Python block builder."""
    p = len(m)
    bins = ref_utils.fd_binaries(p)
    blocks = [ref_utils.binary2diffmat(np.array(m), bins[-1])]
    for i in range(bins.shape[0] - 1):
        w = 1.0 if unit else float(np.prod(np.asarray(deltas, dtype=float) ** (1 - bins[i])))
        blocks.append(ref_utils.binary2diffmat(np.array(m), bins[i]) * w)
    return sp.vstack(blocks).tocsr()


def gen_dmats():
    cases = [
        ([7], [0.3]), ([4, 5], [0.3, 0.7]), ([5, 5], [0.2, 0.2]), ([4, 4, 4], [0.5, 0.25, 0.125]),
        ([4, 4, 5], [0.5, 0.25, 0.125]), ([3, 3, 3, 3], [0.5, 0.25, 0.125, 0.3]),
        ([3, 3, 3, 4], [0.5, 0.25, 0.125, 0.3]),
    ]
    for m, dl in cases:
        tag = "x".join(map(str, m))
        arrays = {}
        D = ref_utils.create_D(dims=np.array(m), deltas=None)
        arrays["py_none_r"], arrays["py_none_c"], arrays["py_none_v"] = coo(D)
        arrays["py_none_shape"] = np.array(D.shape)
        if len(m) > 1:
            D = ref_utils.create_D(dims=np.array(m), deltas=dl)
            arrays["py_w_r"], arrays["py_w_c"], arrays["py_w_v"] = coo(D)
            arrays["py_w_shape"] = np.array(D.shape)
        for key, unit in (("cpp", False), ("cppunit", True)):
            D = ref_D_cpp(m, dl, unit)
            arrays[key + "_r"], arrays[key + "_c"], arrays[key + "_v"] = coo(D)
            arrays[key + "_shape"] = np.array(D.shape)
        save(f"dmat_{tag}", dict(m=m, deltas=dl), **arrays)
    # unequal meshes the reference rejects (mixed-partial quirk)
    bad = []
    for m in ([4, 3, 5], [4, 5, 4], [5, 3, 5], [3, 3, 4, 3], [3, 4, 3, 3]):
        try:
            ref_utils.create_D(dims=np.array(m), deltas=None)
            bad.append((m, False))
        except ValueError:
            bad.append((m, True))
    save("dmat_mismatch", dict(cases=[dict(m=m, raises=r) for m, r in bad]))


# ------------------------------------------------------------ restated C++ loops
def soft(z, lam):
    return np.sign(z) * np.maximum(np.abs(z) - lam, 0.0)


def rcpp_admm_update(D, Oty, W, lam, theta, u, rho, fixed=None, snaps=(1, 5, 20)):
    """rcpp-code/MultivarTV/src/solvers.cpp:96-136, line by line (TOL = 1e-4, solvers.hpp:19)."""
    TOL = 1e-4
    Dt = D.T.tocsr()
    crossD = Dt @ D
    crossO = sp.diags(W)
    ntheta, rowsD = D.shape[1], D.shape[0]
    alpha = D @ theta
    counter, max_counter = 1, 3000
    spcrosses = (crossO + rho * crossD).tocsc()
    dual_norm = primal_norm = 1.0
    eps_dual = eps_primal = TOL
    hist, snap = [], {}
    while (dual_norm > eps_dual or primal_norm > eps_primal) if fixed is None else (counter - 1 < fixed):
        uold = u.copy()
        b = Oty + rho * (Dt @ (alpha + u))
        theta = splu(spcrosses).solve(b)
        alpha = soft(D @ theta - u, lam / rho)
        primal = alpha - D @ theta
        u = u + primal
        dual = rho * (Dt @ (u - uold))
        dual_norm = np.linalg.norm(dual)
        primal_norm = np.linalg.norm(primal)
        eps_dual = TOL * (math.sqrt(ntheta) + np.linalg.norm(Dt @ u))
        eps_primal = TOL * (math.sqrt(rowsD) + max(np.linalg.norm(D @ theta), np.linalg.norm(alpha)))
        hist.append([primal_norm, dual_norm, eps_primal, eps_dual, rho])
        r_n, s_n = np.linalg.norm(primal), np.linalg.norm(dual)
        if r_n > 10 * s_n:
            rho, u = 2.0 * rho, (1.0 / 2.0) * u
        elif s_n > 10 * r_n:
            rho, u = (1.0 / 2.0) * rho, 2.0 * u
        spcrosses = (crossO + rho * crossD).tocsc()
        counter += 1
        if counter - 1 in snaps:
            snap[counter - 1] = theta.copy()
        if counter > max_counter:
            break
    return theta, u, rho, counter - 1, np.array(hist), snap


def cpp_admm_update(D, Oty, W, lam, theta, ymean, fixed=None, snaps=(1, 5)):
    """cpp-code/solvers.cpp:90-130, line by line (TOL = 1e-3, solvers.hpp:14); matrix fixed
    at crossO + lambda*crossD by the caller (:144 / :209)."""
    TOL = 1e-3
    Dt = D.T.tocsr()
    lu = splu((sp.diags(W) + lam * (Dt @ D)).tocsc())
    alpha = D @ theta
    u = np.full(D.shape[0], 1.0 / lam)
    thetaold = np.full_like(theta, ymean - 0.1)
    counter, max_counter = 1, 2000
    rho = int(lam)
    hist, snap = [], {}
    while np.any(np.abs(theta - thetaold) > TOL) if fixed is None else (counter - 1 < fixed):
        thetaold = theta
        b = Oty + rho * (Dt @ (alpha + u))
        theta = lu.solve(b)
        with np.errstate(divide="ignore"):
            thr = lam / float(rho) if rho != 0 else np.inf
        alpha = soft(D @ theta - u, thr)
        dual = rho * (Dt @ (alpha + u))
        primal = alpha - D @ theta
        u = u + primal
        counter += 1
        if counter > max_counter:
            raise RuntimeError("Failed to converge!")
        r_n, s_n = math.sqrt(primal @ primal), math.sqrt(dual @ dual)
        hist.append([r_n, s_n, float(rho)])
        if r_n > 20 * s_n:
            rho_next, u = 20 * rho, 0.05 * u
        elif s_n > 20 * r_n:
            rho_next, u = 0.1 * rho, 10 * u
        else:
            rho_next = rho
        rho = int(rho_next)
        if counter - 1 in snaps:
            snap[counter - 1] = theta.copy()
    return theta, u, rho, counter - 1, np.array(hist), snap


def deltas_b(m):
    """rcpp create_deltas on lattice data in [0,1]: (1 + 2e-4) / m_j."""
    return [(1.0 + 2e-4) / mj for mj in m]


def gen_rcpp():
    specs = [
        ("rcpp_1d_200", [200], 0.5, None),
        ("rcpp_2d_32", [32, 32], 0.5, None),
        ("rcpp_2d_24x40", [24, 40], 1.0, None),
        ("rcpp_3d_12", [12, 12, 12], 1.0, None),
        ("rcpp_3d_8x8x11", [8, 8, 11], 1.0, None),
        ("rcpp_4d_5", [5, 5, 5, 5], 1.0, None),
        ("rcpp_2d_scat", [20, 20], 0.3, 1500),
    ]
    for name, m, lam, nscat in specs:
        N = int(np.prod(m))
        if nscat is None:
            y = towers(m)
            Oty, W = y.copy(), np.ones(N)
            deltas = deltas_b(m)
        else:
            data, yd, _ = towers_scattered(nscat, len(m))
            # lattice mesh min-EPS..max+EPS (rcpp…/utils.cpp:234-254) and nearest point (:267-304)
            lo, hi = data.min(0) - 1e-4, data.max(0) + 1e-4
            axes = [np.linspace(lo[j], hi[j], m[j]) for j in range(len(m))]
            idx = np.zeros(nscat, dtype=np.int64)
            stride = 1
            for j in range(len(m)):
                idx += np.abs(data[:, j:j + 1] - axes[j][None, :]).argmin(1) * stride
                stride *= m[j]
            W = np.bincount(idx, minlength=N).astype(float)
            Oty = np.bincount(idx, weights=yd, minlength=N)
            y = yd
            deltas = [(data[:, j].max() - data[:, j].min() + 2e-4) / m[j] for j in range(len(m))]
        D = ref_D_cpp(m, deltas)
        theta0 = np.full(N, y.mean())
        u0 = np.zeros(D.shape[0])
        rho0 = lam / 5.0
        th, u, rho, it, hist, snap = rcpp_admm_update(D, Oty, W, lam, theta0.copy(), u0.copy(), rho0)
        thf, uf, rhof, itf, histf, snapf = rcpp_admm_update(D, Oty, W, lam, theta0.copy(), u0.copy(), rho0,
                                                            fixed=20)
        save(name, dict(m=m, lam=lam, rho0=rho0, deltas=deltas, iters=it, rho=rho, variant="rcpp",
                        E=int(D.shape[0])),
             Oty=Oty, W=W, theta0=theta0, theta=th, u=u, hist=hist,
             fixed_theta=thf, fixed_u=uf, fixed_rho=np.array(rhof), fixed_hist=histf,
             snap1=snapf[1], snap5=snapf[5], snap20=snapf[20])
    # warm-started lambda path (rcpp…/solvers.cpp:204-222): theta, u, rho carried over
    m = [16, 16]
    y = towers(m)
    D = ref_D_cpp(m, deltas_b(m))
    lams = [2.0, 1.0, 0.5]
    theta, u, rho = np.full(256, y.mean()), np.zeros(D.shape[0]), lams[0] / 5.0
    outs = {}
    for k, lam in enumerate(lams):
        theta, u, rho, it, _, _ = rcpp_admm_update(D, y, np.ones(256), lam, theta, u, rho)
        outs[f"theta{k}"], outs[f"u{k}"] = theta, u
        outs[f"rho{k}"], outs[f"iters{k}"] = np.array(rho), np.array(it)
    save("rcpp_path_2d_16", dict(m=m, lams=lams, deltas=deltas_b(m)), y=y, **outs)


def gen_cpp():
    for name, m, lam, unit in [("cpp_2d_16", [16, 16], 3.0, False), ("cpp_3d_8_unit", [8, 8, 8], 2.0, True),
                               ("cpp_2d_12_frac", [12, 12], 0.5, False)]:
        N = int(np.prod(m))
        y = towers(m)
        deltas = [(1.0 + 0.02) / mj for mj in m]  # cpp create_deltas EPS = 0.01
        D = ref_D_cpp(m, deltas, unit)
        theta0 = np.full(N, y.mean())
        th, u, rho, it, hist, snap = cpp_admm_update(D, y, np.ones(N), lam, theta0.copy(), y.mean())
        save(name, dict(m=m, lam=lam, deltas=deltas, unit=unit, iters=it, rho=rho, variant="cpp",
                        ymean=float(y.mean())),
             y=y, theta0=theta0, theta=th, u=u, hist=hist, **{f"snap{k}": v for k, v in snap.items()})


# ------------------------------------------------------------ reference Python
def gen_py():
    # config 1: 1D n = 1000 through the reference mbs_one cache path (code/solvers.py:42-51)
    n = 1000
    data = (np.arange(n, dtype=float) / (n - 1)).reshape(n, 1)
    from multivartv_amd.synth import normal_noise
    x = data[:, 0]
    f = np.where(x > 0.8, 1.0, np.where(x < 0.2, 0.5, 0.0))
    y = f + 0.5 * normal_noise(0, n)
    for m, lam in ((1000, 2.0), (250, 2.0), (1000, 0.5)):
        meshob = ref_utils.mesh_coords(data, mesh_dims=np.array([m]))
        mesh = meshob["mesh"]
        O = ref_utils.nearest_interp_matrix(data, mesh)
        Ot = O.transpose()
        D = ref_utils.create_D(dims=np.array([m]), deltas=None)
        Dt = D.transpose()
        cache2 = Ot.dot(y.reshape(n, 1))
        cache1 = splu((Ot.dot(O) + lam * Dt.dot(D)).tocsc())
        out = ref_solvers.mbs_one(data, y, np.array([m]), mesh=mesh, tune=lam,
                                  cache=[cache1, cache2, D, Dt, D.shape[0], O, Ot, mesh, m])
        save(f"py_1d_n{n}_m{m}_lam{lam:g}", dict(n=n, m=[m], lam=lam, variant="py"),
             data=data, y=y, mesh=mesh, theta=np.asarray(out["theta.hat"]).ravel(),
             fitted=np.asarray(out["fitted"]).ravel(), W=np.asarray(Ot.dot(O).diagonal()).ravel(),
             Oty=np.asarray(cache2).ravel())
    # 2D no-cache mbs_one (tune := lam_max_pinv, code/solvers.py:23-40) and the mbs path (:91-141)
    n, p = 600, 2
    data, y, ftrue = towers_scattered(n, p)
    m = np.array([8, 8])
    out = ref_solvers.mbs_one(data, y, m)
    meshob = ref_utils.mesh_coords(data, mesh_dims=m)
    save("py_2d_mbs_one_nocache", dict(n=n, m=m.tolist(), variant="py"),
         data=data, y=y, mesh=meshob["mesh"], deltas=np.array(meshob["deltas"]),
         theta=np.asarray(out["theta.hat"]).ravel(), fitted=np.asarray(out["fitted"]).ravel())
    outp = ref_solvers.mbs(data, y, m, ftrue=ftrue, ntune=4)
    fits = outp["minmse.fits"]
    save("py_2d_mbs_path", dict(n=n, m=m.tolist(), ntune=4, variant="py"),
         data=data, y=y, ftrue=ftrue, theta=np.asarray(fits["theta.hat"]).ravel(),
         minmse=np.array(outp["minmse"]), minlam=np.array(outp["minmse.lam"]))
    # mesh_coords ordering quirk for p = 3 (meshgrid 'xy', code/utils.py:188)
    data3, _, _ = towers_scattered(50, 3)
    mo = ref_utils.mesh_coords(data3, mesh_dims=np.array([3, 4, 5]))
    save("py_mesh_coords_3d", dict(m=[3, 4, 5]), data=data3, mesh=mo["mesh"], deltas=np.array(mo["deltas"]))
    # reference unit tests' own pins (code/test_utils.py)
    save("py_unit_pins", dict(
        t2v_222=int(ref_utils.t2v_unit(dims=np.array([3, 3, 3]), ind=np.array([2, 2, 2]))),
        v2t_26=[int(v) for v in ref_utils.v2t_unit(dims=np.array([3, 3, 3]), ind=26)],
        nearest=[int(v) for v in ref_utils.nearest1(np.array([0.1, 0.9]), np.array([[0], [0.5], [1.0]]))],
        mesh_delta=float(np.round(ref_utils.mesh_coords(np.linspace(0.01, 0.99, 10).reshape(10, 1),
                                                        mesh_dims=np.array([6]))["deltas"][0], 2))))


if __name__ == "__main__":
    gen_dmats()
    gen_rcpp()
    gen_cpp()
    gen_py()
