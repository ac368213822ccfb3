"""The research code's C++ API (variant A, cpp-code/solvers.hpp:85-129) through include/mvtv/solvers.hpp:
``mvtv::mbs`` (cpp-code/solvers.cpp:277-310) and ``mvtv::mbs_one`` without cache (:134-152), run by
multivartv_amd/lib/mvtv_mbs --cpp / --cpp-one against fixtures from the oracle's restatement
(tests/golden/gen_golden_cpp_mbs.py).

* reference CV (cache on the full data, fold 0's path for every fold's test MSE, refit on the last
  path's matrix) and the corrected CV, each on a given lambda grid: the MSE matrix to 1e-7, the chosen
  row exactly, the refit's theta / fitted to 5e-7 of max|theta|: the W != I theta-solve is PCG to the
  default rtol 1e-10 against the fixture's SuperLU, whose forward error is up to cond(A) * 1e-10 (Jacobi-PCG
  lands 1.00e-7, the spectrally preconditioned PCG 1.0007e-7 of max|theta| from SuperLU on cpp_mbs_2d_refcv);
* the automatic grid: lambda_max from the reference's CG (cpp-code/utils.cpp:354-404), which runs on the
  singular D^T D with an inconsistent right-hand side and moves by ~1e-3 relative under 1e-15 changes of
  O^T y, so it is checked to 1e-2 and the grid against its own formula;
* mbs_one without cache: unit block weights and crossO + lambda crossD, theta to 1e-7.
"""
import os
import subprocess

import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")
from conftest import load_golden  # noqa: E402

pytestmark = pytest.mark.gpu
CLI = os.path.join(os.path.dirname(mv.__file__), "lib", "mvtv_mbs")


def _run(tmp_path, mode, x, y, m, n_lambda, folds, lambdas=None, seed=0, fixed_cv=False):
    n, p = x.shape
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    hdr = np.array([n, p, n_lambda if lambdas is None else len(lambdas), folds, seed,
                    0 if lambdas is None else 1, int(fixed_cv)], dtype=np.int64)
    parts = [hdr.tobytes(), np.asarray(m, dtype=np.float64).tobytes(), np.asfortranarray(x).tobytes(order="F"),
             np.asarray(y, dtype=np.float64).tobytes()]
    if lambdas is not None:
        parts.append(np.asarray(lambdas, dtype=np.float64).tobytes())
    fin.write_bytes(b"".join(parts))
    r = subprocess.run([CLI, mode, str(fin), str(fout)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return fout.read_bytes()


def _mbs(tmp_path, g, meta, lambdas=None, n_lambda=0, fixed_cv=False):
    b = _run(tmp_path, "--cpp", g["data"], g["y"], meta["m"], n_lambda, meta["folds"], lambdas=lambdas,
             seed=meta["seed"], fixed_cv=fixed_cv)
    nl, best, N, n = np.frombuffer(b[:32], dtype=np.int64)
    v = np.frombuffer(b[32:], dtype=np.float64)
    out = {"best": int(best), "lambda_max": v[0], "lambdas": v[1:1 + nl]}
    o = 1 + nl
    out["mse_mat"] = v[o:o + nl * meta["folds"]].reshape(meta["folds"], nl).T
    o += nl * meta["folds"]
    out["theta"], out["fitted"] = v[o:o + N], v[o + N:o + N + n]
    return out


@pytest.mark.parametrize("name", ["cpp_mbs_2d_refcv", "cpp_mbs_2d_fixedcv"])
def test_cxx_mbs_variant_a_on_given_grid(tmp_path, name):
    meta, g = load_golden(name)
    got = _mbs(tmp_path, g, meta, lambdas=g["lambdas"], fixed_cv=not meta["reference_cv"])
    np.testing.assert_array_equal(got["lambdas"], g["lambdas"])
    np.testing.assert_allclose(got["mse_mat"], g["mse_mat"], rtol=1e-7)
    assert got["best"] == meta["best"]
    tol = 5e-7 * np.max(np.abs(g["theta"]))
    assert np.max(np.abs(got["theta"] - g["theta"])) <= tol
    assert np.max(np.abs(got["fitted"] - g["fitted"])) <= tol


def test_cxx_mbs_variant_a_lambda_max(tmp_path):
    meta, g = load_golden("cpp_mbs_2d_refcv")
    got = _mbs(tmp_path, g, meta, n_lambda=meta["n_lambda"])
    assert got["lambda_max"] == pytest.approx(meta["lambda_max"], rel=1e-2)
    lm = got["lambda_max"]
    grid = np.exp(np.linspace(np.log(lm * 1e-5), np.log(lm), meta["n_lambda"]))[::-1]
    np.testing.assert_allclose(got["lambdas"], grid, rtol=1e-13)


def test_cxx_mbs_one_variant_a_without_cache(tmp_path):
    meta, g = load_golden("cpp_mbs_one_nocache_3d")
    b = _run(tmp_path, "--cpp-one", g["data"], g["y"], meta["m"], 0, 0, lambdas=[meta["lam"]])
    N, n = np.frombuffer(b[:16], dtype=np.int64)
    v = np.frombuffer(b[16:], dtype=np.float64)
    tol = 1e-7 * np.max(np.abs(g["theta"]))
    assert np.max(np.abs(v[:N] - g["theta"])) <= tol
    assert np.max(np.abs(v[N:N + n] - g["fitted"])) <= tol
