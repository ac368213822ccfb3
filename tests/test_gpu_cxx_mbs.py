"""The C++ host API's mbs_impl (include/mvtv/solvers.hpp, csrc/solvers.cpp; the released package's
mbs_impl, rcpp-code/MultivarTV/src/solvers.cpp:305-376) against the Python driver multivartv_amd.cv,
which is itself checked against the oracle (tests/test_gpu_cv.py). Both drive the same C ABI, so on a
given lambda grid they agree to rounding: the chosen index exactly, theta / fitted / MSEs to 1e-12
(mean(y), which starts every path, and the MSEs are sums: pairwise in numpy, sequential in the C++
host, as in Armadillo); with the lambda_max grid the grids agree to
rounding of the two linspace formulas and the results to 1e-7.

Runs multivartv_amd/lib/mvtv_mbs (built by `make -C multivartv_amd/csrc`) as a child process."""
import os
import subprocess

import numpy as np
import pytest

mv = pytest.importorskip("multivartv_amd")
from multivartv_amd import cv  # noqa: E402

pytestmark = pytest.mark.gpu
CLI = os.path.join(os.path.dirname(mv.__file__), "lib", "mvtv_mbs")


def _run_cli(tmp_path, x, y, m, n_lambda, folds, lambdas=None, seed=0):
    n, p = x.shape
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    hdr = np.array([n, p, n_lambda if lambdas is None else len(lambdas), folds, seed,
                    0 if lambdas is None else 1, 0], dtype=np.int64)
    parts = [hdr.tobytes(), np.asarray(m, dtype=np.float64).tobytes(),
             np.asfortranarray(x).tobytes(order="F"), y.astype(np.float64).tobytes()]
    if lambdas is not None:
        parts.append(np.asarray(lambdas, dtype=np.float64).tobytes())
    fin.write_bytes(b"".join(parts))
    r = subprocess.run([CLI, str(fin), str(fout)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    b = fout.read_bytes()
    nl, ind, N, nn = np.frombuffer(b[:32], dtype=np.int64)
    v = np.frombuffer(b[32:], dtype=np.float64)
    out, o = {}, 0
    for name, k in (("lambdas", nl), ("cv", nl), ("model_mses", nl), ("theta", N), ("fitted", nn), ("resid", nn)):
        out[name] = v[o:o + k]
        o += k
    out["ind"] = int(ind)
    return out


def _problem(n, p, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 1, size=(n, p))
    f = np.where(np.all(x > 0.55, axis=1), 1.0, 0.0)
    return x, f + 0.3 * rng.standard_normal(n)


@pytest.mark.parametrize("folds", [1, 3])
def test_cxx_mbs_impl_matches_python_on_given_grid(tmp_path, folds):
    x, y = _problem(500, 2, seed=folds)
    m = [12, 10]
    lambdas = np.exp(np.linspace(np.log(2.0), np.log(0.02), 5))
    got = _run_cli(tmp_path, x, y, m, 0, folds, lambdas=lambdas, seed=5)
    ref = cv.mbs_impl(x, y, m, lambdas=lambdas, folds=folds, seed=5)
    np.testing.assert_array_equal(got["lambdas"], lambdas)
    np.testing.assert_allclose(got["cv"], ref["cv.mses"], rtol=1e-12)
    assert got["ind"] == ref["lambda_minmse_ind"]
    np.testing.assert_allclose(got["theta"], ref["theta_hat"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(got["fitted"], ref["fitted"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(got["resid"], ref["residuals"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(got["model_mses"], [md["mse"] for md in ref["models"]], rtol=1e-12)


def test_cxx_mbs_impl_lambda_max_grid(tmp_path):
    x, y = _problem(400, 3, seed=9)
    m = [6, 6, 6]
    got = _run_cli(tmp_path, x, y, m, 6, 1)
    ref = cv.mbs_impl(x, y, m, n_lambda=6, folds=1)
    lam_ref = np.array([md["lambda"] for md in ref["models"]])
    np.testing.assert_allclose(got["lambdas"], lam_ref, rtol=1e-13)
    np.testing.assert_allclose(got["cv"], ref["cv.mses"], rtol=1e-7)
    assert got["ind"] == ref["lambda_minmse_ind"]
    np.testing.assert_allclose(got["theta"], ref["theta_hat"], rtol=1e-7, atol=1e-9)
