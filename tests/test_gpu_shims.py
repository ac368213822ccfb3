"""GPU: the reference-shaped host APIs (Python code/solvers.py mirror, C++ solvers.hpp mirror)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden

mv = pytest.importorskip("multivartv_amd")
from multivartv_amd import solvers, utils  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["py_1d_n1000_m1000_lam2", "py_1d_n1000_m250_lam2"])
def test_config1_through_mbs_one_cache_path(name):
    """BASELINE config 1 via the reference's own API shape (code/solvers.py:mbs_one, cache path)."""
    meta, g = load_golden(name)
    m = np.array(meta["m"])
    cache = solvers.make_cache(g["data"], g["y"], m, sigma=meta["lam"], weighted=False)  # create_D(m, None)
    np.testing.assert_array_equal(cache.mesh, g["mesh"])
    out = solvers.mbs_one(g["data"], g["y"], m, tune=meta["lam"], cache=cache)
    assert set(out) == {"mesh", "theta.hat", "fitted", "data", "y", "eps", "m", "counter"}
    ref = g["theta"]
    assert np.max(np.abs(out["theta.hat"].ravel() - ref)) <= 1e-9 * np.max(np.abs(ref))
    assert np.max(np.abs(out["fitted"].ravel() - g["fitted"])) <= 1e-9 * np.max(np.abs(ref))
    cache.problem.close()


def test_reference_test_mbs_one():
    """code/test_solvers.py:24-29 on the same inputs: at lambda_max, mean(theta) = mean(fitted) = mean(y)."""
    rng = np.random.RandomState(117)
    n = 10000
    x1 = rng.uniform(-1, 1, n)
    x2 = rng.uniform(-1, 1, n)
    data = np.concatenate((x1.reshape((n, 1)), x2.reshape((n, 1))), 1)
    z = 2 * np.maximum(0, x1 + x2)
    ytrue = np.exp(z) - (z + z ** 2 / 2 + z ** 3 / 6)
    y = ytrue + rng.normal(0, 1, n)
    out = solvers.mbs_one(data, y, np.array([10, 10]))
    a = np.round(np.mean(out["theta.hat"]), 3)
    b = np.round(np.mean(out["fitted"]), 3)
    c = np.round(np.mean(y), 3)
    assert a == b == c


def test_mbs_path_with_reference_tuners():
    """code/solvers.py:mbs with the reference's own lambda grid (the auto grid is a SuperLU artefact)."""
    meta, g = load_golden("py_2d_mbs_path")
    from oracle import mvtv_oracle as O
    _, _, tuners, _ = O.mbs_path_py(g["data"], g["y"], meta["m"], ftrue=g["ftrue"], ntune=meta["ntune"])
    out = solvers.mbs(g["data"], g["y"], np.array(meta["m"]), ftrue=g["ftrue"], tuners=tuners)
    assert out["minmse.lam"] == pytest.approx(float(g["minlam"]), rel=1e-12)
    assert out["minmse"] == pytest.approx(float(g["minmse"]), rel=1e-9)
    np.testing.assert_allclose(out["minmse.fits"]["theta.hat"].ravel(), g["theta"], rtol=1e-9, atol=1e-10)


def test_mbs_one_nocache_reference_lambda_max():
    """code/solvers.py:23-40 without a cache: tune := lam_max_pinv (SuperLU on the singular D^T D),
    reproduced by utils.lam_max_pinv; theta against the reference's own output."""
    meta, g = load_golden("py_2d_mbs_one_nocache")
    out = solvers.mbs_one(g["data"], g["y"], np.array(meta["m"]))
    np.testing.assert_allclose(out["theta.hat"].ravel(), g["theta"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(out["fitted"].ravel(), g["fitted"], rtol=1e-9, atol=1e-12)


def test_mbs_path_auto_grid():
    """code/solvers.py:mbs with ntune only: the lambda grid from lam_max_pinv * prod(deltas) (:115-117)."""
    meta, g = load_golden("py_2d_mbs_path")
    out = solvers.mbs(g["data"], g["y"], np.array(meta["m"]), ftrue=g["ftrue"], ntune=meta["ntune"])
    assert out["minmse.lam"] == pytest.approx(float(g["minlam"]), rel=1e-12)
    assert out["minmse"] == pytest.approx(float(g["minmse"]), rel=1e-9)
    np.testing.assert_allclose(out["minmse.fits"]["theta.hat"].ravel(), g["theta"], rtol=1e-9, atol=1e-10)


def test_cpp_host_api(tmp_path):
    """include/mvtv/solvers.hpp: create_cache_objects + mbs_path (warm start) on a 2D scattered fit."""
    exe = tmp_path / "cpp_api"
    src = os.path.join(ROOT, "tests", "cpp", "cpp_api_main.cpp")
    lib = os.path.join(ROOT, "multivartv_amd", "lib")
    subprocess.check_call(["g++", "-std=c++17", "-O2", src, "-I", os.path.join(ROOT, "include"), "-L", lib, "-lmvtv",
                           f"-Wl,-rpath,{lib}", "-o", str(exe)])
    out = subprocess.check_output([str(exe)], timeout=300).decode().split()
    vals = dict(zip(out[::2], map(float, out[1::2])))
    assert vals["n_models"] == 3
    assert vals["best"] >= 0 and vals["minmse"] > 0
    assert vals["fitted_ok"] == 1
