"""CPU tests of the host-side logic around the hot path (no GPU)."""
import numpy as np
import pytest

from conftest import load_golden
from multivartv_amd import synth, utils
from oracle import mvtv_oracle as O


@pytest.mark.parametrize("name", ["py_1d_n1000_m1000_lam2", "py_1d_n1000_m250_lam2", "py_2d_mbs_one_nocache",
                                  "py_mesh_coords_3d"])
def test_mesh_and_nearest_match_reference(name):
    meta, g = load_golden(name)
    mesh = utils.mesh_coords(g["data"], meta["m"])["mesh"]
    np.testing.assert_array_equal(mesh, g["mesh"])            # incl. the p >= 3 'xy' ordering quirk
    np.testing.assert_array_equal(utils.nearest_index(g["data"], mesh), O.nearest_index(g["data"], mesh))


def test_nearest_random_and_nontensor():
    rng = np.random.default_rng(0)
    data = rng.uniform(-1, 2, size=(300, 3))
    mesh = utils.mesh_coords(rng.uniform(0, 1, size=(50, 3)), [4, 5, 6])["mesh"]
    np.testing.assert_array_equal(utils.nearest_index(data, mesh), O.nearest_index(data, mesh))
    scattered = rng.uniform(0, 1, size=(40, 2))                 # not a tensor grid: brute force path
    np.testing.assert_array_equal(utils.nearest_index(data[:, :2], scattered), O.nearest_index(data[:, :2], scattered))


def test_interp_weights():
    idx = np.array([0, 2, 2, 5])
    W, oty = utils.interp_weights(idx, 6, [1.0, 2.0, 3.0, 4.0])
    np.testing.assert_array_equal(W, [1, 0, 2, 0, 0, 1])
    np.testing.assert_array_equal(oty, [1, 0, 5, 0, 0, 4])


def test_synthetic_generator_is_counter_based():
    a = synth.towers([16, 8, 4])
    b = synth.towers([16, 8, 4], threads=1, chunk=7)
    np.testing.assert_array_equal(a, b)
    z = synth.normal_noise(100, 5)
    np.testing.assert_array_equal(z, synth.normal_noise(0, 105)[100:])
    big = synth.normal_noise(0, 200000)
    assert abs(big.mean()) < 0.01 and abs(big.std() - 1) < 0.01


def test_fastdiv_formula():
    """The invariant-divisor division used for node decoding (mvtv_internal.h FastDiv)."""
    rng = np.random.default_rng(1)
    for d in [1, 2, 3, 7, 64, 127, 128, 511, 512, 1000, 4095, 65537, 2**31 - 1]:
        shift = 0
        while (1 << shift) < d:
            shift += 1
        mul = ((1 << 32) * ((1 << shift) - d)) // d + 1 if d > 1 else 0
        if d == 1:
            shift = 0
        n = np.concatenate([rng.integers(0, 2**32, 20000, dtype=np.uint64), np.array([0, 1, d - 1, d, 2**32 - 1],
                                                                                    dtype=np.uint64)])
        hi = (n * np.uint64(mul)) >> np.uint64(32)
        q = (hi + n) >> np.uint64(shift)
        np.testing.assert_array_equal(q, n // np.uint64(d))


def test_slab_plane_bounds():
    from multivartv_amd import slab
    b = slab.plane_bounds(512, 8)
    assert b[0] == 0 and b[-1] == 512 and np.all(np.diff(b) == 64)
    b = slab.plane_bounds(10, 4)
    assert b[0] == 0 and b[-1] == 10 and np.all(np.diff(b) >= 2)
    with pytest.raises(ValueError):
        slab.plane_bounds(3, 4)


def test_slab_desc_layout_matches_header():
    import ctypes
    from multivartv_amd import slab
    assert ctypes.sizeof(slab.SlabDesc) == 32          # int64 x3 + int32 x2 (include/mvtv/mvtv.h)
    assert [f[0] for f in slab.SlabDesc._fields_] == ["m_global", "z_begin", "z_end", "ghost_lo", "ghost_hi"]


def test_create_D_and_lam_max_pinv_match_reference_fixtures():
    """utils.create_D is the Python reference's D (bit-identical to the oracle's, itself pinned to
    the reference) and utils.lam_max_pinv gives the reference's SuperLU value on the no-cache
    fixture (320.0, tests/golden/py_2d_mbs_one_nocache.npz)."""
    from multivartv_amd import utils as U
    from oracle import mvtv_oracle as O
    for m in ([8, 8], [3, 3, 3, 3], [4, 4, 4], [7]):
        for dl in (None, [0.1, 0.2, 0.3, 0.4][:len(m)]):
            if len(m) == 1 and dl is not None:
                with pytest.raises(ValueError):
                    U.create_D(m, dl)
                continue
            D1, D2 = U.create_D(m, dl), O.build_D(m, O.block_table(len(m), dl, "py"))
            assert D1.shape == D2.shape and (D1 != D2).nnz == 0
    with pytest.raises(ValueError):
        U.create_D([4, 5, 3])
    meta, g = load_golden("py_2d_mbs_one_nocache")
    mesh, deltas = U.mesh_coords(g["data"], meta["m"])["mesh"], U.mesh_coords(g["data"], meta["m"])["deltas"]
    idx = U.nearest_index(g["data"], mesh)
    _, oty = U.interp_weights(idx, 64, g["y"])
    assert U.lam_max_pinv(U.create_D(meta["m"], deltas), oty) == 320.0
