"""Host model of the factorised line solve (k_trir / k_trigr / k_trisr, mvtv_spectral.hip).

After the transforms along the other dimensions, every line of the last dimension carries c0 I + c1 T with T the
Neumann Laplacian tridiag(-1, [1, 2, ..., 2, 1], -1) — the operator the reference factorises with SuperLU every ADMM
iteration (rcpp-code/MultivarTV/src/solvers.cpp:113), restricted to one line. The kernels solve it as
x = (F + B - f) / D with two first-order recursions and the mirror closure, segment-parallel. This numpy model follows
the kernels' steps one for one (segments from zero carries, one scan per line over the segments' sums, the mirror
2 x 2 closure, the recursions rerun with their carries; the slab form: per-rank sums, the chunk owner's scan over the
ranks, phase 3) and checks them against a dense solve, including the ill-conditioned end (c1 / c0 = 1e7) and ragged
last segments / uneven rank blocks. No GPU."""
import numpy as np
import pytest


def _dense(c0, c1, f):
    m = len(f)
    T = np.diag(np.r_[1.0, 2.0 * np.ones(m - 2), 1.0]) - np.diag(np.ones(m - 1), 1) - np.diag(np.ones(m - 1), -1)
    return np.linalg.solve(c0 * np.eye(m) + c1 * T, f)


def _consts(c0, c1):
    D = np.sqrt(c0 * (c0 + 4.0 * c1))
    den = 1.0 / (c0 + 2.0 * c1 + D)
    return 2.0 * c1 * den, (c0 + D) * den, D   # r, 1 - r (cancellation-free), D


def _powt(r, t, n):
    """(r^n, 1 - r^n) by squaring, as powt_pow: 1 - r^(a+b) = t_a + r^a t_b."""
    y = (1.0, 0.0)
    x = (r, t)
    while n:
        if n & 1:
            y = (y[0] * x[0], y[1] + y[0] * x[1])
        x = (x[0] * x[0], x[1] + x[0] * x[1])
        n >>= 1
    return y


def _rerun(g, r, fin, bin_, D):
    """phase 3 of one segment: g <- B (backward with its carry), then x_i = (B_i + r F_{i-1}) / D."""
    g = g.copy()
    b = bin_
    for i in range(len(g) - 1, -1, -1):
        b = g[i] + r * b
        g[i] = b
    out = np.empty_like(g)
    fv = fin
    for i in range(len(g)):
        gn = g[i + 1] if i + 1 < len(g) else bin_
        out[i] = (g[i] + r * fv) / D
        fv = g[i] + r * (fv - gn)
    return out


def _local_sums(g, r):
    fl = bl = 0.0
    for v in g:
        fl = r * fl + v
    for v in g[::-1]:
        bl = r * bl + v
    return fl, bl


def line_solve(c0, c1, f, sl):
    """k_trir / k_trigr: segments of sl rows (the last one shorter when sl does not divide m)."""
    m = len(f)
    r, t, D = _consts(c0, c1)
    bounds = list(range(0, m, sl)) + [m]
    segs = [f[bounds[k]:bounds[k + 1]] for k in range(len(bounds) - 1)]
    sums = [_local_sums(s, r) for s in segs]
    rl = [_powt(r, t, len(s))[0] for s in segs]
    fin, acc = [], 0.0
    for k, (fl, _) in enumerate(sums):
        fin.append(acc)
        acc = acc * rl[k] + fl
    bin_, bcc = [0.0] * len(segs), 0.0
    for k in range(len(segs) - 1, -1, -1):
        bin_[k] = bcc
        bcc = bcc * rl[k] + sums[k][1]
    pm, tm = _powt(r, t, m)
    idet = 1.0 / (tm + pm * tm)   # 1 / (1 - r^2m)
    fm1, bm = (bcc + pm * acc) * idet, (acc + pm * bcc) * idet
    pf = pb = 1.0
    for k in range(len(segs)):
        kb = len(segs) - 1 - k
        fin[k] += pf * fm1
        bin_[kb] += pb * bm
        pf *= rl[k]
        pb *= rl[kb]
    return np.concatenate([_rerun(s, r, fin[k], bin_[k], D) for k, s in enumerate(segs)])


def slab_line_solve(c0, c1, f, G):
    """k_trisr phase 1 / k_trisr_iface / phase 3: rank k owns rows [floor(m k / G), floor(m (k + 1) / G))."""
    m = len(f)
    r, t, D = _consts(c0, c1)
    b = [(m * k) // G for k in range(G + 1)]
    blocks = [f[b[k]:b[k + 1]] for k in range(G)]
    co = [_local_sums(x, r) for x in blocks]           # phase 1: 2 numbers per line and rank
    rb = [_powt(r, t, len(x))[0] for x in blocks]
    lr_f, acc = [], 0.0                                 # the interface (chunk owner)
    for k in range(G):
        lr_f.append(acc)
        acc = acc * rb[k] + co[k][0]
    lr_b, bcc = [0.0] * G, 0.0
    for k in range(G - 1, -1, -1):
        lr_b[k] = bcc
        bcc = bcc * rb[k] + co[k][1]
    pm, tm = _powt(r, t, m)
    idet = 1.0 / (tm + pm * tm)
    fm1, bm = (bcc + pm * acc) * idet, (acc + pm * bcc) * idet
    pf = pb = 1.0
    for k in range(G):
        kb = G - 1 - k
        lr_f[k] += pf * fm1
        lr_b[kb] += pb * bm
        pf *= rb[k]
        pb *= rb[kb]
    return np.concatenate([_rerun(x, r, lr_f[k], lr_b[k], D) for k, x in enumerate(blocks)])


CASES = [(1.0, 0.0), (1.0, 1e-3), (1.0, 1.0), (3.7, 0.2), (1.0, 1e2), (1e-3, 5.0), (1.0, 1e4)]


@pytest.mark.parametrize("m,sl", [(512, 32), (512, 16), (128, 32), (64, 16), (500, 32), (37, 10), (101, 16), (1009, 16)])
@pytest.mark.parametrize("c0,c1", CASES)
def test_segmented_line_solve_matches_dense(m, sl, c0, c1):
    f = np.random.default_rng(m * 7 + sl).standard_normal(m) + 2.0
    x, ref = line_solve(c0, c1, f, sl), _dense(c0, c1, f)
    # the dense LU of the same matrix carries ~eps * cond; the recursions stay at ~eps / (1 - r)
    cond = (c0 + 4.0 * c1) / c0
    assert np.abs(x - ref).max() <= max(1e-13, 4e-16 * cond) * np.abs(ref).max()


@pytest.mark.parametrize("m,G", [(512, 8), (512, 2), (133, 2), (64, 3), (40, 4), (128, 8)])
@pytest.mark.parametrize("c0,c1", CASES)
def test_slab_line_solve_matches_single(m, G, c0, c1):
    f = np.random.default_rng(m + G).standard_normal(m)
    x1 = line_solve(c0, c1, f, 16 if m % 16 == 0 else 1)
    xs = slab_line_solve(c0, c1, f, G)
    assert np.abs(xs - x1).max() <= 1e-12 * max(1.0, np.abs(x1).max())


def test_extreme_coupling_beats_dense_against_long_double():
    """c1 / c0 = 1e7 (sigma far above the identity): the recursions against a long-double Thomas solve, where a
    double LU of the same matrix is off by ~1e-11."""
    m, c0, c1 = 512, 1.0, 1e7
    f = np.random.default_rng(3).standard_normal(m) + 5.0
    a = np.full(m, -np.longdouble(c1))
    bdiag = np.full(m, np.longdouble(c0) + 2 * np.longdouble(c1))
    bdiag[0] -= np.longdouble(c1)
    bdiag[-1] -= np.longdouble(c1)
    d = f.astype(np.longdouble)
    cp = np.zeros(m, dtype=np.longdouble)
    cp[0] = a[0] / bdiag[0]
    d[0] = d[0] / bdiag[0]
    for i in range(1, m):
        den = bdiag[i] - a[i] * cp[i - 1]
        cp[i] = a[i] / den
        d[i] = (d[i] - a[i] * d[i - 1]) / den
    ref = d.copy()
    for i in range(m - 2, -1, -1):
        ref[i] = d[i] - cp[i] * ref[i + 1]
    x = line_solve(c0, c1, f, 32)
    assert float(np.abs(x - ref).max() / np.abs(ref).max()) <= 1e-12
