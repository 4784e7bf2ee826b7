"""CPU checks of the association-test restatement (--run-mode association_test,
src/main_meth.cpp:206-264, src/data.cpp:385-417, src/utilities.cpp:269-282).

The reference computes p-values with Boost.Math (students_t / normal
complemented CDFs), which is absent here: the oracle's t tail is pinned
against SciPy's published implementation (scipy.stats.t.sf, Cephes incbet),
as SURVEY §8(c) prescribes, and the statistic against an independent numpy
restatement."""
import math

import numpy as np
import pytest
from scipy import stats as S

from _data import make_problem
from oracle import pyoracle as O


@pytest.mark.parametrize("df", [1, 2, 3, 7, 30, 59, 60, 61, 200, 998, 9998, 49998, 99998, 199998])
def test_t_tail_matches_scipy(df):
    ts = np.concatenate([np.linspace(0, 8, 81), [10, 15, 20, 30, 40, 60, 100, 1e3]])
    for t in ts:
        ref = S.t.sf(t, df)
        got = O.t_sf(t, df)
        if ref < 1e-300:
            assert got < 1e-290
            continue
        assert abs(got - ref) <= 5e-12 * ref + 1e-300, (df, t, got, ref)
        assert abs(O.t_sf(-t, df) - S.t.sf(-t, df)) <= 5e-12 * ref + 4e-16  # = 1 - sf(t)


def test_t_tail_against_arbitrary_precision():
    mp = pytest.importorskip("mpmath")
    mp.mp.dps = 40
    for df in (59.0, 998.0, 99998.0):
        for t in (0.3, 2.0, 2.9, 3.1, 6.0, 17.0):
            x = mp.mpf(df) / (mp.mpf(df) + mp.mpf(t) ** 2)
            ref = mp.betainc(mp.mpf(df) / 2, mp.mpf(1) / 2, 0, x, regularized=True) / 2
            assert abs(O.t_sf(t, df) - float(ref)) <= 5e-12 * float(ref), (df, t)


def test_lnbeta_half_series_continuity():
    mp = pytest.importorskip("mpmath")
    mp.mp.dps = 40
    for a in (0.5, 3.0, 29.5, 30.0, 30.5, 100.0, 5e4, 1e6):
        ref = float(mp.log(mp.beta(mp.mpf(a), mp.mpf(1) / 2)))
        assert abs(O.load().orc_lnbeta_half(a) - ref) < 1.5e-14, a  # lgamma branch below a = 30


def test_reg1d_pval_is_the_simple_regression_t_test():
    rng = np.random.default_rng(5)
    for n, slope in ((50, 0.0), (500, 0.05), (5000, 0.3), (20000, 1.0)):
        x = rng.normal(size=n)
        y = slope * x + rng.normal(size=n)
        p = O.reg1d_pval(x.sum(), (x * x).sum(), (x * y).sum(), y.sum(), (y * y).sum(), n)
        ref = S.linregress(x, y).pvalue
        assert abs(p - ref) <= 1e-8 * ref + 1e-300, (n, p, ref)


def test_loo_matches_numpy_restatement():
    N, Mt = 800, 300
    X, y, beta = make_problem(N, Mt, kind=1)
    est = beta / np.sqrt(N) * 0.9  # an estimate file holds x1_hat / sqrt(N)
    p, st = O.assoc_loo(X, y, est)
    mave, msig = O.marker_stats(X)
    x1 = est * np.sqrt(N)
    z1 = O.ax(X, mave, msig, x1)
    ymod = y - z1
    for j in range(0, Mt, 7):
        ym = ymod + X[j] / np.sqrt(N) * x1[j]
        ref = S.linregress(X[j], ym)
        assert np.allclose(st[j], [X[j].sum(), (X[j] ** 2).sum(), X[j] @ ym, ym.sum(), ym @ ym], rtol=1e-12)
        assert abs(p[j] - ref.pvalue) <= 1e-7 * ref.pvalue + 1e-300
    # causal markers are detected
    causal = beta != 0
    assert np.median(p[causal]) < 0.05 < np.median(p[~causal])


def test_se_matches_scipy_normal():
    rng = np.random.default_rng(1)
    r1 = np.concatenate([rng.normal(size=200) * 0.05, [0.0, -0.0, 1e-3, -1e-3]])
    gam1, N = 3.7, 1000
    p = O.assoc_se(r1, gam1, N)
    sd = math.sqrt(1.0 / (gam1 * N))
    ref = S.norm.cdf(0, loc=r1, scale=sd)
    ref = np.where(r1 <= 0, 1 - ref, ref)
    assert np.allclose(p, ref, rtol=1e-13, atol=1e-16)
