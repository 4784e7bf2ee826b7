"""Degenerate shapes at the C ABI's lower bounds (N >= 2, Mt >= nranks):
one marker, two samples, one marker per rank.  Operators, marker statistics
and the one-pass CG operator's VAMP run against the oracle, as in
tests/test_gpu_parity.py (reductions to 1e-13 relative, integer counts
exact)."""
import numpy as np
import pytest

from conftest import relerr

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)


@pytest.mark.parametrize("N,Mt", [(2, 1), (3, 5), (17, 1), (5, 2), (2, 7)])
def test_operators_tiny(N, Mt):
    X = O.generate_markers(9, 0, N, 0, Mt)
    mave, msig = O.marker_stats(X)
    rng = np.random.default_rng(2)
    x, u = rng.normal(size=Mt), rng.normal(size=N)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        assert relerr(d.get_mave(), mave) < 1e-13
        assert relerr(d.get_msig(), msig) < 1e-13
        assert relerr(d.Ax(x), O.ax(X, mave, msig, x)) < 1e-13
        assert relerr(d.ATx(u), O.atx(X, mave, msig, u)) < 1e-13


@pytest.mark.parametrize("N,Mt", [(17, 1), (33, 3), (40, 2), (12000, 3)])  # 12000: a team plan, 61 empty teams
def test_vamp_tiny(N, Mt):
    X = O.generate_markers(4, 0, N, 0, Mt)
    beta = np.zeros(Mt)
    beta[0] = 0.7
    mave, msig = O.marker_stats(X)
    rng = np.random.default_rng(4)
    y = O.standardize_phen(((X - mave[:, None]) * msig[:, None]).T @ beta + rng.normal(0, 0.5, N))
    its = 5
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=0.0)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        v = va.Vamp(d, va.VampOptions(max_iter=its, stop_criteria_thr=0.0), true_signal=beta)
        v.infere(keep_hist=True)
        s = v.summary()
        x1h = v.x1_hist[: s["iterations"], : d.M]
    assert s["iterations"] == ref["iterations"]
    assert s["cg_iters"] == ref["cg_iters"].tolist()
    assert s["ons_iters"] == ref["ons_iters"].tolist()
    for k in range(s["iterations"]):
        assert relerr(x1h[k], ref["x1_hist"][k]) <= 1e-10, k
