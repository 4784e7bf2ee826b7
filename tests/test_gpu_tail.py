"""The linear iteration's tail without the host (vamp.cpp; DESIGN.md §4.4
item 5): one reduction launch per vector length, gam1 formed by that
launch's last block, the EM round's mixture update (and the merging of close
variances) formed by the EM round's last block, and the next iteration's
prelude + CG start queued before the host's one wait, its scalars formed by
the denoiser's last block.  The host checks the device's mixture and scalars
against its own bit for bit every iteration (a difference fails the run);
here the runs with the queued-ahead start on and off must agree bit for bit,
also when the stop criterion fires (the start queued for the iteration that
never runs is discarded), and both must match the oracle
(src/vamp.cpp:110-438)."""
import numpy as np
import pytest

from conftest import relerr
from _data import make_problem

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)

N, MT = 1500, 3001
KEYS = ("iterations", "cg_iters", "ons_iters", "L")
ARRAYS = ("x1_hist", "r1_hist", "params", "metrics", "x1_final")


def _gpu(X, y, beta, **kw):
    with va.Data(N, MT) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        v = va.Vamp(d, va.VampOptions(**kw), true_signal=beta)
        x1 = v.infere(keep_hist=True)
        s = v.summary()
        n = s["iterations"]
        s["x1_hist"], s["r1_hist"], s["x1_final"] = v.x1_hist[:n, :d.M].copy(), v.r1_hist[:n, :d.M].copy(), x1
    return s


# (the oracle stops the first case at iteration 13 of 40; the mixture goes
# from 10 components to 6 by merges in the first five iterations)
@pytest.mark.parametrize("kw", [dict(max_iter=40, stop_criteria_thr=1e-2),
                                dict(max_iter=12, stop_criteria_thr=0.0),
                                dict(max_iter=12, stop_criteria_thr=0.0, learn_vars=0, merge_vars_thr=0.0)],
                         ids=["stop_fires", "fixed", "fixed_vars_no_merge"])
def test_queued_start_bitwise_and_oracle(monkeypatch, kw):
    X, y, beta = make_problem(N, MT)
    out = {}
    for on in (1, 0):
        monkeypatch.setenv("VAMPOMI_PRE_AHEAD", str(on))
        out[on] = _gpu(X, y, beta, **kw)
    for k in KEYS:
        assert out[1][k] == out[0][k], k
    for k in ARRAYS:
        np.testing.assert_array_equal(np.asarray(out[1][k]), np.asarray(out[0][k]), err_msg=k)
    ref = O.vamp_infere(X, y, MT, true_signal=beta, keep_hist=True, **kw)
    s = out[1]
    assert s["iterations"] == ref["iterations"]
    if kw["stop_criteria_thr"] > 0:
        assert s["iterations"] < kw["max_iter"]  # the stop fired with a start queued ahead
    assert s["cg_iters"] == ref["cg_iters"].tolist()
    assert s["ons_iters"] == ref["ons_iters"].tolist()
    assert s["L"] == ref["L"].tolist()
    for it in range(s["iterations"]):
        assert relerr(s["x1_hist"][it], ref["x1_hist"][it]) <= 1e-10, it
        assert relerr(s["r1_hist"][it], ref["r1_hist"][it]) <= 1e-10, it
