"""GPU parity across the option space of main_meth (src/options.hpp:62-104):
mixture shape, EM iterations and tolerance, learn_vars, learn_prior_delay,
damping rho, merge threshold, gam1 / h2 starts, CG tolerance and cap,
alpha_scale, a warm start from an estimate file — linear and probit, each
against the CPU oracle with the same bars as the default runs."""
import numpy as np
import pytest

from conftest import relerr
import os

from _data import PROBIT_K, make_problem, oracle_with_spread, record_probit_ratio

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)

N, MT = 600, 1100

CASES = {
    "one_slab": dict(vars=(0.0, 1e-3), probs=(0.9, 0.1)),
    "three_slabs": dict(vars=(0.0, 1e-5, 1e-3, 1e-1), probs=(0.97, 0.02, 0.008, 0.002)),
    "em3_tight": dict(EM_max_iter=3, EM_err_thr=1e-4),
    "fixed_vars": dict(learn_vars=0),
    "late_prior": dict(learn_prior_delay=4),
    "no_damping": dict(rho=1.0),
    "strong_damping": dict(rho=0.2),
    "no_merge": dict(merge_vars_thr=0.0),
    "gam1_h2": dict(gam1=1e-3, h2=0.3),
    "cg_loose": dict(CG_err_tol=1e-3, CG_max_iter=4),
    "cg_tight": dict(CG_err_tol=1e-9),
}


def _gpu(X, y, beta, model, alpha_scale=1.0, x1hat_init=None, **kw):
    with va.Data(N, MT, alpha_scale=alpha_scale) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        v = va.Vamp(d, va.VampOptions(model=model, **kw), true_signal=beta, x1hat_init=x1hat_init)
        v.infere(keep_hist=True)
        s = v.summary()
        n = s["iterations"]
        s["x1_hist"], s["r1_hist"] = v.x1_hist[:n, :d.M].copy(), v.r1_hist[:n, :d.M].copy()
    return s


def _check(s, ref, spread=None):
    assert s["iterations"] == ref["iterations"]
    assert s["cg_iters"] == ref["cg_iters"].tolist()
    assert s["ons_iters"] == ref["ons_iters"].tolist()
    assert s["L"] == ref["L"].tolist()
    its = s["iterations"]
    gaps = {key: np.array([relerr(s[f"{key}_hist"][k], ref[f"{key}_hist"][k]) for k in range(its)])
            for key in ("x1", "r1")}
    if spread is not None:  # probit: the bar is PROBIT_K x the oracle's rank-count spread
        test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
        for key in ("x1", "r1"):
            record_probit_ratio(test, key, gaps[key], spread[key][:its])
    for k in range(its):
        for key in ("x1", "r1"):
            bar = 1e-10 if spread is None else max(1e-10, PROBIT_K * spread[key][k])
            assert gaps[key][k] <= bar, (key, k)


@pytest.mark.parametrize("case", sorted(CASES))
def test_linear_options(case):
    X, y, beta = make_problem(N, MT, seed=5)
    kw = dict(max_iter=12, stop_criteria_thr=0.0, **CASES[case])
    ref = O.vamp_infere(X, y, MT, true_signal=beta, **kw)
    _check(_gpu(X, y, beta, "linear", **kw), ref)


@pytest.mark.parametrize("case", ["three_slabs", "em3_tight", "fixed_vars", "no_damping", "cg_loose"])
def test_probit_options(case):
    X, y, beta = make_problem(N, MT, seed=5)
    yb = (y > 0).astype(np.float64)
    kw = dict(max_iter=10, stop_criteria_thr=0.0, model="bin_class", **CASES[case])
    ref, spread = oracle_with_spread(X, yb, beta, MT, ranks=(2, 3), **kw)
    _check(_gpu(X, yb, beta, **kw), ref, spread)


def test_alpha_scale_and_warm_start():
    X, y, beta = make_problem(N, MT, seed=6, kind=1)
    init = beta * 0.5 + 1e-3 * np.cos(np.arange(MT))
    kw = dict(max_iter=10, stop_criteria_thr=0.0)
    ref = O.vamp_infere(X, y, MT, true_signal=beta, x1hat_init=init, alpha_scale=0.5, **kw)
    _check(_gpu(X, y, beta, "linear", alpha_scale=0.5, x1hat_init=init, **kw), ref)
