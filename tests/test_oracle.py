"""The CPU oracle (oracle/vamp_oracle.c) against independent numpy
restatements of the reference formulas, and its own invariants.

PARITY UNPINNED: the reference ships no tests or fixtures and cannot be built
here; these checks pin the restatement to the reference's
formulas as written (file:line in each test), not to reference outputs.
"""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

from conftest import relerr
from _data import make_problem, sharded_oracle
from oracle import pyoracle as O


def test_generator_exact_and_deterministic():
    a = O.generate_markers(9, 0, 333, 5, 7)
    b = O.generate_markers(9, 0, 333, 5, 7)
    assert np.array_equal(a, b)
    # dyadic: multiples of 2^-17, |x| <= 6
    assert np.all(a * 2 ** 17 == np.round(a * 2 ** 17)) and np.abs(a).max() <= 6
    # a shard starting at S equals rows S.. of the full matrix (index-keyed)
    full = O.generate_markers(9, 0, 333, 0, 12)
    assert np.array_equal(full[5:12], a)
    big = O.generate_markers(1, 0, 2000, 0, 500)
    assert abs(big.mean()) < 0.01 and abs(big.var() - 1) < 0.01
    m = O.generate_markers(1, 1, 2000, 0, 200)
    assert m.min() >= 0 and m.max() <= 1 and 0.2 < m.mean() < 0.8


def test_bernoulli_index_keyed():
    b1 = O.bern_bits(5, 3, 0, 4000)
    assert 0.45 < b1.mean() < 0.55
    assert np.array_equal(O.bern_bits(5, 3, 1000, 100), b1[1000:1100])  # rank-count invariant
    assert not np.array_equal(O.bern_bits(5, 4, 0, 4000), b1)  # fresh draw per iteration


@pytest.mark.parametrize("Mt,P", [(2000, 1), (2000, 3), (7, 8), (500000, 8), (13, 5)])
def test_divide_work(Mt, P):
    # src/utilities.cpp:214-229
    lens = [Mt // P + (1 if r < Mt % P else 0) for r in range(P)]
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    for r in range(P):
        M, S, Mm = O.divide_work(Mt, P, r)
        assert (M, S) == (lens[r], starts[r])
        assert Mm == (Mt // P + 1 if Mt % P else Mt // P)


def test_marker_stats_formula():
    X = O.generate_markers(2, 1, 501, 0, 40)
    X[3] = 0.25  # zero variance -> msig = 1 (src/data.cpp:275-276)
    mave, msig = O.marker_stats(X)
    assert relerr(mave, X.mean(axis=1)) < 1e-14
    sd = X.std(axis=1, ddof=1)
    ref = np.where(sd > 0, 1 / np.where(sd > 0, sd, 1), 1.0)
    assert relerr(msig, ref) < 1e-13 and msig[3] == 1.0
    _, msig2 = O.marker_stats(X, alpha_scale=0.5)  # 1/pow(sd, alpha_scale) (:270-273)
    assert relerr(msig2, np.where(sd > 0, 1 / np.where(sd > 0, sd, 1) ** 0.5, 1.0)) < 1e-13


def test_ax_atx_formula():
    X = O.generate_markers(4, 0, 300, 0, 450)
    mave, msig = O.marker_stats(X)
    A = ((X - mave[:, None]) * msig[:, None]).T / np.sqrt(300)  # N x M, standardised / sqrt(N)
    rng = np.random.default_rng(0)
    x, u = rng.normal(size=450), rng.normal(size=300)
    assert relerr(O.ax(X, mave, msig, x), A @ x) < 1e-13
    assert relerr(O.atx(X, mave, msig, u), A.T @ u) < 1e-13


def _posterior_mean(y, gam1, probs, vars_):
    s = 1 / gam1
    w = np.array([p / np.sqrt(v + s) * np.exp(-y * y / (2 * (v + s))) for p, v in zip(probs, vars_)])
    w = w / w.sum()
    return y * sum(wk * v / (v + s) for wk, v in zip(w, vars_))


def test_denoiser_is_the_spike_and_slab_posterior_mean():
    # src/vamp.cpp:440-492: g1 = E[x | r], g1d = d g1 / d r (Tweedie)
    probs = np.array(O.DEFAULT_PROBS)
    vars_ = np.array(O.DEFAULT_VARS) * 1000
    for gam1 in (1e-3, 0.5, 3.0):
        for y in (-40.0, -3.0, -0.2, 0.0, 0.7, 5.0, 60.0):
            g = O.g1(y, gam1, probs, vars_)
            # y + sigma*pkd/pk cancels when the spike dominates: absolute, scaled by |y|
            assert abs(g - _posterior_mean(y, gam1, probs, vars_)) <= 1e-13 * max(1.0, abs(y))
            h = 1e-5 * max(1.0, abs(y))
            num = (_posterior_mean(y + h, gam1, probs, vars_) - _posterior_mean(y - h, gam1, probs, vars_)) / (2 * h)
            assert O.g1d(y, gam1, probs, vars_) == pytest.approx(num, rel=1e-5, abs=1e-9)
    assert O.g1(1.5, 1e11, probs, vars_) == 1.5 and O.g1d(1.5, 1e11, probs, vars_) == 1  # |sigma| < 1e-10


def test_read_phen(tmp_path):
    p = tmp_path / "a.phen"
    vals = [1.5, -0.25, 3.0, 2.0, -1.0]
    p.write_text("".join("%d %d %0.10f\n" % (i, i, v) for i, v in enumerate(vals)))
    y = O.read_phen(str(p), 5, standardize=False)
    assert np.array_equal(y, vals)
    ys = O.read_phen(str(p), 5, standardize=True)
    v = np.array(vals)
    assert relerr(ys, v * np.sqrt((len(v) - 1) / ((v - v.mean()) ** 2).sum())) < 1e-15  # scaled, not centred
    q = tmp_path / "b.phen"
    q.write_text(" 0 0 7.0\n")  # leading blank: the regex split's empty first token shifts the fields
    assert O.read_phen(str(q), 1, standardize=False)[0] == 0.0
    na = tmp_path / "na.phen"
    na.write_text("0 0 1\n1 1 NA\n")
    with pytest.raises(IOError):
        O.read_phen(str(na), 2)


def _run(N, Mt, **kw):
    X, y, beta = make_problem(N, Mt)
    return O.vamp_infere(X, y, Mt, true_signal=beta, **kw), (X, y, beta)


def test_vamp_oracle_learns_the_signal():
    r, (X, y, beta) = _run(1000, 2000, max_iter=20, stop_criteria_thr=0.0)
    assert r["iterations"] == 20
    corr = np.corrcoef(r["x1_final"], beta)[0, 1]
    assert corr > 0.8
    assert r["metrics"][-1, 2] > 0.7  # R2 of the LMMSE estimate
    # reference-equivalent pass count: 6 + 2[it>1] + 2(k1+k2) per iteration
    k = r["cg_iters"] + r["ons_iters"]
    assert r["a_passes"] == sum(6 + 2 * (i > 0) + 2 * k[i] for i in range(20))


def test_vamp_oracle_default_stop():
    r, _ = _run(1000, 2000, max_iter=50)  # stop_criteria_thr 0.01 (src/options.hpp:77)
    assert 2 <= r["iterations"] < 50


def test_vamp_oracle_thread_count_invariant():
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r); from _data import make_problem, sharded_oracle;"
            "from oracle import pyoracle as O; X, y, b = make_problem(500, 900);"
            "r = O.vamp_infere(X, y, 900, true_signal=b, max_iter=6, stop_criteria_thr=0.0);"
            "print(r['x1_final'].tobytes().hex()[:64], r['x1_final'].sum().hex())"
            % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.dirname(os.path.abspath(__file__))))
    outs = set()
    for t in ("1", "3", "8"):
        env = dict(os.environ, OMP_NUM_THREADS=t)
        outs.add(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                                check=True).stdout)
    assert len(outs) == 1, outs


@pytest.mark.parametrize("model", ["linear", "bin_class"])
@pytest.mark.parametrize("P", [2, 3])
def test_vamp_oracle_shard_invariance(P, model):
    """Marker sharding over P ranks (src/utilities.cpp:207-239) reproduces the
    single-rank run: the index-keyed Bernoulli makes it rank-count invariant.
    Linear: to 1e-12.  Probit: the iteration counts exactly, the values to
    the model's conditioning (alpha2 ~ 1 - 4e-8 at iteration 1 amplifies the
    all-reduce order by ~1e8)."""
    N, Mt, its = 600, 1100, 8
    X, y, beta = make_problem(N, Mt)
    if model == "bin_class":
        y = (y > 0).astype(np.float64)
    one = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=0.0, model=model)
    res = sharded_oracle(X, y, beta, Mt, P, max_iter=its, stop_criteria_thr=0.0, model=model)
    x = np.concatenate([r["x1_final"] for r in res])
    assert relerr(x, one["x1_final"]) < (1e-12 if model == "linear" else 1e-6)
    for r in res:
        assert r["cg_iters"].tolist() == one["cg_iters"].tolist()
        assert r["ons_iters"].tolist() == one["ons_iters"].tolist()
        assert r["L"].tolist() == one["L"].tolist()
        assert np.allclose(r["params"], one["params"], rtol=1e-11 if model == "linear" else 1e-5)


def test_update_prior_one_em_pass_numpy():
    """updatePrior (src/vamp.cpp:531-643), one EM pass without merging, against
    a numpy restatement of the responsibilities and moment updates."""
    rng = np.random.default_rng(3)
    N = 800
    r1 = np.concatenate([rng.normal(size=700) * 0.02, rng.normal(size=300) * 0.3])
    gam1 = 40.0
    probs = np.array([0.9, 0.06, 0.04])
    vars_ = np.array([0.0, 1e-3, 5e-2]) * N
    p, v = O.update_prior(r1, gam1, probs, vars_, N, EM_max_iter=1, merge_vars_thr=0.0)
    nv = 1 / gam1
    lam = 1 - probs[0]
    om = probs[1:] / lam
    vmax = vars_.max()
    num = lam * om[None, :] * np.exp(-(r1[:, None] ** 2) / 2 * (vmax - vars_[None, 1:]) / (vars_[None, 1:] + nv)
                                     / (vmax + nv)) / np.sqrt(vars_[None, 1:] + nv) / np.sqrt(2 * np.pi)
    s = num.sum(1)
    beta = num / s[:, None]
    pin = 1 / (1 + (1 - lam) / np.sqrt(2 * np.pi * nv) * np.exp(-(r1 ** 2) / 2 * vmax / nv / (nv + vmax)) / s)
    lam_new = pin.sum() / len(r1)
    g = gam1 * r1[:, None] / (1 / vars_[None, 1:] + gam1)
    vv = 1 / (1 / vars_[1:] + gam1)
    gam = beta * (g ** 2 + vv[None, :])
    res = (beta * pin[:, None]).sum(0)
    res_g = (gam * pin[:, None]).sum(0)
    exp_v = np.concatenate([[0.0], res_g / res])
    exp_p = np.concatenate([[1 - lam_new], lam_new * res / pin.sum()])
    assert np.allclose(v, exp_v, rtol=1e-12) and np.allclose(p, exp_p, rtol=1e-12)
    # merging: equal slabs collapse into one component carrying both weights
    p2, v2 = O.update_prior(r1, gam1, [0.9, 0.05, 0.05], np.array([0.0, 1e-3, 1e-3]) * N, N, EM_max_iter=1,
                            learn_vars=0)
    assert len(p2) == 2 and abs(p2.sum() - 1) < 1e-12
