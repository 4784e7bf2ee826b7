"""GPU parity of the association tests (--run-mode association_test,
src/main_meth.cpp:206-264, src/data.cpp:385-417, src/utilities.cpp:269-282)
through the C ABI against the oracle.

Bars:
* the five per-marker sums to 1e-13 relative;
* the p-value function: the device's p from its own sums equals the oracle's
  linear_reg1d_pvals of those sums to 1e-12;
* end to end, p-values to 1e-10 relative, or to 10x the formula's own
  sensitivity to summation order where that is larger: the reference forms
  variances as sumsqx - sumx^2/n, which for raw methylation values cancels
  ~50-fold, and a tail p-value multiplies the relative error of t by ~t^2.
  The sensitivity is measured per marker as the change of the oracle's p when
  its sequential sums are replaced by numpy's pairwise sums;
* SE p-values to 1e-14."""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import relerr
from _data import make_problem

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)


def _estimate(beta, N, scale=0.9, seed=0):
    rng = np.random.default_rng(seed)
    return (beta * scale + rng.normal(size=beta.shape) * 1e-3) / np.sqrt(N)  # as an _it_K.bin holds it


def _order_spread(X, y, est, po):
    """|p(oracle sums) - p(pairwise sums)| / p per marker (numpy restatement)."""
    N = X.shape[1]
    mave, msig = O.marker_stats(X)
    x1 = est * np.sqrt(N)
    ymod = y - O.ax(X, mave, msig, x1)
    ym = ymod[None, :] + X / np.sqrt(N) * x1[:, None]
    sums = np.stack([X.sum(1), (X * X).sum(1), (X * ym).sum(1), ym.sum(1), (ym * ym).sum(1)], axis=1)
    pp = np.array([O.reg1d_pval(*s, N) for s in sums])
    return np.abs(pp - po) / np.maximum(po, 1e-300)


def _sums_extended(X, y, est, chunk=64):
    """The five per-marker sums of the float64 terms (raw x, y_mark = y_mod +
    x/sqrt(N)*x1_hat, their float64 products) accumulated in x87 extended
    precision: the reference value of each sum to ~1e-18, against which both
    the device's tree sums and the oracle's sequential sums are rounding."""
    N = X.shape[1]
    mave, msig = O.marker_stats(X)
    x1 = est * np.sqrt(N)
    ymod = y - O.ax(X, mave, msig, x1)
    out = np.zeros((X.shape[0], 5))
    L = np.longdouble
    for a in range(0, X.shape[0], chunk):
        Xc = X[a:a + chunk]
        ym = ymod[None, :] + Xc / np.sqrt(N) * x1[a:a + chunk, None]
        out[a:a + chunk] = np.stack([Xc.sum(1, dtype=L), (Xc * Xc).sum(1, dtype=L), (Xc * ym).sum(1, dtype=L),
                                     ym.sum(1, dtype=L), (ym * ym).sum(1, dtype=L)], axis=1)
    return out


def _check_loo(p, st, po, sto, spread, exact=None):
    for q in range(5):
        if exact is None:
            assert relerr(st[:, q], sto[:, q]) < 1e-13, q
        else:
            # at large N the oracle's SEQUENTIAL sums carry ~sqrt(N)*eps of their
            # own: the device is held to 1e-13 of the extended-precision sums,
            # and to the oracle within twice the oracle's own rounding
            assert relerr(st[:, q], exact[:, q]) < 1e-13, q
            assert relerr(st[:, q], sto[:, q]) < max(1e-13, 2 * relerr(sto[:, q], exact[:, q])), q
    tol = np.maximum(1e-10, 10 * spread)
    ok = np.abs(p - po) <= tol * po + 1e-300
    assert ok.all(), (p[~ok][:5], po[~ok][:5], spread[~ok][:5])


def _check_pfun(p, st, N):
    pf = np.array([O.reg1d_pval(*s, N) for s in st])
    assert np.all(np.abs(p - pf) <= 1e-12 * pf + 1e-300)


@pytest.mark.parametrize("N,Mt,kind", [(1000, 2000, 0), (1000, 2000, 1), (4099, 333, 1), (257, 1031, 0)])
def test_loo_parity(N, Mt, kind):
    X, y, beta = make_problem(N, Mt, kind=kind)
    est = _estimate(beta, N)
    po, sto = O.assoc_loo(X, y, est)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        p, st = d.assoc_loo(est)
    _check_pfun(p, st, N)
    _check_loo(p, st, po, sto, _order_spread(X, y, est, po))
    assert np.median(p[beta != 0]) < np.median(p[beta == 0])


def test_loo_extreme_p_values():
    """Strong effects: p-values down to ~1e-300 keep their relative accuracy."""
    N, Mt = 20000, 64
    X, y, beta = make_problem(N, Mt, kind=0, lam=0.3, h2=0.95)
    est = np.zeros(Mt)  # no leave-one-out add-back: plain marginal tests on y
    po, sto = O.assoc_loo(X, y, est)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        p, st = d.assoc_loo(est)
    assert po.min() < 1e-30
    _check_pfun(p, st, N)
    _check_loo(p, st, po, sto, _order_spread(X, y, est, po))


def test_every_loo_variant_is_bitwise_identical():
    """All association-pass variants (markers per wave, unroll, IEEE vs
    fma-corrected division) give the same sums bit for bit."""
    from vampomi_amd import _lib

    N, Mt = 4099, 301
    X, y, beta = make_problem(N, Mt, kind=1)
    est = _estimate(beta, N)
    lib = va.load()
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        ref = None
        for v in range(8):
            _lib.check(lib.vampomi_dev_set_variant(d.ctx, 2, v))
            p, st = d.assoc_loo(est)
            if ref is None:
                ref = (p, st)
            assert np.array_equal(st, ref[1]) and np.array_equal(p, ref[0]), v
        _lib.check(lib.vampomi_dev_set_variant(d.ctx, 2, 16))  # the default


@pytest.mark.parametrize("N,Mt,kind", [(4099, 301, 1), (20000, 64, 0), (5, 7, 0), (257, 5, 1)])
def test_workgroup_loo_variants(N, Mt, kind):
    """Variants 8-19 (loo_wg_kernel: the waves of a workgroup share its G
    markers and split the rows) against the oracle with the LOO bars, odd N
    (the zero pad row) and fewer markers than a workgroup takes included;
    variants with the same number of waves W are bitwise identical."""
    from vampomi_amd import _lib

    X, y, beta = make_problem(N, Mt, kind=kind)
    est = _estimate(beta, N)
    po, sto = O.assoc_loo(X, y, est)
    spread = _order_spread(X, y, est, po)
    lib = va.load()
    by_w = {}
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        for v, w in ((8, 8), (9, 8), (10, 8), (11, 8), (12, 4), (13, 4), (14, 4), (15, 4), (16, 8), (17, 2), (18, 2),
                     (19, 2)):
            _lib.check(lib.vampomi_dev_set_variant(d.ctx, 2, v))
            assert d.kernel_name(2, 1, v).startswith("loo_wg_kernel"), d.kernel_name(2, 1, v)
            p, st = d.assoc_loo(est)
            _check_pfun(p, st, N)
            _check_loo(p, st, po, sto, spread)
            if w in by_w:
                assert np.array_equal(st, by_w[w]), v
            by_w[w] = st
        _lib.check(lib.vampomi_dev_set_variant(d.ctx, 2, 16))  # the default


def test_se_parity():
    N, Mt = 1000, 2000
    X, y, beta = make_problem(N, Mt)
    rng = np.random.default_rng(3)
    r1 = np.concatenate([rng.normal(size=Mt - 4) * 0.05, [0.0, -0.0, 1e-3, -1e-3]])
    gam1 = 2.5
    po = O.assoc_se(r1, gam1, N)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        p = d.assoc_se(r1, gam1)
    assert np.allclose(p, po, rtol=1e-14, atol=1e-16)


def test_cli_association_files(tmp_path):
    N, Mt = 600, 1500
    X, y, beta = make_problem(N, Mt, kind=1)
    Xp = tmp_path / "ex.bin"
    X.astype("<f8").tofile(Xp)
    yp = tmp_path / "ex.phen"
    yp.write_text("".join("%d %d %0.10f\n" % (i, i, v) for i, v in enumerate(y)))
    est = _estimate(beta, N)
    ep = tmp_path / "ex_it_7.bin"
    est.astype("<f8").tofile(ep)
    r1 = est * 3
    rp = tmp_path / "ex_r1_it_7.bin"
    r1.astype("<f8").tofile(rp)
    base = [va.CLI_PATH, "--meth-file", str(Xp), "--phen-file", str(yp), "--N", str(N), "--Mt", str(Mt),
            "--out-dir", str(tmp_path), "--out-name", "as", "--run-mode", "association_test"]
    r = subprocess.run(base + ["--pval-method", "loo", "--estimate-file", str(ep)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(tmp_path / "as_it_7_pval_loo.bin", dtype="<f8")
    yo = O.read_phen(str(yp), N, True)
    po, _ = O.assoc_loo(X, yo, est)
    assert got.shape == (Mt,) and np.all(np.abs(got - po) <= 1e-10 * po + 1e-300)
    r = subprocess.run(base + ["--pval-method", "se", "--r1-file", str(rp), "--gam1", "3.5"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.fromfile(tmp_path / "as_it_7_pval_se.bin", dtype="<f8")
    assert np.allclose(got, O.assoc_se(r1, 3.5, N), rtol=1e-14, atol=1e-16)
    r = subprocess.run(base + ["--pval-method", "loo", "--estimate-file", str(tmp_path / "noiter.bin")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "cannot parse the iteration" in r.stdout


def test_c5_samples_whole_vector_vs_oracle():
    """configs[4]'s sample count, N = 100,000 methylation-like, at a reduced
    Mt: the WHOLE p-value and sums vectors against the oracle's assoc_loo
    (src/data.cpp:385-417, src/main_meth.cpp:245-264) with the bars above."""
    N, Mt = 100000, 2000
    X, y, beta = make_problem(N, Mt, seed=9, kind=1, lam=0.05, h2=0.5)
    est = _estimate(beta, N)
    po, sto = O.assoc_loo(X, y, est)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        p, st = d.assoc_loo(est)
    _check_pfun(p, st, N)
    _check_loo(p, st, po, sto, _order_spread(X, y, est, po), _sums_extended(X, y, est))
    assert np.median(p[beta != 0]) < np.median(p[beta == 0])


def test_c5_full_shard_properties():
    """The whole per-GPU C5 shard (N = 100,000 x 62,500 methylation-like
    markers, 50 GB; eight of them are configs[4]): the device sums equal a
    float64 restatement on 16 markers spread over the shard (first, last,
    power-of-two boundaries, random), the p-values equal the oracle's p-value
    function of those sums, and the causal markers stand out."""
    N, Mt = 100000, 62500
    with va.Data(N, Mt) as d:
        d.generate(9, va.GEN_METH)
        beta = d.simulate_phen(10, lam=0.05, h2=0.5)
        y = d.get_phen()
        est = _estimate(beta, N)
        p, st = d.assoc_loo(est)
        z1 = d.Ax(est * np.sqrt(N))
        ymod = y - z1
        rng = np.random.default_rng(5)
        picks = sorted({0, 1, Mt - 2, Mt - 1, 8191, 8192, 32767, 32768, 61439, 61440,
                        *rng.integers(0, Mt, 6).tolist()})
        for j in picks:
            x = d.get_meth_data(j, 1)[0]
            ym = ymod + x / np.sqrt(N) * (est[j] * np.sqrt(N))
            ref = [x.sum(), x @ x, x @ ym, ym.sum(), ym @ ym]
            assert np.allclose(st[j], ref, rtol=1e-11), j
            q = O.reg1d_pval(*ref, N)
            assert abs(p[j] - q) <= 1e-8 * q
        _check_pfun(p[picks], st[picks], N)
        assert np.all((p >= 0) & (p <= 1)) and np.all(np.isfinite(st))
        assert np.all(st[:, 0] > 0) and np.all(st[:, 1] > 0)  # methylation values in (0, 1)
        # 3,090 causal markers share h2 = 0.5: they stand out, the null ones are uniform
        assert np.median(p[beta != 0]) < 0.02 and 0.4 < np.median(p[beta == 0]) < 0.6


def test_c5_full_shard_vs_oracle():
    """The WHOLE per-GPU C5 shard (N = 100,000 x 62,500 methylation-like
    markers, 50 GB; eight of them are configs[4]) against the oracle's
    assoc_loo on the same matrix (bit-identical generator): every marker's
    five sums to 1e-12 relative (the oracle's sequential sums carry ~sqrt(N)
    eps of their own at this N), the p-value function to 1e-12, and every
    p-value to 1e-10 relative or, where that fails, to 10x the formula's own
    sensitivity to summation order measured on that marker (the bars above)."""
    N, Mt, seed = 100000, 62500, 13
    with va.Data(N, Mt) as d:
        d.generate(seed, va.GEN_METH)
        beta = d.simulate_phen(seed + 1, lam=0.05, h2=0.5)
        y = d.get_phen()
        est = _estimate(beta, N)
        p, st = d.assoc_loo(est)
    X = O.generate_markers(seed, va.GEN_METH, N, 0, Mt)
    po, sto = O.assoc_loo(X, y, est)
    for q in range(5):
        assert relerr(st[:, q], sto[:, q]) < 1e-12, q
    _check_pfun(p, st, N)
    bad = np.nonzero(np.abs(p - po) > 1e-10 * po + 1e-300)[0]
    # (at this N about 2.5 % of the markers: those whose statistic cancels
    # most; each is held to its own measured sensitivity below)
    assert len(bad) < Mt // 10, len(bad)
    if len(bad):  # the sensitivity on those markers (y_mod over the whole shard)
        mave, msig = O.marker_stats(X)
        x1 = est * np.sqrt(N)
        ymod = y - O.ax(X, mave, msig, x1)
        Xb = X[bad]
        ym = ymod[None, :] + Xb / np.sqrt(N) * x1[bad, None]
        sums = np.stack([Xb.sum(1), (Xb * Xb).sum(1), (Xb * ym).sum(1), ym.sum(1), (ym * ym).sum(1)], axis=1)
        pp = np.array([O.reg1d_pval(*q, N) for q in sums])
        spread = np.abs(pp - po[bad]) / np.maximum(po[bad], 1e-300)
        ok = np.abs(p[bad] - po[bad]) <= np.maximum(1e-10, 10 * spread) * po[bad] + 1e-300
        assert ok.all(), (bad[~ok][:5], p[bad][~ok][:5], po[bad][~ok][:5])
    assert np.median(p[beta != 0]) < 0.02 and 0.4 < np.median(p[beta == 0]) < 0.6
