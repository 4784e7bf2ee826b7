"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bars (BASELINE.json north_star): x1_hat / r1 within 1e-10 relative fp64
(norm-wise, SURVEY §0.2 explains why not element-wise), integer iteration and
CG counts identical.  Operators and generators: bit-exact where the
arithmetic is exact (synthetic data, Bernoulli draws), 1e-13 relative where it
is a reduction.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import relerr

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)


def _problem(N, Mt, seed=3, kind=0, n_causal=None, h2=0.8):
    X = O.generate_markers(seed, kind, N, 0, Mt)
    rng = np.random.default_rng(seed)
    nc = n_causal or max(1, Mt // 10)
    beta = np.zeros(Mt)
    idx = rng.choice(Mt, nc, replace=False)
    beta[idx] = rng.normal(0, np.sqrt(h2 / nc), nc)
    mave, msig = O.marker_stats(X)
    g = ((X - mave[:, None]) * msig[:, None]).T @ beta
    y = O.standardize_phen(g + rng.normal(0, np.sqrt(1 - h2), N))
    return X, y, beta


@pytest.mark.parametrize("N,Mt,kind", [(64, 128, 0), (301, 517, 0), (1000, 333, 1), (4099, 77, 0)])
def test_generator_and_stats(N, Mt, kind):
    Xo = O.generate_markers(5, kind, N, 0, Mt)
    with va.Data(N, Mt) as d:
        d.generate(5, kind)
        Xg = d.get_meth_data()
        assert np.array_equal(Xg, Xo), "device generator must be bit-identical to the oracle's"
        mo, so = O.marker_stats(Xo)
        assert relerr(d.get_mave(), mo) < 1e-13
        assert relerr(d.get_msig(), so) < 1e-13


@pytest.mark.parametrize("N,Mt", [(64, 128), (301, 517), (1000, 2000), (4099, 1031)])
def test_ax_atx(N, Mt):
    X, y, _ = _problem(N, Mt)
    mave, msig = O.marker_stats(X)
    rng = np.random.default_rng(1)
    x = rng.normal(size=Mt)
    u = rng.normal(size=N)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        assert relerr(d.Ax(x), O.ax(X, mave, msig, x)) < 1e-13
        assert relerr(d.ATx(u), O.atx(X, mave, msig, u)) < 1e-13
        # adjoint identity <A x, u> == <x, A^T u>
        lhs, rhs = d.Ax(x) @ u, x @ d.ATx(u)
        assert abs(lhs - rhs) <= 1e-12 * (abs(lhs) + 1e-300) * 10


def test_lmmse_pcg_denoise():
    N, Mt = 500, 900
    X, y, _ = _problem(N, Mt)
    mave, msig = O.marker_stats(X)
    rng = np.random.default_rng(2)
    v = rng.normal(size=Mt)
    tau, gam2 = 2.0, 0.7
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        ref = tau * O.atx(X, mave, msig, O.ax(X, mave, msig, v)) + gam2 * v
        assert relerr(d.lmmse_mult(v, tau, gam2), ref) < 1e-13
        assert np.all(d.lmmse_mult(np.zeros(Mt), tau, gam2) == 0)
        mu, it = d.pcg(v, tau, gam2, tol=1e-10)
        resid = tau * O.atx(X, mave, msig, O.ax(X, mave, msig, mu)) + gam2 * mu - v
        assert np.linalg.norm(resid) / np.linalg.norm(v) < 1e-9
        assert it > 1
        probs = np.array(O.DEFAULT_PROBS)
        vars_s = np.array(O.DEFAULT_VARS) * N
        r1 = rng.normal(size=Mt) * 3
        x1, x1d, sd = d.denoise(r1, 0.8, probs, vars_s)
        gx = np.array([O.g1(t, 0.8, probs, vars_s) for t in r1])
        gdx = np.array([O.g1d(t, 0.8, probs, vars_s) for t in r1])
        assert relerr(x1, gx) < 1e-13
        assert relerr(x1d, gdx) < 1e-13
        assert abs(sd - gdx.sum()) <= 1e-12 * abs(gdx.sum())


def _gpu_vamp(X, y, beta, Mt, headstart=None, op_variant=None, **kw):
    N = X.shape[1]
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        if headstart is not None:
            d.set_variant(5, 1 if headstart else 0)
        if op_variant is not None:
            d.set_variant(3, op_variant)
        d.set_phen(y, standardize=False)
        v = va.Vamp(d, va.VampOptions(**kw), true_signal=beta)
        x1 = v.infere(keep_hist=True)
        s = v.summary()
        n = s["iterations"]
        s["x1_hist"] = v.x1_hist[:n, : d.M].copy()
        s["r1_hist"] = v.r1_hist[:n, : d.M].copy()
        s["x1_final"] = x1
    return s


def _assert_parity(s, ref, tol=1e-10):
    assert s["iterations"] == ref["iterations"]
    assert s["cg_iters"] == ref["cg_iters"].tolist()
    assert s["ons_iters"] == ref["ons_iters"].tolist()
    assert s["L"] == ref["L"].tolist()
    for k in range(s["iterations"]):
        assert relerr(s["x1_hist"][k], ref["x1_hist"][k]) <= tol, f"x1 it {k + 1}"
        assert relerr(s["r1_hist"][k], ref["r1_hist"][k]) <= tol, f"r1 it {k + 1}"
    p, pr = np.array(s["params"]), ref["params"]
    assert np.allclose(p, pr, rtol=1e-9, atol=0)
    m, mr = np.array(s["metrics"]), ref["metrics"]
    assert np.allclose(m, mr, rtol=1e-9, atol=1e-12, equal_nan=True)


@pytest.mark.parametrize("N,Mt,its,thr", [(64, 128, 10, 0.0), (301, 517, 12, 0.0), (1000, 2000, 30, 0.0),
                                          (1000, 2000, 50, 0.01)])
def test_vamp_parity(N, Mt, its, thr):
    X, y, beta = _problem(N, Mt)
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=thr)
    s = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=thr)
    _assert_parity(s, ref)


def test_vamp_parity_methylation_like_no_truth():
    N, Mt = 700, 1500
    X, y, _ = _problem(N, Mt, kind=1)
    ref = O.vamp_infere(X, y, Mt, max_iter=15, stop_criteria_thr=0.0)
    s = _gpu_vamp(X, y, None, Mt, max_iter=15, stop_criteria_thr=0.0)
    _assert_parity(s, ref)
    assert np.isnan(np.array(s["metrics"])[:, 1]).all()  # corr with a zero true signal is 0/0


def test_batched_rhs_bitwise_equal_to_sequential():
    N, Mt = 1000, 2000
    X, y, beta = _problem(N, Mt)
    a = _gpu_vamp(X, y, beta, Mt, max_iter=8, stop_criteria_thr=0.0, batch_rhs=1)
    b = _gpu_vamp(X, y, beta, Mt, max_iter=8, stop_criteria_thr=0.0, batch_rhs=0)
    assert np.array_equal(a["x1_hist"], b["x1_hist"])
    assert a["cg_iters"] == b["cg_iters"] and a["ons_iters"] == b["ons_iters"]
    assert a["a_passes_exec"] < b["a_passes_exec"]


@pytest.mark.parametrize("N,Mt,its,kind", [(1000, 2000, 30, 0), (700, 1500, 20, 1), (301, 517, 12, 0)])
def test_recurrence_mode_matches_bitwise_schedule(N, Mt, its, kind):
    """batch_rhs=2 carries A^T A x2 and A^T A invQ through the CG
    steps instead of a pass: the same vectors up to rounding, the same
    integer counts, exactly one executed pass fewer per iteration after the
    first (iteration 1 has no warm start either way)."""
    X, y, beta = _problem(N, Mt, kind=kind)
    a = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=0.0, batch_rhs=2)
    b = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=0.0, batch_rhs=1)
    assert a["cg_iters"] == b["cg_iters"] and a["ons_iters"] == b["ons_iters"] and a["L"] == b["L"]
    for k in range(its):
        assert relerr(a["x1_hist"][k], b["x1_hist"][k]) <= 1e-11, f"x1 it {k + 1}"
        assert relerr(a["r1_hist"][k], b["r1_hist"][k]) <= 1e-11, f"r1 it {k + 1}"
    assert np.allclose(np.array(a["params"]), np.array(b["params"]), rtol=1e-11, atol=0)
    assert b["a_passes_exec"] - a["a_passes_exec"] == its
    assert a["a_passes_ref"] == b["a_passes_ref"]
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=0.0)
    _assert_parity(a, ref)


@pytest.mark.parametrize("N,Mt,its,kind", [(1000, 2000, 30, 0), (700, 1500, 20, 1), (301, 517, 12, 0)])
def test_ax_recurrence_mode(N, Mt, its, kind):
    """batch_rhs=3 (default) also carries A x2 through the CG steps (AW +=
    alpha * A p) and computes z1 = A x1 as one more right-hand side of the first
    CG pass: no pass outside the CG, 2*max(k1, k2) per iteration, the same
    integer counts, values within rounding of the bitwise schedule and within
    the parity bar of the oracle."""
    X, y, beta = _problem(N, Mt, kind=kind)
    a = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=0.0, batch_rhs=3)
    b = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=0.0, batch_rhs=2)
    assert a["cg_iters"] == b["cg_iters"] and a["ons_iters"] == b["ons_iters"] and a["L"] == b["L"]
    for k in range(its):
        assert relerr(a["x1_hist"][k], b["x1_hist"][k]) <= 1e-11, f"x1 it {k + 1}"
        assert relerr(a["r1_hist"][k], b["r1_hist"][k]) <= 1e-11, f"r1 it {k + 1}"
    assert np.allclose(np.array(a["params"]), np.array(b["params"]), rtol=1e-11, atol=0)
    assert np.allclose(np.array(a["metrics"]), np.array(b["metrics"]), rtol=1e-10, atol=1e-13, equal_nan=True)
    assert b["a_passes_exec"] - a["a_passes_exec"] == its + 1  # + iteration 1's own z1 pass
    assert a["a_passes_exec"] == 1 + sum(2 * max(p, q) for p, q in zip(a["cg_iters"], a["ons_iters"]))  # + A^T y
    assert a["a_passes_ref"] == b["a_passes_ref"]
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=0.0)
    _assert_parity(a, ref)


@pytest.mark.parametrize("N,Mt,its,kind", [(1000, 2000, 30, 0), (4099, 3001, 12, 1), (301, 517, 12, 0),
                                            (10000, 2500, 8, 0)])
def test_onepass_mode(N, Mt, its, kind):
    """batch_rhs=4 reads X once per CG step (A^T q and A d in one pass, q = A p
    and A r carried as N-vector recurrences): the same integer counts as
    batch_rhs=3, values within rounding of it and within the parity bar of the
    oracle, and 1 + max(k1, k2) executed passes per iteration (A r0 with z1,
    then one per CG step).  N > 2048 exercises the tile exchange between the
    workgroups of a team."""
    X, y, beta = _problem(N, Mt, kind=kind)
    a = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=0.0, batch_rhs=4)
    b = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=0.0, batch_rhs=3)
    errs = [max(relerr(a["x1_hist"][k], b["x1_hist"][k]), relerr(a["r1_hist"][k], b["r1_hist"][k]))
            for k in range(its)]
    print("onepass vs batch_rhs=3, max rel err per iteration:", ["%.1e" % e for e in errs])
    assert a["cg_iters"] == b["cg_iters"] and a["ons_iters"] == b["ons_iters"] and a["L"] == b["L"]
    assert max(errs) <= 1e-11
    assert np.allclose(np.array(a["params"]), np.array(b["params"]), rtol=1e-11, atol=0)
    assert np.allclose(np.array(a["metrics"]), np.array(b["metrics"]), rtol=1e-10, atol=1e-13, equal_nan=True)
    assert a["a_passes_exec"] == 1 + _onepass_passes(a["cg_iters"], a["ons_iters"])  # + A^T y
    assert a["a_passes_ref"] == b["a_passes_ref"]
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=0.0)
    _assert_parity(a, ref)


def _onepass_passes(cg, ons, headstart=True):
    """Executed passes of the one-pass schedule: 1 + max(k1, k2) per
    iteration; with the head start, from iteration 2 on, the Onsager solve's
    first step rides in the pass that starts the x2 solve: 1 + max(k1, k2 - 1)."""
    return sum(1 + (max(p, q - 1) if headstart and i > 0 else max(p, q)) for i, (p, q) in enumerate(zip(cg, ons)))


@pytest.mark.parametrize("N,Mt,its,kind,opv", [(1000, 2000, 30, 0, None), (4099, 3001, 12, 1, None),
                                                (301, 517, 12, 0, None), (10000, 2500, 10, 0, None),
                                                (3000, 2000, 10, 1, 1000 + 2 * 100 + 2),
                                                (3000, 2000, 10, 0, 1000 + 4 * 100 + 4),
                                                (1000, 2000, 6, 0, 1000 + 1 * 100 + 0)])
def test_headstart(N, Mt, its, kind, opv):
    """The head start (pcg.cpp): the Onsager solve takes its first CG step in
    the pass that starts the x2 solve, from A.bern formed one iteration early.
    Every step is still the reference's: the same CG, Onsager and mixture
    counts as without it, values within rounding (the plain products are
    summed in another order), within the parity bar of the oracle, and
    max(k1, k2 - 1) + 1 passes per iteration from iteration 2 on.  Team plans
    forced by opv cover the hand-off kernel at small N."""
    X, y, beta = _problem(N, Mt, kind=kind)
    a = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=0.0, headstart=True, op_variant=opv)
    b = _gpu_vamp(X, y, beta, Mt, max_iter=its, stop_criteria_thr=0.0, headstart=False, op_variant=opv)
    errs = [max(relerr(a["x1_hist"][k], b["x1_hist"][k]), relerr(a["r1_hist"][k], b["r1_hist"][k]))
            for k in range(its)]
    print("head start vs none, max rel err per iteration:", ["%.1e" % e for e in errs])
    assert a["cg_iters"] == b["cg_iters"] and a["ons_iters"] == b["ons_iters"] and a["L"] == b["L"]
    assert max(errs) <= 1e-11
    assert np.allclose(np.array(a["params"]), np.array(b["params"]), rtol=1e-11, atol=0)
    assert np.allclose(np.array(a["metrics"]), np.array(b["metrics"]), rtol=1e-10, atol=1e-13, equal_nan=True)
    assert a["a_passes_exec"] == 1 + _onepass_passes(a["cg_iters"], a["ons_iters"], True)
    assert b["a_passes_exec"] == 1 + _onepass_passes(b["cg_iters"], b["ons_iters"], False)
    assert a["a_passes_ref"] == b["a_passes_ref"]
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=0.0)
    _assert_parity(a, ref)


def test_headstart_cg_limits():
    """CG_max_iter reached inside the head start: the Onsager solve stops after
    max_iter steps of its own (its first in the head-start pass), exactly as
    without the head start; max_iter 1 and 2 included."""
    N, Mt = 800, 1500
    X, y, beta = _problem(N, Mt)
    for cgmax in (1, 2, 3):
        a = _gpu_vamp(X, y, beta, Mt, max_iter=5, stop_criteria_thr=0.0, CG_max_iter=cgmax, headstart=True)
        b = _gpu_vamp(X, y, beta, Mt, max_iter=5, stop_criteria_thr=0.0, CG_max_iter=cgmax, headstart=False)
        assert a["cg_iters"] == b["cg_iters"] and a["ons_iters"] == b["ons_iters"], cgmax
        assert max(a["ons_iters"]) <= cgmax and max(a["cg_iters"]) <= cgmax
        for k in range(5):
            assert relerr(a["x1_hist"][k], b["x1_hist"][k]) <= 1e-11, (cgmax, k)
        ref = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=5, stop_criteria_thr=0.0, CG_max_iter=cgmax)
        _assert_parity(a, ref)


def test_deterministic_repeat():
    N, Mt = 777, 1234
    X, y, beta = _problem(N, Mt)
    a = _gpu_vamp(X, y, beta, Mt, max_iter=6, stop_criteria_thr=0.0)
    b = _gpu_vamp(X, y, beta, Mt, max_iter=6, stop_criteria_thr=0.0)
    assert np.array_equal(a["x1_hist"], b["x1_hist"])


def _write_inputs(tmp, X, y, beta):
    Xp = os.path.join(tmp, "ex.bin")
    X.astype("<f8").tofile(Xp)  # marker-major: M blocks of N doubles (README.md:15)
    yp = os.path.join(tmp, "ex.phen")
    with open(yp, "w") as f:
        for i, v in enumerate(y):
            f.write("%d %d %0.10f\n" % (i, i, v))  # simulation/data_sim.py:68
    tp = os.path.join(tmp, "ex_ts.bin")
    beta.astype("<f8").tofile(tp)
    return Xp, yp, tp


def test_cli_drop_in_files(tmp_path):
    N, Mt, its = 400, 900, 6
    X, y, beta = _problem(N, Mt)
    Xp, yp, tp = _write_inputs(str(tmp_path), X, y, beta)
    out_g = tmp_path / "gpu"
    out_o = tmp_path / "orc"
    out_g.mkdir()
    out_o.mkdir()
    cmd = [va.CLI_PATH, "--meth-file", Xp, "--phen-file", yp, "--N", str(N), "--Mt", str(Mt), "--out-dir",
           str(out_g), "--out-name", "ex", "--iterations", str(its), "--stop-criteria-thr", "0",
           "--true-signal-file", tp]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    yo = O.read_phen(yp, N, True)
    ref = O.vamp_infere(X, yo, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=0.0, out_dir=str(out_o),
                        out_name="ex")
    for name in ("ex_params.csv", "ex_metrics.csv", "ex_prior.csv"):
        a = (out_g / name).read_bytes()
        b = (out_o / name).read_bytes()
        assert len(a) == len(b), name
        # header identical, NUL holes identical, row offsets identical
        nl = b.index(b"\n") + 1
        assert a[:nl] == b[:nl]
        assert [i for i, c in enumerate(a) if c == 0] == [i for i, c in enumerate(b) if c == 0]
        ra = [r for r in a.replace(b"\0", b"").decode().splitlines()[1:] if r]
        rb = [r for r in b.replace(b"\0", b"").decode().splitlines()[1:] if r]
        assert len(ra) == len(rb)
        for la, lb in zip(ra, rb):
            fa = [float(t) for t in la.split(",")]
            fb = [float(t) for t in lb.split(",")]
            assert fa[0] == fb[0]
            assert np.allclose(fa, fb, rtol=1e-9, atol=2e-15, equal_nan=True), (la, lb)
    for it in range(1, its + 1):
        for pat in ("ex_it_%d.bin", "ex_r1_it_%d.bin"):
            a = np.fromfile(out_g / (pat % it), dtype="<f8")
            b = np.fromfile(out_o / (pat % it), dtype="<f8")
            assert a.shape == b.shape == (Mt,)
            assert relerr(a, b) <= 1e-10
    assert relerr(np.fromfile(out_g / ("ex_it_%d.bin" % its), dtype="<f8"), ref["x1_final"]) <= 1e-10


def test_cli_resume_from_estimate_file(tmp_path):
    N, Mt = 300, 640
    X, y, beta = _problem(N, Mt)
    Xp, yp, tp = _write_inputs(str(tmp_path), X, y, beta)
    init = np.random.default_rng(4).normal(size=Mt) * 0.01
    ip = tmp_path / "init.bin"
    init.astype("<f8").tofile(ip)
    yo = O.read_phen(yp, N, True)
    ref = O.vamp_infere(X, yo, Mt, x1hat_init=init, max_iter=5, stop_criteria_thr=0.0)
    with va.Data(N, Mt) as d:
        d.read_methylation_data(Xp)
        d.read_phen(yp)
        assert relerr(d.get_phen(), yo) == 0.0
        v = va.Vamp(d, va.VampOptions(max_iter=5, stop_criteria_thr=0.0), x1hat_init=init)
        v.infere(keep_hist=True)
        s = v.summary()
        s["x1_hist"], s["r1_hist"] = v.x1_hist[:5], v.r1_hist[:5]
    _assert_parity(s, ref)


def test_errors_are_statuses(tmp_path):
    with va.Data(100, 50) as d:
        with pytest.raises(va.VampomiError) as e:
            d.Ax(np.zeros(50))
        assert e.value.status == 6  # ERR_STATE
        with pytest.raises(va.VampomiError) as e:
            d.read_methylation_data(str(tmp_path / "missing.bin"))
        assert e.value.status == 4
        p = tmp_path / "na.phen"
        p.write_text("0 0 1.0\n1 1 NA\n")
        with pytest.raises(va.VampomiError) as e:
            d.read_phen(str(p))
        assert e.value.status == 5


def test_c2_shape_properties():
    """BASELINE config 2 shape (N=10k, Mt=50k, 4 GB) on one GPU: size-independent checks."""
    N, Mt = 10000, 50000
    with va.Data(N, Mt) as d:
        d.generate(2024, va.GEN_GAUSS)
        beta = d.simulate_phen(7, lam=0.1, h2=0.8)
        Xs = d.get_meth_data(12345, 3)
        for k in range(3):
            xo = np.array([O.load().orc_gauss_dyadic(2024, 12345 + k, j) for j in range(0, N, 997)])
            assert np.array_equal(Xs[k, ::997], xo)
        rng = np.random.default_rng(0)
        x, u = rng.normal(size=Mt), rng.normal(size=N)
        ax, atx = d.Ax(x), d.ATx(u)
        assert abs(ax @ u - x @ atx) <= 1e-11 * abs(ax @ u)
        assert relerr(d.Ax(2 * x + 3 * beta), 2 * ax + 3 * d.Ax(beta)) < 1e-13  # linearity
        a = va.Vamp(d, va.VampOptions(max_iter=3, stop_criteria_thr=0.0, batch_rhs=1), true_signal=beta)
        a.infere(keep_hist=True)
        b = va.Vamp(d, va.VampOptions(max_iter=3, stop_criteria_thr=0.0, batch_rhs=0), true_signal=beta)
        b.infere(keep_hist=True)
        assert np.array_equal(a.x1_hist[:3], b.x1_hist[:3])
        # x1 = 0 at iteration 1, so its correlations are 0/0 (the reference writes -nan)
        assert np.isnan(a.metrics[0, 1]) and np.all(np.isfinite(a.metrics[1:3]))
        assert np.all(a.metrics[1:3, 3] > 0.1)  # x2 correlates with the true signal


def test_every_kernel_variant_is_correct():
    """All entries of the A.x / A^T.u tuning tables (tools/kbench.py) agree with the oracle."""
    import ctypes as C
    from vampomi_amd import _lib

    N, Mt = 4099, 1031  # ragged in both dimensions
    X, _, _ = _problem(N, Mt)
    mave, msig = O.marker_stats(X)
    rng = np.random.default_rng(3)
    x, u = rng.normal(size=Mt), rng.normal(size=N)
    ax_ref, atx_ref = O.ax(X, mave, msig, x), O.atx(X, mave, msig, u)
    lib = va.load()
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        for which, nvar in ((0, 7), (1, 8)):
            for v in range(nvar):
                _lib.check(lib.vampomi_dev_set_variant(d.ctx, which, v))
                if which == 0:
                    assert relerr(d.Ax(x), ax_ref) < 1e-13, ("ax", v)
                else:
                    assert relerr(d.ATx(u), atx_ref) < 1e-13, ("atx", v)
        # variants are settings of this context only: a fresh one runs the defaults
        with va.Data(N, Mt) as e:
            e.load_meth(X)
            assert e.kernel_name(1, 2, 1) != d.kernel_name(1, 2, 1)
            assert e.kernel_name(1, 2, 1) == "atx_kernel<4, 2, 1, 4, true>"  # the per-K default (G=4, UJ=4)
            assert relerr(e.ATx(u), atx_ref) < 1e-13


def test_rccl_code_path_single_rank(tmp_path):
    """The multi-rank data path (RCCL communicator, N-vector and scalar
    all-reduces, division after the reduce) on a 1-rank communicator gives
    bitwise the same run as the direct path when <d,p> is formed the same way
    (VAMPOMI_DP_SEPARATE=1), and the same run to 1e-12 with the multi-rank
    default <d,p> = tau*|A p|^2 + gam2*|p|^2 (one collective fewer per CG step)."""
    import sys

    code = r'''
import sys, numpy as np
sys.path[:0] = [%r, %r]
import vampomi_amd as va
from _data import make_problem
X, y, beta = make_problem(800, 1500)
with va.Data(800, 1500) as d:
    d.load_meth(X); d.set_phen(y, standardize=False)
    v = va.Vamp(d, va.VampOptions(max_iter=5, stop_criteria_thr=0.0), true_signal=beta)
    v.infere(keep_hist=True)
    np.save(sys.argv[1], v.x1_hist[:5, :1500])
''' % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for force, sep in (("0", "0"), ("1", "1"), ("1", "0")):
        f = tmp_path / f"x{force}{sep}.npy"
        env = dict(os.environ, VAMPOMI_FORCE_RCCL=force, VAMPOMI_DP_SEPARATE=sep)
        r = subprocess.run([sys.executable, "-c", code, str(f)], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(np.load(f))
    assert np.array_equal(outs[0], outs[1])
    for it in range(5):
        a, b = outs[0][it], outs[2][it]
        assert np.linalg.norm(a - b) <= 1e-12 * max(np.linalg.norm(a), 1e-300), it

