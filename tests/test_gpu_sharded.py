"""The multi-rank (marker-sharded) engine on the GPU: P ranks as threads of
this process, each with its own context on device 0, joined by the
test-only loopback communicator (VAMPOMI_COMM=loopback: an in-process
rendezvous summing in rank order).  Every multi-rank code path of the engine
runs — divide_work shards with S > 0, per-rank A.x partials + all-reduce +
division, synced and local reductions, the EM / Onsager / noise-precision
all-reduces, file offsets — except RCCL itself, which
tests/test_gpu_parity.py::test_rccl_code_path_single_rank covers.  Results
must match the single-rank GPU run (linear) or the oracle's bars (probit,
association tests)."""
import os
import threading
import time

import numpy as np
import pytest

from conftest import relerr
from _data import PROBIT_K, make_problem, oracle_with_spread, record_probit_ratio

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)


def run_ranks(monkeypatch, P, N, Mt, fn, timeout=100):
    """fn(rank, data) on P threads, one context each; returns the results by rank."""
    monkeypatch.setenv("VAMPOMI_COMM", "loopback")
    cid = os.urandom(va.UNIQUE_ID_BYTES)
    res, errs = [None] * P, []

    def work(r):
        try:
            with va.Data(N, Mt, rank=r, nranks=P, comm_id=cid, device=0) as d:
                res[r] = fn(r, d)
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append((r, e))

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(P)]
    [t.start() for t in th]
    deadline = time.monotonic() + timeout
    [t.join(max(0.0, deadline - time.monotonic())) for t in th]
    stuck = [r for r, t in enumerate(th) if t.is_alive()]
    assert not stuck, f"ranks {stuck} stuck in a collective; errors of the others: {errs}"
    assert not errs, errs
    return res


def _vamp(d, X, y, beta, model="linear", **kw):
    d.load_meth(X[d.S:d.S + d.M])
    d.set_phen(y, standardize=False)
    v = va.Vamp(d, va.VampOptions(model=model, **kw), true_signal=beta[d.S:d.S + d.M])
    x1 = v.infere(keep_hist=True)
    s = v.summary()
    n = s["iterations"]
    s["x1_hist"], s["r1_hist"], s["x1_final"] = v.x1_hist[:n, :d.M].copy(), v.r1_hist[:n, :d.M].copy(), x1
    s["S"], s["M"] = d.S, d.M
    return s


def _cat(parts, key):
    return np.concatenate([p[key] for p in parts], axis=-1)


@pytest.mark.parametrize("P", [2, 3])
def test_sharded_operators(monkeypatch, P):
    N, Mt = 1001, 2003
    X, y, _ = make_problem(N, Mt)
    mave, msig = O.marker_stats(X)
    rng = np.random.default_rng(8)
    x, u = rng.normal(size=Mt), rng.normal(size=N)

    def fn(r, d):
        d.load_meth(X[d.S:d.S + d.M])
        return d.S, d.M, d.Ax(x[d.S:d.S + d.M]), d.ATx(u), d.get_mave(), d.get_msig()

    res = run_ranks(monkeypatch, P, N, Mt, fn)
    assert [r[0] for r in res] == [O.divide_work(Mt, P, k)[1] for k in range(P)]
    for r in res:  # A.x is all-reduced: every rank holds the whole product
        assert relerr(r[2], O.ax(X, mave, msig, x)) < 1e-13
    assert relerr(np.concatenate([r[3] for r in res]), O.atx(X, mave, msig, u)) < 1e-13
    assert relerr(np.concatenate([r[4] for r in res]), mave) < 1e-14
    assert relerr(np.concatenate([r[5] for r in res]), msig) < 1e-14


@pytest.mark.parametrize("P", [2, 4])
def test_sharded_team_ax(monkeypatch, P):
    """A.x on the team plan (N above ~16k: ax_team_kernel) on P ranks: each
    rank's team slots, its reduction, the all-reduce and /sqrt(N); odd N, and
    fewer markers per rank than teams (empty teams write zero slots)."""
    N, Mt = 20001, 403
    X = O.generate_markers(11, 1, N, 0, Mt)
    mave, msig = O.marker_stats(X)
    x = np.random.default_rng(9).normal(size=Mt)

    def fn(r, d):
        d.load_meth(X[d.S:d.S + d.M])
        return d.kernel_name(0, 1), d.Ax(x[d.S:d.S + d.M])

    res = run_ranks(monkeypatch, P, N, Mt, fn)
    ref = O.ax(X, mave, msig, x)
    for name, ax in res:
        assert name.startswith("ax_team_kernel<"), name
        assert relerr(ax, ref) < 1e-13
        assert np.array_equal(ax, res[0][1])  # the same all-reduced vector on every rank


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_sharded_linear_vamp_matches_single_rank(monkeypatch, P):
    N, Mt, its = 1000, 2000, 12
    X, y, beta = make_problem(N, Mt)
    kw = dict(max_iter=its, stop_criteria_thr=0.0)
    with va.Data(N, Mt) as d:
        one = _vamp(d, X, y, beta, **kw)
    parts = run_ranks(monkeypatch, P, N, Mt, lambda r, d: _vamp(d, X, y, beta, **kw))
    for p in parts:
        assert p["cg_iters"] == one["cg_iters"] and p["ons_iters"] == one["ons_iters"] and p["L"] == one["L"]
        assert np.allclose(p["params"], one["params"], rtol=1e-11)
        assert np.allclose(p["metrics"], one["metrics"], rtol=1e-11, equal_nan=True)
    for k in range(its):
        assert relerr(_cat(parts, "x1_hist")[k], one["x1_hist"][k]) < 1e-12, k
        assert relerr(_cat(parts, "r1_hist")[k], one["r1_hist"][k]) < 1e-12, k
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, **kw)
    assert relerr(_cat(parts, "x1_final"), ref["x1_final"]) < 1e-10
    assert parts[0]["cg_iters"] == ref["cg_iters"].tolist()


@pytest.mark.parametrize("P", [2, 4, 8])
def test_sharded_probit(monkeypatch, P):
    """Mt = 2003: shards of unequal size at every P (divide_work's remainder)."""
    N, Mt, its = 1000, 2003, 12
    X, y, beta = make_problem(N, Mt)
    yb = (y > 0).astype(np.float64)
    kw = dict(max_iter=its, stop_criteria_thr=0.0, model="bin_class")
    ref, spread = oracle_with_spread(X, yb, beta, Mt, **kw)
    parts = run_ranks(monkeypatch, P, N, Mt, lambda r, d: _vamp(d, X, yb, beta, **kw))
    for p in parts:
        assert p["cg_iters"] == ref["cg_iters"].tolist() and p["ons_iters"] == ref["ons_iters"].tolist()
        m = np.array(p["metrics"])
        for o in (0, 6):
            assert np.array_equal(m[:, o:o + 4], ref["metrics"][:, o:o + 4])
    gap = np.array([relerr(_cat(parts, "x1_hist")[k], ref["x1_hist"][k]) for k in range(its)])
    record_probit_ratio(f"test_sharded_probit[{P}]", "x1", gap, spread["x1"][:its])
    for k in range(its):
        assert gap[k] <= max(1e-10, PROBIT_K * spread["x1"][k]), k


@pytest.mark.parametrize("P", [3, 4, 8])
def test_sharded_association_and_test_mode(monkeypatch, P):
    N, Mt = 900, 1501
    X, y, beta = make_problem(N, Mt, kind=1)
    est = beta * 0.9

    def fn(r, d):
        d.load_meth(X[d.S:d.S + d.M])
        d.set_phen(y, standardize=False)
        p, st = d.assoc_loo(est[d.S:d.S + d.M])
        return p, st, d.test_metrics(est[d.S:d.S + d.M]), d.assoc_se(est[d.S:d.S + d.M], 2.0)

    res = run_ranks(monkeypatch, P, N, Mt, fn)
    assert [r[1].shape[0] for r in res] == [O.divide_work(Mt, P, k)[0] for k in range(P)]
    po, sto = O.assoc_loo(X, y, est)
    st = np.concatenate([r[1] for r in res])
    p = np.concatenate([r[0] for r in res])
    for q in range(5):
        assert relerr(st[:, q], sto[:, q]) < 1e-13
    pf = np.array([O.reg1d_pval(*s, N) for s in st])
    assert np.all(np.abs(p - pf) <= 1e-12 * pf + 1e-300)
    ro, co = O.test_metrics(X, y, est)
    for r in res:
        assert abs(r[2][0] - ro) <= 1e-12 * abs(ro) and abs(r[2][1] - co) <= 1e-12 * abs(co)
    assert np.allclose(np.concatenate([r[3] for r in res]), O.assoc_se(est, 2.0, N), rtol=1e-14, atol=1e-16)


def test_eight_ranks_team_operator_matches_single_rank(monkeypatch):
    """configs[2]'s rank count at C2's sample count: N = 10,000 (the team
    operator with teams of 2 on every rank, the head start) and Mt = 16,003
    (Mt % 8 = 3: three shards one marker longer), 8 loopback ranks against
    the one-rank run: counts exact, x1_hat / r1 within 1e-12 at every
    iteration (only the rank-ordered A.x / A d / scalar sums differ)."""
    N, Mt, its, P = 10000, 16003, 8, 8
    X, y, beta = make_problem(N, Mt, seed=6)
    kw = dict(max_iter=its, stop_criteria_thr=0.0)
    with va.Data(N, Mt) as d:
        one = _vamp(d, X, y, beta, **kw)
        assert d.stats().op.launches > 0

    def fn(r, d):
        s = _vamp(d, X, y, beta, **kw)
        s["op_launches"] = d.stats().op.launches
        s["op_name"] = d.kernel_name(3, 2)
        return s

    parts = run_ranks(monkeypatch, P, N, Mt, fn, timeout=300)
    assert [p["M"] for p in parts] == [O.divide_work(Mt, P, k)[0] for k in range(P)]
    for p in parts:
        assert p["op_launches"] > 0 and "team" in p["op_name"], p["op_name"]
        assert p["cg_iters"] == one["cg_iters"] and p["ons_iters"] == one["ons_iters"] and p["L"] == one["L"]
        assert np.allclose(p["params"], one["params"], rtol=1e-11)
    for k in range(its):
        assert relerr(_cat(parts, "x1_hist")[k], one["x1_hist"][k]) < 1e-12, k
        assert relerr(_cat(parts, "r1_hist")[k], one["r1_hist"][k]) < 1e-12, k


def test_pcg_warm_start_on_some_ranks_only(monkeypatch):
    """vampomi_pcg with mu0 on rank 0 and NULL on rank 1: the zero-vector test
    is collective (both ranks run the warm-start pass), rank 1 starts from a
    zero slice; equals the one-rank solve from [mu0_0, 0]."""
    N, Mt = 700, 1301
    X, _, _ = make_problem(N, Mt, seed=9)
    rng = np.random.default_rng(4)
    v = rng.normal(size=Mt)
    mu0 = rng.normal(size=Mt) * 0.1
    M0, S1, _ = O.divide_work(Mt, 2, 0)
    mu0_full = np.concatenate([mu0[:M0], np.zeros(Mt - M0)])
    tau, gam2 = 1.7, 0.4
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        one, it1 = d.pcg(v, tau, gam2, mu0=mu0_full, tol=1e-9, max_iter=200)

    def fn(r, d):
        d.load_meth(X[d.S:d.S + d.M])
        return d.pcg(v[d.S:d.S + d.M], tau, gam2, mu0=mu0[:M0] if r == 0 else None, tol=1e-9, max_iter=200)

    parts = run_ranks(monkeypatch, 2, N, Mt, fn)
    assert [p[1] for p in parts] == [it1, it1]
    assert relerr(np.concatenate([p[0] for p in parts]), one) < 1e-12


def _run_ranks_collect(monkeypatch, P, N, Mt, fn, timeout=60):
    """Like run_ranks, but returns each rank's exception (or None) instead of asserting."""
    monkeypatch.setenv("VAMPOMI_COMM", "loopback")
    cid = os.urandom(va.UNIQUE_ID_BYTES)
    errs = [None] * P

    def work(r):
        try:
            with va.Data(N, Mt, rank=r, nranks=P, comm_id=cid, device=0) as d:
                fn(r, d)
        except BaseException as e:  # noqa: BLE001 - returned
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(P)]
    [t.start() for t in th]
    deadline = time.monotonic() + timeout
    [t.join(max(0.0, deadline - time.monotonic())) for t in th]
    assert not [r for r, t in enumerate(th) if t.is_alive()], "a rank is still waiting"
    return errs


def test_rank_local_failure_releases_the_other_ranks(monkeypatch):
    """A collective entry point that fails on one rank (here an argument error
    in updatePrior) poisons the communicator: the rank waiting in its own
    collective fails at once with the cause, instead of after a timeout."""
    N, Mt = 300, 500
    X, _, _ = make_problem(N, Mt)

    def fn(r, d):
        d.load_meth(X[d.S:d.S + d.M])
        if r == 1:
            time.sleep(0.5)  # rank 0 is inside its all-reduce by now
            d.update_prior(np.zeros(d.M), 1.0, [], [])  # L = 0: ERR_ARG on this rank only
        else:
            d.Ax(np.ones(d.M))

    t0 = time.monotonic()
    errs = _run_ranks_collect(monkeypatch, 2, N, Mt, fn)
    assert time.monotonic() - t0 < 30
    assert isinstance(errs[1], va.VampomiError) and "mixture components" in str(errs[1])
    assert isinstance(errs[0], va.VampomiError) and "rank 1 aborted" in str(errs[0]), errs[0]


def test_divergent_collectives_fail_on_every_rank(monkeypatch):
    """Ranks that issue different collectives (sequence, size or call site)
    fail together, each naming every rank's collective."""
    N, Mt = 300, 500
    X, _, _ = make_problem(N, Mt)

    def fn(r, d):
        d.load_meth(X[d.S:d.S + d.M])
        if r == 0:
            d.Ax(np.ones(d.M))  # the A.x all-reduce (N doubles)
        else:
            d.barrier()  # a 1-double all-reduce

    errs = _run_ranks_collect(monkeypatch, 2, N, Mt, fn)
    for e in errs:
        assert isinstance(e, va.VampomiError) and "ranks disagree on the collective" in str(e), e
        assert "rank 0:" in str(e) and "rank 1:" in str(e)


def test_side_stream_removed():
    """Rounds 2-5 ran the prefetched EM / denoiser on a second HIP stream
    (set_variant(4)); it never shortened an iteration (0.5 % slower at one
    rank, unused by the host-free multi-rank tail) and was removed in round 6
    (DESIGN.md §6).  The hook now refuses, so no caller believes it is on."""
    with va.Data(1001, 2003) as d:
        with pytest.raises(va.VampomiError) as e:
            d.set_variant(4, 1)
        assert e.value.status == 1  # ERR_ARG


@pytest.mark.parametrize("P", [1, 2])
def test_team_operator_beside_the_writer(monkeypatch, tmp_path, P):
    """N = 12,000: the one-pass operator runs as teams of 4 workgroups that
    must all be resident.  With the iteration writer's kernel + copy stream
    busy, every team launch still completes (no hand-off timeout) and the
    results are bitwise those of the run without files; the files hold what
    the history holds."""
    N, Mt, its = 12000, 3001, 8
    X, y, beta = make_problem(N, Mt, seed=4)
    out = {}
    for busy in (0, 1):
        def fn(r, d, busy=busy):
            kw = dict(out_dir=str(tmp_path / f"b{busy}"), out_name="t") if busy else {}
            return _vamp(d, X, y, beta, max_iter=its, stop_criteria_thr=0.0, **kw)

        if busy:
            (tmp_path / "b1").mkdir()
        if P == 1:
            with va.Data(N, Mt) as d:
                out[busy] = [fn(0, d)]
        else:
            out[busy] = run_ranks(monkeypatch, P, N, Mt, fn, timeout=300)
    for a, b in zip(out[0], out[1]):
        for k in ("iterations", "cg_iters", "ons_iters", "L"):
            assert a[k] == b[k], k
        for k in ("x1_hist", "r1_hist", "params"):
            np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)
    x1 = np.concatenate([p["x1_hist"] for p in out[1]], axis=1)
    r1 = np.concatenate([p["r1_hist"] for p in out[1]], axis=1)
    for it in range(1, its + 1):
        np.testing.assert_array_equal(np.fromfile(tmp_path / "b1" / f"t_it_{it}.bin", dtype="<f8"), x1[it - 1])
        np.testing.assert_array_equal(np.fromfile(tmp_path / "b1" / f"t_r1_it_{it}.bin", dtype="<f8"), r1[it - 1])


def test_headstart_agreed_over_ranks(monkeypatch):
    """The head start changes the collective sequence (its launch's all-reduce
    replaces ax_dev's), and each rank reads its own switch (VAMPOMI_HEADSTART,
    set_variant(5)).  With the switch off on ONE rank the job must neither hang
    nor mismatch: op_prepare agrees the choice over the ranks, so both ranks
    run without it and equal the one-rank run with it off (bitwise: the same
    schedule, the same rank-ordered sums)."""
    N, Mt, its = 1001, 2003, 8
    X, y, beta = make_problem(N, Mt)
    kw = dict(max_iter=its, stop_criteria_thr=0.0)
    with va.Data(N, Mt) as d:
        d.set_variant(5, 0)
        off = _vamp(d, X, y, beta, **kw)

    def fn(r, d):
        if r == 1:
            d.set_variant(5, 0)
        return _vamp(d, X, y, beta, **kw)

    parts = run_ranks(monkeypatch, 2, N, Mt, fn)
    for p in parts:
        assert p["cg_iters"] == off["cg_iters"] and p["ons_iters"] == off["ons_iters"]
        assert np.allclose(p["params"], off["params"], rtol=1e-11)
    for k in range(its):
        assert relerr(_cat(parts, "x1_hist")[k], off["x1_hist"][k]) < 1e-12, k


def test_rank_local_switches_between_runs(monkeypatch):
    """a rank-local set_variant(5) (and a one-rank timing hook on
    the operator) between two runs of a job must not make the ranks issue
    different collectives.  The choice is agreed at vampomi_vamp_begin, the
    one point every rank reaches, so the second run -- head start off on
    rank 1 only -- runs without it on both ranks (bitwise the one-rank run
    with it off) and the first run with it (bitwise the one-rank default)."""
    import ctypes as C

    N, Mt, its = 1001, 2003, 6
    X, y, beta = make_problem(N, Mt)
    kw = dict(max_iter=its, stop_criteria_thr=0.0)
    one = {}
    for hs in (1, 0):
        with va.Data(N, Mt) as d:
            d.set_variant(5, hs)
            one[hs] = _vamp(d, X, y, beta, **kw)

    def fn(r, d):
        first = _vamp(d, X, y, beta, **kw)
        if r == 1:
            d.set_variant(5, 0)
            ms = C.c_double()
            va.load().vampomi_dev_time_pass(d.ctx, 3, 1, 1, C.byref(ms))  # plans this rank's operator, no agreement
        return first, _vamp(d, X, y, beta, **kw)

    parts = run_ranks(monkeypatch, 2, N, Mt, fn)
    for run, hs in ((0, 1), (1, 0)):
        ps = [p[run] for p in parts]
        for p in ps:
            assert p["cg_iters"] == one[hs]["cg_iters"] and p["ons_iters"] == one[hs]["ons_iters"]
        for k in range(its):
            assert relerr(_cat(ps, "x1_hist")[k], one[hs]["x1_hist"][k]) < 1e-12, (run, k)


def test_multi_rank_tail_switch_agreed_over_ranks(monkeypatch):
    """the host-free tail (VAMPOMI_MR_TAIL, set_variant(6)) changes
    the tail's collective sequence, so a rank-local choice must not reach the
    collectives: op_agree agrees it at vampomi_vamp_begin with the operator and
    head-start choices.  Rank 1 alone turns it off: both ranks run the
    host-waiting tail (no divergent all-reduce: the loopback communicator would
    fail the job on one), the same host waits on both, bitwise the run with it
    off everywhere."""
    N, Mt = 1001, 2003
    X, y, beta = make_problem(N, Mt)
    kw = dict(max_iter=8, stop_criteria_thr=0.0)

    def fn_off_on_one(r, d):
        if r == 1:
            d.set_variant(6, 0)
        s = _vamp(d, X, y, beta, **kw)
        s["host_syncs"] = d.stats().host_syncs
        return s

    mixed = run_ranks(monkeypatch, 2, N, Mt, fn_off_on_one)
    monkeypatch.setenv("VAMPOMI_MR_TAIL", "0")
    off = run_ranks(monkeypatch, 2, N, Mt, lambda r, d: dict(_vamp(d, X, y, beta, **kw),
                                                             host_syncs=d.stats().host_syncs))
    monkeypatch.delenv("VAMPOMI_MR_TAIL")
    on = run_ranks(monkeypatch, 2, N, Mt, lambda r, d: dict(_vamp(d, X, y, beta, **kw),
                                                            host_syncs=d.stats().host_syncs))
    assert mixed[0]["host_syncs"] == mixed[1]["host_syncs"] == off[0]["host_syncs"] > on[0]["host_syncs"]
    for k in range(kw["max_iter"]):
        assert np.array_equal(_cat(mixed, "x1_hist")[k], _cat(off, "x1_hist")[k]), k
    assert mixed[0]["cg_iters"] == off[0]["cg_iters"]


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("kw", [dict(max_iter=10, stop_criteria_thr=0.0), dict(max_iter=30, stop_criteria_thr=0.01),
                                dict(max_iter=8, stop_criteria_thr=0.0, EM_max_iter=3, EM_err_thr=1e-9),
                                dict(max_iter=8, stop_criteria_thr=0.0, learn_prior_delay=4)],
                         ids=["fixed", "stops", "em3", "delay"])
def test_multi_rank_tail_without_host_waits_bitwise(monkeypatch, P, kw):
    """Several ranks (VAMPOMI_MR_TAIL, default on): the linear iteration's tail
    runs without host waits -- gam1, the EM round's mixture update and the next
    prelude's scalars are formed on the device after the all-reduce of their
    sums (vk::tail_post), and the next prelude + CG start are queued before
    the host's one wait.  Bitwise the run with the host waiting at every
    level (VAMPOMI_MR_TAIL=0), also when the stop criterion fires, with
    several EM rounds (the host path) and with the prior's learning delayed."""
    N, Mt = 1001, 2003
    X, y, beta = make_problem(N, Mt)
    out = {}

    def fn(r, d):
        s = _vamp(d, X, y, beta, **kw)
        s["host_syncs"] = d.stats().host_syncs
        return s

    for mt in ("0", "1"):
        monkeypatch.setenv("VAMPOMI_MR_TAIL", mt)
        out[mt] = run_ranks(monkeypatch, P, N, Mt, fn)
    if "EM_max_iter" not in kw and "learn_prior_delay" not in kw:  # (the host path of those settings is kept)
        assert out["1"][0]["host_syncs"] < out["0"][0]["host_syncs"], (out["1"][0]["host_syncs"],
                                                                      out["0"][0]["host_syncs"])
    for a, b in zip(out["0"], out["1"]):
        for k in ("iterations", "cg_iters", "ons_iters", "L"):
            assert a[k] == b[k], k
        for k in ("x1_hist", "r1_hist", "params", "metrics"):
            np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("kw", [dict(), dict(CG_max_iter=2), dict(CG_max_iter=1), dict(hs=0)],
                         ids=["default", "cg_max2", "cg_max1", "no_headstart"])
def test_folded_cg_decisions_bitwise(monkeypatch, P, kw):
    """Several ranks (VAMPOMI_CG_FOLD, default on): each CG step's decision is
    formed by the next step's operator launch from the all-reduced sums
    (vk::OpFold; the two CgStates alternate), and by a decision launch only
    when no step follows (CG_max_iter reached).  Bitwise the run with a
    decision launch after every step (VAMPOMI_CG_FOLD=0), with and without
    the head start, and with the solve cut at 1 and 2 steps; the team
    operator (N = 12,000) and the whole-column plan (N = 1,001)."""
    kw = dict(kw)
    hs = kw.pop("hs", 1)
    for N, Mt, its in ((1001, 2003, 6), (12000, 3001, 4)):
        X, y, beta = make_problem(N, Mt, seed=8)
        out = {}

        def fn(r, d):
            d.set_variant(5, hs)
            return _vamp(d, X, y, beta, max_iter=its, stop_criteria_thr=0.0, **kw)

        for fo in ("0", "1"):
            monkeypatch.setenv("VAMPOMI_CG_FOLD", fo)
            out[fo] = run_ranks(monkeypatch, P, N, Mt, fn, timeout=300)
        for a, b in zip(out["0"], out["1"]):
            for k in ("iterations", "cg_iters", "ons_iters", "L"):
                assert a[k] == b[k], (N, k)
            for k in ("x1_hist", "r1_hist", "params"):
                np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=f"{N} {k}")
