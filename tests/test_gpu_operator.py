"""The one-pass CG operator (kernels.h: atax) on its own, every plan.

One application computes, for K <= 2 systems, q = A r/diag [+ beta q_old]
and p [= z + beta p] (the fused CG direction update), then from ONE read of X

    d = tau * A^T q + gam2 * p        (lmmse_mult, src/vamp.cpp:645-662)
    A d                                (data::Ax, src/data.cpp:340-373)
    <d, p>

with A = (X - mave) * msig / sqrt(N) (data::ATx src/data.cpp:294-333).
Checked against numpy on the explicit matrix (norm-relative 1e-12), for the
whole-column kernel and every team plan (team sizes 1..32, each hand-off
configuration) that exists for the shape, including odd N (the zero pad row)
and shapes where the last team member holds a short tile.  Team results
are also bitwise repeatable.
"""
import numpy as np
import pytest

from conftest import relerr

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker: the generator and marker statistics)

SHAPES = [(1000, 3000, 0), (10000, 4000, 0), (50001, 1500, 1), (100000, 600, 1),
          (50001, 7, 0)]  # fewer markers than teams: empty teams
# every configuration of atax_team.hip's kTmCfg (0-6) at every team size
CANDIDATES = [0] + [T * 10 + c for T in (1, 2, 4, 8, 16, 32) for c in range(7)]


def _ref(X, mave, msig, ar, qo, p, z, beta, diag, tau, gam2):
    N = X.shape[1]
    Xc = X - mave[:, None]
    q = ar / diag
    pp = p.copy()
    if z is not None:
        q = q + beta[:, None] * qo
        pp = z + beta[:, None] * p
    t = (Xc @ q.T).T * msig[None, :] / np.sqrt(N)
    d = tau * t + gam2 * pp
    ad = (Xc.T @ (msig[None, :] * d).T).T / np.sqrt(N)
    return d, ad, np.sum(d * pp, axis=1)


@pytest.fixture(scope="module", params=SHAPES, ids=lambda s: "N%d_M%d" % s[:2])
def problem(request):
    N, Mt, kind = request.param
    X = O.generate_markers(11, kind, N, 0, Mt)
    mave, msig = O.marker_stats(X)
    d = va.Data(N, Mt)
    d.load_meth(X)
    yield N, Mt, X, mave, msig, d
    d.close()


def _plans(d):
    ok = []
    for v in CANDIDATES:
        try:
            d.set_variant(3, v)
        except va.VampomiError:
            continue
        ok.append(v)
    d.set_variant(3, -1)
    return ok


def test_operator_every_plan_vs_numpy(problem):
    N, Mt, X, mave, msig, d = problem
    plans = _plans(d)
    assert plans, "no operator plan for N=%d" % N
    if N > 20000:
        assert all(v >= 10 for v in plans), plans  # whole columns cannot hold these N
        assert any(v >= 20 for v in plans), plans  # teams with a hand-off do
    rng = np.random.default_rng(N)
    diag, tau, gam2 = 1.7, 0.9, 0.35
    for K in (1, 2):
        ar, qo = rng.normal(size=(K, N)), rng.normal(size=(K, N))
        p, z = rng.normal(size=(K, Mt)), rng.normal(size=(K, Mt))
        beta = rng.uniform(0.1, 0.9, size=K)
        for fused in (False, True):
            zz, qq, bb = (z, qo, beta) if fused else (None, None, None)
            rd, rad, rdp = _ref(X, mave, msig, ar, qq, p, zz, bb, diag, tau, gam2)
            for v in plans:
                d.set_variant(3, v)
                gd, gad, gdp = d.op_apply(ar, p, diag, tau, gam2, z=zz, qo=qq, beta=bb)
                what = "plan %d (%s) K=%d fused=%d" % (v, d.kernel_name(3, K), K, fused)
                assert relerr(gd, rd) < 1e-12, (what, relerr(gd, rd))
                assert relerr(gad, rad) < 1e-12, (what, relerr(gad, rad))
                assert np.allclose(gdp, rdp, rtol=1e-12, atol=0), (what, gdp, rdp)
    d.set_variant(3, -1)


def test_operator_team_plans_bitwise_repeatable(problem):
    N, Mt, X, mave, msig, d = problem
    plans = [v for v in _plans(d) if v >= 20] or _plans(d)
    rng = np.random.default_rng(1)
    ar, p = rng.normal(size=(2, N)), rng.normal(size=(2, Mt))
    for v in plans[:3]:
        d.set_variant(3, v)
        a = d.op_apply(ar, p, 1.0, 1.0, 0.5)
        b = d.op_apply(ar, p, 1.0, 1.0, 0.5)
        for x, y in zip(a, b):
            assert np.array_equal(x, y), v
    d.set_variant(3, -1)


def test_team_launches_from_two_contexts_on_one_gpu():
    """Two contexts of one process on the same GPU (ranks as threads, as the
    loopback tests run them) launching team grids at the same time: each
    grid needs every CU, so the launches are ordered on the device
    (engine.cpp team_launch); without that the two grids can each hold part
    of the CUs and time out."""
    import threading

    N, Mt = 50001, 1500
    X = O.generate_markers(5, 1, N, 0, Mt)
    mave, msig = O.marker_stats(X)
    rng = np.random.default_rng(3)
    ar, p = rng.normal(size=(2, N)), rng.normal(size=(2, Mt))
    ref = _ref(X, mave, msig, ar, None, p, None, None, 1.3, 0.8, 0.4)
    errs, outs = [], []

    def work():
        try:
            with va.Data(N, Mt) as d:
                d.load_meth(X)
                for _ in range(6):
                    outs.append(d.op_apply(ar, p, 1.3, 0.8, 0.4))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=work) for _ in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a context is stuck"
    assert not errs, errs
    assert len(outs) == 12
    for gd, gad, gdp in outs:
        assert relerr(gd, ref[0]) < 1e-12 and relerr(gad, ref[1]) < 1e-12
        assert np.array_equal(gd, outs[0][0]) and np.array_equal(gad, outs[0][1])



@pytest.mark.parametrize("N,Mt", [(20000, 2000), (50001, 300), (100000, 600), (50001, 7), (33000, 1000)])
def test_ax_team_plan_vs_numpy(N, Mt):
    """data::Ax (src/data.cpp:340-373) on the team plan (ax_team_kernel, the
    default above ~16k samples) against numpy on the explicit matrix and
    against the tile plan (variant 0): odd N (the zero pad row), fewer markers
    than teams (empty teams write zero slots), every team size the plan picks;
    bitwise repeatable."""
    X = O.generate_markers(7, 1, N, 0, Mt)
    mave, msig = O.marker_stats(X)
    x = np.random.default_rng(5).normal(size=Mt)
    ref = ((X - mave[:, None]) * (msig * x)[:, None]).sum(axis=0) / np.sqrt(N)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        assert d.kernel_name(0, 1).startswith("ax_team_kernel<")
        a = d.Ax(x)
        b = d.Ax(x)
        d.set_variant(0, 0)
        assert d.kernel_name(0, 1).startswith("ax_partial_kernel<")
        tile = d.Ax(x)
    assert relerr(a, ref) < 1e-13
    assert relerr(a, tile) < 1e-13
    assert np.array_equal(a, b)
