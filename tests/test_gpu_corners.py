"""GPU parity in corners the default runs do not reach: the PCG entry point
with a warm start and with the Onsager stop (vamp::precondCG_solver,
src/vamp.cpp:664-757, restated in numpy below), and VAMP runs with very few
markers (one A.x chunk, fewer markers than one A^T wave group) and with N
much smaller or larger than Mt."""
import numpy as np
import pytest

from conftest import relerr
from _data import make_problem

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)


def pcg_numpy(X, mave, msig, v, mu0, tau, gam2, onsager, max_iter, tol):
    """precondCG_solver, line by line (numpy dots; the engine's differ only in
    summation order)."""
    N = X.shape[1]

    def lmmse(u):
        if not np.any(u):
            return np.zeros_like(u)
        return tau * O.atx(X, mave, msig, O.ax(X, mave, msig, u)) + gam2 * u

    diag = tau * (N - 1) / N + gam2
    mu = mu0.copy()
    r = v - lmmse(mu)
    z = r / diag
    p = z.copy()
    prev, its = 0.0, 0
    norm_v = np.sqrt(v @ v)
    for i in range(max_iter):
        its = i + 1
        d = lmmse(p)
        rz = r @ z
        alpha = rz / (d @ p)
        mu = mu + alpha * p
        if onsager:
            ons = gam2 * (v @ mu)
            rel = abs((ons - prev) / ons) if ons != 0 else 1
            if rel < 1e-8:
                break
            prev = ons
        beta = rz ** -1
        r = r - d * alpha
        z = r / diag
        beta *= r @ z
        p = z + beta * p
        if np.sqrt(r @ r) / norm_v < tol:
            break
    return mu, its


@pytest.mark.parametrize("warm,onsager", [(False, False), (True, False), (False, True), (True, True)])
def test_pcg_entry_point(warm, onsager):
    N, Mt = 700, 1300
    X, _, _ = make_problem(N, Mt, seed=9)
    mave, msig = O.marker_stats(X)
    rng = np.random.default_rng(4)
    v = rng.normal(size=Mt)
    mu0 = rng.normal(size=Mt) * 0.1 if warm else np.zeros(Mt)
    tau, gam2 = 1.7, 0.4
    ref, its = pcg_numpy(X, mave, msig, v, mu0, tau, gam2, onsager, 200, 1e-9)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        mu, it = d.pcg(v, tau, gam2, mu0=mu0 if warm else None, onsager=onsager, tol=1e-9, max_iter=200)
    assert it == its
    assert relerr(mu, ref) < 1e-11


@pytest.mark.parametrize("N,Mt", [(500, 40), (300, 7), (64, 3000), (6000, 120)])
def test_vamp_shapes(N, Mt):
    X, y, beta = make_problem(N, Mt, seed=2)
    kw = dict(max_iter=8, stop_criteria_thr=0.0)
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, **kw)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        v = va.Vamp(d, va.VampOptions(**kw), true_signal=beta)
        v.infere(keep_hist=True)
        s = v.summary()
        x1 = v.x1_hist[: s["iterations"], : d.M]
    assert s["cg_iters"] == ref["cg_iters"].tolist() and s["ons_iters"] == ref["ons_iters"].tolist()
    for k in range(s["iterations"]):
        assert relerr(x1[k], ref["x1_hist"][k]) <= 1e-10, k


@pytest.mark.parametrize("em,lv,merge", [(1, 1, 0.5), (3, 1, 0.5), (4, 0, 0.0), (2, 1, 5.0)])
def test_update_prior_entry_point(em, lv, merge):
    N, Mt = 900, 2100
    X, _, _ = make_problem(N, Mt, seed=12)
    rng = np.random.default_rng(em)
    r1 = np.concatenate([rng.normal(size=Mt - 300) * 0.02, rng.normal(size=300) * 0.4])
    vars_s = np.array(O.DEFAULT_VARS) * N
    po, vo = O.update_prior(r1, 35.0, O.DEFAULT_PROBS, vars_s, N, EM_max_iter=em, learn_vars=lv, merge_vars_thr=merge)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        p, v = d.update_prior(r1, 35.0, O.DEFAULT_PROBS, vars_s, EM_max_iter=em, learn_vars=lv, merge_vars_thr=merge)
    assert len(p) == len(po)
    assert np.allclose(p, po, rtol=1e-12, atol=0) and np.allclose(v, vo, rtol=1e-12, atol=0)


def test_device_memory_plan_matches_the_allocations(tmp_path):
    """vampomi_dev_mem_plan (the CPU-side budget tests/test_op_plan.py checks
    for c3full at n = 2, 4, 8) against the device memory a C2-sized context
    really takes during a run with the team operator and the writer on."""
    import ctypes as C

    import torch

    N, Mt = 10000, 50000
    torch.cuda.init()
    free0, _ = torch.cuda.mem_get_info()
    with va.Data(N, Mt) as d:
        d.generate(3, va.GEN_GAUSS)
        beta = d.simulate_phen(4)
        v = va.Vamp(d, va.VampOptions(max_iter=2, stop_criteria_thr=0.0, out_dir=str(tmp_path), out_name="m"),
                    true_signal=beta)
        v.begin()
        v.step()
        free1, _ = torch.cuda.mem_get_info()
        v.step()
        v.end()
        cus = torch.cuda.get_device_properties(0).multi_processor_count
    b = C.c_int64()
    assert va.load().vampomi_dev_mem_plan(N, Mt, 1, 0, cus, 0, 1, C.byref(b)) == 0
    used = free0 - free1
    assert abs(used - b.value) <= 256 * 2**20 + 0.02 * b.value, (used / 2**20, b.value / 2**20)


def test_read_ceiling_hook():
    """vampomi_dev_read_ceiling (the same-run roofline of bench.py): a pure read
    stream of the resident matrix, the faster of its two shapes; plausible
    rates, bytes within the matrix, no effect on the operators' results; a
    matrix too small for either shape is an argument error, not a launch."""
    N, Mt = 10000, 5000
    X = O.generate_markers(3, 0, N, 0, Mt)
    x = np.random.default_rng(1).normal(size=Mt)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        before = d.Ax(x)
        c = d.read_ceiling(5)
        assert 0 < c["bytes"] <= 8.0 * Mt * ((N + 15) // 16 * 16)
        assert 1000.0 < c["GBs"] < 10000.0, c
        assert np.array_equal(d.Ax(x), before)
    with va.Data(100, 10) as d:
        d.load_meth(O.generate_markers(3, 0, 100, 0, 10))
        with pytest.raises(va.VampomiError):
            d.read_ceiling(3)
