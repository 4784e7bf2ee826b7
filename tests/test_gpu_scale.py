"""GPU parity at the BASELINE configs' own sizes (VERDICT r01 "configs
untested"), plus the CLI on files the reference itself wrote.

* C3's samples, N = 100,000 methylation-like (configs[2]/[4]):
  - against the oracle at a reduced Mt (the oracle finishes in seconds):
    x1_hat / r1 within 1e-10 norm-relative per iteration, iteration / CG /
    Onsager / mixture counts exact;
  - the full 62,500-marker per-GPU shard (50 GB): the production schedule and
    batch_rhs 3 against batch_rhs 1 (bitwise the reference's sequential
    order, tests/test_gpu_parity.py) within 1e-11, counts equal;
  - the same shard split over two ranks (loopback communicator) against the
    one-rank run.
* C2 (configs[1], N = 10,000 x Mt = 50,000) whole, with the production
  one-pass CG operator (batch_rhs 4), against the oracle for 6 iterations.
* main_meth.exe on tests/golden/datasim.* (written by the reference's
  simulation/data_sim.py) against tests/golden/oracle_datasim.npz.
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import relerr
from _data import make_problem
from test_gpu_sharded import run_ranks

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")


def _run(d, y=None, beta=None, **kw):
    if y is not None:
        d.set_phen(y, standardize=False)
    v = va.Vamp(d, va.VampOptions(**kw), true_signal=beta)
    v.infere(keep_hist=True)
    s = v.summary()
    n = s["iterations"]
    s["x1_hist"], s["r1_hist"] = v.x1_hist[:n, :d.M].copy(), v.r1_hist[:n, :d.M].copy()
    return s


def _counts_equal(a, b):
    assert a["iterations"] == b["iterations"]
    assert list(a["cg_iters"]) == list(b["cg_iters"]), (a["cg_iters"], b["cg_iters"])
    assert list(a["ons_iters"]) == list(b["ons_iters"]), (a["ons_iters"], b["ons_iters"])
    assert list(a["L"]) == list(b["L"])


def test_c3_samples_reduced_markers_vs_oracle():
    N, Mt, its = 100000, 2000, 8
    X, y, beta = make_problem(N, Mt, seed=7, kind=1)
    kw = dict(max_iter=its, stop_criteria_thr=0.0)
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, **kw)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        s = _run(d, y, beta, **kw)
    _counts_equal(s, ref)
    for k in range(its):
        assert relerr(s["x1_hist"][k], ref["x1_hist"][k]) <= 1e-10, k
        assert relerr(s["r1_hist"][k], ref["r1_hist"][k]) <= 1e-10, k
    assert np.allclose(np.array(s["params"]), ref["params"], rtol=1e-9, atol=0)


C3_SHARD = dict(N=100000, Mt=62500, its=6, seed=20250711)


@pytest.fixture(scope="module")
def c3_shard_runs():
    """The full per-GPU C3 shard on one rank, for batch_rhs 1, 3 and the default."""
    c = C3_SHARD
    out = {}
    with va.Data(c["N"], c["Mt"]) as d:
        d.generate(c["seed"], va.GEN_METH)
        beta = d.simulate_phen(c["seed"] + 1, lam=0.1, h2=0.8)
        for b in (1, 3, va.VampOptions().batch_rhs):
            out[b] = _run(d, None, beta, max_iter=c["its"], stop_criteria_thr=0.0, batch_rhs=b)
    out["beta"] = beta
    return out


def test_c3_full_shard_schedules_agree(c3_shard_runs):
    base = c3_shard_runs[1]  # the reference's sequential order, bit for bit (batch_rhs 0 == 1)
    for b in sorted(k for k in c3_shard_runs if k not in (1, "beta")):
        s = c3_shard_runs[b]
        _counts_equal(s, base)
        for k in range(s["iterations"]):
            assert relerr(s["x1_hist"][k], base["x1_hist"][k]) <= 1e-11, (b, k)
            assert relerr(s["r1_hist"][k], base["r1_hist"][k]) <= 1e-11, (b, k)
    assert all(c >= 1 for c in base["cg_iters"])


def test_c3_full_shard_two_ranks(monkeypatch, c3_shard_runs):
    c = C3_SHARD
    one = c3_shard_runs[va.VampOptions().batch_rhs]

    def fn(r, d):
        d.generate(c["seed"], va.GEN_METH)  # index-keyed: each rank generates its own columns
        beta = d.simulate_phen(c["seed"] + 1, lam=0.1, h2=0.8)
        return _run(d, None, beta, max_iter=c["its"], stop_criteria_thr=0.0)

    parts = run_ranks(monkeypatch, 2, c["N"], c["Mt"], fn, timeout=400)
    for p in parts:
        _counts_equal(p, one)
    for k in range(one["iterations"]):
        assert relerr(np.concatenate([p["x1_hist"][k] for p in parts]), one["x1_hist"][k]) <= 1e-12, k
        assert relerr(np.concatenate([p["r1_hist"][k] for p in parts]), one["r1_hist"][k]) <= 1e-12, k


@pytest.fixture(scope="module")
def c2_problem():
    return make_problem(10000, 50000, seed=11)


def test_c2_whole_production_schedule_vs_oracle(c2_problem):
    N, Mt, its = 10000, 50000, 6
    X, y, beta = c2_problem
    kw = dict(max_iter=its, stop_criteria_thr=0.0)
    ref = O.vamp_infere(X, y, Mt, true_signal=beta, **kw)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        s = _run(d, y, beta, **kw)  # batch_rhs default: the one-pass CG operator at this shape
        st = d.stats()
    assert va.VampOptions().batch_rhs == 4 and st.op.launches > 0, "the one-pass operator did not run"
    _counts_equal(s, ref)
    for k in range(its):
        assert relerr(s["x1_hist"][k], ref["x1_hist"][k]) <= 1e-10, k
        assert relerr(s["r1_hist"][k], ref["r1_hist"][k]) <= 1e-10, k


def test_c2_bench_window_vs_oracle_fixture(c2_problem):
    """Iterations 1-25 of C2 on the production schedule (the driver's bench
    times 6-25) against the oracle's run committed in
    tests/golden/oracle_c2_window.npz (made by make_c2_window.py in the build
    container): every iteration's CG / Onsager / mixture counts exact, params
    within 1e-9, the norms and four +-1 projections of x1_hat / r1 within the
    1e-10 norm bar (a projection moves by at most sqrt(M) * ||delta||), and
    the whole x1_hat / r1 vectors at iterations 6, 15 and 25 within 1e-10."""
    import sys

    sys.path.insert(0, G)
    from make_c2_window import probes

    z = np.load(os.path.join(G, "oracle_c2_window.npz"))
    N, Mt, its = int(z["N"]), int(z["Mt"]), int(z["its"])
    X, y, beta = c2_problem
    assert X.shape == (Mt, N)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        s = _run(d, y, beta, max_iter=its, stop_criteria_thr=0.0)
    assert s["iterations"] == its
    assert s["cg_iters"] == z["cg_iters"].tolist() and s["ons_iters"] == z["ons_iters"].tolist()
    assert s["L"] == z["L"].tolist()
    assert np.allclose(np.array(s["params"]), z["params"], rtol=1e-9, atol=0)
    P = probes(Mt)
    for key in ("x1", "r1"):
        h = s[f"{key}_hist"]
        nrm = z[f"{key}_norm"]
        assert np.all(np.abs(np.linalg.norm(h, axis=1) - nrm) <= 1e-10 * nrm), key
        bound = 1e-10 * np.sqrt(Mt) * nrm[:, None]
        assert np.all(np.abs(h @ P.T - z[f"{key}_proj"]) <= bound), key
        for q, k in enumerate(z["keep_its"]):
            assert relerr(h[k - 1], z[key][q]) <= 1e-10, (key, k)
        if f"{key}_blocks" in z:  # (round 6 fixture)
            got, want = block_checks(h, P), z[f"{key}_blocks"]
            nb = want.shape[1]
            # the whole vector's 1e-10 bar spent on one block: its norm moves by at most ||delta||, a
            # projection on a +-1 probe by at most sqrt(block length) * ||delta||
            tol = 1e-10 * nrm[:, None, None] * np.array([1.0, np.sqrt(Mt / nb + 1), np.sqrt(Mt / nb + 1)])[None, None, :]
            bad = np.abs(got - want) > tol
            assert not np.any(bad), (key, np.argwhere(bad)[:5])


def test_cli_on_reference_written_files(tmp_path):
    """main_meth.exe reads the files data_sim.py wrote (marker-major .bin, PLINK
    .phen, _ts.bin) through the device readers and reproduces the oracle's run
    on them: _it_K.bin / _r1_it_K.bin within 1e-10, CSV rows within 1e-9, the
    per-iteration CG / Onsager counts exact."""
    z = np.load(os.path.join(G, "oracle_datasim.npz"))
    its = int(z["its"])
    vars_ = ",".join(repr(v) for v in O.DEFAULT_VARS)
    probs = ",".join(repr(v) for v in O.DEFAULT_PROBS)
    r = subprocess.run([va.CLI_PATH, "--meth-file", os.path.join(G, "datasim.bin"),
                        "--phen-file", os.path.join(G, "datasim.phen"),
                        "--true-signal-file", os.path.join(G, "datasim_ts.bin"), "--N", "100", "--Mt", "200",
                        "--iterations", str(its), "--stop-criteria-thr", str(float(z["thr"])), "--vars", vars_,
                        "--probs", probs, "--seed", str(0x5EED5EED), "--out-dir", str(tmp_path), "--out-name", "g"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    counts = [tuple(map(int, m)) for m in re.findall(r"it \d+: CG iterations (\d+), onsager CG iterations (\d+)",
                                                     r.stdout)]
    assert [c[0] for c in counts] == z["cg_iters"].tolist()
    assert [c[1] for c in counts] == z["ons_iters"].tolist()
    # per iteration, as the reference prints them (src/vamp.cpp:396-401)
    times = [float(t) for t in re.findall(r"Total iteration time = ([0-9.eE+-]+)", r.stdout)]
    so_far = [float(t) for t in re.findall(r"Total computation time so far = ([0-9.eE+-]+)", r.stdout)]
    assert len(times) == its and len(so_far) == its and all(t > 0 for t in times)
    assert np.allclose(np.cumsum(times), so_far, rtol=1e-4)
    # and the solves' share of it ("CG took", "onsager took", src/vamp.cpp:313-316, :326-333)
    solves = [float(t) for t in re.findall(r"CG and onsager \(one pass over the markers per step for both\) took "
                                           r"([0-9.eE+-]+) seconds", r.stdout)]
    assert len(solves) == its and all(0 < s <= t for s, t in zip(solves, times))
    for q, k in enumerate(z["keep_its"]):
        x1 = np.fromfile(tmp_path / f"g_it_{k}.bin", dtype="<f8")
        r1 = np.fromfile(tmp_path / f"g_r1_it_{k}.bin", dtype="<f8")
        assert relerr(x1, z["x1"][q]) <= 1e-10, k
        assert relerr(r1, z["r1"][q]) <= 1e-10, k

    def rows(b):
        lines = bytes(b).decode().replace("\0", "").splitlines()[1:]
        return np.array([[float(t) for t in ln.split(",")] for ln in lines if ln.strip()])

    for name in ("params", "metrics"):
        got = rows(open(tmp_path / f"g_{name}.csv", "rb").read())
        want = rows(z[f"csv_{name}"])
        assert got.shape == want.shape
        assert np.allclose(got, want, rtol=1e-9, atol=1e-12, equal_nan=True), name


@pytest.mark.parametrize("name", ["datasim", "gen"])
def test_device_operators_vs_reference_outputs(name):
    """Device marker statistics, A.x and A^T.u against the REFERENCE's own
    src/data.cpp outputs (tests/golden/ref_data_pin.npz, tests/test_ref_pin.py):
    1e-13 relative (fixed-order device reductions vs the reference's OpenMP ones)."""
    import sys

    sys.path.insert(0, G)
    from make_ref_golden import case_matrix, probe_vectors

    pin = np.load(os.path.join(G, "ref_data_pin.npz"))
    X = case_matrix(name)
    M, N = X.shape
    x, u = probe_vectors(N, M)
    for a, tag in ((1.0, ""), (0.7, "_a07")):
        with va.Data(N, M, alpha_scale=a) as d:
            if name == "datasim":
                d.read_methylation_data(os.path.join(G, "datasim.bin"))  # the device reader on the reference's file
            else:
                d.load_meth(X)
            assert relerr(d.get_mave(), pin[f"{name}_mave{tag}"]) <= 1e-13
            assert relerr(d.get_msig(), pin[f"{name}_msig{tag}"]) <= 1e-13
            if a == 1.0:
                assert relerr(d.Ax(x), pin[f"{name}_ax"]) <= 1e-13
                assert relerr(d.ATx(u), pin[f"{name}_atx"]) <= 1e-13
                if name == "datasim":
                    for s in (0, 1):
                        d.read_phen(os.path.join(G, "datasim.phen"), standardize=bool(s))
                        assert np.array_equal(d.get_phen(), pin[f"datasim_phen_std{s}"]), s


def test_c3_full_shard_window_vs_oracle_fixture():
    """The WHOLE per-GPU C3 shard (N = 100,000 x 62,500 methylation-like
    markers, 50 GB; eight of them are configs[2]) on the production schedule
    (the team operator at T = 32, the head start), iterations 1-12 -- the
    window `bench.py --config c3` times is 3-12 -- against the CPU oracle's run
    of the same problem committed in tests/golden/oracle_c3_window.npz (made
    by make_c3_window.py in the build container: X from the index-keyed
    generator, bit-identical here, y / beta stored).  Every iteration: CG /
    Onsager / mixture counts exact, params within 1e-9, the norms and four
    +-1 projections of x1_hat / r1 within the 1e-10 norm bar (a projection
    moves by at most sqrt(M) * ||delta||), and per block of 256 contiguous
    markers its norm and two +-1 projections within the same bar on the
    block (a localized error moves its block's checks to first order);
    the whole x1_hat / r1 at iterations 3, 7 and 12 within 1e-10
    (src/vamp.cpp:110-438)."""
    import sys

    sys.path.insert(0, G)
    from make_c2_window import probes
    from make_c3_window import block_checks

    z = np.load(os.path.join(G, "oracle_c3_window.npz"))
    N, Mt, its = int(z["N"]), int(z["Mt"]), int(z["its"])
    with va.Data(N, Mt) as d:
        d.generate(int(z["seed"]), int(z["kind"]))
        s = _run(d, z["y"], z["beta"], max_iter=its, stop_criteria_thr=0.0)
        st = d.stats()
    assert st.op.launches > 0, "the one-pass team operator did not run"
    assert s["iterations"] == its
    assert s["cg_iters"] == z["cg_iters"].tolist() and s["ons_iters"] == z["ons_iters"].tolist()
    assert s["L"] == z["L"].tolist()
    assert np.allclose(np.array(s["params"]), z["params"], rtol=1e-9, atol=0)
    P = probes(Mt)
    for key in ("x1", "r1"):
        h = s[f"{key}_hist"]
        nrm = z[f"{key}_norm"]
        assert np.all(np.abs(np.linalg.norm(h, axis=1) - nrm) <= 1e-10 * nrm), key
        bound = 1e-10 * np.sqrt(Mt) * nrm[:, None]
        assert np.all(np.abs(h @ P.T - z[f"{key}_proj"]) <= bound), key
        for q, k in enumerate(z["keep_its"]):
            assert relerr(h[k - 1], z[key][q]) <= 1e-10, (key, k)
