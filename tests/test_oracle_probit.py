"""CPU checks of the probit restatement (oracle/vamp_oracle.c, infere_bin_class,
src/vamp_probit.cpp) — independent formulas (scipy) and the committed golden
fixtures.  Parity vs the reference itself is unpinned."""
import math
import os

import numpy as np
import pytest
import scipy.special as sp
from scipy.stats import norm

from conftest import relerr
from _data import make_problem
from oracle import pyoracle as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_erfcx_matches_scipy_and_keeps_the_reference_clamps():
    xs = np.concatenate([np.linspace(-10, 10, 4001), [-1e-300, 0.0, 1e-300, -9.999999, 9.999999]])
    for x in xs:
        # x < 0: exp(x^2) amplifies the rounding of x^2 by 2x^2 (both libraries)
        tol = 2e-15 + (4 * x * x * 1.2e-16 if x < 0 else 0.0)
        assert abs(O.erfcx(x) - sp.erfcx(x)) <= tol * sp.erfcx(x), x
    # src/utilities.cpp:295-298: +inf below -10, lowest() above 10
    assert O.erfcx(-10.0000001) == math.inf
    assert O.erfcx(10.0000001) == -np.finfo(np.float64).max
    assert math.isnan(O.erfcx(math.nan))


@pytest.mark.parametrize("tau1", [1e-6, 0.05, 1.0, 37.0])
def test_probit_denoiser_is_the_truncated_gaussian_mean(tau1):
    """g1_bin_class(p) = p + s*phi(sc)/Phi(sc)/(tau1*sqrt(1+1/tau1)), c = p/sqrt(1+1/tau1),
    s = 2y-1; g1d_bin_class is its derivative in p (src/vamp_probit.cpp:469-488)."""
    sq = math.sqrt(1 + 1 / tau1)
    for y in (0.0, 1.0):
        s = 2 * y - 1
        for p in np.linspace(-6, 6, 121) * sq:
            x = s * p / sq
            ref = p + s * math.exp(norm.logpdf(x) - norm.logcdf(x)) / tau1 / sq
            assert abs(O.g1_bin(p, tau1, y) - ref) <= 1e-12 * max(1.0, abs(ref)), (p, y)
            h = 1e-5 * sq
            fd = (O.g1_bin(p + h, tau1, y) - O.g1_bin(p - h, tau1, y)) / (2 * h)
            assert abs(O.g1d_bin(p, tau1, y) - fd) < 1e-6
            assert -1e-12 <= O.g1d_bin(p, tau1, y) <= 1 + 1e-12


def test_probit_p1_is_index_keyed_standard_normal():
    a = O.probit_p1(9, 20000)
    assert np.array_equal(a[:100], O.probit_p1(9, 100))
    assert abs(a.mean()) < 0.03 and abs(a.std() - 1) < 0.03
    assert not np.array_equal(a[:100], O.probit_p1(10, 100))


def _row_len(n):
    return 5 + 22 * n + 1


@pytest.mark.parametrize("name", ["probit_c1", "probit_c1_stop"])
def test_oracle_reproduces_golden_probit(name, tmp_path):
    g = np.load(os.path.join(G, f"oracle_{name}.npz"), allow_pickle=False)
    X, y, beta = make_problem(1000, 2000)
    yb = (y > 0).astype(np.float64)
    r = O.vamp_infere(X, yb, 2000, true_signal=beta, max_iter=int(g["its"]), stop_criteria_thr=float(g["thr"]),
                      model="bin_class", out_dir=str(tmp_path), out_name="p")
    assert r["iterations"] == int(g["iterations"])
    for k in ("cg_iters", "ons_iters", "L"):
        assert r[k].tolist() == g[k].tolist(), k
    for i, k in enumerate(g["keep_its"]):
        assert relerr(r["x1_hist"][k - 1], g["x1"][i]) < 1e-12
        assert relerr(r["r1_hist"][k - 1], g["r1"][i]) < 1e-12
    assert np.allclose(r["params"], g["params"], rtol=1e-11)
    assert np.allclose(r["metrics"], g["metrics"], rtol=1e-11, equal_nan=True)
    for k in ("params", "metrics", "prior"):
        assert (tmp_path / f"p_{k}.csv").read_bytes() == g[f"csv_{k}"].tobytes(), k


def test_probit_csv_byte_contract():
    """infere_bin_class writes no header (setup_io creates empty files) and
    row `it` at it*strlen(row): 8 params, 12 metrics, and prior rows whose
    length follows L, so later shorter rows overlap earlier longer ones."""
    g = np.load(os.path.join(G, "oracle_probit_c1.npz"), allow_pickle=False)
    its = int(g["iterations"])
    for case, n in (("params", 8), ("metrics", 12)):
        b = g[f"csv_{case}"].tobytes()
        rl = _row_len(n)
        assert len(b) == (its + 1) * rl and b[:rl] == b"\0" * rl
        for it in range(1, its + 1):
            row = b[it * rl:(it + 1) * rl]
            assert row[:5] == b"%5d" % it and row.endswith(b"\n")
    # confusion counts are integers summing to N; accuracy = (TP+TN)/N
    m = g["metrics"]
    for o in (0, 6):
        assert np.all(m[:, o:o + 4].sum(axis=1) == 1000)
        assert np.allclose(m[:, o + 4], (m[:, o] + m[:, o + 1]) / 1000)
    # prior: replay the writes of (L, probs, vars) rows
    pr = g["prior"]
    buf = bytearray()
    for it in range(1, its + 1):
        L = int(pr[it - 1, 0])
        vals = pr[it - 1, :1 + 2 * L]  # L, probs[L], vars[L] (packed, zero padded)
        row = ("%5d" % it + "".join(", %20.15f" % v for v in vals) + "\n").encode()
        off = it * len(row)
        if len(buf) < off + len(row):
            buf.extend(b"\0" * (off + len(row) - len(buf)))
        buf[off:off + len(row)] = row
    assert bytes(buf) == g["csv_prior"].tobytes()


def test_probit_learns_the_signal():
    g = np.load(os.path.join(G, "oracle_probit_c1.npz"), allow_pickle=False)
    m = g["metrics"]
    assert m[-1, 10] > 0.9 and m[-1, 11] > 0.7  # accuracy of x2, corr(x2, beta)
    assert np.isnan(m[0, 5])  # x1 = 0 at iteration 1: corr 0/0


def _wave64(v):
    t = list(v)
    o = 32
    while o:
        for l in range(o):
            t[l] = t[l] + t[l + o]
        o >>= 1
    return t[0]


def _block256(th):
    return ((_wave64(th[:64]) + _wave64(th[64:128])) + _wave64(th[128:192])) + _wave64(th[192:256])


def _dev_red_py(a, b, nblk):
    """kernels.hip's grouping of a reduction (dots_part, block_put_sums, red_final), in Python floats."""
    n, stride = len(a), nblk * 256
    part = []
    for bk in range(nblk):
        th = []
        for t in range(256):
            acc = 0.0
            for e in range(bk * 256 + t, n, stride):
                acc += float(a[e]) * float(b[e])
            th.append(acc)
        part.append(_block256(th))
    th = []
    for t in range(256):
        acc = 0.0
        for bk in range(t, nblk, 256):
            acc += part[bk]
        th.append(acc)
    return _block256(th)


def test_association_modes():
    """The oracle's association modes (vamp_oracle.c, the probit bar's
    measurement): the default is orc_dot; DEVICE groups a sum exactly as
    kernels.hip's reductions do (checked against a Python restatement of
    dots_part / block_put_sums / red_final, bit for bit) and <d,p> as the team
    operator does; REFRUN with one thread is the reference's sequential loop
    and with several a reordering of the same chunk sums."""
    import ctypes as C

    lib = O.load()
    P = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    rng = np.random.default_rng(11)
    for n in (1, 300, 5000, 70001):
        a, b = rng.normal(size=n), rng.normal(size=n)
        O.set_assoc()
        assert lib.orc_assoc_dot(P(a), P(b), n, 0) == lib.orc_dot(P(a), P(b), n)
        O.set_assoc(O.ASSOC_DEVICE, 16, 256)
        if n <= 5000:
            nblk = max(1, min(1024, -(-n // 512)))
            assert lib.orc_assoc_dot(P(a), P(b), n, 0) == _dev_red_py(a, b, nblk), n
            assert lib.orc_assoc_dot(P(a), P(b), n, 3) == _dev_red_py(a, b, -(-n // 256)), n  # the EM round's grid
        O.set_assoc(O.ASSOC_REFRUN, 1, 0, 5)
        seq = 0.0
        for i in range(n):
            seq += float(a[i]) * float(b[i])
        assert lib.orc_assoc_dot(P(a), P(b), n, 0) == seq
        O.set_assoc(O.ASSOC_REFRUN, 8, 0, 5)
        got = {lib.orc_assoc_dot(P(a), P(b), n, 0) for _ in range(16)}
        assert all(abs(g - seq) <= 1e-12 * (np.sum(np.abs(a * b)) + 1e-300) for g in got)
        if n >= 5000:
            assert len(got) > 1  # the arrival order differs from call to call
    O.set_assoc()
    # <d, p> of the operator: member-owned columns per workgroup, lanes over workgroups, butterfly
    M = 4099
    d, p = rng.normal(size=M), rng.normal(size=M)
    for T, grid in ((16, 256), (2, 256), (1, 256)):
        nteams = grid // T
        part = []
        for bk in range(grid):
            g, member = bk >> 3, (bk >> 3) % T
            team = g // T + (nteams >> 3) * (bk & 7)
            if T > 1:
                cols = [team + m * nteams for m in range(max(0, -(-(M - team) // nteams))) if (m & (T - 1)) == member]
            else:
                cols = range(team * M // nteams, (team + 1) * M // nteams)
            acc = 0.0
            for c in cols:
                acc += float(d[c]) * float(p[c])
            part.append(acc)
        lanes = []
        for l in range(64):
            acc = 0.0
            for bk in range(l, grid, 64):
                acc += part[bk]
            lanes.append(acc)
        assert lib.orc_dev_dp(P(d), P(p), M, T, grid) == _wave64(lanes), T
