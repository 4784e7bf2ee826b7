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
