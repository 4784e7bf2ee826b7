"""Committed fixtures (tests/golden, made by tests/golden/make_golden.py).

* datasim.*  — written by the reference's own simulation/data_sim.py (seeded):
  they pin the input formats our readers accept.
* oracle_*.npz — regression pins of the CPU oracle (parity unpinned vs the
  reference itself: DESIGN.md §Oracle).
"""
import os

import numpy as np
import pytest

from conftest import relerr
from _data import make_problem
from oracle import pyoracle as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
N_DS, M_DS = 100, 200


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def test_datasim_formats_match_the_reference_layout():
    # data_sim.py:58 packs X.transpose().ravel(): M blocks of N doubles
    X = np.fromfile(os.path.join(G, "datasim.bin"), dtype="<f8").reshape(M_DS, N_DS)
    beta = np.fromfile(os.path.join(G, "datasim_ts.bin"), dtype="<f8")
    raw = O.read_phen(os.path.join(G, "datasim.phen"), N_DS, standardize=False)
    assert raw.shape == (N_DS,) and beta.shape == (M_DS,)
    assert (beta != 0).sum() == int(M_DS * 0.1)  # CM = int(M*lam), data_sim.py:38
    resid = raw - X.T @ beta  # y = X beta + N(0, 1-h2), h2 = 0.8 (data_sim.py:46-47)
    assert 0.05 < resid.var() < 0.5
    assert abs(np.corrcoef(raw, X.T @ beta)[0, 1]) > 0.7
    lines = open(os.path.join(G, "datasim.phen")).read().splitlines()
    assert lines[3].split()[:2] == ["3", "3"]  # "%d %d %0.10f" (data_sim.py:68)


def _check_oracle_case(name, X, y, Mt, beta):
    g = load(f"oracle_{name}.npz")
    r = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=int(g["its"]), stop_criteria_thr=float(g["thr"]))
    assert r["iterations"] == int(g["iterations"])
    assert r["cg_iters"].tolist() == g["cg_iters"].tolist()
    assert r["ons_iters"].tolist() == g["ons_iters"].tolist()
    assert r["L"].tolist() == g["L"].tolist()
    for i, k in enumerate(g["keep_its"]):
        assert relerr(r["x1_hist"][k - 1], g["x1"][i]) < 1e-12
        assert relerr(r["r1_hist"][k - 1], g["r1"][i]) < 1e-12
    assert np.allclose(r["params"], g["params"], rtol=1e-11)
    assert np.allclose(r["metrics"], g["metrics"], rtol=1e-11, equal_nan=True)


def test_oracle_reproduces_golden_datasim():
    X = np.fromfile(os.path.join(G, "datasim.bin"), dtype="<f8").reshape(M_DS, N_DS)
    y = O.read_phen(os.path.join(G, "datasim.phen"), N_DS, True)
    beta = np.fromfile(os.path.join(G, "datasim_ts.bin"), dtype="<f8")
    _check_oracle_case("datasim", X, y, M_DS, beta)


@pytest.mark.parametrize("name", ["c1", "c1_stop"])
def test_oracle_reproduces_golden_c1(name):
    X, y, beta = make_problem(1000, 2000)
    _check_oracle_case(name, X, y, 2000, beta)


@pytest.mark.parametrize("case,fields", [("params", 6), ("metrics", 7)])
def test_golden_csv_byte_contract(case, fields):
    """src/utilities.cpp:366-401: header at offset 0, row `it` at it*strlen(row),
    "%5d" then ", %20.15f" per value, NUL-filled holes."""
    g = load("oracle_c1.npz")
    b = g[f"csv_{case}"].tobytes()
    header = b[: b.index(b"\n") + 1]
    assert header.count(b", ") == fields - 1 and b"\0" not in header
    row_len = 5 + 22 * (fields - 1) + 1
    its = int(g["iterations"])
    assert len(b) == (its + 1) * row_len
    assert b[len(header):row_len] == b"\0" * (row_len - len(header))
    for it in range(1, its + 1):
        row = b[it * row_len:(it + 1) * row_len]
        assert row.endswith(b"\n") and row[:5] == b"%5d" % it
        vals = row[5:-1].split(b", ")[1:]
        assert len(vals) == fields - 1 and all(len(v) == 20 for v in vals)
    if case == "metrics":  # corr(x1, x0) at it 1 is 0/0 -> glibc prints "-nan"
        assert b[row_len:2 * row_len].split(b",")[2].strip() == b"-nan"


def test_golden_prior_csv_header_only():
    # linear model: the prior row write is commented out (src/vamp.cpp:392)
    b = load("oracle_c1.npz")["csv_prior"].tobytes()
    fields = b.decode().strip().split(", ")
    assert fields[:2] == ["iteration", "number of components"]
    assert fields[2:12] == [f"prob{i}" for i in range(10)] and fields[12:] == [f"var{i}" for i in range(10)]
