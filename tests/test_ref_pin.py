"""The oracle pinned to the REFERENCE's own code: src/data.cpp's
compute_markers_statistics, ATx/dot_product, Ax and read_phen, compiled where
they lie (oracle/Makefile `ref`, oracle/ref_data_harness.cpp).

* tests/golden/ref_data_pin.npz holds the reference's outputs on the files its
  own simulation/data_sim.py wrote and on a ragged generated problem
  (tests/golden/make_ref_golden.py); the oracle must reproduce them here, on
  any host.
* Where the reference is built (oracle/_ref/ref_data: the build container),
  the reference is also run live on further shapes and compared.

Bars: A.x bit for bit (the reference sums each sample over markers in index
order, as the oracle); marker means within 1e-15, scales and A^T.u within
4e-15 relative (the reference's `omp simd reduction`s reassociate those sums:
measured 1e-16..1.1e-15, growing with N); read_phen bit for bit.
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import relerr
from oracle import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ref_data")

import sys  # noqa: E402

sys.path.insert(0, G)
from make_ref_golden import CASES, case_matrix, probe_vectors  # noqa: E402

PIN = np.load(os.path.join(G, "ref_data_pin.npz"))


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference_operators(name):
    X = case_matrix(name)
    M, N = X.shape
    x, u = probe_vectors(N, M)
    for a, tag in ((1.0, ""), (0.7, "_a07")):
        mave, msig = O.marker_stats(X, a)
        assert relerr(mave, PIN[f"{name}_mave{tag}"]) <= 1e-15
        assert relerr(msig, PIN[f"{name}_msig{tag}"]) <= 4e-15
    mave, msig = O.marker_stats(X)
    # the reference's own statistics feed its operators: compare the operators on them
    mr, sr = PIN[f"{name}_mave"], PIN[f"{name}_msig"]
    assert np.array_equal(O.ax(X, mr, sr, x), PIN[f"{name}_ax"])
    assert relerr(O.atx(X, mr, sr, u), PIN[f"{name}_atx"]) <= 4e-15


def test_oracle_read_phen_matches_reference():
    for s in (0, 1):
        y = O.read_phen(os.path.join(G, "datasim.phen"), 100, bool(s))
        assert np.array_equal(y, PIN[f"datasim_phen_std{s}"]), s


def _ref(*args):
    subprocess.run([REF, *map(str, args)], check=True, capture_output=True,
                   env=dict(os.environ, OMP_NUM_THREADS="4"))


@pytest.mark.skipif(not os.path.exists(REF), reason="reference not built here (oracle/Makefile ref)")
@pytest.mark.parametrize("N,M,kind,seed", [(64, 128, 0, 1), (777, 301, 1, 2), (4099, 63, 0, 3), (2, 5, 1, 4)])
def test_reference_live(N, M, kind, seed, tmp_path):
    X = O.generate_markers(seed, kind, N, 0, M)
    xp = str(tmp_path / "X.bin")
    X.tofile(xp)
    x, u = probe_vectors(N, M)
    x.tofile(tmp_path / "x.bin")
    u.tofile(tmp_path / "u.bin")
    _ref("stats", xp, N, M, 1.0, tmp_path / "mave", tmp_path / "msig")
    mr, sr = np.fromfile(tmp_path / "mave"), np.fromfile(tmp_path / "msig")
    mave, msig = O.marker_stats(X)
    assert relerr(mave, mr) <= 1e-15 and relerr(msig, sr) <= 4e-15
    _ref("ax", xp, N, M, tmp_path / "x.bin", tmp_path / "ax")
    assert np.array_equal(O.ax(X, mr, sr, x), np.fromfile(tmp_path / "ax"))
    _ref("atx", xp, N, M, tmp_path / "u.bin", tmp_path / "atx")
    assert relerr(O.atx(X, mr, sr, u), np.fromfile(tmp_path / "atx")) <= 4e-15
