"""GPU parity of --run-mode test (src/main_meth.cpp:112-205): R2 test and the
squared z correlation per estimate file, and the _test.csv layout."""
import os
import subprocess

import numpy as np
import pytest

from _data import make_problem

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)


@pytest.mark.parametrize("N,Mt,kind", [(700, 900, 1), (4099, 333, 0)])
def test_test_metrics_parity(N, Mt, kind):
    X, y, beta = make_problem(N, Mt, kind=kind)
    with va.Data(N, Mt) as d:
        d.load_meth(X)
        d.set_phen(y, standardize=False)
        for s in (0.0, 0.5, 0.9, 1.3):
            est = beta * s
            r2, c2 = d.test_metrics(est)
            ro, co = O.test_metrics(X, y, est)
            assert abs(r2 - ro) <= 1e-12 * max(1.0, abs(ro))
            if s == 0.0:
                assert np.isnan(c2) and np.isnan(co)  # z = 0: 0/0
            else:
                assert abs(c2 - co) <= 1e-12 * abs(co)


def test_cli_test_mode(tmp_path):
    N, Mt, Nt, its = 500, 800, 300, 4
    X, y, beta = make_problem(N, Mt, seed=3)
    Xt = O.generate_markers(77, 0, Nt, 0, Mt)  # held-out samples: another generator stream, same effects
    mave, msig = O.marker_stats(Xt)
    yt = O.standardize_phen(O.ax(Xt, mave, msig, beta * np.sqrt(Nt)) + 0.3 * np.sin(np.arange(Nt)))
    for name, A, v in (("train", X, y), ("test", Xt, yt)):
        A.astype("<f8").tofile(tmp_path / f"{name}.bin")
        (tmp_path / f"{name}.phen").write_text("".join("%d %d %0.10f\n" % (i, i, t) for i, t in enumerate(v)))
    out = tmp_path / "out"
    out.mkdir()
    cli = va.CLI_PATH
    r = subprocess.run([cli, "--meth-file", str(tmp_path / "train.bin"), "--phen-file", str(tmp_path / "train.phen"),
                        "--N", str(N), "--Mt", str(Mt), "--out-dir", str(out), "--out-name", "ex", "--iterations",
                        str(its), "--stop-criteria-thr", "0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    # the text form of one estimate file (read_vec_from_file, src/utilities.cpp:104-122)
    e3 = np.fromfile(out / "ex_it_3.bin", dtype="<f8")
    (out / "txt_it_3.txt").write_text("\n".join("%.17g" % v for v in e3))
    for est_name, rng, csv in (("ex_it_1.bin", "1,4", "ex_test.csv"), ("txt_it_3.txt", "3,3", "tx_test.csv")):
        r = subprocess.run([cli, "--run-mode", "test", "--meth-file-test", str(tmp_path / "test.bin"),
                            "--phen-file-test", str(tmp_path / "test.phen"), "--N-test", str(Nt), "--Mt", str(Mt),
                            "--N", str(N), "--estimate-file", str(out / est_name), "--test-iter-range", rng,
                            "--out-dir", str(out), "--out-name", csv[:2]], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        b = (out / csv).read_bytes()
        assert b.startswith(b"iteration, R2 test, z correlation test\n")
        lo, hi = map(int, rng.split(","))
        row_len = 5 + 22 * 2 + 1
        yo = O.read_phen(str(tmp_path / "test.phen"), Nt, True)
        for it in range(lo, hi + 1):
            row = b[it * row_len:(it + 1) * row_len].decode()
            f = [float(t) for t in row.split(",")]
            assert int(f[0]) == it
            est = np.fromfile(out / f"ex_it_{it}.bin", dtype="<f8")
            ro, co = O.test_metrics(Xt, yo, est)
            assert abs(f[1] - ro) <= 2e-15 + 1e-12 * abs(ro)
            if it == 1:  # x1_hat = 0 at iteration 1: z = 0, the correlation is 0/0 (-nan in the file)
                assert np.isnan(f[2]) and np.isnan(co)
            else:
                assert abs(f[2] - co) <= 2e-15 + 1e-12 * abs(co)
