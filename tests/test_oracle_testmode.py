"""CPU check of the --run-mode test restatement (src/main_meth.cpp:112-205,
calc_stdev src/utilities.cpp:183-205) against numpy."""
import numpy as np

from _data import make_problem
from oracle import pyoracle as O


def test_test_metrics_formula():
    N, Mt = 700, 900
    X, y, beta = make_problem(N, Mt, kind=1)
    est = beta * 0.9  # file units: x1_hat / sqrt(N), and y = A(beta sqrt(N)) + noise (tests/_data.py)
    r2, c2 = O.test_metrics(X, y, est)
    mave, msig = O.marker_stats(X)
    z = ((X - mave[:, None]) * msig[:, None]).T @ (est * np.sqrt(N)) / np.sqrt(N)
    sd = np.std(y, ddof=1)
    assert abs(r2 - (1 - ((y - z) ** 2).sum() / (sd * sd * N))) < 1e-12
    assert abs(c2 - np.corrcoef(z, y)[0, 1] ** 2) < 0.05  # not centred: <z,y>/(|z||y|), y ~ mean 0
    assert abs(c2 - (z @ y) ** 2 / ((z @ z) * (y @ y))) < 1e-12
    assert 0.3 < r2 < 1
