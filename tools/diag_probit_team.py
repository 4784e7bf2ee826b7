"""Diagnostic: probit prior-row errors against the oracle at N = 12,000 (team
operator), per iteration, for batch_rhs 3 (two passes per CG step) and 4."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from _data import make_problem, oracle_with_spread  # noqa: E402
import test_gpu_probit as T  # noqa: E402

N, Mt = 12000, 1500
X, y, beta = make_problem(N, Mt)
y = (y > 0).astype(np.float64)
ref, spread = oracle_with_spread(X, y, beta, Mt, max_iter=8, stop_criteria_thr=0.0, model="bin_class")
po = ref["prior"]
tol = np.maximum(1e-9, 10 * np.max(spread["params"], axis=1, keepdims=True))
print("spread params max per it", np.max(spread["params"], axis=1))
for br in (3, 4):
    s = T._gpu_probit(X, y, beta, Mt, max_iter=8, stop_criteria_thr=0.0, batch_rhs=br)
    pg = np.array(s["prior"])
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = np.where(po != 0, np.abs(pg - po) / np.abs(po), np.abs(pg - po))
    print("batch_rhs", br, "cg", s["cg_iters"], "L", s["L"])
    for i in range(pg.shape[0]):
        bad = np.where(np.abs(pg[i] - po[i]) > tol[i] * np.abs(po[i]) + 1e-300)[0]
        print(" it", i + 1, "max rel %.2e tol %.2e" % (np.nanmax(rel[i]), tol[i, 0]), "bad cols", bad[:8],
              "vals", pg[i, bad[:3]], po[i, bad[:3]])
