"""C2 bench-window fixture: the CPU oracle's run of the C2 problem
(BASELINE configs[1], N = 10,000 x Mt = 50,000 i.i.d. Gaussian, tests/_data.py
make_problem seed 11) over iterations 1-25, the window the driver's bench
times (--warmup 5 --steps 20: iterations 6-25).

Stored (tests/golden/oracle_c2_window.npz, ~2.5 MB):
* x1_hat and r1 (the _it_K.bin / _r1_it_K.bin values, x / sqrt(N)) at the
  iterations in KEEP_ITS;
* for EVERY iteration: the norms of x1 / r1, their projections on four fixed
  +-1 probe vectors, params, metrics, CG / Onsager / mixture-size counts.

The inputs are regenerated bit for bit from the index-keyed generators on any
host, so only outputs are stored.  Run in the build container (OpenMP over its
cores; the oracle's reductions reassociate with the thread count at the 1e-15
level, far inside the 1e-10 bar):

    python tests/golden/make_c2_window.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from _data import make_problem  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

N, MT, SEED, ITS = 10000, 50000, 11, 25
KEEP_ITS = (6, 15, 25)


def probes(M: int) -> np.ndarray:
    """Four fixed +-1 vectors of length M (splitmix64 bits; the same on every host)."""
    lib = O.load()
    P = np.empty((4, M))
    for k in range(4):
        P[k] = [1.0 if (lib.orc_splitmix64(0xC2C2 + k * 1000003 + i) >> 63) else -1.0 for i in range(M)]
    return P


def main():
    t0 = time.time()
    X, y, beta = make_problem(N, MT, seed=SEED)
    ref = O.vamp_infere(X, y, MT, true_signal=beta, max_iter=ITS, stop_criteria_thr=0.0)
    assert ref["iterations"] == ITS
    P = probes(MT)
    keep = np.array(KEEP_ITS)
    np.savez(os.path.join(HERE, "oracle_c2_window.npz"),
             N=N, Mt=MT, seed=SEED, its=ITS, keep_its=keep,
             x1=ref["x1_hist"][keep - 1], r1=ref["r1_hist"][keep - 1],
             x1_norm=np.linalg.norm(ref["x1_hist"], axis=1), r1_norm=np.linalg.norm(ref["r1_hist"], axis=1),
             x1_proj=ref["x1_hist"] @ P.T, r1_proj=ref["r1_hist"] @ P.T,
             params=ref["params"], metrics=ref["metrics"], cg_iters=ref["cg_iters"], ons_iters=ref["ons_iters"],
             L=ref["L"], threads=int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    print(f"oracle_c2_window.npz: {ITS} iterations in {time.time() - t0:.0f} s; cg {ref['cg_iters'].tolist()} "
          f"ons {ref['ons_iters'].tolist()}")


if __name__ == "__main__":
    main()
