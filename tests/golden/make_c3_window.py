"""C3 shard bench-window fixture: the CPU oracle's run of the whole per-GPU C3
shard (BASELINE configs[2]'s samples, N = 100,000 methylation-like, 62,500 of
its 500,000 markers; eight such shards are configs[2]) over iterations 1-12,
the window `bench.py --config c3` times (--warmup 2 --steps 10: 3-12).

The problem: X = the index-keyed methylation-like design (seed 31, kind 1,
bit-identical on the device, `Data.generate`), y / beta = tests/_data.py
phen_from_markers (standardised phenotype).  Stored
(tests/golden/oracle_c3_window.npz, ~3.5 MB):
* the inputs the device cannot regenerate by itself: y and beta;
* for EVERY iteration: the norms of x1_hat / r1, their projections on four
  fixed +-1 probe vectors, params, metrics, CG / Onsager / mixture counts;
* for EVERY iteration, per block of NBLK contiguous markers (round 6,
  ADVICE r05: a localized error must not hide in the whole-vector norms):
  the block's norm and its projections on two of the probes (block_checks);
* x1_hat and r1 at the iterations in KEEP_ITS.

Run in the build container (50 GB for X; ~10 min on 8 cores):

    python tests/golden/make_c3_window.py
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
sys.path.insert(0, HERE)

from _data import phen_from_markers  # noqa: E402
from make_c2_window import probes  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

N, MT, SEED, KIND, ITS = 100000, 62500, 31, 1, 12
KEEP_ITS = (3, 7, 12)
NBLK = 256


def block_checks(H, P):
    """Per row of H (iterations x M) and block of NBLK contiguous markers: the
    block's norm and its projections on probes P[0] and P[1] -> (its, NBLK, 3)."""
    M = H.shape[1]
    edges = np.linspace(0, M, NBLK + 1).astype(np.int64)
    out = np.zeros((H.shape[0], NBLK, 3))
    for b in range(NBLK):
        h = H[:, edges[b]:edges[b + 1]]
        out[:, b, 0] = np.linalg.norm(h, axis=1)
        out[:, b, 1] = h @ P[0, edges[b]:edges[b + 1]]
        out[:, b, 2] = h @ P[1, edges[b]:edges[b + 1]]
    return out


def main():
    t0 = time.time()
    X = O.generate_markers(SEED, KIND, N, 0, MT)
    y, beta = phen_from_markers(X, SEED, lam=0.1, h2=0.8)
    print(f"inputs: {time.time() - t0:.0f} s", flush=True)
    ref = O.vamp_infere(X, y, MT, true_signal=beta, max_iter=ITS, stop_criteria_thr=0.0)
    assert ref["iterations"] == ITS
    del X
    P = probes(MT)
    keep = np.array(KEEP_ITS)
    np.savez_compressed(os.path.join(HERE, "oracle_c3_window.npz"),
                        N=N, Mt=MT, seed=SEED, kind=KIND, its=ITS, keep_its=keep, y=y, beta=beta,
                        x1=ref["x1_hist"][keep - 1], r1=ref["r1_hist"][keep - 1],
                        x1_norm=np.linalg.norm(ref["x1_hist"], axis=1), r1_norm=np.linalg.norm(ref["r1_hist"], axis=1),
                        x1_proj=ref["x1_hist"] @ P.T, r1_proj=ref["r1_hist"] @ P.T,
                        x1_blocks=block_checks(ref["x1_hist"], P), r1_blocks=block_checks(ref["r1_hist"], P),
                        params=ref["params"], metrics=ref["metrics"], cg_iters=ref["cg_iters"],
                        ons_iters=ref["ons_iters"], L=ref["L"])
    print(f"oracle_c3_window.npz: {ITS} iterations in {time.time() - t0:.0f} s; cg {ref['cg_iters'].tolist()} "
          f"ons {ref['ons_iters'].tolist()}")


if __name__ == "__main__":
    main()
