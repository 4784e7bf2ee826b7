"""C4 shard sensitivity fixture: how far the reference's own probit result
moves under a change of summation order, measured on the oracle at the whole
per-GPU C4 shard (BASELINE configs[3]: N = 50,000 samples; 50,000 of its
200,000 markers), 8 iterations (src/vamp_probit.cpp:19-488).

The problem: X = the index-keyed Gaussian design (seed 20250711, bit-identical
on the device, `Data.generate`), y / beta = tests/_data.py phen_from_markers
thresholded at 0.  Stored (tests/golden/oracle_c4_spread.npz):
* the inputs the device cannot regenerate by itself: y (0/1) and beta;
* the single-rank oracle run's per-iteration x1 / r1 norms, params and counts
  (the GPU test re-runs the oracle on the GPU box's host and checks it is this
  run, bit for bit);
* per variant, per iteration, the norm-relative change of x1 / r1 (and
  element-wise of params, metrics, prior rows) against the single-rank run:
  ranks P = 2, 3 (what `mpirun -np` changes), P = 64, 128 virtual shards (the
  sums over markers split as finely as the device's team slots split them),
  and orc_atx's sample sums in blocks of 128 rows, alone and with 128 shards
  (the device's A^T sums over lanes, waves and team members).

tests/test_gpu_probit.py::test_c4_full_shard_vs_oracle holds the device to
PROBIT_K x the largest of these per iteration.  Run in the build container
(20 GB for X; about 25 min on 8 cores):

    python tests/golden/make_c4_spread.py
    python tests/golden/make_c4_spread.py --add 256 512 1024   # finer virtual shards
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

from _data import oracle_with_spread, phen_from_markers  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

N, MT, SEED, ITS = 50000, 50000, 20250711, 8
RANKS = (2, 3, 64, 128)
BLOCKS = ((1, 128), (128, 128))
GEN_GAUSS = 0


def c4_inputs(X):
    y, beta = phen_from_markers(X, SEED + 1, lam=0.1, h2=0.8)
    return (y > 0).astype(np.float64), beta


def main():
    """`make_c4_spread.py` makes the fixture; `make_c4_spread.py --add P ...`
    adds P-rank variants to the committed one (the single-rank run is redone,
    the stored variants kept)."""
    add = [int(a) for a in sys.argv[sys.argv.index("--add") + 1:]] if "--add" in sys.argv else None
    t0 = time.time()
    X = O.generate_markers(SEED, GEN_GAUSS, N, 0, MT)
    y, beta = c4_inputs(X)
    kw = dict(model="bin_class", max_iter=ITS, stop_criteria_thr=0.0)
    ref = O.vamp_infere(X, y, MT, true_signal=beta, **kw)
    print(f"single rank: {time.time() - t0:.0f} s", flush=True)
    pv = {}
    if add:
        old = np.load(os.path.join(HERE, "oracle_c4_spread.npz"))
        assert np.array_equal(old["ref_x1_norm"], np.linalg.norm(ref["x1_hist"], axis=1)), "not the stored run"
        for i, v in enumerate(old["variants"]):
            pv[tuple(int(a) for a in v)] = {key: old[f"spread_{key}"][i] for key in ("x1", "r1", "params", "metrics",
                                                                                    "prior")}
        oracle_with_spread(X, y, beta, MT, ranks=tuple(add), blocks=(), ref=ref, per_variant=pv, **kw)
    else:
        oracle_with_spread(X, y, beta, MT, ranks=RANKS, blocks=BLOCKS, ref=ref, per_variant=pv, **kw)
    variants = sorted(pv)
    out = dict(N=N, Mt=MT, seed=SEED, its=ITS, y=y.astype(np.uint8), beta=beta,
               ref_x1_norm=np.linalg.norm(ref["x1_hist"], axis=1), ref_r1_norm=np.linalg.norm(ref["r1_hist"], axis=1),
               ref_params=ref["params"], ref_cg=ref["cg_iters"], ref_ons=ref["ons_iters"], ref_L=ref["L"],
               variants=np.array(variants, dtype=np.int64))
    for key in ("x1", "r1", "params", "metrics", "prior"):
        out[f"spread_{key}"] = np.stack([pv[v][key] for v in variants])
    np.savez_compressed(os.path.join(HERE, "oracle_c4_spread.npz"), **out)
    for v in variants:
        print(v, "x1", np.array2string(pv[v]["x1"], precision=2), "r1", np.array2string(pv[v]["r1"], precision=2))
    print(f"oracle_c4_spread.npz: {time.time() - t0:.0f} s; cg {ref['cg_iters'].tolist()} "
          f"ons {ref['ons_iters'].tolist()}")


if __name__ == "__main__":
    main()
