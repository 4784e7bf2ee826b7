"""C4 shard parity fixture (round 6): how far the reference's OWN runs move
from one another on the whole per-GPU C4 probit shard (BASELINE configs[3]:
N = 50,000 samples; 50,000 of its 200,000 markers), 8 iterations
(src/vamp_probit.cpp:19-488), and where the device's own grouping of the sums
lands, measured on the oracle.

The problem: X = the index-keyed Gaussian design (seed 20250711, bit-identical
on the device, `Data.generate`), y / beta = tests/_data.py phen_from_markers
thresholded at 0.  Stored (tests/golden/oracle_c4_spread.npz):
* the inputs the device cannot regenerate by itself: y (0/1) and beta;
* the restatement's run (ORC_ASSOC_DEFAULT): per-iteration x1 / r1 norms,
  params and counts (the GPU test re-runs it on the GPU box's host and checks
  it is this run);
* the ensemble of the reference's own runs (tests/_data.py
  reference_ensemble): one rank at OMP_NUM_THREADS = 4 ... 128, four arrival
  orders of the threads' sums each (inner_prod's `omp parallel for
  reduction`, src/utilities.cpp:138-158; sum_d and the EM sums sequential as
  the reference writes them), and 2 and 3 ranks (`mpirun -np`).  Per variant,
  per iteration: the norm-relative change of x1 / r1 (element-wise of params,
  metrics, prior rows) against the restatement's run.  The GPU test's bar is
  PROBIT_K_ENSEMBLE x the 90th percentile over these variants;
* (tests/golden/oracle_c4_devorder.npz) the device-order run
  (ORC_ASSOC_DEVICE at the C4 plan: teams of 16, 256 workgroups): its x1 / r1
  at every iteration as float32 differences from the restatement's run
  (exact to ~1e-16 relative after adding back), its counts and params.  The
  GPU test checks the GPU lands on it.

Run in the build container (20 GB for X; about 2 h on 8 cores for the
ensemble, 10 min for the device-order part):

    python tests/golden/make_c4_spread.py [ensemble] [device]
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

from _data import phen_from_markers, reference_ensemble  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

N, MT, SEED, ITS = 50000, 50000, 20250711, 8
GEN_GAUSS = 0
DEV_T, DEV_GRID = 16, 256  # the C4 shard's operator plan on a 256-CU MI355X (tests/test_op_plan.py)


def c4_inputs(X):
    y, beta = phen_from_markers(X, SEED + 1, lam=0.1, h2=0.8)
    return (y > 0).astype(np.float64), beta


def main():
    parts = [a for a in sys.argv[1:] if a in ("ensemble", "device")] or ["ensemble", "device"]
    t0 = time.time()
    X = O.generate_markers(SEED, GEN_GAUSS, N, 0, MT)
    y, beta = c4_inputs(X)
    kw = dict(model="bin_class", max_iter=ITS, stop_criteria_thr=0.0)
    ref = O.vamp_infere(X, y, MT, true_signal=beta, **kw)
    print(f"restatement: {time.time() - t0:.0f} s; cg {ref['cg_iters'].tolist()} ons {ref['ons_iters'].tolist()}",
          flush=True)
    base = dict(N=N, Mt=MT, seed=SEED, its=ITS, ref_x1_norm=np.linalg.norm(ref["x1_hist"], axis=1),
                ref_r1_norm=np.linalg.norm(ref["r1_hist"], axis=1), ref_params=ref["params"], ref_cg=ref["cg_iters"],
                ref_ons=ref["ons_iters"], ref_L=ref["L"])
    if "device" in parts:
        O.set_assoc(O.ASSOC_DEVICE, DEV_T, DEV_GRID)
        try:
            dv = O.vamp_infere(X, y, MT, true_signal=beta, **kw)
        finally:
            O.set_assoc()
        assert np.array_equal(dv["cg_iters"], ref["cg_iters"]) and np.array_equal(dv["ons_iters"], ref["ons_iters"])
        np.savez_compressed(os.path.join(HERE, "oracle_c4_devorder.npz"), **base, dev_T=DEV_T, dev_grid=DEV_GRID,
                            dev_x1_diff=(dv["x1_hist"] - ref["x1_hist"]).astype(np.float32),
                            dev_r1_diff=(dv["r1_hist"] - ref["r1_hist"]).astype(np.float32),
                            dev_params=dv["params"], dev_L=dv["L"])
        dgap = np.linalg.norm(dv["x1_hist"] - ref["x1_hist"], axis=1) / np.linalg.norm(ref["x1_hist"], axis=1)
        print(f"device order: {time.time() - t0:.0f} s; vs restatement", np.array2string(dgap, precision=2),
              flush=True)
    if "ensemble" in parts:
        pv = reference_ensemble(X, y, beta, MT, ref, **kw)
        variants = sorted(pv)
        out = dict(base, y=y.astype(np.uint8), beta=beta, variants=np.array(variants, dtype=np.int64))
        for key in ("x1", "r1", "params", "metrics", "prior"):
            out[f"spread_{key}"] = np.stack([pv[v][key] for v in variants])
        np.savez_compressed(os.path.join(HERE, "oracle_c4_spread.npz"), **out)
        for v in variants:
            print(v, "x1", np.array2string(pv[v]["x1"], precision=2), flush=True)
        print("x1 q90", np.array2string(np.quantile(out["spread_x1"], 0.9, axis=0), precision=2))
    print(f"done: {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
