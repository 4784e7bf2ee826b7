"""Regenerate the committed golden fixtures (run in the build container only;
it reads /root/reference, which does not exist on the GPU box).

1. ``datasim_*``: the reference's own input generator,
   /root/reference/simulation/data_sim.py, executed with seeded numpy/random
   (it is unseeded upstream, data_sim.py:35,40-42,47), N=100, M=200.  These
   are files in the reference's formats (marker-major .bin, PLINK .phen,
   _ts.bin) written by the reference's code: they pin our readers.
2. ``oracle_*``: outputs of the CPU oracle (PARITY UNPINNED restatement, see
   oracle/vamp_oracle.h) on (a) the data_sim fixture and (b) the generated C1
   problem (tests/_data.py, N=1000, Mt=2000): per-iteration x1/r1 at selected
   iterations, params, metrics, CG/Onsager/L counts and the three CSV files'
   raw bytes.  They are regression pins for the oracle and GPU references.
   ``oracle_probit_*``: the same for the probit model (--model bin_class) on
   the C1 problem's liability thresholded at 0.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import random
import runpy
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from _data import make_problem  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

REF_DATASIM = "/root/reference/simulation/data_sim.py"
KEEP_ITS = (1, 2, 3, 5, 10, 20, 30)


def run_data_sim(N=100, M=200, seed=12345):
    argv = sys.argv
    np.random.seed(seed)
    random.seed(seed)
    sys.argv = ["data_sim.py", "--out-dir", HERE, "--out-name", "datasim", "--N", str(N), "--M", str(M)]
    try:
        runpy.run_path(REF_DATASIM, run_name="__main__")
    finally:
        sys.argv = argv


def oracle_case(name, X, y, Mt, beta, its, thr, model="linear"):
    with tempfile.TemporaryDirectory() as td:
        r = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=its, stop_criteria_thr=thr, out_dir=td,
                          out_name="g", model=model)
        csv = {k: open(os.path.join(td, f"g_{k}.csv"), "rb").read() for k in ("params", "metrics", "prior")}
    keep = [k for k in KEEP_ITS if k <= r["iterations"]] + [r["iterations"]]
    keep = sorted(set(keep))
    np.savez_compressed(
        os.path.join(HERE, f"oracle_{name}.npz"),
        iterations=r["iterations"], cg_iters=r["cg_iters"], ons_iters=r["ons_iters"], L=r["L"],
        params=r["params"], metrics=r["metrics"], keep_its=np.array(keep),
        x1=r["x1_hist"][np.array(keep) - 1], r1=r["r1_hist"][np.array(keep) - 1],
        csv_params=np.frombuffer(csv["params"], dtype=np.uint8), csv_metrics=np.frombuffer(csv["metrics"], np.uint8),
        csv_prior=np.frombuffer(csv["prior"], dtype=np.uint8), a_passes=r["a_passes"], its=its, thr=thr,
        model=model, x1_final=r["x1_final"], prior=r.get("prior", np.zeros(0)))
    print(name, r["iterations"], r["cg_iters"].tolist(), r["ons_iters"].tolist())


def main():
    run_data_sim()
    N, M = 100, 200
    X = np.fromfile(os.path.join(HERE, "datasim.bin"), dtype="<f8").reshape(M, N)
    y = O.read_phen(os.path.join(HERE, "datasim.phen"), N, True)
    beta = np.fromfile(os.path.join(HERE, "datasim_ts.bin"), dtype="<f8")
    oracle_case("datasim", X, y, M, beta, 20, 0.0)
    X, y, beta = make_problem(1000, 2000)
    oracle_case("c1", X, y, 2000, beta, 30, 0.0)
    oracle_case("c1_stop", X, y, 2000, beta, 50, 0.01)
    # probit (src/vamp_probit.cpp): the same liability thresholded at 0
    yb = (y > 0).astype(np.float64)
    oracle_case("probit_c1", X, yb, 2000, beta, 30, 0.0, model="bin_class")
    oracle_case("probit_c1_stop", X, yb, 2000, beta, 50, 0.01, model="bin_class")


if __name__ == "__main__":
    main()
