"""Regenerate tests/golden/ref_data_pin.npz: outputs of the REFERENCE's own
data-class operators (src/data.cpp compiled where it lies, oracle/_ref/ref_data,
see oracle/ref_data_harness.cpp) on (a) the files the reference's
simulation/data_sim.py wrote (tests/golden/datasim.*) and (b) a ragged
methylation-like problem from the index-keyed generator (regenerated bit for
bit by tests from the seed).  Build-container only (needs /root/reference).

    make -C oracle ref && python tests/golden/make_ref_golden.py
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = os.path.join(ROOT, "oracle", "_ref", "ref_data")

CASES = {"datasim": dict(N=100, M=200), "gen": dict(N=1001, M=517, seed=9, kind=1)}


def probe_vectors(N, M):
    """Exactly representable inputs for A.x (M) and A^T.u (N)."""
    x = np.array([((i * 7919) % 1001 - 500) / 256.0 for i in range(M)])
    u = np.array([((j * 104729) % 997 - 498) / 512.0 for j in range(N)])
    return x, u


def case_matrix(name):
    c = CASES[name]
    if name == "datasim":
        return np.fromfile(os.path.join(HERE, "datasim.bin"), dtype="<f8").reshape(c["M"], c["N"])
    from oracle import pyoracle as O
    return O.generate_markers(c["seed"], c["kind"], c["N"], 0, c["M"])


def ref(*args, env=None):
    e = dict(os.environ, OMP_NUM_THREADS="1")
    subprocess.run([REF, *map(str, args)], check=True, capture_output=True, env=e)


def main():
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for name, c in CASES.items():
            N, M = c["N"], c["M"]
            X = case_matrix(name)
            xp = os.path.join(td, "X.bin")
            X.astype("<f8").tofile(xp)
            x, u = probe_vectors(N, M)
            x.tofile(os.path.join(td, "x.bin"))
            u.tofile(os.path.join(td, "u.bin"))
            for a, tag in ((1.0, ""), (0.7, "_a07")):
                ref("stats", xp, N, M, a, os.path.join(td, "mave"), os.path.join(td, "msig"))
                out[f"{name}_mave{tag}"] = np.fromfile(os.path.join(td, "mave"))
                out[f"{name}_msig{tag}"] = np.fromfile(os.path.join(td, "msig"))
            ref("ax", xp, N, M, os.path.join(td, "x.bin"), os.path.join(td, "o"))
            out[f"{name}_ax"] = np.fromfile(os.path.join(td, "o"))
            ref("atx", xp, N, M, os.path.join(td, "u.bin"), os.path.join(td, "o"))
            out[f"{name}_atx"] = np.fromfile(os.path.join(td, "o"))
        for s in (0, 1):
            ref("phen", os.path.join(HERE, "datasim.phen"), 100, s, os.path.join(td, "p"))
            out[f"datasim_phen_std{s}"] = np.fromfile(os.path.join(td, "p"))
    np.savez_compressed(os.path.join(HERE, "ref_data_pin.npz"), **out)
    print(sorted(out))


if __name__ == "__main__":
    main()
