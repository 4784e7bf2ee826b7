"""Deterministic test problems built only from the index-keyed generators and
the oracle's fixed-order arithmetic, so inputs are bit-identical on every host
(no BLAS, no numpy RNG)."""
from __future__ import annotations

import numpy as np

from oracle import pyoracle as O


def make_problem(N: int, Mt: int, seed: int = 3, kind: int = 0, lam: float = 0.1, h2: float = 0.8):
    """X (Mt, N) marker-major, y (N, standardised like read_phen), beta (Mt)."""
    lib = O.load()
    X = O.generate_markers(seed, kind, N, 0, Mt)
    mave, msig = O.marker_stats(X)
    beta = np.zeros(Mt)
    causal = np.array([(lib.orc_splitmix64(seed * 7919 + i) >> 11) * 2.0 ** -53 < lam for i in range(Mt)])
    cm = max(int(causal.sum()), 1)
    g = np.array([lib.orc_gauss_dyadic(seed + 101, i, 0) for i in range(Mt)])
    beta[causal] = g[causal] * np.sqrt(h2 / cm)
    z = O.ax(X, mave, msig, beta * np.sqrt(N))  # sum_i (X_i - mave_i) msig_i beta_i, fixed order
    noise = np.array([lib.orc_gauss_dyadic(seed + 202, -1, j) for j in range(N)])
    y = O.standardize_phen(z + np.sqrt(1 - h2) * noise)
    return X, y, beta
