"""Deterministic test problems built only from the index-keyed generators and
the oracle's fixed-order arithmetic, so inputs are bit-identical on every host
(no BLAS, no numpy RNG)."""
from __future__ import annotations

import os
import threading

import numpy as np

from oracle import pyoracle as O


def make_problem(N: int, Mt: int, seed: int = 3, kind: int = 0, lam: float = 0.1, h2: float = 0.8):
    """X (Mt, N) marker-major, y (N, standardised like read_phen), beta (Mt)."""
    X = O.generate_markers(seed, kind, N, 0, Mt)
    y, beta = phen_from_markers(X, seed, lam, h2)
    return X, y, beta


def phen_from_markers(X, seed: int = 3, lam: float = 0.1, h2: float = 0.8):
    """make_problem's phenotype for a given design X (Mt, N): (y, beta)."""
    lib = O.load()
    Mt, N = X.shape
    mave, msig = O.marker_stats(X)
    beta = np.zeros(Mt)
    causal = np.array([(lib.orc_splitmix64(seed * 7919 + i) >> 11) * 2.0 ** -53 < lam for i in range(Mt)])
    cm = max(int(causal.sum()), 1)
    g = np.array([lib.orc_gauss_dyadic(seed + 101, i, 0) for i in range(Mt)])
    beta[causal] = g[causal] * np.sqrt(h2 / cm)
    z = O.ax(X, mave, msig, beta * np.sqrt(N))  # sum_i (X_i - mave_i) msig_i beta_i, fixed order
    noise = np.array([lib.orc_gauss_dyadic(seed + 202, -1, j) for j in range(N)])
    y = O.standardize_phen(z + np.sqrt(1 - h2) * noise)
    return y, beta


class ThreadComm:
    """In-process SUM all-reduce for P threads acting as ranks (summed in rank order)."""

    def __init__(self, P):
        self.P = P
        self.bar = threading.Barrier(P)
        self.buf = {}
        self.lock = threading.Lock()

    def make(self, rank):
        def ar(a):
            with self.lock:
                self.buf[rank] = a.copy()
            self.bar.wait()
            if rank == 0:  # one sum, in rank order, for every rank (P ranks summing P buffers each is O(P^2 n))
                tot = np.zeros_like(a)
                for r in range(self.P):
                    tot += self.buf[r]
                self.tot = tot
            self.bar.wait()
            a[:] = self.tot  # (rank 0 replaces self.tot only after every rank reached the next call's barrier)
        return ar


def sharded_oracle(X, y, beta, Mt, P, **kw):
    """The oracle on P marker shards (divide_work), one thread per rank."""
    comm = ThreadComm(P)
    res = [None] * P

    def work(r):
        # OpenMP threads per rank: the host's cores shared out (each rank's
        # thread has its own OpenMP team; 128 ranks x all cores would thrash)
        O.set_omp_threads(max(1, (os.cpu_count() or 1) // P))
        M, S, _ = O.divide_work(Mt, P, r)
        res[r] = O.vamp_infere(X[S:S + M], y, Mt, S=S, rank=r, nranks=P,
                               true_signal=None if beta is None else beta[S:S + M], allreduce=comm.make(r), **kw)

    th = [threading.Thread(target=work, args=(r,)) for r in range(P)]
    [t.start() for t in th]
    [t.join() for t in th]
    return res


def oracle_with_spread(X, y, beta, Mt, ranks=(2, 3, 4), blocks=(), ref=None, per_variant=None, **kw):
    """The single-rank oracle run plus the reference's own sensitivity to the
    summation order: per iteration, the largest norm-relative change of
    x1 / r1 (and element-wise of params, metrics, prior) when the same
    problem runs
    * on P ranks for P in `ranks` (the all-reduce order, exactly what
      `mpirun -np P` changes for the reference; P = 64 or 128 "virtual
      shards" split the sums over markers as finely as the device's team
      slots do), and
    * with orc_atx summing samples in blocks of B rows for (P, B) in `blocks`
      (the sums over samples, which a rank count never splits).
    Returns (ref, spread) with spread["x1"], spread["r1"] of shape
    (iterations,) and spread["params"] like ref["params"].  `ref` may be
    passed in (the single-rank run, already made); `per_variant` (a dict)
    receives each variant's own spread."""
    if ref is None:
        ref = O.vamp_infere(X, y, Mt, true_signal=beta, **kw)
    kw = {k: v for k, v in kw.items() if k not in ("out_dir", "out_name")}  # files: single-rank run only
    n = ref["iterations"]
    sp = {"x1": np.zeros(n), "r1": np.zeros(n), "params": np.zeros_like(ref["params"]),
          "metrics": np.zeros_like(ref["metrics"])}
    for P, B in [(P, 0) for P in ranks] + list(blocks):
        O.set_atx_block(B)
        try:
            res = sharded_oracle(X, y, beta, Mt, P, **kw) if P > 1 else \
                [O.vamp_infere(X, y, Mt, true_signal=beta, **kw)]
        finally:
            O.set_atx_block(0)
        assert res[0]["iterations"] == n, "the reference's own iteration count depends on the summation order"
        own = {}
        for key in ("x1", "r1"):
            h = np.concatenate([r[f"{key}_hist"] for r in res], axis=1)
            num = np.linalg.norm(h - ref[f"{key}_hist"], axis=1)
            den = np.maximum(np.linalg.norm(ref[f"{key}_hist"], axis=1), 1e-300)
            own[key] = num / den
        for key in ("params", "metrics", "prior"):
            if key not in ref:
                continue
            a, b = res[0][key], ref[key]
            with np.errstate(invalid="ignore", divide="ignore"):
                own[key] = np.where(np.isnan(a) & np.isnan(b), 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-300))
        for key, e in own.items():
            sp[key] = np.maximum(sp.get(key, np.zeros_like(e)), e)
        if per_variant is not None:
            per_variant[(P, B)] = own
    return ref, sp


# The reference's own runs: one rank with OMP_NUM_THREADS = T sums each
# inner_prod over T contiguous chunks and adds the threads' sums in arrival
# order (src/utilities.cpp:138-158; ORC_ASSOC_REFRUN, vamp_oracle.c), and
# `mpirun -np P` splits every sum over markers over the ranks (divide_work).
# Every member of this ensemble is a run the reference itself performs.
REF_THREADS = (4, 8, 16, 32, 64, 128)


def reference_ensemble(X, y, beta, Mt, ref, threads=REF_THREADS, seeds=(1, 2, 3, 4), ranks=(2, 3), **kw):
    """Per-variant spread (norm-relative change of x1 / r1 per iteration, and
    element-wise of params, metrics, prior) of the reference's own runs around
    the oracle's restatement run `ref`: one rank at T threads x arrival-order
    seeds, and P ranks.  Returns {(kind, a, b): own} with kind 0 = (T, seed),
    1 = (P ranks, 0)."""
    out = {}
    n = ref["iterations"]

    def own_of(res):
        own = {}
        for key in ("x1", "r1"):
            h = np.concatenate([r[f"{key}_hist"] for r in res], axis=1)
            num = np.linalg.norm(h - ref[f"{key}_hist"], axis=1)
            den = np.maximum(np.linalg.norm(ref[f"{key}_hist"], axis=1), 1e-300)
            own[key] = num / den
        for key in ("params", "metrics", "prior"):
            if key in ref:
                a, b = res[0][key], ref[key]
                with np.errstate(invalid="ignore", divide="ignore"):
                    own[key] = np.where(np.isnan(a) & np.isnan(b), 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-300))
        return own

    kw = {k: v for k, v in kw.items() if k not in ("out_dir", "out_name")}
    for T in threads:
        for sd in seeds:
            O.set_assoc(O.ASSOC_REFRUN, T, 0, sd)
            try:
                r = O.vamp_infere(X, y, Mt, true_signal=beta, **kw)
            finally:
                O.set_assoc()
            assert r["iterations"] == n
            out[(0, T, sd)] = own_of([r])
    for P in ranks:
        res = sharded_oracle(X, y, beta, Mt, P, **kw)
        assert res[0]["iterations"] == n
        out[(1, P, 0)] = own_of(res)
    return out


def ensemble_quantile(per_variant: dict, key: str, q: float = 0.9):
    """The q-quantile over the ensemble's variants, per iteration (or element)."""
    return np.quantile(np.stack([v[key] for v in per_variant.values()]), q, axis=0)


# The probit parity bar's multiple of the oracle's own rank-count spread
# (DESIGN.md §3): the GPU must stay within PROBIT_K x the amount by which the
# reference's own result moves when its all-reduce order changes.  Set to
# about twice the largest gap / spread ratio measured over every probit GPU
# test (record_probit_ratio; VAMPOMI_PROBIT_RATIOS=<file> appends them).
PROBIT_K = 6.0


def record_probit_ratio(test: str, key: str, gap, spread, floor: float = 1e-10):
    """gap / spread per iteration where the bar is the spread's (k * spread >
    floor), appended as one JSON line to $VAMPOMI_PROBIT_RATIOS; returns the
    largest ratio (0 where the floor sets the bar everywhere)."""
    import json
    import os

    gap, spread = np.atleast_1d(np.asarray(gap, dtype=float)), np.atleast_1d(np.asarray(spread, dtype=float))
    m = (spread > 0) & (PROBIT_K * spread > floor)
    r = float(np.max(gap[m] / spread[m])) if np.any(m) else 0.0
    f = os.environ.get("VAMPOMI_PROBIT_RATIOS")
    if f:
        with open(f, "a") as fh:
            g1 = gap.reshape(len(gap), -1).max(axis=1) if gap.ndim > 1 else gap  # per iteration (params: rows)
            s1 = spread.reshape(len(spread), -1).max(axis=1) if spread.ndim > 1 else spread
            fh.write(json.dumps({"test": test, "key": key, "max_ratio": r, "n": int(np.sum(m)),
                                 "gap": [float(g) for g in g1[:16]], "spread": [float(v) for v in s1[:16]]}) + "\n")
    return r
