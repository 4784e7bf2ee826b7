"""Benchmark workloads (BASELINE.json configs) — shapes only, no device code.

c2 (default): N=10,000 x Mt=50,000 i.i.d. Gaussian design (configs[1]).  With
    n GPUs: weak scaling at constant per-GPU bytes AND constant aspect ratio
    Mt/N = 5, i.e. N = 10,000*sqrt(n), Mt = 50,000*sqrt(n), so that the
    spectrum of A^T A (and with it the CG iteration counts) stays comparable.
c3: the per-GPU shard of configs[2] (N=100,000, 62,500 methylation-like
    markers per GPU); n=8 is exactly N=100,000 x Mt=500,000.
"""
from __future__ import annotations

import math

GEN_GAUSS, GEN_METH = 0, 1


def workload(cfg: str, n: int) -> dict:
    if cfg == "c3":
        return {"workload": "c3-shard", "N": 100000, "Mt": 62500 * n, "kind": GEN_METH}
    if n == 1:
        return {"workload": "c2", "N": 10000, "Mt": 50000, "kind": GEN_GAUSS}
    s = math.sqrt(n)
    return {"workload": "c2-weak", "N": int(round(10000 * s)), "Mt": int(round(50000 * s)), "kind": GEN_GAUSS}
