"""Benchmark workloads (BASELINE.json configs) — shapes only, no device code.

c2 (default): N=10,000 x Mt=50,000 i.i.d. Gaussian design (configs[1]).  With
    n GPUs: weak scaling over markers, the reference's own sharding (MPI ranks
    split the markers, src/utilities.cpp:207-239): N = 10,000 samples and
    50,000 markers (4 GB) per GPU, Mt = 50,000*n.  Every GPU runs the same
    one-pass CG operator as at n = 1 (K*N fits the CU's LDS); the CG counts
    follow the problem (Mt/N grows with n) and are reported per iteration.
c3: the per-GPU shard of configs[2] (N=100,000, 62,500 methylation-like
    markers per GPU); n=8 is exactly N=100,000 x Mt=500,000.
c4: probit model (configs[3], --model bin_class): N=50,000 with 50,000
    Gaussian markers per GPU and a binary phenotype; n=4 is exactly
    N=50,000 x Mt=200,000.
c4full: configs[3] whole (N=50,000 x Mt=200,000, 80 GB) on any number of
    GPUs (strong scaling; it fits one MI355X).
c5: LOO association test (configs[4], --run-mode association_test
    --pval-method loo): N=100,000 with 62,500 methylation-like markers per
    GPU; n=8 is exactly N=100,000 x Mt=500,000.
c3full: configs[2] itself, N=100,000 x Mt=500,000 methylation-like (400 GB),
    fixed, markers sharded over n >= 2 GPUs (strong scaling: 200 GB per GPU at
    n = 2, 50 GB at n = 8).  It does not fit one MI355X (288 GB).
auto: the bench default, c2 at n = 1 and its weak-scaling form c2-weak at
    n > 1 (the same 50,000 x 10,000 shard per GPU, so the driver's 1 -> 8
    curve stays within one workload family); bench.py adds the c3full
    (configs[2]) phase to the n > 1 line.
c3big: configs[2]'s samples with 300,000 methylation-like markers per GPU,
    i.e. 240 GB of the 288 GB HBM3E resident on one MI355X (the
    1-GPU row at a reduced Mt); n=2 covers Mt=600,000 > configs[2]'s 500,000.
"""
from __future__ import annotations

GEN_GAUSS, GEN_METH = 0, 1


def workload(cfg: str, n: int) -> dict:
    if cfg == "auto":
        cfg = "c2"
    if cfg == "c3full":
        if n < 2:
            raise ValueError("c3full (400 GB) needs n >= 2 GPUs; at n = 1 use c2 or c3big")
        return {"workload": "c3full", "N": 100000, "Mt": 500000, "kind": GEN_METH, "model": "linear",
                "scaling": "strong"}
    if cfg == "c3":
        return {"workload": "c3-shard", "N": 100000, "Mt": 62500 * n, "kind": GEN_METH, "model": "linear"}
    if cfg == "c4":
        return {"workload": "c4-shard", "N": 50000, "Mt": 50000 * n, "kind": GEN_GAUSS, "model": "bin_class"}
    if cfg == "c5":
        return {"workload": "c5-shard", "N": 100000, "Mt": 62500 * n, "kind": GEN_METH, "model": "loo"}
    if cfg == "c3big":
        return {"workload": "c3big", "N": 100000, "Mt": 300000 * n, "kind": GEN_METH, "model": "linear"}
    if cfg == "c4full":
        return {"workload": "c4", "N": 50000, "Mt": 200000, "kind": GEN_GAUSS, "model": "bin_class"}
    if n == 1:
        return {"workload": "c2", "N": 10000, "Mt": 50000, "kind": GEN_GAUSS, "model": "linear"}
    return {"workload": "c2-weak", "N": 10000, "Mt": 50000 * n, "kind": GEN_GAUSS, "model": "linear"}
