"""Kernel tuning sweep for the A.x / A^T.u passes (run on the GPU box).

    python tools/kbench.py [N] [Mt] [reps] [which: ax,atx,loo,op]   (OP_PLANS=v1,v2: operator plans)

Prints, per variant and batch width K, the average launch time and the
algorithmic HBM rate 8*N*M + 8*K*N + 8*(2+K)*M bytes per launch.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import vampomi_amd as va  # noqa: E402
from vampomi_amd import _lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
Mt = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
lib = va.load()
d = va.Data(N, Mt)
d.generate(1, va.GEN_GAUSS)
rng = np.random.default_rng(0)
x, u = rng.normal(size=Mt), rng.normal(size=N)
only = sys.argv[4].split(",") if len(sys.argv) > 4 else ["ax", "atx", "loo"]
res = {"N": N, "Mt": Mt, "reps": reps, "ax": {}, "atx": {}, "loo": {}}
ref_ax, ref_atx = None, None
for which, name, Ks, nvar in ((0, "ax", tuple(int(k) for k in os.environ.get("AX_KS", "1,2,3").split(",")), 8), (1, "atx", (1, 2), 8)):
    if name not in only:
        continue
    for v in range(nvar):
        _lib.check(lib.vampomi_dev_set_variant(d.ctx, which, v))
        # correctness against variant 0 (chunking may differ: 1e-13)
        if which == 0:
            out = d.Ax(x)
            ref_ax = out if v == 0 else ref_ax
            err = float(np.linalg.norm(out - ref_ax) / np.linalg.norm(ref_ax))
        else:
            out = d.ATx(u)
            ref_atx = out if v == 0 else ref_atx
            err = float(np.linalg.norm(out - ref_atx) / np.linalg.norm(ref_atx))
        row = {"relerr_vs_v0": err}
        for K in Ks:
            ms = C.c_double()
            _lib.check(lib.vampomi_dev_time_pass(d.ctx, which, K, 2, C.byref(ms)))  # warm
            _lib.check(lib.vampomi_dev_time_pass(d.ctx, which, K, reps, C.byref(ms)))
            b = 8.0 * N * Mt + 8.0 * K * N + 8.0 * (2 + K) * Mt
            row[f"K{K}"] = {"us": round(ms.value * 1e3, 1), "GBs": round(b / (ms.value * 1e-3) / 1e9, 1)}
        res[name][v] = row
        print(name, v, json.dumps(row), flush=True)
    _lib.check(lib.vampomi_dev_set_variant(d.ctx, which, 0))
if "op" in only:  # the one-pass CG operator (A^T q and A d from one read of X), every plan for this N
    res["op"] = {}
    plans = os.environ.get("OP_PLANS")
    cands = [int(v) for v in plans.split(",")] if plans else \
        [-1, 0] + [T * 10 + c for T in (1, 2, 4, 8, 16, 32) for c in range(5)]
    for v in cands:
        try:
            d.set_variant(3, v)
        except va.VampomiError:
            continue
        row = {"kernel": d.kernel_name(3, 2)}
        for K in (1, 2):
            ms = C.c_double()
            _lib.check(lib.vampomi_dev_time_pass(d.ctx, 3, K, 2, C.byref(ms)))
            _lib.check(lib.vampomi_dev_time_pass(d.ctx, 3, K, reps, C.byref(ms)))
            b = 8.0 * N * Mt + 8.0 * K * N + 8.0 * (2 + K) * Mt
            row[f"K{K}"] = {"us": round(ms.value * 1e3, 1), "GBs": round(b / (ms.value * 1e-3) / 1e9, 1)}
        res["op"][v] = row
        print("op", v, json.dumps(row), flush=True)
    d.set_variant(3, -1)
if "loo" in only:
    d.set_phen(rng.normal(size=N), standardize=False)
    est = rng.normal(size=Mt) * 1e-3
    ref = None
    for v in range(int(os.environ.get("LOO_VARIANTS", "20"))):
        _lib.check(lib.vampomi_dev_set_variant(d.ctx, 2, v))
        p, st = d.assoc_loo(est)
        ref = st if ref is None else ref
        ms = C.c_double()
        _lib.check(lib.vampomi_dev_time_pass(d.ctx, 2, 1, 2, C.byref(ms)))
        _lib.check(lib.vampomi_dev_time_pass(d.ctx, 2, 1, reps, C.byref(ms)))
        b = 8.0 * N * Mt + 8.0 * N + 48.0 * Mt
        row = {"kernel": d.kernel_name(2, 1, v), "bitwise_eq_v0": bool(np.array_equal(st, ref)),
               "us": round(ms.value * 1e3, 1), "GBs": round(b / (ms.value * 1e-3) / 1e9, 1)}
        res["loo"][v] = row
        print("loo", v, json.dumps(row), flush=True)
    _lib.check(lib.vampomi_dev_set_variant(d.ctx, 2, 0))
print(json.dumps(res))
