"""Workgroup start/end skew of the one-pass operator (an experiment build:
atax_team.hip with TM_TS=1, e.g. make EXTRA_FLAGS=-DTM_TS=1 OBJDIR=../build_ts
LIBDIR=../lib_ts, run with VAMPOMI_LIB=<that .so> VAMPOMI_OP_TS=1).

    python tools/op_skew.py [N] [Mt] [launches] [K]

Per launch: the kernel span (first start .. last end), the spread of the
workgroups' start and end times, the mean wait of a workgroup for the last
one (what a perfectly balanced launch would save), and per XCD the mean end
time relative to the first start; then whether the slow XCDs / teams are
the same from launch to launch (rank correlation of team end times)."""
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
nl = int(sys.argv[3]) if len(sys.argv) > 3 else 6
K = int(sys.argv[4]) if len(sys.argv) > 4 else 2
var = int(sys.argv[5]) if len(sys.argv) > 5 else -1  # operator plan (vampomi_dev_set_variant(c, 3, var))
lib = va.load()
d = va.Data(N, Mt)
d.generate(1, va.GEN_GAUSS)
T, S, TR, grid, nslots = (C.c_int() for _ in range(5))
ns64 = C.c_int64()
name = C.create_string_buffer(128)
if var != -1:
    d.set_variant(3, var)
_lib.check(lib.vampomi_dev_op_plan(N, Mt, 256, var, K, C.byref(T), C.byref(S), C.byref(TR), C.byref(grid),
                                   C.byref(ns64), name, 128))
print("plan", name.value.decode(), "T", T.value, "grid", grid.value, flush=True)
ms = C.c_double()
_lib.check(lib.vampomi_dev_time_pass(d.ctx, 3, K, 3, C.byref(ms)))  # warm
ends = []
out = {"N": N, "Mt": Mt, "K": K, "kernel": name.value.decode(), "launches": []}
for rep in range(nl):
    _lib.check(lib.vampomi_dev_time_pass(d.ctx, 3, K, 1, C.byref(ms)))
    buf = (C.c_ulonglong * (4 * 1024))()
    n = C.c_int()
    _lib.check(lib.vampomi_dev_op_timestamps(d.ctx, buf, 4 * 1024, C.byref(n)))
    a = np.frombuffer(buf, dtype=np.uint64, count=n.value).reshape(-1, 4).astype(np.float64)
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) * 0.01, (a[:, 1] - t0) * 0.01  # us
    xcc = a[:, 2].astype(int) & 0xF
    span = en.max()
    g = grid.value
    team = np.array([(b & 7) + 8 * ((b >> 3) // T.value) for b in range(g)])
    tend = np.array([en[team == t].max() for t in range(g // T.value)])
    per_xcc = {int(x): round(float(en[xcc == x].mean()), 2) for x in sorted(set(xcc))}
    row = {"event_us": round(ms.value * 1e3, 1), "span_us": round(float(span), 1),
           "start_spread_us": round(float(st.max() - st.min()), 2),
           "end_min_us": round(float(en.min()), 1), "end_spread_us": round(float(en.max() - en.min()), 2),
           "mean_wait_for_last_us": round(float(span - en.mean()), 2),
           "team_end_spread_us": round(float(tend.max() - tend.min()), 2), "end_by_xcc": per_xcc}
    ends.append(tend)
    out["launches"].append(row)
    print(json.dumps(row), flush=True)
E = np.array(ends)
if len(E) > 1:
    r = np.argsort(np.argsort(E, axis=1), axis=1)
    cc = np.corrcoef(r)
    out["team_rank_corr_mean"] = float((cc.sum() - len(E)) / (len(E) * (len(E) - 1)))
    print("mean rank correlation of team end times between launches:", round(out["team_rank_corr_mean"], 3))
print(json.dumps(out))
