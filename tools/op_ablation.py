"""Ablations of the one-pass CG operator at one shape, in ONE process on one
device, against the same process's pure read stream of the same matrix
(vampomi_dev_read_ceiling), so box-to-box variance cancels (run on the GPU box):

    VAMPOMI_LIB=<TM_DBG build .so> python tools/op_ablation.py [N] [Mt] [reps] [rounds]

Each ablation removes one component of the operator's per-column work
(VAMPOMI_OP_DBG bits, honoured by team kernels only in TM_DBG builds; results
are wrong while set): 8 the streaming waves' A d accumulation, 2048 their LDS
q reads, 4096 the hand-off wave's whole chain (polls, member sum, epilogue, d
stores, publishes: it only keeps the step barriers), 1|2 its granule waits and
publishes, 1024 the owners' d stores, 4 the streaming butterfly.  Rounds
alternate every setting; the table gives the median per setting, its
difference to dbg 0 and each time against the stream.
"""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import vampomi_amd as va  # noqa: E402
from vampomi_amd import _lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
Mt = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
K = 2
SETTINGS = [(0, "baseline"), (8, "no A d accumulation"), (2048, "no LDS q reads"), (8 | 2048, "neither"),
            (1024, "no owner d stores"), (1 | 2, "no granule waits / publishes"),
            (4096, "no hand-off work at all"), (4096 | 8 | 2048, "streaming dot only (no hand-off, A d, q reads)"),
            (4, "no streaming butterfly")]

lib = va.load()
d = va.Data(N, Mt)
d.generate(1, va.GEN_GAUSS)
name = d.kernel_name(3, K)
if os.environ.get("OP_ABL_ONE"):
    # one library (a TM_ABL build has its ablation baked in; the production library none): the operator's
    # launch time and the same process's read stream, as one JSON line (tools/op_ablation_libs.sh)
    ms = C.c_double()
    _lib.check(lib.vampomi_dev_time_pass(d.ctx, 3, K, 3, C.byref(ms)))
    _lib.check(lib.vampomi_dev_time_pass(d.ctx, 3, K, reps, C.byref(ms)))
    c = d.read_ceiling(9)
    print(json.dumps({"lib": os.environ.get("VAMPOMI_LIB", "production"), "kernel": name, "op_us": round(ms.value * 1e3, 1),
                      "stream_us": round(c["us_med"], 1)}), flush=True)
    sys.exit(0)
times = {s: [] for s, _ in SETTINGS}
ceil = []
for r in range(rounds):
    for s, _ in SETTINGS:
        os.environ["VAMPOMI_OP_DBG"] = str(s)
        ms = C.c_double()
        _lib.check(lib.vampomi_dev_time_pass(d.ctx, 3, K, 3, C.byref(ms)))  # warm
        _lib.check(lib.vampomi_dev_time_pass(d.ctx, 3, K, reps, C.byref(ms)))
        times[s].append(ms.value * 1e3)
        print(f"round {r} dbg {s}: {ms.value * 1e3:.1f} us", flush=True)
    os.environ["VAMPOMI_OP_DBG"] = "0"
    c = d.read_ceiling(9)
    ceil.append(c["us_med"])
    print(f"round {r} stream: {c['us_med']:.1f} us ({c['variant']})", flush=True)
os.environ["VAMPOMI_OP_DBG"] = "0"
alg = 8.0 * N * Mt + 8.0 * K * N + 8.0 * (2 + K) * Mt
stream = statistics.median(ceil)
base = statistics.median(times[0])
print(f"\n{name} K = {K}, N = {N}, Mt = {Mt}; {rounds} rounds x {reps} launches; library "
      f"{os.environ.get('VAMPOMI_LIB', 'default')}")
print(f"same-process read stream of the matrix: {stream:.1f} us (median of {rounds} x 9)")
print(f"{'dbg':>6} {'us':>8} {'-base':>7} {'/stream':>8}  component removed")
rows = []
for s, what in SETTINGS:
    t = statistics.median(times[s])
    rows.append({"dbg": s, "what": what, "us": round(t, 1), "minus_base_us": round(t - base, 1),
                 "over_stream": round(t / stream, 4), "all_us": [round(x, 1) for x in times[s]]})
    print(f"{s:6d} {t:8.1f} {t - base:+7.1f} {t / stream:8.4f}  {what}")
print(json.dumps({"kernel": name, "N": N, "Mt": Mt, "K": K, "stream_us": round(stream, 1), "alg_bytes": alg,
                  "rows": rows}))
