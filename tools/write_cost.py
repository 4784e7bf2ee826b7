"""Where the per-iteration output files cost time: vamp_begin and every
vamp_step timed on the host, with and without out_dir, C2 (device-generated).

    python tools/write_cost.py [out_parent]
"""
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402

import vampomi_amd as va  # noqa: E402

parent = sys.argv[1] if len(sys.argv) > 1 else None
d = va.Data(10000, 50000)
d.generate(20250711, va.GEN_GAUSS)
beta = d.simulate_phen(20250712, lam=0.1, h2=0.8)
res = {}
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["nowrite", "write", "nowrite2", "write2"]
for mode in modes:
    out = tempfile.mkdtemp(prefix="vampomi_wc_", dir=parent) if mode.startswith("write") else ""
    v = va.Vamp(d, va.VampOptions(max_iter=25, stop_criteria_thr=0.0, out_dir=out, out_name="c2"), true_signal=beta)
    t0 = time.perf_counter()
    v.begin()
    t1 = time.perf_counter()
    steps = []
    for _ in range(25):
        a = time.perf_counter()
        v.step()
        steps.append((time.perf_counter() - a) * 1e3)
    t2 = time.perf_counter()
    v.end()
    t3 = time.perf_counter()
    res[mode] = {"begin_ms": round((t1 - t0) * 1e3, 3), "end_ms": round((t3 - t2) * 1e3, 3),
                 "step1_ms": round(steps[0], 3), "step2_ms": round(steps[1], 3),
                 "steps6_25_ms_mean": round(sum(steps[5:]) / 20, 4), "last_step_ms": round(steps[-1], 3),
                 "total_ms": round((t3 - t0) * 1e3, 2)}
    print(mode, json.dumps(res[mode]), flush=True)
    if out:
        shutil.rmtree(out, ignore_errors=True)
d.close()
