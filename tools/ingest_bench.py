"""Streaming ingest rate (vampomi_load_meth_file): write a marker-major fp64
file of the given shape (generated on the device, dumped in chunks), then
time loading it into a fresh context (parallel pread -> pinned staging ->
HBM, plus the marker statistics), and check it bit for bit.

    python tools/ingest_bench.py [N] [M] [path] [threads...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import vampomi_amd as va  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
M = int(sys.argv[2]) if len(sys.argv) > 2 else 25000
path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.environ.get("TMPDIR", "/tmp"), "vampomi_ingest.bin")
threads = sys.argv[4:] or ["1", "4", "8", "16"]
gb = 8.0 * N * M / 1e9
t0 = time.perf_counter()
with va.Data(N, M) as d:
    d.generate(5, va.GEN_METH)
    ref_rows = d.get_meth_data(M // 2, 2)
    ref_mave = d.get_mave()
    with open(path, "wb") as f:
        step = max(1, (1 << 30) // (8 * N))
        for i0 in range(0, M, step):
            f.write(d.get_meth_data(i0, min(step, M - i0)).astype("<f8").tobytes())
t_write = time.perf_counter() - t0
res = {"N": N, "M": M, "GB": round(gb, 2), "write_s": round(t_write, 1), "runs": []}
for nt in threads:
    os.environ["VAMPOMI_IO_THREADS"] = nt
    with va.Data(N, M) as d:
        t0 = time.perf_counter()
        d.read_methylation_data(path)
        el = time.perf_counter() - t0
        ok = bool(np.array_equal(d.get_meth_data(M // 2, 2), ref_rows) and np.array_equal(d.get_mave(), ref_mave))
    res["runs"].append({"threads": int(nt), "s": round(el, 3), "GB/s": round(gb / el, 2), "bitwise": ok})
    print(json.dumps(res["runs"][-1]), flush=True)
os.remove(path)
print(json.dumps(res))
