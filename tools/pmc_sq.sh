#!/bin/bash
# Occupancy, instruction-mix and wait-cycle counters of the A / A^T kernels
# (one rocprofv3 --pmc pass of 8 SQ counters, kernel dispatch rows only).
#   gpurun -- bash tools/pmc_sq.sh [config]      (bench.py --config, default c2)
set -u
CFG=${1:-c2}
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcsq_$CFG
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_INSTS_SALU -d "$OUT/SQ" -o run --output-format csv -- \
    python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline --no-timing > "$OUT/SQ.log" 2>&1 || exit $?
python - "$OUT" <<'PY' > "$OUT/summary.json"
import csv, glob, json, os, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "SQ", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    if not any(s in k for s in ("atax", "ax_partial", "atx_kernel", "loo_kernel")):
        continue
    per = defaultdict(dict)
    for (disp, c), v in d.items():
        per[disp][c] = sum(v)
    busy = [p for p in per.values() if p.get("SQ_BUSY_CYCLES", 0) > 0]
    mx = max(p.get("SQ_WAVE_CYCLES", 0) for p in busy) if busy else 0
    real = [p for p in busy if p.get("SQ_WAVE_CYCLES", 0) >= 0.05 * mx]
    if not real:
        continue
    avg = {c: sum(p.get(c, 0) for p in real) / len(real) for c in real[0]}
    avg["dispatches"] = len(real)
    if avg.get("SQ_WAVE_CYCLES"):
        avg["wait_any_frac_of_wave_cycles"] = avg.get("SQ_WAIT_ANY", 0) / avg["SQ_WAVE_CYCLES"]
        avg["wait_inst_any_frac_of_wave_cycles"] = avg.get("SQ_WAIT_INST_ANY", 0) / avg["SQ_WAVE_CYCLES"]
    out[k.split("(")[0]] = avg
print(json.dumps(out, indent=1))
PY
cat "$OUT/summary.json"
