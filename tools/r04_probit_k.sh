#!/bin/bash
# The probit parity bar's measured gap / spread ratios (tests/_data.py
# record_probit_ratio): every probit GPU test, ratios appended to a file.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r04k
mkdir -p "$OUT"
export TMPDIR=/tmp
export VAMPOMI_PROBIT_RATIOS=$PWD/$OUT/ratios.jsonl
rm -f "$VAMPOMI_PROBIT_RATIOS"
timeout -k 10 600 python -u -m pytest tests/test_gpu_probit.py tests/test_gpu_options.py tests/test_gpu_sharded.py \
    -m gpu -q --timeout 300 --timeout-method thread -k "probit or bin_class or c4" > "$OUT/pytest.log" 2>&1
rc=$?
tail -n 5 "$OUT/pytest.log"
python - "$VAMPOMI_PROBIT_RATIOS" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
best = {}
for r in rows:
    k = r["key"]
    if r["max_ratio"] > best.get(k, (0, ""))[0]:
        best[k] = (r["max_ratio"], r["test"])
for k, (v, t) in sorted(best.items()):
    print(f"{k:7s} max gap/spread {v:.3f}  ({t})")
print("overall", max(v for v, _ in best.values()))
PY
exit $rc
