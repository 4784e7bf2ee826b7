"""The probit parity bar's measured gap / spread ratios (tests/_data.py
record_probit_ratio writes one JSON row per checked iteration set): the
maximum per key, and overall.

    python tools/probit_ratios.py gpurun_out/<tag>/ratios.jsonl
"""
import json
import sys

rows = [json.loads(line) for line in open(sys.argv[1])]
best = {}
for r in rows:
    k = r["key"]
    if r["max_ratio"] > best.get(k, (0.0, ""))[0]:
        best[k] = (r["max_ratio"], r["test"])
for k, (v, t) in sorted(best.items()):
    print(f"{k:7s} max gap/spread {v:.3f}  ({t})")
print("overall", max(v for v, _ in best.values()) if best else None)
