"""The probit parity bar's measured gap / spread ratios (tests/_data.py
record_probit_ratio writes one JSON row per checked iteration set): the
maximum per key, and overall; then the device-order rows (gap to the
oracle in the device's order of the sums, from iteration 3 on).

    python tools/probit_ratios.py gpurun_out/<tag>/ratios.jsonl
"""
import json
import sys

rows = [json.loads(line) for line in open(sys.argv[1])]
best = {}
dev = [r for r in rows if "gap_dev" in r and "key" in r]
for r in rows:
    if "max_ratio" not in r:
        continue
    k = r["key"]
    if r["max_ratio"] > best.get(k, (0.0, ""))[0]:
        best[k] = (r["max_ratio"], r["test"])
for k, (v, t) in sorted(best.items()):
    print(f"{k:7s} max gap/spread {v:.3f}  ({t})")
print("overall", max(v for v, _ in best.values()) if best else None)
for r in dev:
    g, q = r["gap_dev"][2:], r["gap_seq"][2:]
    if g:
        print(f"{r['test']:28s} {r['key']}: max gap to the device order {max(g):.2e} (restatement {max(q):.2e})")
