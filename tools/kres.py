"""Per-kernel VGPRs / spills / occupancy from hipcc -Rpass-analysis=kernel-resource-usage output.

    hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [substring]
"""
import re
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    if pat in k:
        print(f"{k[:60]:60s} vgpr {v.get('VGPRs')} spill {v.get('VGPRs Spill')} occ {v.get('Occupancy [waves/SIMD]')}")
