"""Per-launch durations of the one-pass operator in a rocprofv3 kernel trace,
grouped by the kernel that ran before it and by its position in the CG
solve (the first launch after the solve's A.x pass, the later ones), and the
idle gap before each.

    python tools/trace_op.py gpurun_out/prof/run_kernel_trace.csv [skip_fraction]
"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
rows = rows[int(len(rows) * skip):]


def short(r):
    return r["Kernel_Name"].split("(")[0].replace("void vk::", "").replace("vk::", "").split("<")[0]


by_prev, by_pos, gaps = collections.defaultdict(list), collections.defaultdict(list), collections.defaultdict(list)
pos = 0
for i, r in enumerate(rows):
    n = short(r)
    if n == "ax_partial_kernel":
        pos = 0
    if n != "atax_team_kernel":
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if d < 50:  # gated launch (the step queued after the solve stopped)
        continue
    prev = rows[i - 1] if i else None
    pn = short(prev) if prev else "-"
    by_prev[pn].append(d)
    by_pos[min(pos, 9)].append(d)
    if prev:
        gaps[pn].append((int(r["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3)
    pos += 1
print("operator launches by the kernel before them:")
for k, v in sorted(by_prev.items(), key=lambda kv: -len(kv[1])):
    print("  %-28s n=%4d mean %7.1f us  min %7.1f  max %7.1f  gap before %.1f us" %
          (k, len(v), statistics.mean(v), min(v), max(v), statistics.mean(gaps[k]) if gaps[k] else 0))
print("by position in the solve (0 = first launch after the A.x pass):")
for k in sorted(by_pos):
    v = by_pos[k]
    print("  %d: n=%4d mean %7.1f us  min %7.1f  max %7.1f" % (k, len(v), statistics.mean(v), min(v), max(v)))
