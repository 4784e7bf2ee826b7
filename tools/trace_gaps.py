"""Summarise a rocprofv3 kernel trace: per-kernel time, and the idle gaps
between consecutive kernels grouped by (previous, next) kernel.

    python tools/trace_gaps.py gpurun_out/prof3/run_kernel_trace.csv [skip_fraction]
"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.4
sel = rows[int(len(rows) * skip):]
busy, cnt, gaps = collections.Counter(), collections.Counter(), []
prev = prevn = None
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].split("(")[0].replace("void vk::", "").replace("vk::", "")
    busy[n] += e - s
    cnt[n] += 1
    if prev is not None:
        gaps.append((s - prev, n, prevn))
    prev, prevn = e, n
T = int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])
print("span %.2f ms, kernels %.2f ms, gaps %.2f ms" % (T / 1e6, sum(busy.values()) / 1e6,
                                                     sum(g for g, _, _ in gaps if g > 0) / 1e6))
for n, b in busy.most_common(16):
    print("%-44s %5d %8.3f ms  avg %7.1f us" % (n[:44], cnt[n], b / 1e6, b / cnt[n] / 1e3))
gb = collections.defaultdict(list)
for g, n, p in gaps:
    gb[(p[:28], n[:28])].append(g)
for k, v in sorted(gb.items(), key=lambda kv: -sum(kv[1]))[:10]:
    print("%-62s n=%4d mean %6.1f us total %.2f ms" % (k, len(v), statistics.mean(v) / 1e3, sum(v) / 1e6))
