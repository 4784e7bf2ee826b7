"""Per-kernel statistics from a rocprofv3 kernel trace, with the gated launches
of the A / A^T / association kernels counted apart.

The CG loop queues its next step before the current one has decided
(pcg.cpp): after the last step of a solve one queued step runs with its gate
closed, and each of its kernels returns at once (a few microseconds).  The
bench's HIP-event timing drops those launches; so does this summary, which is
the one to compare with bench.py's avg_launch_us.  A launch is gated when it
took less than 5% of the kernel's longest launch.

    python tools/kstats.py run_kernel_trace.csv > kernel_stats_real.csv
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
dur = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    dur[n].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "GatedCalls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
for n, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    gated = []
    if any(k in n for k in ("ax_partial_kernel", "atx_kernel", "atax_kernel", "atax_team_kernel", "loo_kernel")):
        cut = 0.05 * max(d)
        gated = [x for x in d if x < cut]
        d = [x for x in d if x >= cut]
    if not d:
        continue
    w.writerow([n, len(d), len(gated), sum(d), round(sum(d) / len(d), 1), min(d), max(d)])
