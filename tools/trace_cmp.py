"""Per-iteration kernel time of one or more rocprofv3 kernel traces of the
C2 line, side by side: iterations are delimited by the first launch of each
VAMP iteration (prelude_cg_init_kernel; `--mark K` another kernel launched
once per iteration, e.g. probit_denoise_kernel for the probit model); the first `skip` and the last
iteration are dropped (warm-up; the run's end).  Rows: us per iteration per
kernel (mean), the non-operator kernels' sum, and the idle gaps and span of
the median iteration (a profiler buffer flush can stall the host for ~10 ms
inside one iteration).

    python tools/trace_cmp.py a/run_kernel_trace.csv b/run_kernel_trace.csv [--skip 8] [--mark K]
"""
import csv
import sys
from collections import defaultdict

OPS = ("atax_team_kernel", "atax_team_plain_kernel", "ax_partial_kernel", "ax_team_kernel", "atx_kernel")  # the passes over X


def short(name):
    n = name.replace("void ", "").replace("vk::", "")
    return n.split("(")[0][:34]


def per_iter(path, skip, mark="prelude_cg_init_kernel"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
    its = list(zip(starts[skip:-1], starts[skip + 1:]))
    if not its:
        raise SystemExit(f"{path}: fewer than {skip + 2} iterations")
    tot = defaultdict(float)
    gl, sl = [], []
    for a, b in its:
        sl.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
        end, g = None, 0.0
        for r in rows[a:b]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            tot[short(r["Kernel_Name"])] += (e - s) / 1e3
            if end is not None and s > end:
                g += (s - end) / 1e3
            end = max(end or e, e)
        gl.append(g + max(0, int(rows[b]["Start_Timestamp"]) - end) / 1e3)
    n = len(its)
    out = {k: v / n for k, v in tot.items()}
    nona = sum(v for k, v in out.items() if not k.startswith(OPS))
    return n, out, nona, sorted(gl)[n // 2], sorted(sl)[n // 2]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 8
    if "--skip" in sys.argv:
        args.remove(str(skip))
    mark = sys.argv[sys.argv.index("--mark") + 1] if "--mark" in sys.argv else "prelude_cg_init_kernel"
    if "--mark" in sys.argv:
        args.remove(mark)
    res = [per_iter(p, skip, mark) for p in args]
    names = sorted({k for r in res for k in r[1]}, key=lambda k: -max(r[1].get(k, 0) for r in res))
    print("us per iteration".ljust(36) + "".join(f"{'trace ' + str(i):>12s}" for i in range(len(res))))
    print("iterations".ljust(36) + "".join(f"{r[0]:12d}" for r in res))
    for k in names:
        print(k.ljust(36) + "".join(f"{r[1].get(k, 0.0):12.1f}" for r in res))
    for label, j in (("non-operator kernels", 2), ("gaps (median iteration)", 3), ("span (median iteration)", 4)):
        print(label.ljust(36) + "".join(f"{r[j]:12.1f}" for r in res))
    print("A-pass fraction of span".ljust(36) +
          "".join(f"{sum(v for k, v in r[1].items() if k.startswith(OPS)) / r[4]:12.4f}" for r in res))


if __name__ == "__main__":
    main()
