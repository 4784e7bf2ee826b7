"""Side-stream overlap in a rocprofv3 kernel trace: for every kernel of the
prefetched denoiser/EM (em_kernel, denoise_kernel) the time it ran together
with a kernel of another queue (the main stream's reductions), per kernel.

    python tools/trace_overlap.py gpurun_out/prof_c2/<pid>_kernel_trace.csv [out.json]
"""
import collections
import csv
import json
import sys

SIDE = ("em_kernel", "denoise_kernel")


def name(r):
    return r["Kernel_Name"].split("(")[0].replace("void vk::", "").replace("vk::", "")


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    qkey = "Queue_Id" if rows and "Queue_Id" in rows[0] else "Stream_Id"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r), r.get(qkey, "")) for r in rows]
    res = collections.defaultdict(lambda: {"launches": 0, "busy_us": 0.0, "overlapped_us": 0.0,
                                           "with": collections.Counter(), "queues": set()})
    for i, (s, e, n, q) in enumerate(ev):
        if not n.startswith(SIDE):
            continue
        d = res[n.split("<")[0]]
        d["launches"] += 1
        d["busy_us"] += (e - s) / 1e3
        d["queues"].add(q)
        # kernels of other queues that ran inside [s, e)
        iv = []
        for j in range(max(0, i - 64), min(len(ev), i + 64)):
            s2, e2, n2, q2 = ev[j]
            if j == i or q2 == q:
                continue
            a, b = max(s, s2), min(e, e2)
            if b > a:
                iv.append((a, b))
                d["with"][n2.split("<")[0]] += 1
        iv.sort()
        tot, cur = 0, None
        for a, b in iv:  # union of the overlapping intervals
            if cur and a <= cur[1]:
                cur[1] = max(cur[1], b)
            else:
                if cur:
                    tot += cur[1] - cur[0]
                cur = [a, b]
        if cur:
            tot += cur[1] - cur[0]
        d["overlapped_us"] += tot / 1e3
    summary = {k: {"launches": v["launches"], "busy_us": round(v["busy_us"], 1),
                   "overlapped_us": round(v["overlapped_us"], 1),
                   "overlap_frac": round(v["overlapped_us"] / v["busy_us"], 3) if v["busy_us"] else 0.0,
                   "queues": sorted(v["queues"]), "ran_beside": dict(v["with"].most_common(6))}
               for k, v in res.items()}
    print(json.dumps(summary, indent=1))
    if out:
        json.dump({"trace": path, "side_stream_kernels": summary}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
