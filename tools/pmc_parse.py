"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE dispatch rows per kernel.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half
the bytes of a wide (16 B/lane) coalesced streaming read, so the fetched bytes
are 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B streaming stores (our
partial-sum stores are 8 B/lane: reported as measured, uncalibrated).

Gated dispatches (a CG step queued after its solve had stopped returns at
once: tools/kstats.py) are counted apart: a dispatch whose counter is below 1%
of the kernel's largest is gated; the averages are over the others.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
out = {}
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        if "ax_partial" in k or "atx_kernel" in k or "atax_kernel" in k or "atax_team_kernel" in k or "loo_kernel" in k or "loo_wg_kernel" in k:
            d = out.setdefault(k, {})
            real = [x for x in v if x >= 0.01 * max(v)] or v
            d[counter + "_KB_avg"] = sum(real) / len(real)
            d["dispatches"] = len(real)
            d["gated_dispatches_" + counter] = len(v) - len(real)
for k, d in out.items():
    if "FETCH_SIZE_KB_avg" in d:
        d["hbm_read_bytes_per_launch"] = 2 * d["FETCH_SIZE_KB_avg"] * 1024  # gfx950 x2 correction
    if "WRITE_SIZE_KB_avg" in d:
        d["hbm_write_bytes_per_launch"] = d["WRITE_SIZE_KB_avg"] * 1024
    d["traffic_bytes_per_launch"] = d.get("hbm_read_bytes_per_launch", 0) + d.get("hbm_write_bytes_per_launch", 0)
print(json.dumps(out, indent=1))
