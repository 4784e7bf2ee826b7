"""main_meth.exe at C2 with and without its per-iteration output files
(src/vamp.cpp:235-249 _it_K.bin / _r1_it_K.bin, :388-393 CSV rows): the
drop-in user's rate.  Writes the C2 problem (N = 10,000 x Mt = 50,000,
tests/_data.py make_problem seed 11) as marker-major .bin + PLINK .phen into a
scratch directory, then runs the CLI alternately with --out-dir and without,
--iterations 25 --stop-criteria-thr 0, and reports iterations/s from the CLI's
own "total computation time" (vampomi_infere: all iterations, writes included).

    python tools/cli_write_ab.py [scratch_dir] [reps]
"""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import vampomi_amd as va  # noqa: E402
from _data import make_problem  # noqa: E402

N, MT, ITS = 10000, 50000, 25
base = tempfile.mkdtemp(prefix="vampomi_cli_", dir=sys.argv[1] if len(sys.argv) > 1 else None)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
try:
    X, y, beta = make_problem(N, MT, seed=11)
    X.astype("<f8").tofile(os.path.join(base, "c2.bin"))
    del X
    with open(os.path.join(base, "c2.phen"), "w") as f:
        f.write("".join("%d %d %0.10f\n" % (i, i, v) for i, v in enumerate(y)))
    cmd = [va.CLI_PATH, "--meth-file", os.path.join(base, "c2.bin"), "--phen-file", os.path.join(base, "c2.phen"),
           "--N", str(N), "--Mt", str(MT), "--iterations", str(ITS), "--stop-criteria-thr", "0"]
    out = {"nowrite": [], "write": []}
    for r in range(reps):
        for mode in ("nowrite", "write"):
            extra = []
            if mode == "write":
                od = os.path.join(base, f"out{r}")
                os.makedirs(od, exist_ok=True)
                extra = ["--out-dir", od, "--out-name", "c2"]
            p = subprocess.run(cmd + extra, capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                raise SystemExit(p.stdout[-2000:] + p.stderr[-2000:])
            secs = float(re.search(r"total computation time = ([0-9.eE+-]+) s", p.stdout).group(1))
            out[mode].append(ITS / secs)
            print(mode, round(ITS / secs, 2), "it/s", flush=True)
    files = sorted(os.listdir(os.path.join(base, "out0")))
    res = {"workload": "c2 via main_meth.exe (N=10000, Mt=50000, 25 iterations, iteration 1 included)",
           "it_s_nowrite": [round(v, 3) for v in out["nowrite"]], "it_s_write": [round(v, 3) for v in out["write"]],
           "ratio_write_over_nowrite": round(max(out["write"]) / max(out["nowrite"]), 4),
           "files_per_run": len(files)}
    print(json.dumps(res))
finally:
    shutil.rmtree(base, ignore_errors=True)
