"""Per-kernel register use and spills of a HIP source file (gfx950), from the
compiler's kernel-resource-usage remarks:

    python tools/regcheck.py vampomi_amd/csrc/atax_team.hip [name-filter]
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950",
                      "-I" + ROOT + "/include", "-I" + ROOT + "/vampomi_amd/csrc", "-c", src, "-o", "/dev/null",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))
for r in rows:
    if flt in r["name"]:
        print("%-100s VGPR %3d AGPR %3d spill(s/v) %3d/%3d scratch %d" % (
            r["name"][:100], r.get("VGPRs", 0), r.get("AGPRs", 0), r.get("SGPRs Spill", 0), r.get("VGPRs Spill", 0),
            r.get("ScratchSize [bytes/lane]", 0)))
