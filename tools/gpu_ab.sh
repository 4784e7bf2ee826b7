#!/bin/bash
# A/B of environment settings on one box, alternating, each a C2 bench line
# (or --config given by AB_CONFIG) and a rocprofv3 kernel-stats run.
#   gpurun -- bash tools/gpu_ab.sh "VAMPOMI_CG_EPT=2" "VAMPOMI_CG_EPT=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/ab
mkdir -p "$OUT"
export TMPDIR=/tmp
CFG=${AB_CONFIG:-c2}
STEPS=${AB_STEPS:-20}
for rep in 1 2 3; do
    i=0
    for setting in "$@"; do
        i=$((i + 1))
        env $setting timeout -k 10 300 python bench.py --config "$CFG" --steps "$STEPS" --warmup 5 --no-cpu-baseline \
            > "$OUT/v${i}_$rep.log" 2>&1 || { echo "v$i rep $rep failed"; tail -5 "$OUT/v${i}_$rep.log"; exit 1; }
        python - "$OUT/v${i}_$rep.log" "$setting" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:32s} {d['value']:9.3f} it/s  {d['ms_per_step']:8.3f} ms/step  op {d['roofline']['avg_launch_us']:8.1f} us")
PY
    done
done
i=0
for setting in "$@"; do
    i=$((i + 1))
    export $setting
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_v$i" -o run --output-format csv -- \
        python bench.py --config "$CFG" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_v$i.log" 2>&1 || exit 1
    unset "${setting%%=*}"
    echo "== $setting"
    head -8 "$OUT/prof_v$i/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-40,120-220
done
