#!/bin/bash
# One GPU call's steps, in order, each under its own time limit; the call ends
# at the first step that fails (its log under gpurun_out/<tag>/):
#
#   gpurun -- bash tools/gpu_session.sh <tag> <step> [<step> ...]
#
# steps:
#   suite        the GPU test suite (durations of the slowest tests)
#   fullshard    the whole-shard oracle tests alone (C3, C4, C5)
#   tests        the GPU tests named in $TESTS (pytest arguments; $TESTK: a -k expression)
#   rehearse     bench.py's n > 1 flow with 8 loopback rank threads on this GPU
#   bitwise      12 VAMP iterations (linear and probit; N x Mt = $BWN x $BWM, default 10000 x 20000) on this build and on
#                $OLD (default build_ab/, make -C vampomi_amd/csrc OBJDIR=../../build_ab/obj LIBDIR=../../build_ab/lib BINDIR=../../build_ab/bin at the base commit), compared bit for bit
#   ab           C2 lines alternating this build and $OLD, $ROUNDS rounds
#   envab        C2 lines alternating the settings in $ENVAB ("A=1;A=2;...")
#   envtrace     a kernel trace of the C2 line ($ENVCFG: another config, $ENVSTEPS steps) per setting in $ENVAB,
#                per-iteration kernel times side by side
#   trace        rocprofv3 kernel trace of the C2 line + the gap analysis
#   trace_old    the same for $OLD
#   hiptrace     rocprofv3 HIP API + kernel trace of a short C2 line
#   timing       the C2 rate at timing period 4 / 16 / none
#   probit_k     every probit test, the parity bar's gap / spread ratios
#   launcher     the default C2 line over a 1-rank RCCL communicator, and the
#                2-rank launcher on a 1-GPU box (one failure line, rc != 0)
#   rccl         the 1-rank RCCL path against the direct one (rates, timing on/off, traces compared)
#   ceiling      the HBM read ceiling of this box (tools/hbm_ceiling, 4 GB and 50 GB buffers)
#   ablation     the C2 operator's components removed one at a time (tools/op_ablation.py, build_dbg/: TM_DBG=1)
#   benchc2      the default C2 line, both CPU legs
#   c4           the probit shard's line and its per-iteration kernel trace
#   bases        rank 0's 1-GPU bases (tools/one_gpu_bases.py)
#   final        smoke, the default C2 line (both CPU legs), its kernel stats
#                and PMC traffic; the same for C3; C4 and C5 lines
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
OLD=${OLD:-$PWD/build_ab/lib/libvampomi.so}
ROUNDS=${ROUNDS:-3}
step() {
    local name=$1 tmo=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 2 "$OUT/$name.log" | cut -c1-400
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
brief() {
    grep '^{' "$OUT/$1.log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('$1', d['value'], d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'), d.get('a_kernel_frac_of_step'))" | tee -a "$OUT/ab.txt"
}
C2=(python bench.py --steps 20 --warmup 5 --no-cpu-baseline)
prof() {
    step "rocprof_$1" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$1" -o run --output-format csv -- \
        python bench.py --config "$1" --steps "$2" --warmup 5 --no-cpu-baseline
}
for s in "$@"; do
    case $s in
    suite)
        step suite 900 python -u -m pytest tests -m gpu -x -q --durations=12 --timeout 400 --timeout-method thread ;;
    fullshard)
        step fullshard 900 python -u -m pytest tests/test_gpu_scale.py::test_c3_full_shard_window_vs_oracle_fixture \
            tests/test_gpu_probit.py::test_c4_full_shard_vs_oracle \
            tests/test_gpu_assoc.py::test_c5_full_shard_vs_oracle -m gpu -v --durations=0 --timeout 400 \
            --timeout-method thread ;;
    tests)       # TESTS="<pytest args>": a subset, the probit gap / spread ratios recorded
        export VAMPOMI_PROBIT_RATIOS=$PWD/$OUT/ratios.jsonl
        step tests 900 python -u -m pytest $TESTS ${TESTK:+-k "$TESTK"} -m gpu -v --durations=8 --timeout 300 \
            --timeout-method thread
        [ -f "$VAMPOMI_PROBIT_RATIOS" ] && python tools/probit_ratios.py "$VAMPOMI_PROBIT_RATIOS" | tee "$OUT/probit_k.txt"
        unset VAMPOMI_PROBIT_RATIOS ;;
    rehearse)
        step rehearse 400 python bench.py --rehearse 8 --steps 3 --warmup 1 --deadline-s 380 ;;
    bitwise)
        for m in linear bin_class; do
            step bw_new_$m 200 python tools/lib_bitwise.py run "$OUT/new_$m.npz" "${BWN:-10000}" "${BWM:-20000}" 12 $m
            step bw_old_$m 200 env VAMPOMI_LIB="$OLD" python tools/lib_bitwise.py run "$OUT/old_$m.npz" \
                "${BWN:-10000}" "${BWM:-20000}" 12 $m
            python tools/lib_bitwise.py cmp "$OUT/new_$m.npz" "$OUT/old_$m.npz" | tee -a "$OUT/bitwise.txt"
        done ;;
    ab)
        for r in $(seq "$ROUNDS"); do
            step ab_new_$r 200 "${C2[@]}" && brief ab_new_$r
            step ab_old_$r 200 env VAMPOMI_LIB="$OLD" "${C2[@]}" && brief ab_old_$r
        done ;;
    envab)
        IFS=';' read -r -a settings <<< "${ENVAB:-}"
        for r in $(seq "$ROUNDS"); do
            i=0
            for e in "${settings[@]}"; do
                i=$((i + 1))
                step env${i}_$r 200 env $e "${C2[@]}" && brief env${i}_$r
            done
        done ;;
    envtrace)    # a kernel trace of the C2 line per setting in $ENVAB, compared per iteration
        IFS=';' read -r -a settings <<< "${ENVAB:-}"
        i=0
        traces=()
        for e in "${settings[@]}"; do
            i=$((i + 1))
            step envtrace$i 300 env $e rocprofv3 --kernel-trace --stats -d "$OUT/prof_env$i" -o run --output-format csv \
                -- python bench.py --config "${ENVCFG:-c2}" --steps "${ENVSTEPS:-20}" --warmup 5 --no-cpu-baseline --no-timing
            traces+=("$(find "$OUT/prof_env$i" -name 'run_kernel_trace.csv' | head -1)")
        done
        python tools/trace_cmp.py "${traces[@]}" | tee "$OUT/envtrace_cmp.txt" ;;
    trace)
        step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
            python bench.py --steps 20 --warmup 5 --no-cpu-baseline
        f=$(find "$OUT/prof" -name 'run_kernel_trace.csv' | head -1)
        python tools/trace_gaps.py "$f" 0.3 > "$OUT/gaps.txt" && head -34 "$OUT/gaps.txt" ;;
    trace_old)
        VAMPOMI_LIB="$OLD" step trace_old 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_old" -o run \
            --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
        f=$(find "$OUT/prof_old" -name 'run_kernel_trace.csv' | head -1)
        python tools/trace_gaps.py "$f" 0.3 > "$OUT/gaps_old.txt" && head -34 "$OUT/gaps_old.txt" ;;
    hiptrace)
        step hiptrace 300 rocprofv3 --hip-trace --kernel-trace -d "$OUT/hprof" -o run --output-format csv -- \
            python bench.py --steps 6 --warmup 2 --no-cpu-baseline ;;
    timing)
        for r in $(seq "$ROUNDS"); do
            step tp4_$r 200 "${C2[@]}" --timing-period 4 && brief tp4_$r
            step tp16_$r 200 "${C2[@]}" --timing-period 16 && brief tp16_$r
            step tpnone_$r 200 "${C2[@]}" --no-timing && brief tpnone_$r
        done ;;
    probit_k)
        export VAMPOMI_PROBIT_RATIOS=$PWD/$OUT/ratios.jsonl
        rm -f "$VAMPOMI_PROBIT_RATIOS"
        step probit_k 600 python -u -m pytest tests/test_gpu_probit.py tests/test_gpu_options.py \
            tests/test_gpu_sharded.py -m gpu -q --timeout 300 --timeout-method thread -k "probit or bin_class or c4"
        python tools/probit_ratios.py "$VAMPOMI_PROBIT_RATIOS" | tee "$OUT/probit_k.txt"
        unset VAMPOMI_PROBIT_RATIOS ;;
    launcher)
        step bench_c2_rccl1 200 env VAMPOMI_FORCE_RCCL=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
        echo "== spawn2_on_one_gpu ($(date +%T))"
        timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --deadline-s 240 > "$OUT/spawn2.log" 2>&1
        echo "rc=$?" >> "$OUT/spawn2.log"
        tail -n 2 "$OUT/spawn2.log" | cut -c1-2500 ;;
    rccl)        # the 1-rank RCCL path against the direct one: rates with and without event timing, traces
        for r in $(seq "$ROUNDS"); do
            step rc_dir_$r 200 "${C2[@]}" && brief rc_dir_$r
            step rc_rccl_$r 200 env VAMPOMI_FORCE_RCCL=1 "${C2[@]}" && brief rc_rccl_$r
            step rc_dir_nt_$r 200 "${C2[@]}" --no-timing && brief rc_dir_nt_$r
            step rc_rccl_nt_$r 200 env VAMPOMI_FORCE_RCCL=1 "${C2[@]}" --no-timing && brief rc_rccl_nt_$r
        done
        step trace_dir 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_dir" -o run --output-format csv -- \
            python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-timing
        VAMPOMI_FORCE_RCCL=1 step trace_rccl 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rccl" -o run \
            --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-timing
        python tools/trace_cmp.py "$(find "$OUT/prof_dir" -name 'run_kernel_trace.csv' | head -1)" \
            "$(find "$OUT/prof_rccl" -name 'run_kernel_trace.csv' | head -1)" | tee "$OUT/trace_cmp.txt" ;;
    ceiling)     # the HBM read ceiling (tools/hbm_ceiling: every byte of a 4 GB / 50 GB buffer read once)
        step ceiling_4 200 tools/hbm_ceiling 4 15
        step ceiling_50 300 tools/hbm_ceiling 50 5 ;;
    ablation)    # the C2 operator's components, one at a time, against the same process's read stream (TM_DBG build)
        step ablation 400 env VAMPOMI_LIB="$PWD/build_dbg/lib/libvampomi.so" python tools/op_ablation.py 10000 50000 40 3 ;;
    ablibs)      # the C2 operator with a component removed at compile time (TM_ABL builds), against production
        step ablibs 600 bash tools/op_ablation_libs.sh 3 ;;
    benchc2)     # the default C2 line with both CPU legs
        step bench_c2 400 python bench.py --steps 20 --warmup 5 ;;
    c4)          # the probit shard: its line, and a kernel trace of 10 iterations (A passes against the rest)
        step bench_c4 400 python bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline
        step trace_c4 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv -- \
            python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline --no-timing
        python tools/trace_cmp.py "$(find "$OUT/prof_c4" -name 'run_kernel_trace.csv' | head -1)" --skip 2 \
            --mark probit_denoise_kernel | tee "$OUT/trace_c4.txt"
        python tools/trace_gaps.py "$(find "$OUT/prof_c4" -name 'run_kernel_trace.csv' | head -1)" 0.3 \
            > "$OUT/gaps_c4.txt" ;;
    bases)
        step bases 200 python tools/one_gpu_bases.py ;;
    final)
        step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
        step bench_c2 400 python bench.py --steps 20 --warmup 5
        prof c2 20
        step pmc_c2 300 bash tools/pmc.sh c2
        step bench_c3 400 python bench.py --config c3 --steps 10 --warmup 2
        prof c3 6
        step pmc_c3 300 bash tools/pmc.sh c3
        step bench_c4 400 python bench.py --config c4 --steps 6 --warmup 2   # iterations 3-8: inside test_c4_full_shard_vs_oracle
        step bench_c5 300 python bench.py --config c5 --steps 5 --warmup 1 ;;
    *)
        echo "unknown step $s"; exit 2 ;;
    esac
done
echo done
