#!/bin/bash
# One GPU job: a tag and a list of steps, each under its own time limit; the first failing step ends
# the job (no retries, nothing after a fault). Replaces the one-shot tools/runs/r*/ scripts.
#
#   tools/gpu_job.sh TAG STEP [STEP ...]
#
# STEP                        runs                                                         limit
#   tests[=PYTEST_ARGS]       python -u -m pytest PYTEST_ARGS (default: tests) -m gpu -x -v 1100 s
#   bench[=BENCH_ARGS]        python3 bench.py BENCH_ARGS            -> bench.json         900 s
#   bench8emu[=BENCH_ARGS]    DFAMD_EMULATE_HOSTS=1 python3 bench.py --gpus 8 BENCH_ARGS  900 s
#   strip[=ARGS]              python3 tools/strip_timing.py ARGS                           400 s
#   prof[=BENCH_ARGS]         rocprofv3 --kernel-trace --stats -- python3 bench.py ...     600 s
#   py=SCRIPT[,ARGS]          python3 SCRIPT ARGS (commas become spaces)                   400 s
#   rocpy=SCRIPT[,ARGS]       rocprofv3 --kernel-trace --stats -- python3 SCRIPT ARGS       400 s
#   sh=SCRIPT[,ARGS]          bash SCRIPT ARGS (a tools/ script)                           400 s
#   smoke                     __graft_entry__.smoke()                                      300 s
#   ab=CFG,MODE,A,B[,ROUNDS]  tools/ab.py one-handle A/B of tunings A vs B (k=v, several joined by +), 60-call
#                             windows, 24 untimed calls after each switch, wall only -> ab.jsonl           300 s
#   trace=PLANE,MODE,CALLS[,k=v ...]  rocprofv3 kernel trace of tools/plane_loop.py with the RNG on the sweep
#                             stream (DFAMD_RNG_OVERLAP=0: every kernel timed alone) -> split.csv          200 s
#   pmc=PLANE,MODE,CALLS[,k=v ...]    tools/pmc_plane.sh: SQ counter passes + a kernel trace -> pmc.json  600 s
#   final                     the closing run: tests, smoke, bench, rocprofv3 of the bench (as four steps)
# Outputs: gpurun_out/TAG/<i>_<step>.{log,json}. Every earlier one-off tools/job_*.sh is one line of these steps
# (tools/README.md, "Recipes").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1; shift
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
steps=()
for step in "$@"; do
  if [ "$step" = final ]; then steps+=(tests smoke bench prof=--cpu-baseline,off); else steps+=("$step"); fi
done
i=0
for step in "${steps[@]}"; do
  i=$((i + 1))
  name=${step%%=*}
  arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  arg=${arg//,/ }
  base="$O/${i}_${name}"
  echo "[gpu_job $(date +%T)] step $i: $name $arg"
  case $name in
    tests) timeout -k 10 1100 python -u -m pytest ${arg:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 \
             --timeout-method thread > "$base.log" 2>&1; rc=$?; tail -3 "$base.log" ;;
    bench) timeout -k 10 900 python3 bench.py $arg > "$base.json" 2> "$base.log"; rc=$?
           [ $rc -eq 0 ] && python3 tools/bench_summary.py "$base.json" ;;
    bench8emu) start=$(date +%s)
           DFAMD_EMULATE_HOSTS=1 DFAMD_BENCH_TIMEOUT=870 timeout -k 10 900 python3 bench.py --gpus 8 $arg > "$base.json" 2> "$base.log"; rc=$?
           echo "wall_s $(( $(date +%s) - start ))" | tee "$base.wall"
           [ $rc -eq 0 ] && python3 tools/bench_summary.py "$base.json" ;;
    strip) timeout -k 10 400 python3 tools/strip_timing.py $arg > "$base.json" 2> "$base.log"; rc=$?; cat "$base.json" ;;
    prof) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$base.d" -o run -- \
             python3 "$ROOT/bench.py" $arg > "$base.log" 2>&1); rc=$?
          [ $rc -eq 0 ] && python3 tools/rocprof_split.py "$base.d/run_kernel_trace.csv" > "$base.split.csv" && head -25 "$base.split.csv" ;;
    py) set -- $arg; script=$1; shift
        timeout -k 10 400 python3 "$script" "$@" > "$base.log" 2>&1; rc=$?; tail -30 "$base.log" ;;
    rocpy) set -- $arg; script=$1; shift
        (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$base.d" -o run -- \
            python3 "$ROOT/$script" "$@" > "$base.log" 2>&1); rc=$?
        [ $rc -eq 0 ] && python3 tools/rocprof_split.py "$base.d/run_kernel_trace.csv" > "$base.split.csv" && head -25 "$base.split.csv" ;;
    sh) set -- $arg; script=$1; shift
        timeout -k 10 400 bash "$script" "$@" > "$base.log" 2>&1; rc=$?; tail -30 "$base.log" ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$base.log" 2>&1; rc=$?; tail -2 "$base.log" ;;
    ab) set -- $arg
        timeout -k 10 300 python3 tools/ab.py --config $1 --mode $2 --rounds ${5:-7} --calls 60 --switch-calls 24 \
          --events 0 --tune-a "${3//+/,}" --tune-b "${4//+/,}" >> "$O/ab.jsonl" 2> "$base.log"; rc=$?
        [ $rc -eq 0 ] && tail -1 "$O/ab.jsonl" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); \
print(d['config'], d['mode'], 'A', d['A'], d['A_median_ms']['wall_ms'], '| B', d['B'], d['B_median_ms']['wall_ms'])" ;;
    trace) set -- $arg; plane=$1; mode=$2; calls=$3; shift 3
        (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
           -d "$base.d" -o run -- python3 "$ROOT/tools/plane_loop.py" $plane $mode $calls "$@" > "$base.log" 2>&1); rc=$?
        [ $rc -eq 0 ] && python3 tools/rocprof_split.py "$base.d/run_kernel_trace.csv" > "$base.split.csv" && \
          grep -E "ypass|zpass|rng_" "$base.split.csv" | head -8 ;;
    pmc) set -- $arg
        PMC_TAG=_$i timeout -k 10 600 bash tools/pmc_plane.sh "$@" > "$base.log" 2>&1; rc=$?; tail -12 "$base.log" ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "[gpu_job] step $i ($name) failed rc=$rc"; tail -40 "$base.log" 2>/dev/null
    exit $rc
  fi
done
echo "[gpu_job $(date +%T)] done"
