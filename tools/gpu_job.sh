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
# Outputs: gpurun_out/TAG/<i>_<step>.{log,json}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1; shift
O=$ROOT/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
i=0
for step in "$@"; do
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
    *) echo "unknown step $name"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "[gpu_job] step $i ($name) failed rc=$rc"; tail -40 "$base.log" 2>/dev/null
    exit $rc
  fi
done
echo "[gpu_job $(date +%T)] done"
