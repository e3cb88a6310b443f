set -o pipefail
# the default bench line, its rocprofv3 kernel summary, then the PMC traffic of every plane of the line
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ahead.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.log || exit 1
python3 tools/bench_summary.py $O/bench.json || true
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline off > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || exit 1
python3 tools/rocprof_split.py $O/prof/run_kernel_trace.csv > $O/prof.split.csv; head -12 $O/prof.split.csv
timeout -k 10 900 python3 tools/pmc_traffic.py --out $O/pmc --json $O/pmc_traffic.json > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 -c "import json; print(json.dumps(json.load(open('$O/pmc_traffic.json'))['per_launch_bytes'], indent=1))"
