set -o pipefail
# the round's closing evidence: full GPU suite, smoke, default bench, its rocprofv3 summary
cd $GRAFT_REPO_ROOT
O=gpurun_out/${FINAL_TAG:-final}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.log || exit 1
python3 tools/bench_summary.py $O/bench.json || true
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline off > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || exit 1
python3 tools/rocprof_split.py $O/prof/run_kernel_trace.csv > $O/prof.split.csv; head -14 $O/prof.split.csv
