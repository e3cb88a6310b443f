set -o pipefail
# table z-pass with the three components' sums interleaved: parity, c3 table alone and in the call
cd $GRAFT_REPO_ROOT
O=gpurun_out/z3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ghost.py tests/test_gpu_ahead.py tests/test_gpu_rungen.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
(cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 40 > $GRAFT_REPO_ROOT/$O/tr.log 2>&1) || exit 1
python3 tools/rocprof_split.py $O/tr/run_kernel_trace.csv > $O/tr.split.csv; grep "pass" $O/tr.split.csv | head -3
(cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trn -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native table 100 > $GRAFT_REPO_ROOT/$O/trn.log 2>&1) || exit 1
python3 tools/rocprof_split.py $O/trn/run_kernel_trace.csv > $O/trn.split.csv; grep "pass" $O/trn.split.csv | head -3
timeout -k 10 300 python3 tools/phase_time.py --config c3 --mode table > $O/phase.json 2>&1; cat $O/phase.json | tail -1
for v in "ylds=2 rows_per_wave=4" "ylds=2 rows_per_wave=2"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 40 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v"; grep "ypass" $O/tr_$n.split.csv | head -1
done
ab() { timeout -k 10 300 python3 tools/ab.py --config $1 --mode $2 --rounds 7 --switch-calls 8 --events ${5:-1} --tune-a "$3" --tune-b "$4" >> $O/ab.jsonl 2>$O/ab.err || exit 1; tail -1 $O/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['mode'], 'A', d['A'], d['A_median_ms'], '| B', d['B'], d['B_median_ms'])"; }
ab c2 packed rng_cus=0 rng_cus=128
ab c2 packed rng_cus=0 rng_cus=64
ab c3 table rng_cus=0 rng_cus=128 0
ab native table rng_cus=0 rng_cus=128 0
ab native packed rng_cus=0 rng_cus=128 0
