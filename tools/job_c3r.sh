set -o pipefail
# c3 table: the per-wave y-pass at 2, 4, 8 rows per wave, alone (RNG on the sweep stream) and in the call
cd $GRAFT_REPO_ROOT
O=gpurun_out/c3r; mkdir -p $O
for v in "rows_per_wave=2" "rows_per_wave=4" "rows_per_wave=8"; do
  n=$(echo $v | tr ' =' '_-')
  (cd /tmp && DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py c3 table 40 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v"; grep "ypass" $O/tr_$n.split.csv | head -2
done
timeout -k 10 300 python3 tools/ab.py --config c3 --mode table --rounds 7 --events 0 --switch-calls 4 --tune-a rows_per_wave=4 --tune-b rows_per_wave=8 > $O/ab.json 2>&1; tail -1 $O/ab.json | cut -c1-300
