set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ghost.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "native or runtime_tuning or ghost" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/ab_multi.py --config native --mode table --tune ylds=3 --tune ylds=2,rows_per_wave=1 > $O/ab.log 2>&1; rc=$?; grep tune $O/ab.log; [ $rc -ne 0 ] && exit $rc
for args in "--tune halo_ghost=0" "--tune halo_ghost=0 --env DFAMD_SOLO_XCHG_US=40" "--tune halo_ghost=1" "--tune halo_ghost=1 --env DFAMD_SOLO_XCHG_US=40"; do
  echo "== strip $args"
  timeout -k 10 300 python3 tools/strip_timing.py --config c4 --mode table --replicate 0 --ns 8 --calls 200 $args >> $O/strip.jsonl 2> $O/strip.err || { tail $O/strip.err; exit 1; }
  tail -2 $O/strip.jsonl
done
