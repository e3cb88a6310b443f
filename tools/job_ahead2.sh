set -o pipefail
# y-pass ahead on the reference's grid (now its default) and on c4/8 table ranks with and without the exchange hold
cd $GRAFT_REPO_ROOT
O=gpurun_out/ahead2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ahead.py tests/test_gpu_ghost.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "native or ahead or ghost_strips" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for t in "halo_ghost=0:ypass_ahead=0" "halo_ghost=0:ypass_ahead=1" "halo_ghost=1:ypass_ahead=0" "halo_ghost=1:ypass_ahead=1"; do
 for h in "" "--env DFAMD_SOLO_XCHG_US=40"; do
  echo "== strip $t $h"
  timeout -k 10 300 python3 tools/strip_timing.py --config c4 --mode table --replicate 0 --ns 8 --calls 200 --tune $t $h >> $O/strip.jsonl 2> $O/strip.err || { tail $O/strip.err; exit 1; }
  tail -2 $O/strip.jsonl | cut -c1-220
 done
done
