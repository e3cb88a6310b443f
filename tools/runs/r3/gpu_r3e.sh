#!/bin/bash
# Occupancy of the overlapped RNG: K3a with 32 / 128 chunks per wave (fewer resident waves) and K1
# with a capped grid, against the defaults, c3 table; event cost with sampled events; parity of the
# new knobs (the runtime-tuning test covers them).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3e}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for tb in "dense_g=32" "dense_g=128" "count_grid=1024" "count_grid=2048" "dense_g=128,count_grid=1024"; do
  timeout -k 10 300 python3 tools/ab.py --torch --config c3 --mode table --rounds 9 --tune-a dense_g=8,count_grid=0 --tune-b $tb \
    >> $O/ab_occupancy.jsonl 2>> $O/ab.err || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
  tail -1 $O/ab_occupancy.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['B'], 'A', d['A_median_ms']['total_ms'], d['A_median_ms']['wall_ms'], 'B', d['B_median_ms']['total_ms'], d['B_median_ms']['wall_ms'])"
done
for cfg in "native packed" "c2 packed" "native table" "c3 table"; do
  timeout -k 10 120 python3 tools/event_cost.py $cfg 9 50 >> $O/event_cost.jsonl 2> $O/ev.err || { echo "event_cost failed"; tail -5 $O/ev.err; exit 1; }
done
cat $O/event_cost.jsonl
