#!/bin/bash
# K1f: count + decoupled look-back scan + compaction in one launch (table mode, dense generation, one GPU).
# Parity first (forced on small planes, the tuning matrix, whole c3 planes), then same-handle A/B
# gen_fused 0 vs 1 on c3/c5 table (overlap on and off) and a serial kernel timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "fused_count or runtime_tuning or bitexact_vs_oracle or native or handoff" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py \
  -k "c3" > $O/pytest_c3.log 2>&1 || { echo "pytest c3 failed"; tail -30 $O/pytest_c3.log; exit 1; }
tail -1 $O/pytest_c3.log
for ov in 0 1; do
  for cfg in c3 c5; do
    DFAMD_RNG_OVERLAP=$ov timeout -k 10 200 python3 tools/ab.py --config $cfg --mode table --rounds 9 --calls 20 \
      --tune-a gen_fused=0 --tune-b gen_fused=1 > $O/ab_${cfg}_ov$ov.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${cfg}_ov$ov.json'));print('$cfg overlap $ov fused0', d['A_median_ms'], 'fused1', d['B_median_ms'])"
  done
done
