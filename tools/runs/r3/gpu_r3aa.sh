#!/bin/bash
# Table mode, c3: room for the RNG beside the sweeps. Dynamic-LDS occupancy caps on the y-pass / z-pass blocks
# (ylds_kb / zlds_kb, same handle A/B) and the y-pass built with per-tap schedule barriers (tapsb) and a
# 5-waves-per-SIMD register budget (tapsbw5); bit-exact subset first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3aa
mkdir -p $O
L=$GRAFT_REPO_ROOT/digital-filtering_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "runtime_tuning" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for b in "ylds_kb=48" "ylds_kb=36" "zlds_kb=32" "zlds_kb=40" "ylds_kb=48,zlds_kb=40" "ylds_kb=36,zlds_kb=32" "ylds_kb=53,zlds_kb=53"; do
  timeout -k 10 200 python3 tools/ab.py --config c3 --mode table --rounds 9 --calls 20 --tune-a ylds_kb=0 --tune-b $b \
    > $O/ab_$b.json || { echo "ab failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$b.json'));print('none', d['A_median_ms'], '$b', d['B_median_ms'])"
done
for i in 1 2; do
  for v in "" _tapsb _tapsbw5; do
    DFAMD_LIB=$L/libdfamd$v.so timeout -k 10 120 python3 tools/ab.py --config c3 --mode table --rounds 7 --calls 20 \
      > $O/lib${v}_$i.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/lib${v}_$i.json'));print('lib$v', d['A_median_ms'])"
  done
done
