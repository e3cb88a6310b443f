#!/bin/bash
# Row-pair y-pass on the reference's grid: equal-byte XCD runs (ycoop_map 0, 8 x longest-run blocks, most of
# them empty) against interleaved tiles (ycoop_map 1: tile t on XCD t % 8, no empty blocks); RNG overlap on and
# off; the no-load ablation likewise. Parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3u
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py \
  -k "native or runtime_tuning" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L=$GRAFT_REPO_ROOT/digital-filtering_amd
for v in "" _nocoefnoise; do
  for ov in 1 0; do
    DFAMD_LIB=$L/libdfamd$v.so DFAMD_RNG_OVERLAP=$ov timeout -k 10 120 python3 tools/ab.py --config native --mode packed --rounds 9 --calls 20 \
      --tune-a ycoop_map=0 --tune-b ycoop_map=1 > $O/ab${v}_ov$ov.json || { echo "ab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab${v}_ov$ov.json'));print('lib$v overlap $ov map0', d['A_median_ms'], 'map1', d['B_median_ms'])"
  done
done
