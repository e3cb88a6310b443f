#!/bin/bash
# Halo overlap (RCCL z-strips: send/recv + unpack on a high-priority stream under the interior strips'
# z-pass): the multi-process GPU tests (emulated hosts), then the bare N = 2 command on c4 with the
# overlap on and off (socket transport: the exchange is far slower than xGMI, so this checks the
# form, not the xGMI gain).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3ay
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_multi.py \
  -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for ov in 1 0; do
  DFAMD_HALO_OVERLAP=$ov DFAMD_EMULATE_HOSTS=1 timeout -k 10 400 python3 bench.py --gpus 2 --config c4 --steps 10 --warmup 3 \
    --other-configs '' --alt-modes off --dropin off --long-run 0 --cpu-baseline off > $O/bench_emu_n2_ov$ov.json 2> $O/bench_emu_n2_ov$ov.err \
    || { echo "emulated bench ov$ov failed"; tail -40 $O/bench_emu_n2_ov$ov.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_emu_n2_ov$ov.json').read().strip())
m=d['multi_gpu']; print('ov$ov emu n2', d['n_gpus'], 'rccl', m['rccl_ranks'], 'parity', d['parity_ok'], d['ms_per_step'], 'same', d.get('ms_per_step_1gpu_same_plane'), d.get('speedup'), 'halo', m.get('halo_ms'), 'per-rank', m.get('per_rank_ms'))"
done
