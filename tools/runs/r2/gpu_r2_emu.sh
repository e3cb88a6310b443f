#!/bin/bash
# Multi-GPU path rehearsed on one GPU: ranks on device 0 with one emulated RCCL host each
# (NCCL_HOSTID; socket transport over loopback). The emulated-host pytest cases, then bench.py under
# torchrun at N = 2 and 4 (c4 split, parity against the unsplit plane on every rank).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r2emu}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_multi.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_multi.log; exit 1; }
tail -3 $O/pytest_multi.log
for n in 2 4; do
  for mode in table packed; do
    DFAMD_EMULATE_HOSTS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 \
      --coeff-mode $mode > $O/bench_emu_n${n}_${mode}.json 2> $O/bench_emu_n${n}_${mode}.err \
      || { echo "bench n=$n $mode failed"; tail -30 $O/bench_emu_n${n}_${mode}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/bench_emu_n${n}_${mode}.json').read().strip().splitlines()[-1])
m=d['multi_gpu']; print($n, '$mode', d['value'], d['ms_per_step'], 'parity', d['parity_ok'], 'ranks', m['rccl_ranks'], 'halo', m['halo_ms_per_call'], m['halo_bytes_per_call'], {k:(v['ms_per_step'],v['parity_ok']) for k,v in (d['other_configs'] or {}).items()})"
  done
done
