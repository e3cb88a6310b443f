#!/bin/bash
# Multi-GPU rehearsal with the final round-3 library on one GPU (emulated RCCL hosts): the bare self-launching
# command at N = 2 in packed (c4 + c5 lines, long run shortened) and in table mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3al
mkdir -p $O
for mode in packed table; do
  DFAMD_EMULATE_HOSTS=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 10 --warmup 3 --coeff-mode $mode \
    --long-run 200 > $O/bench_emu_n2_$mode.json 2> $O/bench_emu_n2_$mode.err \
    || { echo "emulated bench $mode failed"; tail -40 $O/bench_emu_n2_$mode.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_emu_n2_$mode.json').read().strip())
m=d['multi_gpu']; print('$mode emu n2', d['n_gpus'], 'rccl', m['rccl_ranks'], 'parity', d['parity_ok'], d['ms_per_step'], 'same', d.get('ms_per_step_1gpu_same_plane'), d.get('speedup'), 'halo', m.get('halo_ms'))
print({k:(v['ms_per_step'],v['parity_ok']) for k,v in (d['other_configs'] or {}).items()})"
done
