#!/bin/bash
# The driver's multi-GPU command form, rehearsed on one GPU with two emulated RCCL hosts: the bare
# `bench.py --gpus 2` (c4 split, same-plane baseline, c5 split with its 10 000-step long run), final library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r3bj
mkdir -p $O
DFAMD_EMULATE_HOSTS=1 timeout -k 10 1000 python3 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_emu_n2.json 2> $O/bench_emu_n2.err \
  || { echo "emulated bench failed"; tail -40 $O/bench_emu_n2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_emu_n2.json').read().strip())
m=d['multi_gpu']; print('n_gpus', d['n_gpus'], 'rccl', m['rccl_ranks'], 'parity', d['parity_ok'], d['ms_per_step'], 'same', d.get('ms_per_step_1gpu_same_plane'), d.get('speedup'))
c5=d['other_configs']['c5']; print('c5', c5['ms_per_step'], c5['parity_ok'], {k: c5['long_run'][k] for k in c5['long_run'] if k in ('steps','total_s','steady_ms_per_step','variance_ok')})"
