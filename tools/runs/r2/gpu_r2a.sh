#!/bin/bash
# Round-2 first GPU pass: the GPU suite (incl. the multi-process RCCL test at world 1), the default
# bench line (c3 + parity + native/c2), the c4 plane on one GPU, and the per-rank cost of the
# replicated vs split RNG counting for c4 strips (tools/strip_timing.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['parity_ok'], d['roofline']['frac'], {k:(v['ms_per_step'],v['parity_ok']) for k,v in (d['other_configs'] or {}).items()})"
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 --cpu-baseline off --other-configs '' \
  > $O/bench_c4_n1.json 2> $O/bench_c4_n1.err || { echo "bench c4 failed"; tail -20 $O/bench_c4_n1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c4_n1.json')); print('c4', d['value'], d['ms_per_step'], d['parity_ok'], d['roofline']['frac'])"
for mode in packed table; do
  for rep in 1 0; do
    timeout -k 10 300 python tools/strip_timing.py --config c4 --mode $mode --replicate $rep >> $O/strip_c4.jsonl 2>> $O/strip.err \
      || { echo "strip timing failed"; tail -20 $O/strip.err; exit 1; }
  done
done
cat $O/strip_c4.jsonl
