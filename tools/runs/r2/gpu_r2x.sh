#!/bin/bash
# Table y-pass with loads a whole 4-tap group ahead (ydeep): parity, then A/B on c3 table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "runtime_tuning or native_grid or bitexact" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for t in "ydeep=0 ydeep=1" "ydeep=1,rows_per_wave=4 ydeep=1,rows_per_wave=8" "ydeep=0,rows_per_wave=8 ydeep=1,rows_per_wave=2"; do
  set -- $t
  timeout -k 10 300 python tools/ab.py --a DFAMD_RNG_OVERLAP=0 --tune-a $1 --tune-b $2 --config c3 --mode table --rounds 9 --calls 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
done
timeout -k 10 300 python tools/ab.py --tune-a ydeep=0 --tune-b ydeep=1 --config c3 --mode table --rounds 9 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err
timeout -k 10 300 python tools/ab.py --tune-a ydeep=0 --tune-b ydeep=1 --config native --mode table --rounds 9 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err
timeout -k 10 300 python tools/ab.py --tune-a ydeep=0 --tune-b ydeep=1 --config c2 --mode table --rounds 9 --calls 40 >> $O/ab.jsonl 2>> $O/ab.err
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['config'], d['mode'], d['A'], d['A_median_ms']['ypass_ms'], d['A_median_ms']['wall_ms'], d['B'], d['B_median_ms']['ypass_ms'], d['B_median_ms']['wall_ms'])"
