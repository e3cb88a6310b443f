#!/bin/bash
# Round-3 HBM traffic (FETCH_SIZE / WRITE_SIZE in separate --pmc passes, calibrated on tools/hbm_probe's known
# 1 GiB reads and writes) of the c3 sweeps with the final library; result copied to profiles/pmc_traffic.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/pmc_traffic.py --out $GRAFT_REPO_ROOT/gpurun_out/pmc_r3 --json $GRAFT_REPO_ROOT/gpurun_out/pmc_r3/pmc_traffic.json > gpurun_out/pmc_r3.log 2>&1 \
  || { echo "pmc_traffic failed"; tail -30 gpurun_out/pmc_r3.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/pmc_r3/pmc_traffic.json')); print(json.dumps(d['per_launch_bytes'], indent=1)[:2000])"
