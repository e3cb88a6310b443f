#!/bin/bash
# Round-2 PMC traffic of the sweeps (FETCH_SIZE / WRITE_SIZE, one counter per pass, calibrated on
# tools/hbm_probe): the bench line's roofline.traffic source.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/pmc_traffic.py --out $GRAFT_REPO_ROOT/gpurun_out/pmc_r2 --json $GRAFT_REPO_ROOT/gpurun_out/pmc_r2/pmc_traffic.json > gpurun_out/pmc_r2.log 2>&1 \
  || { echo "pmc failed"; tail -30 gpurun_out/pmc_r2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/pmc_r2/pmc_traffic.json')); print(d['per_launch_bytes'])"
