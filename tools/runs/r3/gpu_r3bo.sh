#!/bin/bash
# Stall counters of the final table-mode sweeps on c3 (RNG overlap off; tools/pmc_sweeps.sh passes), for the
# next round's latency-hiding work.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/pmc_sweeps.sh table || exit 1
python3 tools/pmc_summary.py $GRAFT_REPO_ROOT/gpurun_out/pmcsw_table ypass zpass > $GRAFT_REPO_ROOT/gpurun_out/pmcsw_table/summary.json
cat $GRAFT_REPO_ROOT/gpurun_out/pmcsw_table/summary.json
