#!/bin/bash
# Round-end evidence on one MI355X, every GPU step under its own time limit; results land in
# gpurun_out/refresh/ and are copied into profiles/<round>/ by hand. Usage: tools/refresh_profiles.sh
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/refresh
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err
bash tools/gpu_profile.sh refresh/prof > $O/kernel_stats.txt 2>&1
timeout -k 10 900 python3 tools/pmc_traffic.py --out $O/pmc --json $O/pmc_traffic.json > $O/pmc.log 2>&1
echo refresh done
