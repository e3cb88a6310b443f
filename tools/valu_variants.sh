#!/bin/bash
# Where K3r's instructions go (c3 table, one PMC pass each, kernel trace only): SQ_INSTS_VALU / SALU per kernel
# with the timing-only RNG ablations DFAMD_RNG_DEBUG = 0 (as shipped), 1 (no log/sqrt/divide), 4 (no draws:
# fake uniforms), 5 (neither) -> gpurun_out/valu_variants/d<flags>.json. Results are wrong under 1/4/5 by design.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/valu_variants; mkdir -p $O
for d in 0 1 4 5; do
  DFAMD_RNG_DEBUG=$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -d $O/p$d -o run \
     --output-format csv -- python3 $R/tools/plane_loop.py c3 table 6 > $O/p$d.log 2>&1 || { echo "pmc $d failed"; tail -5 $O/p$d.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/p$d rng_ > $O/d$d.json || exit 1
  python3 - $O/d$d.json $d <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    print(f"debug {sys.argv[2]} {k[:50]:50s} VALU {v.get('SQ_INSTS_VALU', 0)/1e6:7.2f}M SALU {v.get('SQ_INSTS_SALU', 0)/1e6:7.2f}M")
PY
done
