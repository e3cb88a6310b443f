#!/bin/bash
# Per-call VALU wave-instructions of table-mode calls (rocprofv3 --pmc SQ_INSTS_VALU, one pass per plane, kernel
# trace only; tools/plane_loop.py <plane> table), written to gpurun_out/valu_issue/valu_issue.json in the form
# bench.py reads from profiles/valu_issue.json (alt_modes.table.roofline_valu.call_issue). Copy it there to adopt it.
# Planes: c3 (the alt-mode line) and native (the reference's grid, the drop-in default).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/valu_issue; mkdir -p $O
for plane in c3 native; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -d $O/p_$plane -o run --output-format csv -- \
     python3 $R/tools/plane_loop.py $plane table 8 > $O/p_$plane.log 2>&1 || { echo "pmc failed ($plane)"; tail -5 $O/p_$plane.log; exit 1; }
  python3 $R/tools/pmc_summary.py $O/p_$plane ypass zpass rng_ > $O/pmc_${plane}_table.json || exit 1
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
out = {"note": "SQ_INSTS_VALU per dispatch (wave-instructions), rocprofv3 --pmc, table mode, one call = one dispatch "
               "of each kernel (the hand-off batch enqueues one generation per call on average); tools/valu_issue.sh",
       "per_call_valu_wave_instr": {}, "by_kernel": {}, "salu_by_kernel": {}}
for plane in ("c3", "native"):
    d = json.load(open(f"{o}/pmc_{plane}_table.json"))
    by = {k: round(v["SQ_INSTS_VALU"]) for k, v in d.items()}
    key = f"{plane}/table"
    out["per_call_valu_wave_instr"][key] = sum(by.values())
    out["by_kernel"][key] = by
    out["salu_by_kernel"][key] = {k: round(v["SQ_INSTS_SALU"]) for k, v in d.items()}
    for k, v in by.items():
        print(f"{key} {k[:60]:60s} VALU {v/1e6:.2f}M")
    print(f"{key} total VALU per call {sum(by.values())/1e6:.2f}M wave-instr")
json.dump(out, open(o + "/valu_issue.json", "w"), indent=1)
PY
