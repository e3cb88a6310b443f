#!/bin/bash
# Per-call VALU wave-instructions of a c3 table call (rocprofv3 --pmc SQ_INSTS_VALU, one pass, kernel trace
# only; tools/plane_loop.py c3 table), written to gpurun_out/valu_issue/valu_issue.json in the form bench.py
# reads from profiles/valu_issue.json (alt_modes.table.roofline_valu.call_issue). Copy it there to adopt it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/valu_issue; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -d $O/p1 -o run --output-format csv -- \
   python3 $R/tools/plane_loop.py c3 table 6 > $O/p1.log 2>&1 || { echo "pmc failed"; tail -5 $O/p1.log; exit 1; }
python3 $R/tools/pmc_summary.py $O ypass zpass rng_ > $O/pmc_c3_table.json
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
d = json.load(open(o + "/pmc_c3_table.json"))
by = {k: round(v["SQ_INSTS_VALU"]) for k, v in d.items()}
tot = sum(by.values())
json.dump({"note": "SQ_INSTS_VALU per dispatch (wave-instructions), rocprofv3 --pmc, c3 table mode, one call = one "
                   "dispatch of each kernel; tools/valu_issue.sh", "per_call_valu_wave_instr": {"c3/table": tot},
           "by_kernel": {"c3/table": by},
           "salu_by_kernel": {"c3/table": {k: round(v["SQ_INSTS_SALU"]) for k, v in d.items()}}},
          open(o + "/valu_issue.json", "w"), indent=1)
for k, v in by.items():
    print(f"{k[:60]:60s} VALU {v/1e6:.2f}M")
print(f"total VALU per call {tot/1e6:.1f}M wave-instr")
PY
