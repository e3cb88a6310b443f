#!/bin/bash
# PMC of K3a (c3 table, RNG overlap off) with and without the fast chunks: VALU / SALU / waves per launch.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for fast in 0 1; do
  O=$R/gpurun_out/r3ah/fast$fast; mkdir -p $O
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SMEM" "SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    DFAMD_K3A_FAST=$fast DFAMD_RNG_OVERLAP=0 timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o run --output-format csv -- \
      python3 $R/tools/ab.py --config c3 --mode table --rounds 2 --calls 3 > $O/p$i.log 2>&1
    rc=$?; echo "fast $fast pass $i rc=$rc"; [ $rc = 0 ] || { tail -5 $O/p$i.log; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $O rng_ > $R/gpurun_out/r3ah/summary_fast$fast.json
  python3 -c "import json; d=json.load(open('$R/gpurun_out/r3ah/summary_fast$fast.json')); [print(k, {c: round(v) for c, v in x.items()}) for k, x in d.items()]"
done
