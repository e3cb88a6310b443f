#!/bin/bash
# PMC counters of the row-pair y-pass on the reference's grid (packed, RNG overlap off), the product
# library and the no-load ablation; one --pmc pass per counter set, kernel trace only.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=$R/digital-filtering_amd
for v in "" _nocoefnoise; do
  O=$R/gpurun_out/r3s/pmc$v; mkdir -p $O
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES" "SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" \
             "SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD"; do
    i=$((i+1))
    DFAMD_LIB=$L/libdfamd$v.so DFAMD_RNG_OVERLAP=0 timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o run --output-format csv -- \
      python3 $R/tools/ab.py --config native --mode packed --rounds 2 --calls 5 > $O/p$i.log 2>&1
    rc=$?
    echo "lib$v pass $i ($set): rc=$rc"
    case $rc in 0) ;; *) echo "stopping after rc=$rc"; tail -5 $O/p$i.log; exit 1;; esac
  done
  python3 $R/tools/pmc_summary.py $O coop2 > $R/gpurun_out/r3s/summary$v.json
  cat $R/gpurun_out/r3s/summary$v.json
done
