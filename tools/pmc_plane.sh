#!/bin/bash
# rocprofv3 counters of one plane's kernels (separate --pmc passes, kernel trace only) driven by
# tools/plane_loop.py, plus one --kernel-trace --stats pass for the durations.
#   tools/pmc_plane.sh PLANE MODE [CALLS] [key=value tuning ...]     e.g. tools/pmc_plane.sh native table 20
# Writes gpurun_out/pmc_PLANE_MODE/{p*,trace}; summary: pmc.json (tools/pmc_summary.py), split.csv.
PLANE=${1:-native}; MODE=${2:-table}; CALLS=${3:-20}
shift 3 2>/dev/null
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_${PLANE}_${MODE}${PMC_TAG}; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/tools/plane_loop.py $PLANE $MODE 200 "$@" > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_split.py $O/trace/run_kernel_trace.csv > $O/split.csv
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o run --output-format csv -- \
    python3 $R/tools/plane_loop.py $PLANE $MODE $CALLS "$@" > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i: rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/p$i.log; exit $rc; }
done
python3 $R/tools/pmc_summary.py $O ypass zpass rng_ > $O/pmc.json
head -30 $O/split.csv
