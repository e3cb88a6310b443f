set -o pipefail
# same-box A/B of two builds: three epochs of noise sets for single-GPU table planes (generation two epochs on)
cd $GRAFT_REPO_ROOT
O=gpurun_out/deep; mkdir -p $O
for lib in libdfamd.so libdfamd_deep.so libdfamd.so libdfamd_deep.so; do
  for cfg in c3 c2; do
    DFAMD_LIB=$GRAFT_REPO_ROOT/digital-filtering_amd/$lib timeout -k 10 200 python3 tools/ab.py --config $cfg --mode table --events 0 --rounds 5 > $O/ab_${lib}_$cfg.json 2>&1 || { tail -3 $O/ab_${lib}_$cfg.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/ab_${lib}_$cfg.json').read().strip().splitlines()[-1]); print('$lib', '$cfg', d['A_median_ms']['wall_ms'], d['B_median_ms']['wall_ms'])"
  done
done
