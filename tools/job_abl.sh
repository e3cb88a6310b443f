set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ec2; mkdir -p $O
python3 - <<'PY' > $O/ec_parity.log 2>&1 || exit 1
import sys; sys.path.insert(0, "digital-filtering_amd"); sys.path.insert(0, "oracle")
import numpy as np, dfamd, oracle as O
for tun in (dict(ylds=3, yt_rows=1, yt_chunk=16, yt_ec=1), dict(ylds=3, yt_rows=1, yt_chunk=8, yt_ec=1), dict(ylds=3, yt_rows=2, yt_chunk=8, yt_ec=1)):
    o = O.Filter(plane=O.PLANE_NATIVE, seed=42); g = dfamd.DigitalFilter(seed=42, device=0, coeff_mode="table", tuning=tun)
    for dt in (1e-8, 1e-5):
        o.filter(dt); g.filter(dt)
    print(tun, all(np.array_equal(g.field(k), o.field(k)) for k in ("u", "v", "w", "T", "rho")), flush=True)
PY
cat $O/ec_parity.log
for lim in 8 100000; do
for v in "ylds=3 yt_rows=1 yt_chunk=16" "ylds=3 yt_rows=1 yt_chunk=16 yt_ec=1" "ylds=3 yt_rows=1 yt_chunk=8 yt_ec=1" "ylds=3 yt_rows=2 yt_chunk=8 yt_ec=1"; do
  n=$(echo $v | tr ' =' '_-')_$lim
  (cd /tmp && DFAMD_TMP_YLIMIT=$lim DFAMD_RNG_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/tr_$n -o run -- python3 $GRAFT_REPO_ROOT/tools/plane_loop.py native table 100 $v > $GRAFT_REPO_ROOT/$O/tr_$n.log 2>&1) || exit 1
  python3 tools/rocprof_split.py $O/tr_$n/run_kernel_trace.csv > $O/tr_$n.split.csv; echo "== $v limit $lim"; grep "ypass_t64" $O/tr_$n.split.csv | head -1
done
done
