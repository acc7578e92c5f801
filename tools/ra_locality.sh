# RoIAlign schedule locality sweep: scheduling curve x resident RoIs per CU
# (VOSDET_RA_WG_PER_CU; 0 = register-limited, 4 at P=7) on the 8-frame launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ra_loc; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for curve in band morton; do
  for k in 0 3 2 1; do
    VOSDET_RA_CURVE=$curve VOSDET_RA_WG_PER_CU=$k RA_ITERS=30 timeout -k 10 120 python -u tools/bench_roialign.py 7 > $O/${curve}_k$k.json 2> $O/${curve}_k$k.err || { echo "bench $curve $k failed"; tail -5 $O/${curve}_k$k.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/${curve}_k$k.json')); print('$curve k=$k', d['avg_launch_us'], d['frac'])"
  done
done
for k in 0 2 1; do
  VOSDET_RA_CURVE=morton VOSDET_RA_WG_PER_CU=$k RA_ITERS=30 timeout -k 10 120 python -u tools/bench_roialign.py 14 > $O/p14_morton_k$k.json 2> $O/p14_k$k.err || { echo "p14 $k failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/p14_morton_k$k.json')); print('p14 morton k=$k', d['avg_launch_us'], d['frac'])"
done
echo done
