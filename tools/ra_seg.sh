# RoIAlign: row segments (VOSDET_RA_SEGS) x workgroups per RoI (VOSDET_RA_PARTS)
# on the 8-frame launch (fewer resident RoIs per XCD at full occupancy).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ra_seg; rm -rf $O; mkdir -p $O
for cfg in "1 1" "2 1" "2 2" "4 2" "4 4" "7 7" "7 4"; do
  set -- $cfg
  VOSDET_RA_SEGS=$1 VOSDET_RA_PARTS=$2 timeout -k 10 200 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -k "fpn" > $O/t_$1_$2.txt 2>&1 || { echo "tests $cfg failed"; tail -20 $O/t_$1_$2.txt; exit 1; }
  for curve in morton band; do
    VOSDET_RA_CURVE=$curve VOSDET_RA_SEGS=$1 VOSDET_RA_PARTS=$2 RA_ITERS=30 timeout -k 10 120 python -u tools/bench_roialign.py 7 > $O/s$1_g$2_$curve.json 2> $O/s$1_g$2_$curve.err || { echo "bench $cfg failed"; tail -5 $O/s$1_g$2_$curve.err; exit 1; }
    python -c "import json; d=json.load(open('$O/s$1_g$2_$curve.json')); print('segs=$1 parts=$2 $curve', d['avg_launch_us'], d['frac'])"
  done
done
for cfg in "1 1" "2 2" "4 4"; do
  set -- $cfg
  VOSDET_RA_SEGS=$1 VOSDET_RA_PARTS=$2 RA_ITERS=30 timeout -k 10 120 python -u tools/bench_roialign.py 14 > $O/p14_s$1_g$2.json 2> $O/p14.err || { echo "p14 failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/p14_s$1_g$2.json')); print('P14 segs=$1 parts=$2', d['avg_launch_us'], d['frac'])"
done
echo done
