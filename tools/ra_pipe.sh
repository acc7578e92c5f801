# Variant-9 (pipelined separable) configurations vs variant 8 on the 8-frame x 1000-RoI launch
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rp
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py tests/test_edge_cases_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
run() { # tag P env...
  tag=$1; P=$2; shift 2
  env "$@" timeout -k 10 120 python -u tools/bench_roialign.py $P > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['avg_launch_us'], d['frac'])"
}
run v8 7 VOSDET_ROIALIGN_VARIANT=8 || exit 1
for cfg in ${1:-24 27 34 37 22 32}; do run v9_$cfg 7 VOSDET_ROIALIGN_VARIANT=9 VOSDET_RA_PIPE=$cfg || exit 1; done
run v8_p14 14 VOSDET_ROIALIGN_VARIANT=8 || exit 1
run v9_p14 14 VOSDET_ROIALIGN_VARIANT=9 VOSDET_RA_PIPE=${2:-24} || exit 1
echo done
