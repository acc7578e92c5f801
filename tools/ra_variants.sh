# RoIAlign candidate variants vs the product on the 8-frame x 1000-RoI launch:
# bit-identity tests, HIP-event timing at P=7 and P=14, optional PMC passes.
# usage: bash tools/ra_variants.sh "<variants>" "<variants for PMC>"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rv
rm -rf $O; mkdir -p $O
VOSDET_TEST_RA_VARIANTS="$1" timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py tests/test_edge_cases_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
run() { # tag P env...
  tag=$1; P=$2; shift 2
  env "$@" timeout -k 10 120 python -u tools/bench_roialign.py $P > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['avg_launch_us'], d['frac'])"
}
for v in 8 $1; do run v$v 7 VOSDET_ROIALIGN_VARIANT=$v || exit 1; done
for v in 8 $1; do run v${v}_p14 14 VOSDET_ROIALIGN_VARIANT=$v || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in $2; do
  for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_LDS"; do
    tag=$(echo $grp | tr ' ' '_')
    VOSDET_ROIALIGN_VARIANT=$v RA_ITERS=5 timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc_v$v/$tag -o run -- python3 tools/bench_roialign.py 7 > $O/pmc_v${v}_$tag.log 2>&1 || { echo "pmc $v $tag failed"; exit 1; }
  done
  VOSDET_ROIALIGN_VARIANT=$v RA_ITERS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_v$v -o run -- python3 tools/bench_roialign.py 7 > $O/trace_v$v.log 2>&1 || { echo "trace failed"; exit 1; }
done
echo done
