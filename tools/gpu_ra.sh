# RoIAlign A/B on the GPU box: parity tests, HIP-event timing of the given
# variants on the 8-frame x 1000-RoI launch, PMC passes and a kernel trace of
# the first variant.  usage: VARIANTS="20 10" PMC=1 bash tools/gpu_ra.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ra}; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_roi_ops_gpu.py} -m gpu -x -q --timeout 200 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -ne 0 ] && { grep -B5 -A40 "Error\|FAILED\|assert" $O/tests.txt | head -80; exit $rc; }
for v in ${VARIANTS:-20 10}; do
  for P in 7 14; do
    VOSDET_ROIALIGN_VARIANT=$v timeout -k 10 120 python -u tools/bench_roialign.py $P > $O/v${v}_p$P.json 2> $O/v${v}_p$P.err || { echo "v$v P$P failed"; tail -5 $O/v${v}_p$P.err; exit 1; }
    python -c "import json;d=json.load(open('$O/v${v}_p$P.json'));print('v$v P$P', d['avg_launch_us'], d['frac'])"
  done
done
if [ -n "$PROBE" ]; then
  timeout -k 10 300 python -u tools/probe_conv_algos.py > $O/probe.json 2> $O/probe.err || { echo probe failed; tail -20 $O/probe.err; exit 1; }
  cat $O/probe.json
fi
[ -z "$PMC" ] && { echo done; exit 0; }
v=$(echo ${VARIANTS:-20} | awk '{print $1}')
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  tag=$(echo $grp | tr ' ' '_')
  VOSDET_ROIALIGN_VARIANT=$v RA_ITERS=5 timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/$tag -o run -- python3 tools/bench_roialign.py 7 > $O/pmc_$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $O/pmc_$tag.log; exit 1; }
done
VOSDET_ROIALIGN_VARIANT=$v RA_ITERS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_roialign.py 7 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
