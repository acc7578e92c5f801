# Product RoIAlign kernel: GPU tests, roofline line, PMC traffic passes summarised
# into profiles/-ready JSON (tools/pmc_summary.py), rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rd
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py tests/test_edge_cases_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/bench_roialign.py 7 > $O/v10.json 2> $O/v10.err || { echo bench failed; tail $O/v10.err; exit 1; }
cat $O/v10.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES" "TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum"; do
  tag=$(echo $grp | tr ' ' '_')
  RA_ITERS=5 timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/$tag -o run -- python3 tools/bench_roialign.py 7 > $O/pmc_$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $O/pmc_$tag.log; exit 1; }
done
python tools/pmc_summary.py $O/pmc sep_buf $O/separable_buf_v10_xcd.json > /dev/null
RA_ITERS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_roialign.py 7 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
