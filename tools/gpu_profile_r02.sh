# round-2 evidence pass: full -m gpu suite, default bench, rocprof kernel trace of
# the bench, RoIAlign PMC traffic passes, bias_act roofline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_suite.txt 2>&1
rc=$?; tail -3 $O/gpu_suite.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail $O/bench_default.err; exit 1; }
tail -c 600 $O/bench_default.json
timeout -k 10 300 python -u tools/bias_act_roofline.py $O/bias_act_roofline.json > $O/bias_act.log 2>&1 || { echo bias_act failed; tail $O/bias_act.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_trace -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-timers > $O/bench_trace.log 2>&1 || { echo trace failed; exit 1; }
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  tag=$(echo $grp | tr ' ' '_')
  VOSDET_ROIALIGN_VARIANT=8 RA_ITERS=5 timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/ra_pmc/$tag -o run -- python3 tools/bench_roialign.py 7 > $O/ra_pmc_$tag.log 2>&1 || { echo "pmc $tag failed"; exit 1; }
done
echo done
