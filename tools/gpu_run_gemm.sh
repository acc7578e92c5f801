# GEMM-epilogue A/B: tests, bench with and without, kernel trace of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gemm; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_epilogue_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for g in 1 0; do
  VOSDET_GEMM_EPILOGUE=$g timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/bench_g$g.json 2> $O/bench_g$g.err || { echo "bench g$g failed"; tail -5 $O/bench_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_g$g.json'));print('gemm=$g', d['value'], d['ms_per_step'], d.get('stages_ms'))"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-timers > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
