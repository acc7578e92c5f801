# Evidence pass at HEAD: full -m gpu suite, smoke, default bench, rocprofv3 kernel
# trace + stats of a short bench.  Output under gpurun_out/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-verify}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_suite.txt 2>&1
rc=$?; tail -3 $O/gpu_suite.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo smoke failed; tail $O/smoke.txt; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail $O/bench_default.err; exit 1; }
tail -c 400 $O/bench_default.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_trace -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-timers > $O/bench_trace.log 2>&1 || { echo trace failed; exit 1; }
echo done
