# quick GPU pass: the given test files, then (optional) the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-quick}; rm -rf $O; mkdir -p $O
timeout -k 10 ${LIMIT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" $O/tests.txt | head -80; exit $rc; }
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
  tail -c 700 $O/bench.json
fi
echo done
