# Round-3 GPU pass: selected tests, the default bench, and the per-shape
# MFMA roofline / conv-algorithm probes.  Every GPU step has its own timeout
# and the chain stops at the first failure.
# usage: TAG=x TESTS="tests/a.py tests/b.py" BENCH="--steps 20" ROOF=1 PROBE=1 bash tools/gpu_r3.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r3}; rm -rf $O; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TLIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/tests.txt 2>&1
  rc=$?; tail -5 $O/tests.txt; [ $rc -ne 0 ] && { grep -B5 -A40 "Error\|FAILED" $O/tests.txt | head -120; exit $rc; }
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
  tail -c 1500 $O/bench.json; grep -i "graph\|capture" $O/bench.err | head -5
fi
if [ -n "$ROOF" ]; then
  timeout -k 10 300 python -u tools/conv_roofline.py $O/conv_roofline.json > $O/conv_roofline.log 2>&1 || { echo roofline failed; tail -20 $O/conv_roofline.log; exit 1; }
  python -c "import json;d=json.load(open('$O/conv_roofline.json'));print({k:v for k,v in d.items() if k!='ops'})"
fi
if [ -n "$PROBE" ]; then
  timeout -k 10 300 python -u tools/probe_conv_algos.py > $O/probe.json 2> $O/probe.err || { echo probe failed; tail -20 $O/probe.err; exit 1; }
  cat $O/probe.json
fi
echo done
