# Round 5: F(4x4) after the V prefetch / scheduling barriers: parity, then probes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "wino4" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
for p in 0 8 1 2 15; do
  echo "probe $p" >> $OUT/probe.jsonl
  VOSDET_WINO4_PROBE=$p timeout -k 10 120 python -u tools/bench_wino4.py 32x256x200x336x256 >> $OUT/probe.jsonl 2>> $OUT/probe.err || { tail $OUT/probe.err; exit 1; }
done
cat $OUT/probe.jsonl
