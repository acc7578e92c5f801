# Round 5: Winograd F(4x4) parity vs torch, then the A/B vs F(2x2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "wino4" > $OUT/tests.txt 2>&1; rc=$?
tail -25 $OUT/tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_wino4.py > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
cat $OUT/ab.jsonl
