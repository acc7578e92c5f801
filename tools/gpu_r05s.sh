# Round 5: fused FPN lateral kernel v2 (two 4-wave workgroups per CU): parity + A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fpn_lateral_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E " $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_fpn_lateral.py > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
cat $OUT/ab.jsonl
