# Round 5: position-split F(4x4) -- bit-identity vs the first form, then P2 timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wino4ps_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E " $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
for ps in 0 1; do
VOSDET_WINO4_PS=$ps timeout -k 10 200 python -u tools/bench_wino4.py > $OUT/ab_ps$ps.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "ps=$ps"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'], d['wino4_rel_err'])" $OUT/ab_ps$ps.jsonl
done
