# Round 5: hand-counted vmcnt F(4x4) form (VOSDET_WINO4_ACC) -- bit-identity vs the
# first form, the six step shapes A/B, then the default bench with each form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wino4_forms_gpu.py -m gpu -v -x -k acc --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E " $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
for acc in 0 1; do
VOSDET_WINO4_ACC=$acc timeout -k 10 200 python -u tools/bench_wino4.py > $OUT/ab_acc$acc.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "acc=$acc"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'], d['wino4_rel_err'])" $OUT/ab_acc$acc.jsonl
done
for acc in 0 1; do
VOSDET_WINO4_ACC=$acc timeout -k 10 300 python -u bench.py > $OUT/bench_acc$acc.json 2> $OUT/bench_acc$acc.err || { tail $OUT/bench_acc$acc.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $OUT/bench_acc$acc.json
done
