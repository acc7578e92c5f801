# Round 5: F(4x4) octets for C4's 7 x 7 res5-head maps -- bit-identity, C4 tests, C4 bench
# with / without octets, and the default bench (its routes must be unchanged).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05aq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wino4_forms_gpu.py tests/test_c4.py tests/test_configs_gpu.py -m gpu -v -x -k "octet or pair or c4 or C4" --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E |FAILED" $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
for o in 0 1; do
VOSDET_WINO4_OCTET=$o timeout -k 10 400 python -u bench.py --config e2e_mask_rcnn_R-50-C4_1x --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4_oct$o.json 2> $OUT/bench_c4_oct$o.err || { tail $OUT/bench_c4_oct$o.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $OUT/bench_c4_oct$o.json
done
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $OUT/bench_default.json
