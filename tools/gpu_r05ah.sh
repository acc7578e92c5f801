# Round 5: full GPU suite + default bench with the mask head on F(4x4) map pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ah
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_suite.txt 2>&1; rc=$?
tail -3 $OUT/gpu_suite.txt; grep -E "^E |FAILED" $OUT/gpu_suite.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['step_roofline']['frac'])" $OUT/bench_default.json
