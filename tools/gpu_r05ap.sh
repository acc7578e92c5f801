# Round 5: P2 / res2 on the row stack -- bit-identity (incl. a 200 x 336 case), the
# bench-config routes, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ap
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wino4_forms_gpu.py tests/test_bench_config_gpu.py tests/test_graph_replay_gpu.py tests/test_timed_loop_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E |FAILED" $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
for r in 1 0 1; do
VOSDET_WINO4_ROWS=$r timeout -k 10 300 python -u bench.py > $OUT/bench_rows$r.json 2> $OUT/bench_rows$r.err || { tail $OUT/bench_rows$r.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['dominant_kernel']['route'], d['dominant_kernel']['avg_launch_us'])" $OUT/bench_rows$r.json
done
