# Round 6: the full GPU suite, smoke, the default bench and the steady-step trace at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r06b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_suite.txt 2>&1; rc=$?
tail -2 $OUT/gpu_suite.txt; grep -E "^E |FAILED" $OUT/gpu_suite.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_roofline']['frac'], d['dominant_kernel']['avg_launch_us'], d['stages_ms'])" $OUT/bench_default.json
TAG=${TAG:-r06b}/trace bash tools/gpu_trace_step.sh > /dev/null || exit 1
head -30 $OUT/trace/steady_step.txt
