# Round 5 session end at HEAD: full GPU suite, smoke, default bench (20 steps), the
# steady-step kernel trace, and the FPN configs (mask head / row stack changed them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ao
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_suite.txt 2>&1; rc=$?
tail -2 $OUT/gpu_suite.txt; grep -E "^E |FAILED" $OUT/gpu_suite.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_roofline']['frac'], d['dominant_kernel']['avg_launch_us'])" $OUT/bench_default.json
for c in e2e_mask_rcnn_X-101-32x8d-FPN_1x e2e_mask_rcnn_R-101-FPN_2x vos_R-101-FPN_3x_gn_dynamic_davis; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('stress_launch', {}).get('frac'))" $OUT/bench_$c.json $c
done
TAG=r05ao/trace bash tools/gpu_trace_step.sh > /dev/null || exit 1
head -8 $OUT/trace/steady_step.txt
