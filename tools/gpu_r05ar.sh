# Round 5 final at HEAD: full GPU suite, smoke, default bench, C4 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ar
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_suite.txt 2>&1; rc=$?
tail -2 $OUT/gpu_suite.txt; grep -E "^E |FAILED" $OUT/gpu_suite.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_roofline']['frac'])" $OUT/bench_default.json
timeout -k 10 400 python -u bench.py --config e2e_mask_rcnn_R-50-C4_1x --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail $OUT/bench_c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'])" $OUT/bench_c4.json
