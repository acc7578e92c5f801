# Round 5: F(4x4) under graph capture (static LDS), then the engine suites + bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_nms_proposals_gpu.py -m gpu -v --timeout 120 --timeout-method thread -k "wino4 or graph" > $OUT/t0.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/t0.txt | tail -2; grep -E "^E " $OUT/t0.txt | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_bench_config_gpu.py tests/test_graph_replay_gpu.py tests/test_timed_loop_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -3
grep -E "FAILED|^E " $OUT/tests.txt | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('dominant_kernel'), d.get('step_roofline',{}).get('frac'))" $OUT/bench_default.json
