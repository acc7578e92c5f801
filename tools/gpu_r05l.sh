# Round 5: the F(4x4) route in the engine -- benched-config / graph-replay / conv
# suites, then the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_bench_config_gpu.py tests/test_graph_replay_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -3
grep -E "FAILED|Error" $OUT/tests.txt | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('dominant_kernel'), d.get('step_roofline',{}).get('frac'))" $OUT/bench_default.json
