# Round 5: P2 lateral fused in the engine: tests + bench; wino4 no-store probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05x
mkdir -p $OUT
export TMPDIR=/tmp
for pr in 0 16 18; do
VOSDET_WINO4_PROBE=$pr timeout -k 10 120 python -u tools/bench_wino4.py 32x256x200x336x256 > $OUT/wino4_probe$pr.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "wino4 probe $pr: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['wino4_us'], d['wino4_exec_frac'])" $OUT/wino4_probe$pr.jsonl)"
done
timeout -k 10 900 python -u -m pytest tests/test_fpn_lateral_gpu.py tests/test_bench_config_gpu.py tests/test_graph_replay_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -3; grep -E "FAILED|^E " $OUT/tests.txt | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('step_roofline',{}).get('frac'))" $OUT/bench_default.json
