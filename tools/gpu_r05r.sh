# Round 5: fused FPN lateral + top-down kernel: parity, A/B at the benched shapes,
# the 32-frame GEMM census, then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fpn_lateral_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E " $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_fpn_lateral.py > $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
cat $OUT/ab.jsonl
timeout -k 10 300 python -u tools/research/gemm_census.py 32 > $OUT/gemm_census.jsonl 2> $OUT/census.err || { tail $OUT/census.err; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('step_roofline',{}).get('frac'))" $OUT/bench_default.json
