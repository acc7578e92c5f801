# Round 5: F(4x4) row stack (vd_conv3x3_wino4_rows_bias_act) -- bit-identity, P3 / P4
# shape timings plain vs rows, route tests, default bench with / without.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05al
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wino4_forms_gpu.py tests/test_bench_config_gpu.py tests/test_graph_replay_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E |FAILED" $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
for m in "" rows; do
WINO4_MOSAIC=$m timeout -k 10 200 python -u tools/bench_wino4.py 32x256x100x168x256 32x256x50x84x256 32x128x100x168x128 32x512x25x42x512 > $OUT/ab_mos_$m.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "mosaic=$m"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'])" $OUT/ab_mos_$m.jsonl
done
for r in 0 1; do
VOSDET_WINO4_ROWS=$r timeout -k 10 300 python -u bench.py > $OUT/bench_rows$r.json 2> $OUT/bench_rows$r.err || { tail $OUT/bench_rows$r.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $OUT/bench_rows$r.json
done
