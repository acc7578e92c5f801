# Round 5: F(4x4) ACC form with per-lane DMA pointers (one 64-bit add a piece) and the
# 12-VALU B^T -- bit-identity vs the first form, stamps, step shapes, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05an
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wino4_forms_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E " $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/wino4_stamps.py > $OUT/stamps_p2.json 2> $OUT/s.err || { tail $OUT/s.err; exit 1; }
cat $OUT/stamps_p2.json
timeout -k 10 200 python -u tools/bench_wino4.py > $OUT/ab.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'])" $OUT/ab.jsonl
timeout -k 10 100 python -u tools/bench_wino4_mosaic.py > $OUT/mosaic.jsonl 2> $OUT/m.err || { tail $OUT/m.err; exit 1; }
cat $OUT/mosaic.jsonl
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $OUT/bench_default.json
