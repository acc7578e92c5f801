# Round 5: F(4x4) with the transform interleaved into the MFMA loop (VOSDET_WINO4_IL=1):
# bit-identity, chunk stamps, step-shape A/B, default bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05aj
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wino4_forms_gpu.py -m gpu -v -x -k "il" --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E " $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
VOSDET_WINO4_IL=2 timeout -k 10 120 python -u tools/wino4_stamps.py > $OUT/stamps_il_p2.json 2> $OUT/s.err || { tail $OUT/s.err; exit 1; }
cat $OUT/stamps_il_p2.json
for il in 0 1; do
VOSDET_WINO4_IL=$il timeout -k 10 200 python -u tools/bench_wino4.py > $OUT/ab_il$il.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "il=$il"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'])" $OUT/ab_il$il.jsonl
done
VOSDET_WINO4_IL=1 timeout -k 10 100 python -u tools/bench_wino4_mosaic.py > $OUT/mosaic_il.jsonl 2> $OUT/m.err || { tail $OUT/m.err; exit 1; }
cat $OUT/mosaic_il.jsonl
for il in 0 1; do
VOSDET_WINO4_IL=$il timeout -k 10 300 python -u bench.py > $OUT/bench_il$il.json 2> $OUT/bench_il$il.err || { tail $OUT/bench_il$il.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $OUT/bench_il$il.json
done
