# Round 5: row stack on the P2-sized shapes (A/B), then the full GPU suite, smoke and
# the default bench at HEAD (res5 on the row stack).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05am
mkdir -p $OUT
export TMPDIR=/tmp
for m in "" rows; do
WINO4_MOSAIC=$m timeout -k 10 200 python -u tools/bench_wino4.py 32x256x200x336x256 32x64x200x336x64 32x512x25x42x512 > $OUT/ab_p2_$m.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "mosaic=$m"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'])" $OUT/ab_p2_$m.jsonl
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_suite.txt 2>&1; rc=$?
tail -2 $OUT/gpu_suite.txt; grep -E "^E |FAILED" $OUT/gpu_suite.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_roofline']['frac'])" $OUT/bench_default.json
