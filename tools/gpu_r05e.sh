# Round 5: RoIAlign variant 11 (pipelined sweep) parity + A/B vs variant 10.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/research/ra_v11_diff.py > $OUT/diff.txt 2>&1 || { cat $OUT/diff.txt; exit 1; }
cat $OUT/diff.txt
timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "separable or schedules" > $OUT/tests.txt 2>&1 || { tail -5 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
rm -f $OUT/ab.jsonl
for v in 10 11 10 11; do
  for P in 7 14; do
    VOSDET_ROIALIGN_VARIANT=$v timeout -k 10 120 python -u tools/bench_roialign.py $P >> $OUT/ab.jsonl 2>> $OUT/ab.err || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['variant'], d['launch'], d['avg_launch_us'], d['frac'])"
