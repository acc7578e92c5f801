# Round 5: RoIAlign pipelined-sweep depths (variants 11 = 2 columns ahead, 13 = 1)
# vs the product (10): bit-identity, then HIP-event A/B at P = 7 and 14.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05f
mkdir -p $OUT
export TMPDIR=/tmp
VOSDET_TEST_RA_VARIANTS="13" timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "separable or schedules" > $OUT/tests.txt 2>&1 || { tail -5 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
rm -f $OUT/ab.jsonl
for v in 10 11 13 10 11 13; do
  for P in 7 14; do
    VOSDET_ROIALIGN_VARIANT=$v timeout -k 10 120 python -u tools/bench_roialign.py $P >> $OUT/ab.jsonl 2>> $OUT/ab.err || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['variant'], d['launch'], d['avg_launch_us'], d['frac'])"
