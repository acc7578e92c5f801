# Round 5: F(4x4) chunk timestamps (STAMP form) on P2 and the mask-head pair shape;
# priority-1 transform A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ai
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/wino4_stamps.py > $OUT/stamps_p2.json 2> $OUT/s.err || { tail $OUT/s.err; exit 1; }
cat $OUT/stamps_p2.json
timeout -k 10 120 python -u tools/wino4_stamps.py 32x256x100x168x256 > $OUT/stamps_p3.json 2> $OUT/s.err || { tail $OUT/s.err; exit 1; }
cat $OUT/stamps_p3.json
for p in 0 1; do
VOSDET_WINO4_PRIO=$p timeout -k 10 200 python -u tools/bench_wino4.py > $OUT/ab_prio$p.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "prio=$p"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'])" $OUT/ab_prio$p.jsonl
done
