# Round 5: where the fused lateral kernel's top-down term costs its time (probes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05v
mkdir -p $OUT
export TMPDIR=/tmp
for pr in 0 1 2 4; do
VOSDET_LATERAL_NB=1 VOSDET_LATERAL_PROBE=$pr timeout -k 10 200 python -u tools/bench_fpn_lateral.py >> $OUT/probe$pr.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
echo "probe $pr"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['K'], d['fused_ms'], d['fused_no_top_ms'])" $OUT/probe$pr.jsonl
done
