# Round 5: F(4x4) channel-block mapping A/B (per XCD vs the 4 blocks of a spatial block
# on one XCD), both forms, the step's shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ab
mkdir -p $OUT
export TMPDIR=/tmp
for ps in 0 1; do for cbx in 1 0; do
VOSDET_WINO4_PS=$ps VOSDET_WINO4_CBX=$cbx timeout -k 10 200 python -u tools/bench_wino4.py > $OUT/ps${ps}_cbx$cbx.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "ps=$ps cbx=$cbx"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'])" $OUT/ps${ps}_cbx$cbx.jsonl
done; done
