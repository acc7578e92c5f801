# Round 5: fused lateral A/B after the top-tensor copy fix; wino4 probes at P2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05w
mkdir -p $OUT
export TMPDIR=/tmp
for nb in 1 2; do
VOSDET_LATERAL_NB=$nb timeout -k 10 200 python -u tools/bench_fpn_lateral.py >> $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
done
python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['nb'], d['K'], d['fused_ms'], d['fused_no_top_ms'], d['old_gemm_plus_add_ms'], d['max_abs_diff'])" $OUT/ab.jsonl
for pr in 0 1 2 4 8 12; do
VOSDET_WINO4_PROBE=$pr timeout -k 10 120 python -u tools/bench_wino4.py 32x256x200x336x256 > $OUT/wino4_probe$pr.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "wino4 probe $pr: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['wino4_us'], d['wino4_exec_frac'])" $OUT/wino4_probe$pr.jsonl)"
done
