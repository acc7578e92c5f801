# Round 5: position-split F(4x4) probes at P2 (32 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05aa
mkdir -p $OUT
export TMPDIR=/tmp
for pp in 4 1 5 8 12; do
VOSDET_WINO4_PS=1 VOSDET_WINO4_PSPROBE=$pp timeout -k 10 120 python -u tools/bench_wino4.py 32x256x200x336x256 > $OUT/ps_probe$pp.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "ps probe $pp: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['wino4_us'], d['wino4_exec_frac'])" $OUT/ps_probe$pp.jsonl)"
done
