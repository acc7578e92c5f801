# Round 5: wino4 non-MFMA critical path composition (probe combinations, P2 32 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05y
mkdir -p $OUT
export TMPDIR=/tmp
for pr in 18 19 22 26 31 17 20 24 28; do
VOSDET_WINO4_PROBE=$pr timeout -k 10 120 python -u tools/bench_wino4.py 32x256x200x336x256 > $OUT/wino4_probe$pr.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "wino4 probe $pr: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['wino4_us'], d['wino4_exec_frac'])" $OUT/wino4_probe$pr.jsonl)"
done
