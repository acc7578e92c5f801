# Round 6: every config's bench line at HEAD (R-101-FPN_2x, X-101-32x8d-FPN with the
# 8(d) P = 14 stress RoIAlign launch, R-50-C4, VOS 480p) and the default line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r06c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['step_roofline']['frac'])" $OUT/bench_default.json
for c in e2e_mask_rcnn_R-101-FPN_2x e2e_mask_rcnn_X-101-32x8d-FPN_1x vos_R-101-FPN_3x_gn_dynamic_davis e2e_mask_rcnn_R-50-C4_1x; do
  timeout -k 10 500 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('stress_launch', {}).get('frac'))" $OUT/bench_$c.json $c
done
