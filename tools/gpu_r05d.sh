# Round 5: every config at HEAD (bench lines) + the default bench, and the RPN
# mask-kernel A/B (prop_time under a kernel trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=gpurun_out/r05d
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt -o run -- python3 $R/tools/prop_time.py 32 > $R/$OUT/prop_prof.log 2>&1 || { tail $R/$OUT/prop_prof.log; exit 1; }
cd $R
cp /tmp/pt/run_kernel_trace.csv $OUT/prop_kernel_trace.csv
python3 tools/prop_breakdown.py $OUT/prop_kernel_trace.csv > $OUT/prop_breakdown.txt; cat $OUT/prop_breakdown.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
tail -c 600 $OUT/bench_default.json
for c in e2e_mask_rcnn_X-101-32x8d-FPN_1x e2e_mask_rcnn_R-101-FPN_2x e2e_mask_rcnn_R-50-C4_1x vos_R-101-FPN_3x_gn_dynamic_davis; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['frames_per_gpu_step'], d['roofline'].get('stress_launch', {}).get('frac'))" $OUT/bench_$c.json $c
done
