# A/B of one environment switch on the default bench, alternated on one box:
# ENV_A / ENV_B (e.g. "VOSDET_SPLIT3_WIDE=0"), REPS rounds of 20-step benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 ${REPS:-2}); do
  for arm in A B; do
    if [ $arm = A ]; then E="${ENV_A:-}"; else E="${ENV_B:-}"; fi
    env $E timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-roofline ${BENCH_ARGS:-} > $OUT/bench_${arm}_$r.json 2> $OUT/bench_${arm}_$r.err || { tail $OUT/bench_${arm}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('stages_ms'))" $OUT/bench_${arm}_$r.json "$arm[$E]"
  done
done
