# Round 6: the two-rank launch rehearsed on one GPU at HEAD (the N>1 timed shape: graph
# replay, one RCCL all_gather per step, side-stream uploads) and the --rccl-gather line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r06f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 2 --share-gpu --steps 6 --warmup 2 --no-cpu-baseline > $OUT/bench_share2.json 2> $OUT/bench_share2.err || { tail -20 $OUT/bench_share2.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('share2', d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'])" $OUT/bench_share2.json
timeout -k 10 400 python -u bench.py --rccl-gather --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_rccl_gather.json 2> $OUT/bench_rccl_gather.err || { tail -20 $OUT/bench_rccl_gather.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rccl', d['value'], d['ms_per_step'], d['config']['parallelism'])" $OUT/bench_rccl_gather.json
