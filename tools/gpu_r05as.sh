# Round 5: the N > 1 launch rehearsed on one GPU at HEAD (two ranks sharing the card,
# gloo carrying the gather since RCCL refuses two ranks on one device), 32 frames each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05as
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 2 --share-gpu --steps 6 --warmup 2 --no-cpu-baseline > $OUT/bench_share2.json 2> $OUT/bench_share2.err || { tail -20 $OUT/bench_share2.err; exit 1; }
tail -c 1500 $OUT/bench_share2.json
