set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_timed_loop_gpu.py tests/test_graph_replay_gpu.py tests/test_rccl_gpu.py -m gpu -v -s --timeout 400 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
timeout -k 10 400 python -u bench.py --rccl-gather --no-cpu-baseline --steps 20 --warmup 5 > $OUT/bench_rccl.json 2> $OUT/bench_rccl.err || exit $?
tail -c 1500 $OUT/bench_rccl.json
timeout -k 10 180 python -u tools/research/concurrent_replay.py --reps 6 > $OUT/concurrent.txt 2>&1; echo "concurrent rc=$?"; tail -8 $OUT/concurrent.txt
