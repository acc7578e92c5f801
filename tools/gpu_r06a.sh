# Round 6: split-bf16 GEMM tests, then the steady-step kernel trace at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r06a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gemm_split3_gpu.py > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
TAG=r06a/trace bash tools/gpu_trace_step.sh > /dev/null || exit 1
head -40 $OUT/trace/steady_step.txt
