# run the given -m gpu test files (default: all) with per-test timeouts
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/gpu_tests.txt}
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $OUT 2>&1
rc=$?
tail -4 $OUT
exit $rc
