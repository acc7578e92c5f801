# Round 5 (session 3 start): step trace at HEAD, then the whole -m gpu suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=r05q/trace bash tools/gpu_trace_step.sh > /dev/null || exit $?
head -45 gpurun_out/r05q/trace/steady_step.txt
OUT=gpurun_out/r05q/suite TEST_LIMIT=720 bash tools/gpu_session.sh
