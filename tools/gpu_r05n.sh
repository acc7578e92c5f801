# Round 5: which change breaks test_graph_replay_gpu -- F(4x4) off, then radix select off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
VOSDET_WINO4=0 timeout -k 10 400 python -u -m pytest tests/test_graph_replay_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/nowino4.txt 2>&1; rc=$?
echo "wino4 off rc=$rc"; grep -E "passed|failed" $OUT/nowino4.txt | tail -1
[ $rc -le 1 ] || exit $rc
VOSDET_RPN_PRESEL=0 timeout -k 10 400 python -u -m pytest tests/test_graph_replay_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/nopresel.txt 2>&1; rc=$?
echo "presel off rc=$rc"; grep -E "passed|failed" $OUT/nopresel.txt | tail -1
