set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/research/graph_prop_dbg.py > $OUT/dbg.txt 2>&1; rc=$?
cat $OUT/dbg.txt | grep -v amdgpu.ids | tail -30
exit $rc
