# Round 5: F(4x4) time breakdown -- the kernel with parts removed (VOSDET_WINO4_PROBE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp
for p in 0 1 2 4 8 5 9 12 13 14 15; do
  echo "probe $p" >> $OUT/probe.jsonl
  VOSDET_WINO4_PROBE=$p timeout -k 10 120 python -u tools/bench_wino4.py 32x256x200x336x256 >> $OUT/probe.jsonl 2>> $OUT/probe.err || { tail $OUT/probe.err; exit 1; }
done
cat $OUT/probe.jsonl
