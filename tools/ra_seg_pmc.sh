# L2 / fabric counters of the RoIAlign segment configurations (separate passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ra_seg_pmc; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for cfg in "1 1" "2 2" "4 4"; do
  set -- $cfg
  for grp in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $grp | tr ' ' '_')
    VOSDET_RA_SEGS=$1 VOSDET_RA_PARTS=$2 RA_ITERS=5 timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/s$1_g$2/$tag -o run -- python3 tools/bench_roialign.py 7 > $O/s$1_g$2_$tag.log 2>&1 || { echo "pmc $cfg $tag failed"; tail -5 $O/s$1_g$2_$tag.log; exit 1; }
  done
  python tools/pmc_summary.py $O/s$1_g$2 sep_buf $O/s$1_g$2.json | grep -E "FETCH|l2_hit"
done
echo done
