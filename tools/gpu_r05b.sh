# Round 5: proposal kernels under a rocprofv3 kernel trace (select A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt -o run -- python3 $R/tools/prop_time.py 32 > $R/$OUT/prop_prof.log 2>&1 || { tail $R/$OUT/prop_prof.log; exit 1; }
cd $R
cp /tmp/pt/run_kernel_stats.csv $OUT/prop_kernel_stats.csv
cp /tmp/pt/run_kernel_trace.csv $OUT/prop_kernel_trace.csv
cut -d, -f1-8 $OUT/prop_kernel_stats.csv | head -20
timeout -k 10 300 python -u -m pytest tests/test_vos_post_gpu.py tests/test_soft_nms_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/vos_post_tests.txt 2>&1 || { tail -40 $OUT/vos_post_tests.txt; exit 1; }
tail -3 $OUT/vos_post_tests.txt
