# Round 5: NMS/proposal parity, the proposal kernels' trace, then a bench trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=gpurun_out/${TAG:-r05c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_nms_proposals_gpu.py tests/test_soft_nms_gpu.py tests/test_edge_cases_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt -o run -- python3 $R/tools/prop_time.py 32 > $R/$OUT/prop_prof.log 2>&1 || { tail $R/$OUT/prop_prof.log; exit 1; }
cd $R
cp /tmp/pt/run_kernel_trace.csv $OUT/prop_kernel_trace.csv
python3 tools/prop_breakdown.py $OUT/prop_kernel_trace.csv > $OUT/prop_breakdown.txt; cat $OUT/prop_breakdown.txt
TAG=${TAG:-r05c}/trace bash tools/gpu_trace_step.sh > /dev/null || exit 1
cat $OUT/trace/post_launches.txt
