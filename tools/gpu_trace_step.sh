# rocprofv3 kernel trace of a short default bench, kept in /tmp on the box (MIOpen's
# NORMAL Find launches thousands of candidate kernels during warm-up, too much to
# ship back); only the steady-step breakdown and the kernel stats come back.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-trace}; rm -rf $O; mkdir -p $O
T=/tmp/vd_trace; rm -rf $T
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-timers ${BENCH_ARGS:-} > $O/bench_trace.log 2>&1 || { echo trace failed; tail -5 $O/bench_trace.log; exit 1; }
python3 tools/analyze_trace.py $T/run_kernel_trace.csv image_to_blob 60 > $O/steady_step.txt || exit 1
python3 tools/kernel_breakdown.py $T/run_kernel_trace.csv roi_align_fpn > $O/roialign_launches.txt || exit 1
for k in nms_prep nms_mask nms_resolve rpn_ class_nms det_limit; do
    python3 tools/kernel_breakdown.py $T/run_kernel_trace.csv $k; done > $O/post_launches.txt || exit 1
for k in conv3x3_wino gemm_split3 gemm1x1 stem_conv; do
    python3 tools/kernel_breakdown.py $T/run_kernel_trace.csv $k; done > $O/conv_gemm_launches.txt || exit 1
cp $T/run_kernel_stats.csv $O/kernel_stats.csv
head -30 $O/steady_step.txt
