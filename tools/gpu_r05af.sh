# Round 5: full GPU suite at the ACC-form default, the step's kernel trace, and one
# SQ PMC pass (LDS conflicts, MFMA busy) over the hand-written and hipBLASLt kernels
# of a short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_suite.txt 2>&1; rc=$?
tail -3 $OUT/gpu_suite.txt; grep -E "^E " $OUT/gpu_suite.txt | head -8
[ $rc -eq 0 ] || exit $rc
TAG=r05af/trace bash tools/gpu_trace_step.sh > /dev/null || exit 1
head -12 $OUT/trace/steady_step.txt
T=/tmp/vd_pmc; rm -rf $T
timeout -s KILL 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex "vd::|Cijk" -d $T -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timers --no-roofline > $OUT/pmc_bench.log 2>&1 || { tail -5 $OUT/pmc_bench.log; exit 1; }
python3 tools/rocpd_pmc_table.py $T/run_results.db $OUT/pmc_step_table.json
