# Round 5: F(4x4) ACC form with the bank-conflict-free swizzled V layout -- bit-identity,
# step-shape A/B vs the first form, an LDS PMC pass, then the default bench with it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ae
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wino4_forms_gpu.py -m gpu -v -x -k acc --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E " $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
for cfg in "0 1" "1 1"; do set -- $cfg
VOSDET_WINO4_ACC=$1 VOSDET_WINO4_VD=$2 timeout -k 10 200 python -u tools/bench_wino4.py > $OUT/ab_acc$1_vd$2.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "acc=$1 vd=$2"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'])" $OUT/ab_acc$1_vd$2.jsonl
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM"
i=0
for pmc in "$P1" "$P2"; do i=$((i+1))
VOSDET_WINO4_ACC=1 timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc_acc1/p$i -o run -- python3 tools/bench_wino4.py 32x256x200x336x256 > $OUT/pmc_acc1_p$i.log 2>&1 || { tail -5 $OUT/pmc_acc1_p$i.log; exit 1; }
done
python3 tools/rocpd_pmc.py conv3x3_wino4 $OUT/pmc_acc1.json $OUT/pmc_acc1/p1/run_results.db $OUT/pmc_acc1/p2/run_results.db > /dev/null
VOSDET_WINO4_ACC=1 timeout -k 10 300 python -u bench.py > $OUT/bench_acc1.json 2> $OUT/bench_acc1.err || { tail $OUT/bench_acc1.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $OUT/bench_acc1.json
