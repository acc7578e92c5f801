# Round 5: F(4x4) V read-ahead distance (VOSDET_WINO4_VD, ACC form) -- bit-identity,
# step-shape A/B, then SQ PMC passes on the benched P2 conv (first form and VD=3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05ad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wino4_forms_gpu.py -m gpu -v -x -k acc --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.txt | tail -2; grep -E "^E " $OUT/tests.txt | head -8
[ $rc -eq 0 ] || exit $rc
for cfg in "0 1" "1 1" "1 2" "1 3"; do set -- $cfg
VOSDET_WINO4_ACC=$1 VOSDET_WINO4_VD=$2 timeout -k 10 200 python -u tools/bench_wino4.py > $OUT/ab_acc$1_vd$2.jsonl 2> $OUT/w.err || { tail $OUT/w.err; exit 1; }
echo "acc=$1 vd=$2"; python3 -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(d['shape'], d['wino4_us'], d['wino4_exec_frac'])" $OUT/ab_acc$1_vd$2.jsonl
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM"
for cfg in "0 1" "1 3"; do set -- $cfg
i=0
for pmc in "$P1" "$P2"; do i=$((i+1))
VOSDET_WINO4_ACC=$1 VOSDET_WINO4_VD=$2 timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc_acc$1_vd$2/p$i -o run -- python3 tools/bench_wino4.py 32x256x200x336x256 > $OUT/pmc_acc$1_vd$2_p$i.log 2>&1 || { tail -5 $OUT/pmc_acc$1_vd$2_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/pmc_acc$1_vd$2 conv3x3_wino4 $OUT/pmc_acc$1_vd$2.json && cat $OUT/pmc_acc$1_vd$2.json
done
