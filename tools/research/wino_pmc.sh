# PMC counters of the P2 Winograd launch (tools/research/wino_sol_probe.py, product
# library, PROBES=0: 13 launches), one rocprofv3 --pmc pass per counter group.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-wino_pmc}; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for P in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
    i=$((i + 1))
    PROBES=0 timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d $O/pmc/p$i -o p -- python3 tools/research/wino_sol_probe.py > $O/pass$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pass$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O/pmc conv3x3_wino2 $O/summary.json > /dev/null && cat $O/summary.json
