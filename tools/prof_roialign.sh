#!/bin/bash
# PMC passes over the RoIAlign microbenchmark (one counter group per pass, as
# the MI355X guide prescribes).  Usage: tools/prof_roialign.sh OUTDIR [variant] [order] [deal]
set -u
OUT=${1:-gpurun_out/prof_ra}
export VOSDET_ROIALIGN_VARIANT=${2:-8}
export ORDER=${3:-1}
export XCD_DEAL=${4:-8}  # read by tools/bench_roialign.py
export RA_ITERS=5
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_ANY" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$tag -o run -- python3 tools/bench_roialign.py 7 > $OUT/$tag.log 2>&1 || { echo "pass $tag failed rc=$?" >> $OUT/failures.txt; exit 1; }
done
