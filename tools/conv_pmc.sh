# PMC passes (one counter group per run) over tools/conv_shape_run.py; per-dispatch
# averages of the matching kernel.  usage: ALGO=wino SHAPE="16 256 200 336" KFILT=wino bash tools/conv_pmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-conv_pmc}; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for grp in "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d /tmp/cpmc_$tag -o run -- python3 tools/conv_shape_run.py ${ALGO:-wino} ${SHAPE:-16 256 200 336} > $O/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $O/$tag.log; exit 1; }
  f=$(ls /tmp/cpmc_$tag/run_counter_collection.csv /tmp/cpmc_$tag/*/run_counter_collection.csv 2>/dev/null | head -1)
  python3 - "$f" "${KFILT:-wino}" > $O/$tag.txt <<'PY'
import csv, sys, collections
v = collections.defaultdict(float); n = collections.Counter(); d = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] not in r["Kernel_Name"]:
        continue
    v[r["Counter_Name"]] += float(r["Counter_Value"]); d[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
for k in v:
    print(k, v[k] / max(1, len(d[k])), "per dispatch over", len(d[k]))
PY
  cat $O/$tag.txt
done
echo done
