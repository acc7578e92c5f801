# PMC passes (one counter group per run) over tools/research/conv3x3_pmc.py
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/conv_pmc; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for grp in "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d /tmp/cpmc_$tag -o run -- python3 tools/research/conv3x3_pmc.py > $O/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $O/$tag.log; exit 1; }
  f=$(ls /tmp/cpmc_$tag/run_counter_collection.csv /tmp/cpmc_$tag/*/run_counter_collection.csv 2>/dev/null | head -1)
  python3 - "$f" > $O/$tag.txt <<'PY'
import csv, sys, collections
v = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "conv3x3" not in r["Kernel_Name"]:
        continue
    v[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in v:
    print(k, v[k] / max(1, n[k] // 1), "per-row-avg-over", n[k])
PY
  cat $O/$tag.txt
done
echo done
