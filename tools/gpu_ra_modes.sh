# Tiled RoIAlign (variant 30) diagnostics on the GPU box: parity tests, then
# HIP-event timing of the 8-frame launch per VOSDET_RA_CFG ("loaders,waves,mode"; mode 0 product, 1 no
# compute, 2 no window DMA) and a kernel trace.
# usage: MODES="- 2,12,0 4,12,1" TAG=x bash tools/gpu_ra_modes.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ram}; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "${TESTK:-tiled}" > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -ne 0 ] && { grep -B5 -A40 "Error\|FAILED\|assert" $O/tests.txt | head -80; exit $rc; }
for m in ${MODES:--}; do
  if [ "$m" = "-" ]; then unset VOSDET_RA_CFG; else export VOSDET_RA_CFG=${m%%:*}; fi
  case $m in *:o1) export VOSDET_RA_ORDER=1;; *) unset VOSDET_RA_ORDER;; esac
  VOSDET_ROIALIGN_VARIANT=30 timeout -k 10 120 python -u tools/bench_roialign.py 7 > $O/m$m.json 2> $O/m$m.err || { echo "mode $m failed"; tail -5 $O/m$m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/m$m.json'));print('mode $m', d['avg_launch_us'], d['frac'])"
done
unset VOSDET_RA_CFG
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
VOSDET_ROIALIGN_VARIANT=30 RA_ITERS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_roialign.py 7 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/trace/run_kernel_stats.csv")):
    if "ratile" in r["Name"] or "fillBuffer" in r["Name"]:
        print(r["Name"][:44], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
echo done
