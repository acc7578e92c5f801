set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/raab
timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/raab/tests.txt 2>&1 || { tail -20 gpurun_out/raab/tests.txt; exit 1; }
tail -1 gpurun_out/raab/tests.txt
for rep in 1 2 3; do for g in 0 1; do
  if [ $g = 1 ]; then export VOSDET_RA_GENERAL=1; else unset VOSDET_RA_GENERAL; fi
  timeout -k 10 120 python -u tools/bench_roialign.py 7 > gpurun_out/raab/g${g}_$rep.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/raab/g${g}_$rep.json'));print('general=$g rep $rep', d['avg_launch_us'], d['frac'])"
done; done
