cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -x -q -k "schedules" --timeout 150 --timeout-method thread > gpurun_out/pf_tests.txt 2>&1; tail -2 gpurun_out/pf_tests.txt
for cfg in "10 none" "10 1000" "16 1000 8" "16 1000 16" "16 1000 32"; do
  set -- $cfg
  if [ "$2" = none ]; then unset XCD_WINDOW; else export XCD_WINDOW=$2; fi
  VOSDET_RA_PF_STRIDE=${3:-16} VOSDET_ROIALIGN_VARIANT=$1 timeout -k 10 100 python tools/bench_roialign.py 7 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['avg_launch_us'], d['frac'])" || exit 1
done
