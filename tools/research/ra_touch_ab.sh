#!/bin/bash
# Variant 18 (touch wave) vs the product kernel: bit-exactness on the schedule
# test, then the roofline launch at several look-aheads.
cd "${GRAFT_REPO_ROOT:-.}"
VOSDET_TEST_RA_VARIANTS="18" timeout -k 10 200 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -x -q -k "schedules" --timeout 150 --timeout-method thread > gpurun_out/touch_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/touch_tests.txt; [ $rc -ne 0 ] && exit $rc
for cfg in "10 0" ${CFGS:-"18 16" "18 32" "18 64" "18 128" "18 256"}; do
  set -- $cfg
  VOSDET_RA_TOUCH_AHEAD=$2 VOSDET_ROIALIGN_VARIANT=$1 timeout -k 10 100 python tools/bench_roialign.py ${P:-7} | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['avg_launch_us'], d['frac'])" || exit 1
done
