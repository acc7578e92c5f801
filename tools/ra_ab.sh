#!/bin/bash
# RoIAlign A/B on the box: the tiled / ring GPU tests, then the 8-frame roofline
# launch for each variant in VARIANTS (and ring diagnostics modes), one JSON line
# each into $D/ab.jsonl (D=gpurun_out/<tag>).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=${D:-gpurun_out/ra_ab}
mkdir -p "$D"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_roi_ops_gpu.py -m gpu -x -v -k "tiled or rows or fpn" \
      --timeout 200 --timeout-method thread > "$D/tests.txt" 2>&1
  rc=$?; tail -3 "$D/tests.txt"; [ $rc -ne 0 ] && exit $rc
fi
: > "$D/ab.jsonl"
for v in ${VARIANTS:-10 30 60}; do
  VOSDET_ROIALIGN_VARIANT=$v timeout -k 10 120 python -u tools/bench_roialign.py ${P:-7} >> "$D/ab.jsonl" 2> "$D/err_$v.txt" || { echo "variant $v failed"; tail -5 "$D/err_$v.txt"; exit 1; }
done
for m in ${MODES:-}; do
  VOSDET_ROIALIGN_VARIANT=60 VOSDET_RA_RING_MODE=$m timeout -k 10 120 python -u tools/bench_roialign.py ${P:-7} | sed "s/^{/{\"ring_mode\": $m, /" >> "$D/ab.jsonl" || exit 1
done
python - "$D/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d.get("variant"), d.get("ring_mode", "-"), d["avg_launch_us"], d["frac"])
PY
