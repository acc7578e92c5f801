#!/bin/bash
# A/B of the GEMM plan pins: the in-tree pins (top-16 heuristic search) vs a fresh
# search over the top VOSDET_GEMM_MAXALGOS (64) hipBLASLt candidates, recorded into
# $O/plans64.txt by a short bench and then benched.  Every GPU step time-limited.
set -o pipefail
O=${O:-gpurun_out/gemm_ab}; mkdir -p $O; rm -f $O/plans64.txt
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 $B > $O/bench_pins16.json 2> $O/bench_pins16.err || exit $?
VOSDET_GEMM_MAXALGOS=64 VOSDET_GEMM_PLANS=$O/plans64.txt VOSDET_GEMM_PLANS_RECORD=1 \
    timeout -k 10 400 $B --steps 3 --warmup 2 --no-roofline --no-timers > $O/search.json 2> $O/search.err || exit $?
VOSDET_GEMM_MAXALGOS=64 VOSDET_GEMM_PLANS=$O/plans64.txt timeout -k 10 300 $B > $O/bench_pins64.json 2> $O/bench_pins64.err || exit $?
timeout -k 10 300 $B > $O/bench_pins16b.json 2> $O/bench_pins16b.err || exit $?
python - <<'PY'
import json, os
O = os.environ.get("O", "gpurun_out/gemm_ab")
for t in ("pins16", "pins64", "pins16b"):
    d = json.loads(open("%s/bench_%s.json" % (O, t)).read().strip().splitlines()[-1])
    print(t, d["value"], d["ms_per_step"], d["stages_ms"])
PY
