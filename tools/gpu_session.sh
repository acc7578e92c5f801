#!/bin/bash
# One GPU session on the box: the -m gpu suite (or the files given in TESTS), then
# optionally the default bench.  Every GPU step under its own time limit, chained
# with &&: a fault, abort or timeout ends the call.
#   OUT=gpurun_out/<tag> TESTS="tests/..." BENCH=1 bash tools/gpu_session.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/session}
mkdir -p "$OUT"
export TMPDIR=/tmp
python - > "$OUT/plans_key.txt" 2>&1 <<'PY'
import ctypes
import torch  # loads torch's hipBLASLt first, as every product process does
from vosdetectron_amd import _lib
b = ctypes.create_string_buffer(256)
_lib.check(_lib.lib().vd_gemm_plans_key(b, 256), "vd_gemm_plans_key")
print(b.value.decode())
PY
timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest ${TESTS:-tests} -m gpu -v --maxfail=5 \
    --timeout 400 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?
tail -5 "$OUT/gpu_tests.txt"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (read them); else stop
if [ "${BENCH:-0}" = "1" ]; then
    timeout -k 10 ${BENCH_LIMIT:-400} python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" \
        2> "$OUT/bench.err" || exit $?
    tail -c 3000 "$OUT/bench.json"
fi
exit $rc
