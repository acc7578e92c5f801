set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_stem_gpu.py tests/test_soft_nms_gpu.py tests/test_nms_proposals_gpu.py tests/test_vos_post_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -4 $O/tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/stem_time.py > $O/stem_time.json 2>&1 || exit $?
cat $O/stem_time.json
timeout -k 10 100 python tools/prop_time.py > $O/prop_u8.txt 2>&1 || exit $?
VOSDET_RESEARCH_LIB=vosdetectron_amd/libvosdet_u24.so timeout -k 10 100 python tools/prop_time.py > $O/prop_u24.txt 2>&1 || exit $?
tail -5 $O/prop_u8.txt $O/prop_u24.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_miopen.json 2> $O/bench_miopen.err || exit $?
VOSDET_STEM=fused timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fused.json 2> $O/bench_fused.err || exit $?
python - <<'PY'
import json
for t in ("miopen", "fused"):
    d = json.loads(open("gpurun_out/r04e/bench_%s.json" % t).read().strip().splitlines()[-1])
    print(t, d["value"], d["ms_per_step"], d["stages_ms"], d["nms"]["latency_us"], d["class_nms"]["avg_us"] if "class_nms" in d else d.get("proposals", {}).get("avg_us"))
PY
exit $rc
