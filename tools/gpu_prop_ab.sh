# proposals / NMS / detections parity, then proposal timing (split and fused NMS)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=prop3 TESTS="tests/test_nms_proposals_gpu.py tests/test_edge_cases_gpu.py tests/test_c4.py tests/test_engine_gpu.py tests/test_reference_api_gpu.py" bash tools/gpu_quick.sh || exit 1
echo split; timeout -k 10 200 python tools/prop_time.py || exit 1
echo nosplit; VOSDET_RPN_SPLIT=0 timeout -k 10 200 python tools/prop_time.py || exit 1
VOSDET_RPN_SPLIT=0 timeout -k 10 200 python -u -m pytest tests/test_nms_proposals_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread 2>&1 | tail -2
