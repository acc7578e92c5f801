# round-2 GPU check: new/changed -m gpu tests first, then the whole suite, then the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_edge_cases_gpu.py tests/test_reference_api_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02_gpu_new.txt 2>&1
rc=$?
tail -5 gpurun_out/r02_gpu_new.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python -u bench.py > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err
rc=$?
tail -c 4000 gpurun_out/r02_bench_default.json
exit $rc
