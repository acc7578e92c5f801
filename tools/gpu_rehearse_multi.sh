# 2-rank RCCL rehearsal of bench.py on a one-GPU box (--share-gpu)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 2 --share-gpu --steps 3 --warmup 1 --batch 2 --no-cpu-baseline --no-roofline --no-timers > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
rc=$?
tail -c 1500 gpurun_out/rehearse2.json; tail -20 gpurun_out/rehearse2.err
exit $rc
