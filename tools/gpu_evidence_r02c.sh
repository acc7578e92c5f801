# Round-2 (third session) evidence pass at HEAD: full -m gpu suite, smoke, the
# default bench (cpu baseline + rooflines), the other BASELINE configs' FPS, and
# an MFMA-busy PMC pass over a short bench.  MIOpen's find-db lives in /tmp for
# the whole call, so only the first bench pays the NORMAL-mode Find.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r02c}; mkdir -p $O
export MIOPEN_USER_DB_PATH=/tmp/vd_miopen_db; mkdir -p $MIOPEN_USER_DB_PATH
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_suite.txt 2>&1
rc=$?; tail -3 $O/gpu_suite.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo smoke failed; tail $O/smoke.txt; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail $O/bench_default.err; exit 1; }
tail -c 300 $O/bench_default.json; echo
exit 0
fi
if [ "${PART}" = 3 ]; then  # N-rank rehearsal on the one-GPU box (gloo collectives)
timeout -k 10 600 python -u bench.py --gpus 2 --share-gpu --steps 4 --warmup 2 --no-cpu-baseline > $O/bench_share2.json 2> $O/bench_share2.err || { echo share2 failed; tail -5 $O/bench_share2.err; exit 1; }
tail -c 400 $O/bench_share2.json; echo
exit 0
fi
for c in e2e_mask_rcnn_R-101-FPN_2x e2e_mask_rcnn_X-101-32x8d-FPN_1x e2e_mask_rcnn_R-50-C4_1x vos_R-101-FPN_3x_gn_dynamic_davis; do
  timeout -k 10 400 python -u bench.py --config $c --batch 8 --steps 5 --no-cpu-baseline --no-roofline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -3 $O/bench_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
T=/tmp/vd_pmc; rm -rf $T
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $T -o run -- python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-timers --no-roofline > $O/pmc_mfma.log 2>&1 || { echo pmc failed; tail -5 $O/pmc_mfma.log; exit 1; }
python3 tools/pmc_step_mfma.py $(ls $T/run_counter_collection.csv $T/*/run_counter_collection.csv 2>/dev/null | head -1) > $O/mfma_pmc_step.json || exit 1
head -c 1500 $O/mfma_pmc_step.json
echo done
