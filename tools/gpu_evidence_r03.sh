# Round-3 evidence at HEAD.  PART=roof: per-conv/GEMM MFMA roofline of one steady
# 16-frame step (tools/conv_roofline.py); PART=cfg: the other BASELINE configs'
# FPS (8 frames per step); PART=pmc: MFMA-busy PMC pass over a short bench;
# PART=share2: 2-rank rehearsal on the one-GPU box (gloo).  MIOpen's find-db lives
# in /tmp for the whole call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03e}; mkdir -p $O
# MIOpen reads the in-tree find-db (vosdetectron_amd/miopen_db, set by the package)
for part in ${PART:-roof}; do
case $part in
roof)
  timeout -k 10 400 python -u tools/conv_roofline.py $O/conv_roofline.json > $O/conv_roofline.log 2>&1 || { echo roofline failed; tail -20 $O/conv_roofline.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/conv_roofline.json'));print({k:v for k,v in d.items() if k!='ops'})" ;;
cfg)
  for c in ${CONFIGS:-e2e_mask_rcnn_R-101-FPN_2x e2e_mask_rcnn_X-101-32x8d-FPN_1x e2e_mask_rcnn_R-50-C4_1x vos_R-101-FPN_3x_gn_dynamic_davis}; do
    timeout -k 10 400 python -u bench.py --config $c --batch 8 --steps 5 --no-cpu-baseline --no-roofline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -3 $O/bench_$c.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'])"
  done ;;
pmc)
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  T=/tmp/vd_pmc; rm -rf $T
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $T -o run -- python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-timers --no-roofline > $O/pmc_mfma.log 2>&1 || { echo pmc failed; tail -5 $O/pmc_mfma.log; exit 1; }
  python3 tools/pmc_step_mfma.py $(ls $T/run_counter_collection.csv $T/*/run_counter_collection.csv 2>/dev/null | head -1) > $O/mfma_pmc_step.json || exit 1
  head -c 600 $O/mfma_pmc_step.json; echo ;;
share2)
  timeout -k 10 600 python -u bench.py --gpus 2 --share-gpu --steps 4 --warmup 2 --no-cpu-baseline > $O/bench_share2.json 2> $O/bench_share2.err || { echo share2 failed; tail -5 $O/bench_share2.err; exit 1; }
  tail -c 400 $O/bench_share2.json; echo ;;
esac
done
echo done
