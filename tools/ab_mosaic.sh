# Same-box A/B of the Winograd layout routing: default (2-D mosaic where it fills
# more of a block) vs VOSDET_WINO_MOSAIC=1 (maps stacked in one column at most).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abmos; rm -rf $O; mkdir -p $O
for rep in 1 2; do for m in 2 1; do
  VOSDET_WINO_MOSAIC=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/m${m}_$rep.json 2> $O/m${m}_$rep.err || { tail -5 $O/m${m}_$rep.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/m${m}_$rep.json').read().strip().splitlines()[-1]);print('mosaic=$m rep $rep', d['value'], d['ms_per_step'])"
done; done
