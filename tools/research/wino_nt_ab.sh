

# Same-box A/B: Winograd with nt LDS-DMA for U (VOSDET_WINO_PROBE=64) or the patch (128)
# vs as shipped -- per-shape probe and the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ntab; rm -rf $O; mkdir -p $O
for m in "" 64 128; do
  VOSDET_WINO_PROBE=$m timeout -k 10 300 python -u tools/wino_mosaic_probe.py > $O/probe_$m.json 2> $O/probe_$m.err || { tail -3 $O/probe_$m.err; exit 1; }
done
for rep in 1 2; do for m in "" 64 128; do
  VOSDET_WINO_PROBE=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $O/b${m}_$rep.json 2> $O/b${m}_$rep.err || { tail -5 $O/b${m}_$rep.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b${m}_$rep.json').read().strip().splitlines()[-1]);print('nt=${m:-0} rep $rep', d['value'], d['ms_per_step'])"
done; done
