#!/bin/bash
# rocprofv3 kernel trace + stats of the RoIAlign roofline launch for one variant:
# per-kernel average durations (the binning passes, the staging kernel, direct).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=${D:-gpurun_out/ra_prof}
rm -rf "$D"; mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in ${VARIANTS:-60}; do
  VOSDET_ROIALIGN_VARIANT=$v RA_ITERS=20 timeout -k 10 180 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$D/v$v" -o run -- python3 tools/bench_roialign.py ${P:-7} \
      > "$D/v$v.log" 2>&1 || { echo "trace $v failed"; tail -5 "$D/v$v.log"; exit 1; }
  f=$(find "$D/v$v" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$D/kernel_stats_v$v.csv"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%-90s %6s %10.1f us" % (r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
