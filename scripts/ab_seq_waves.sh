#!/bin/bash
# C5 (5,000 nodes x 100,000 pods) on 1, 4 and 16 scanning waves of one workgroup (msh_options.seq_waves):
# the serial form without a capacity and the capacity form (15 pods per node). rocprofv3 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/abw}
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in ${WAVES:-1 4 16}; do
  for cap in ${CAPS:-0 15}; do
    tag=n${NODES:-5000}_w${w}_cap$cap
    NODES=${NODES:-5000} SEQ_WAVES=$w SPLIT=serial CAP=$cap WEIGHT=1 NORM=0 MODE=sequential PODS=100000 LAUNCHES=3 timeout -k 10 120 \
      rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o run --output-format csv -- python3 scripts/run_batch.py \
      > "$OUT/$tag.log" 2>&1 || { echo "[$tag] failed"; exit 1; }
    python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, sys, pathlib
for f in pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "seq_" in r["Name"]:
            print(f"{sys.argv[2]:12s} {r['Name'].split('(')[0]:50s} avg_us={float(r['AverageNs'])/1e3:.1f} calls={r['Calls']}")
PY
  done
done
