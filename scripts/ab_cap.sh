#!/bin/bash
# A/B of the capacity form of C5 (5,000 nodes x 100,000 pods, 15 pods per node; rocprofv3 kernel trace of
# scripts/run_batch.py): the current library against variants in scripts/expt/<name>/libminisched_hip.so,
# in the reference list (NORM=0) and MIN-MAX at weight 3 (the KX decode).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/abcap}
mkdir -p "$OUT"
export TMPDIR=/tmp
for variant in ${VARIANTS:-cur cap1}; do
  lib=$PWD/mini-kube-scheduler_amd/libminisched_hip.so
  [ "$variant" != cur ] && lib=$PWD/scripts/expt/$variant/libminisched_hip.so
  for m in "1 0" "3 3"; do
    set -- $m
    tag=${variant}_w$1_n$2
    MSH_LIBRARY=$lib CAP=${CAP:-15} WEIGHT=$1 NORM=$2 MODE=sequential PODS=100000 LAUNCHES=5 timeout -k 10 120 \
      rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o run --output-format csv -- python3 scripts/run_batch.py \
      > "$OUT/$tag.log" 2>&1 || { echo "[$tag] failed"; exit 1; }
    python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, sys, pathlib
for f in pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "seq_" in r["Name"]:
            print(f"{sys.argv[2]:20s} {r['Name'].split('(')[0]:50s} avg_us={float(r['AverageNs'])/1e3:.1f} calls={r['Calls']}")
PY
  done
done
