#!/bin/bash
# A/B of C5 without a capacity (5,000 nodes x 100,000 pods, the headline list w=3 DEFAULT; rocprofv3 kernel
# trace of scripts/run_batch.py): the auto form (pair_kernel with the commit epilogue) and seq_kernel's 64-pod
# blocks (SPLIT=blocks), for the current library and variants in scripts/expt/<name>/libminisched_hip.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/abseq}
mkdir -p "$OUT"
export TMPDIR=/tmp
for variant in ${VARIANTS:-cur}; do
  lib=$PWD/mini-kube-scheduler_amd/libminisched_hip.so
  [ "$variant" != cur ] && lib=$PWD/scripts/expt/$variant/libminisched_hip.so
  for split in ${SPLITS:-auto blocks}; do
    tag=${variant}_${split}
    MSH_LIBRARY=$lib SPLIT=$split WEIGHT=${WEIGHT:-3} NORM=${NORM:-1} MODE=sequential PODS=100000 LAUNCHES=${LAUNCHES:-40} \
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o run --output-format csv -- \
      python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1 || { echo "[$tag] failed"; tail -5 "$OUT/$tag.log"; exit 1; }
    python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, sys, pathlib
for f in pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "seq_" in r["Name"] or "pair_kernel" in r["Name"] or "fold" in r["Name"]:
            print(f"{sys.argv[2]:16s} {r['Name'].split('(')[0]:50s} avg_us={float(r['AverageNs'])/1e3:.2f} "
                  f"min_us={float(r['MinNs'])/1e3:.2f} calls={r['Calls']}")
PY
  done
done
