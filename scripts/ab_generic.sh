#!/bin/bash
# A/B of generic_kernel per 32-batch C3 launch (rocprofv3 kernel trace of scripts/run_batch.py): the current
# library against variants built by scripts/expt/build_variant.py, on the column lists and the reference list.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r6f}
mkdir -p "$OUT"
export TMPDIR=/tmp
# LISTS: "mode weight norm colnorm" entries separated by ';'
IFS=';' read -ra LST <<< "${LISTS:-generic_col 1 0 0;generic_2col 1 0 0;generic 3 1 0;generic 1 0 0;generic_w64 1 0 0;generic_w64 1 0 1}"
for variant in ${VARIANTS:-cur gen_base}; do
  lib=$PWD/mini-kube-scheduler_amd/libminisched_hip.so
  [ "$variant" != cur ] && lib=$PWD/scripts/expt/$variant/libminisched_hip.so
  for m in "${LST[@]}"; do
    set -- $m
    tag=${variant}_$1_$2_$3_$4
    COLNORM=$4 MSH_LIBRARY=$lib WEIGHT=$2 NORM=$3 MODE=$1 PODS=100000 LAUNCHES=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
      -d "$OUT/$tag" -o run --output-format csv -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1 || { echo "[$tag] failed"; exit 1; }
    python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, sys, pathlib
for f in pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "generic_kernel" in r["Name"]:
            print(f"{sys.argv[2]:32s} {r['Name'].split('(')[0]:60s} avg_us={float(r['AverageNs'])/1e3:.1f} calls={r['Calls']}")
PY
  done
done
