#!/bin/bash
# Batches per launch: rocprofv3 kernel trace of 32- and 64-batch C3 launches (headline list) on the current
# library and a variant in scripts/expt/<name>/ (MULTI_MAX 64), scripts/run_batch.py MODE=multi.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/abnb}
mkdir -p "$OUT"
export TMPDIR=/tmp
for arm in cur:32 ${VARIANT:-mm64}:32 ${VARIANT:-mm64}:64 ${VARIANT:-mm64}:96; do
  v=${arm%%:*} nb=${arm##*:}
  lib=$PWD/mini-kube-scheduler_amd/libminisched_hip.so
  [ "$v" != cur ] && lib=$PWD/scripts/expt/$v/libminisched_hip.so
  [ "$nb" = 96 ] && [ "${VARIANT:-mm64}" != mm96 ] && continue
  MSH_LIBRARY=$lib NB=$nb WEIGHT=3 NORM=1 MODE=multi PODS=100000 LAUNCHES=30 timeout -k 10 120 rocprofv3 --kernel-trace \
    --stats -d "$OUT/${v}_$nb" -o run --output-format csv -- python3 scripts/run_batch.py > "$OUT/${v}_$nb.log" 2>&1 \
    || { echo "[$v $nb] failed"; exit 1; }
  python3 - "$OUT/${v}_$nb" "$v nb=$nb" "$nb" <<'PY'
import csv, sys, pathlib
for f in pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "pair" in r["Name"]:
            a = float(r["AverageNs"]) / 1e3
            print(f"{sys.argv[2]:14s} {r['Name'].split('(')[0]:44s} avg_us={a:.1f} per_batch_us={a / int(sys.argv[3]):.3f}")
PY
done
