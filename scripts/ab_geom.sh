#!/bin/bash
# Persistent-kernel geometry A/B on the product library: kernel time per launch (scripts/expt/run) for
# each MSH_WGP_WAVES x MSH_WGP_WPC pair given as "W:WPC" arguments, at 8 and 32 batches per launch.
#   TAG=x scripts/ab_geom.sh 4:8 8:4 16:2 16:1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-geom}
mkdir -p "$OUT"
LIB=mini-kube-scheduler_amd/libminisched_hip.so
for r in $(seq 1 "${REPS:-2}"); do
  for nb in ${NBS:-8 32}; do
    for g in "$@"; do
      MSH_WGP_WAVES=${g%%:*} MSH_WGP_WPC=${g#*:} timeout -k 10 60 scripts/expt/run $LIB "w$g" "$nb" >> "$OUT/ab.jsonl" || exit 1
    done
  done
done
python3 scripts/ab_summary.py "$OUT/ab.jsonl"
