#!/bin/bash
# GPU side of scripts/ab_build.sh: each variant's kernel time per launch at 8 and 32 batches per launch,
# the variants interleaved over REPS rounds. One JSON line each into gpurun_out/$TAG/ab.jsonl.
#   TAG=x REPS=3 scripts/ab_run.sh base quad pipe
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for r in $(seq 1 "${REPS:-3}"); do
  for nb in ${NBS:-8 32}; do
    for v in "$@"; do
      timeout -k 10 60 scripts/expt/run "scripts/expt/libab_$v.so" "$v" "$nb" >> "$OUT/ab.jsonl" || exit 1
    done
  done
done
cat "$OUT/ab.jsonl"
