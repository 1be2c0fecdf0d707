#!/bin/bash
# GPU side of scripts/wg_expt.sh: every variant at 8 and 32 batches per launch, then the product
# library (kernel timing only). One JSON line each into gpurun_out/$TAG/expt.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r3e}
mkdir -p "$OUT"
for nb in 8 32; do
  timeout -k 10 60 scripts/expt/run mini-kube-scheduler_amd/libminisched_hip.so product $nb >> "$OUT/expt.jsonl" || exit 1
  for x in ${EXPTS:-0 1 2 4 7}; do
    timeout -k 10 60 scripts/expt/run scripts/expt/libexpt$x.so expt$x $nb >> "$OUT/expt.jsonl" || exit 1
  done
done
cat "$OUT/expt.jsonl"
