#!/bin/bash
# Round-3 A/B on the box: the product library (persistent multi-batch kernel) against the 2-D grid
# (MSH_WG_PERSIST=0) and the flag-form builds in scripts/expt/, at 8 and 32 batches per launch; then
# the multi-batch / chunk / table-change / scenario GPU tests and the bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3e2
mkdir -p $O
for nb in 8 32; do
  timeout -k 10 60 scripts/expt/run mini-kube-scheduler_amd/libminisched_hip.so persist $nb >> $O/expt.jsonl || exit 1
  MSH_WG_PERSIST=0 timeout -k 10 60 scripts/expt/run mini-kube-scheduler_amd/libminisched_hip.so grid2d $nb >> $O/expt.jsonl || exit 1
  for v in f0 f1 f0s f0n; do timeout -k 10 60 scripts/expt/run scripts/expt/lib$v.so $v $nb >> $O/expt.jsonl || exit 1; done
done
cat $O/expt.jsonl
TAG=r3q2 PYTEST_K="multi_batch or wg_kernel or table_change or scenario or batch_entry" bash scripts/gpu_r3_quick.sh
