#!/bin/bash
# A/B of kernel builds in scripts/expt/ (lib<name>.so) at 20 and 32 batches per launch, plus the
# 8-wave workgroup setting of the base build; one JSON line each into gpurun_out/$TAG/ab.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r3ab}
mkdir -p $O
for nb in 20 32; do
  for v in ${VARIANTS:-base pipe}; do
    timeout -k 10 60 scripts/expt/run scripts/expt/lib$v.so $v $nb >> $O/ab.jsonl || exit 1
  done
  MSH_WG_WAVES=8 timeout -k 10 60 scripts/expt/run scripts/expt/libbase.so base_w8 $nb >> $O/ab.jsonl || exit 1
done
cat $O/ab.jsonl
