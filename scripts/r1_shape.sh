#!/bin/bash
# Shape sweep (fixed vs per-pair cost) of the default library and A/B variants, one process each.
set -o pipefail
mkdir -p gpurun_out
for tag in ${TAGS:-default u16 u16q8}; do
  lib=mini-kube-scheduler_amd/libminisched_hip_${tag}.so
  [ "$tag" = default ] && lib=mini-kube-scheduler_amd/libminisched_hip.so
  MSH_LIBRARY=$lib TAG=$tag timeout -k 10 180 python scripts/scale_grid.py >> gpurun_out/shape.jsonl 2> gpurun_out/shape_$tag.err || exit $?
done
echo shape-done
