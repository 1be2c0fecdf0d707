#!/bin/bash
# Work-queue kernel geometry A/B: workgroup size x workgroups per CU; stamps + timing per point.
set -o pipefail
mkdir -p gpurun_out
for nt in ${NTS:-1024 512 256}; do
  for wg in ${WGS:-0 half}; do
    w=$wg; [ "$wg" = half ] && w=$(( 16 * 64 / nt ))
    [ "$w" = 0 ] && w=""
    tag="nt${nt}_wg${w:-auto}"
    MSH_DYN_THREADS=$nt MSH_BATCH_WG_PER_CU=$w CASES=${CASES:-5000x100000} timeout -k 10 120 python scripts/stamps_dyn.py > gpurun_out/stamps_$tag.jsonl 2>/dev/null || exit $?
    MSH_DYN_THREADS=$nt MSH_BATCH_WG_PER_CU=$w TAG=$tag GRID=${GRID:-5000x100000,5000x1000000} timeout -k 10 120 python scripts/scale_grid.py >> gpurun_out/dyn.jsonl 2>/dev/null || exit $?
  done
done
echo dyn-done
