#!/bin/bash
# PMC of the capacity form of C5 (5,000 nodes x 100,000 pods, 15 pods per node, the reference list) for the
# current library and a variant (MSH_LIBRARY=scripts/expt/<name>/libminisched_hip.so): one --pmc pass per
# counter set, each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r6d}
mkdir -p "$OUT"
export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
for variant in ${VARIANTS:-cur old_cap}; do
  lib=""
  [ "$variant" != cur ] && lib="$PWD/scripts/expt/$variant/libminisched_hip.so"
  for set in SQ1 SQ2; do
    MSH_LIBRARY=${lib:-$PWD/mini-kube-scheduler_amd/libminisched_hip.so} CAP=15 WEIGHT=1 NORM=0 MODE=sequential PODS=100000 LAUNCHES=3 \
      timeout -s KILL 120 rocprofv3 --pmc ${!set} -d "$OUT/${variant}_$set" -o run --output-format csv -- \
      python3 scripts/run_batch.py > "$OUT/${variant}_$set.log" 2>&1 || { echo "[$variant $set] failed"; exit 1; }
    echo "[$variant $set] ok"
  done
done
