#!/bin/bash
# SQ stall anatomy of the batch kernel (one rocprofv3 --pmc pass per counter set).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_sq
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  LAUNCHES=10 timeout -k 10 180 rocprofv3 --pmc "$@" -d "$OUT/$tag" -o run --output-format csv -- python scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run b SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT
run c GRBM_GUI_ACTIVE GRBM_COUNT
echo pmc-sq-done
