#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
run() {
  local tag=$1; shift
  PODS=${PODS:-1000000} LAUNCHES=5 timeout -k 10 240 rocprofv3 --pmc "$@" -d "$OUT/$tag" -o run --output-format csv -- python scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run b SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT
run c GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_INSTS_SMEM
run d SQ_INST_CYCLES_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64
echo pmc2-done
