#!/bin/bash
# PMC passes (each its own rocprofv3 run; --pmc never combined with tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "${PMC_SETS[@]:-}"; do :; done
run() {  # $1 = tag, rest = counters
  local tag=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$OUT/$tag" -o run --output-format csv -- python scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?
  echo "[$tag] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run sq2 SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
run fetch FETCH_SIZE
run write WRITE_SIZE
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
echo pmc-done
