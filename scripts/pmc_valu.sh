#!/bin/bash
# VALU utilisation of the hot kernel at C3 (north_star: "kernel choices justified with rocprof
# counters ... plus VALU utilisation"): one rocprofv3 --pmc pass per counter set (never combined
# with tracing), each under its own hard limit; derived metrics in passes of their own.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_valu
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  PODS=${PODS:-100000} LAUNCHES=20 timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$tag" -o run --output-format csv -- python scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit 1
run b GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run c SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH || exit 1
run d VALUUtilization || echo "VALUUtilization pass failed (derived metric not available?)"
run e VALUBusy || echo "VALUBusy pass failed (derived metric not available?)"
echo pmc-valu-done
