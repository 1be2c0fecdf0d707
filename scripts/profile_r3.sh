#!/bin/bash
# Round-3 profile of the hot kernels, run on the GPU box:
#  1. rocprofv3 --kernel-trace --stats over the headline bench.py command (and the driver's K=20);
#  2. --kernel-trace --stats of single-batch, MIN-MAX, generic and sequential launches (run_batch.py);
#  3. one --pmc pass per counter set (never combined with tracing), each under its own limit.
# Summary: scripts/pmc_r3_summary.py -> profiles/r3_pmc_c3.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_under_rocprof.json" 2> "$OUT/stats.err" || exit 1
echo "[stats] ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_k20" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_k20_under_rocprof.json" 2> "$OUT/stats_k20.err" || exit 1
echo "[stats_k20] ok"
tr() {
  local tag=$1 mode=$2 norm=$3
  NORM=$norm MODE=$mode PODS=100000 LAUNCHES=50 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o run \
    --output-format csv -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
tr stats_single batch 0 || exit 1
tr stats_kx multi 3 || exit 1
tr stats_generic generic 0 || exit 1
tr stats_seq sequential 0 || exit 1
pass() {
  local tag=$1 mode=$2 norm=$3; shift 3
  NORM=$norm MODE=$mode PODS=100000 LAUNCHES=20 timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$tag" -o run --output-format csv \
    -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
LDS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
pass m_sq multi 0 $SQ1 || exit 1
pass m_sq2 multi 0 $SQ2 || exit 1
pass m_lds multi 0 $LDS || exit 1
pass m_grbm multi 0 GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass m_fetch multi 0 FETCH_SIZE || exit 1
pass m_sq3 multi 0 SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA || exit 1
pass m_write multi 0 WRITE_SIZE || exit 1
pass b_sq batch 0 $SQ1 || exit 1
pass b_lds batch 0 $LDS || exit 1
pass b_fetch batch 0 FETCH_SIZE || exit 1
pass b_write batch 0 WRITE_SIZE || exit 1
pass k_sq multi 3 $SQ1 || exit 1
pass g_sq generic 0 $SQ1 || exit 1
pass g_fetch generic 0 FETCH_SIZE || exit 1
pass s_sq sequential 0 $SQ1 || exit 1
pass s_fetch sequential 0 FETCH_SIZE || exit 1
pass s_write sequential 0 WRITE_SIZE || exit 1
python3 scripts/pmc_r3_summary.py "$OUT" "$OUT/r3_pmc_c3.json" > /dev/null && echo profile-r3-done
