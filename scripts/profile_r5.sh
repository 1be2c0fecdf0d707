#!/bin/bash
# Round-5 profile of the hot kernels on the GPU box (each GPU step under its own limit; stop at the first
# failure):
#  1. rocprofv3 --kernel-trace --stats over bench.py (K = 200, the headline line) and the driver's K = 20;
#  2. --kernel-trace --stats of each hot kernel alone (scripts/run_batch.py, C3: 5,000 nodes x 100,000
#     pods per batch): the per-pair kernel 32 batches per launch with the headline plugins (NodeNumber w=3
#     DefaultNormalizeScore), the reference's w=1 list, MIN-MAX and REVERSE at w=3; generic_kernel on the
#     reference list, on the headline list and on NodeNumber + a DEFAULT-normalized column; seq_kernel (C5,
#     headline plugins: pod blocks over workgroups, and MSH_SEQ_SPLIT=serial);
#  3. one --pmc pass per counter set (never combined with tracing).
# Summary: scripts/pmc_r5_summary.py -> profiles/r5_pmc_c3.json (bench.py reads it for the counter
# fractions and the HBM traffic of its roofline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r5
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${SKIP_BENCH_STATS:-0}" != 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
    python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_under_rocprof.json" 2> "$OUT/stats.err" || exit 1
  echo "[stats] ok"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_k20" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_k20_under_rocprof.json" 2> "$OUT/stats_k20.err" || exit 1
  echo "[stats_k20] ok"
fi
# tag mode weight norm kernel
tr() {
  local tag=$1 mode=$2 w=$3 norm=$4 kern=$5
  MSH_SEQ_SPLIT=${SPLIT:-auto} MSH_BATCH_KERNEL=$kern WEIGHT=$w NORM=$norm MODE=$mode PODS=100000 LAUNCHES=30 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
    -d "$OUT/$tag" -o run --output-format csv -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
if [ "${SKIP_TRACE:-0}" != 1 ]; then
  tr stats_multi multi 3 1 pair || exit 1
  tr stats_ref multi 1 0 pair || exit 1
  tr stats_kx multi 3 3 pair || exit 1
  tr stats_rev multi 3 2 pair || exit 1
  tr stats_single batch 3 1 pair || exit 1
  tr stats_generic generic 1 0 generic || exit 1
  tr stats_generic_hl generic 3 1 generic || exit 1
  tr stats_generic_col generic_col 1 0 pair || exit 1
  tr stats_seq sequential 3 1 pair || exit 1
  SPLIT=serial tr stats_seq_serial sequential 3 1 pair || exit 1
fi
pass() {
  local tag=$1 mode=$2 w=$3 norm=$4 kern=$5; shift 5
  MSH_SEQ_SPLIT=${SPLIT:-auto} MSH_BATCH_KERNEL=$kern WEIGHT=$w NORM=$norm MODE=$mode PODS=100000 LAUNCHES=10 timeout -s KILL 90 rocprofv3 --pmc "$@" \
    -d "$OUT/$tag" -o run --output-format csv -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
pass m_sq multi 3 1 pair $SQ1 || exit 1
pass m_sq2 multi 3 1 pair $SQ2 || exit 1
pass m_grbm multi 3 1 pair GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass m_fetch multi 3 1 pair FETCH_SIZE || exit 1
pass m_write multi 3 1 pair WRITE_SIZE || exit 1
pass r_sq multi 1 0 pair $SQ1 || exit 1
pass r_fetch multi 1 0 pair FETCH_SIZE || exit 1
pass r_write multi 1 0 pair WRITE_SIZE || exit 1
pass k_sq multi 3 3 pair $SQ1 || exit 1
pass k_fetch multi 3 3 pair FETCH_SIZE || exit 1
pass k_write multi 3 3 pair WRITE_SIZE || exit 1
pass v_sq multi 3 2 pair $SQ1 || exit 1
pass v_fetch multi 3 2 pair FETCH_SIZE || exit 1
pass v_write multi 3 2 pair WRITE_SIZE || exit 1
pass g_sq generic 1 0 generic $SQ1 || exit 1
pass g_sq2 generic 1 0 generic $SQ2 || exit 1
pass g_grbm generic 1 0 generic GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass g_fetch generic 1 0 generic FETCH_SIZE || exit 1
pass g_write generic 1 0 generic WRITE_SIZE || exit 1
pass gh_sq generic 3 1 generic $SQ1 || exit 1
pass gc_sq generic_col 1 0 pair $SQ1 || exit 1
pass gc_sq2 generic_col 1 0 pair $SQ2 || exit 1
pass s_sq sequential 3 1 pair $SQ1 || exit 1
pass s_grbm sequential 3 1 pair GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
SPLIT=serial pass ss_sq sequential 3 1 pair $SQ1 || exit 1
python3 scripts/pmc_r5_summary.py "$OUT" "$OUT/r5_pmc_c3.json" > /dev/null && echo profile-r5-done
