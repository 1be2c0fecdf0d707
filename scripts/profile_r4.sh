#!/bin/bash
# Round-4 profile of the hot kernels, run on the GPU box (one GPU step per command, each under its own
# limit; stop at the first failure):
#  1. rocprofv3 --kernel-trace --stats over the headline bench.py command (K = 200) and the driver's K = 20;
#  2. --kernel-trace --stats of each hot kernel alone (scripts/run_batch.py): pair_kernel 32 batches per
#     launch, one batch per launch, MIN-MAX; the opt-in class-row kernel; generic_kernel on the reference
#     list and on NodeNumber + a DEFAULT-normalized score column; seq_kernel (C5);
#  3. one --pmc pass per counter set (never combined with tracing).
# Summary: scripts/pmc_r4_summary.py -> profiles/r4_pmc_c3.json (bench.py reads it for the counter
# fractions and the HBM traffic of its roofline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r4
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
tr() {
  local tag=$1 mode=$2 norm=$3 kern=$4
  MSH_BATCH_KERNEL=$kern NORM=$norm MODE=$mode PODS=100000 LAUNCHES=30 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
    -d "$OUT/$tag" -o run --output-format csv -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
tr stats_multi multi 0 pair || exit 1
tr stats_single batch 0 pair || exit 1
tr stats_kx multi 3 pair || exit 1
tr stats_classrows multi 0 classrows || exit 1
tr stats_classrows_kx multi 3 classrows || exit 1
tr stats_generic generic 0 generic || exit 1
tr stats_generic_col generic_col 0 pair || exit 1
tr stats_seq sequential 0 pair || exit 1
pass() {
  local tag=$1 mode=$2 norm=$3 kern=$4; shift 4
  MSH_BATCH_KERNEL=$kern NORM=$norm MODE=$mode PODS=100000 LAUNCHES=10 timeout -s KILL 90 rocprofv3 --pmc "$@" \
    -d "$OUT/$tag" -o run --output-format csv -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
pass m_sq multi 0 pair $SQ1 || exit 1
pass m_sq2 multi 0 pair $SQ2 || exit 1
pass m_grbm multi 0 pair GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass m_fetch multi 0 pair FETCH_SIZE || exit 1
pass m_write multi 0 pair WRITE_SIZE || exit 1
pass k_sq multi 3 pair $SQ1 || exit 1
pass c_sq multi 0 classrows $SQ1 || exit 1
pass g_sq generic 0 generic $SQ1 || exit 1
pass g_grbm generic 0 generic GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass g_fetch generic 0 generic FETCH_SIZE || exit 1
pass gc_sq generic_col 0 pair $SQ1 || exit 1
pass s_sq sequential 0 pair $SQ1 || exit 1
python3 scripts/pmc_r4_summary.py "$OUT" "$OUT/r4_pmc_c3.json" > /dev/null && echo profile-r4-done
