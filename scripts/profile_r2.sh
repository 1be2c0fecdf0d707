#!/bin/bash
# Round-2 profile of the hot kernels (rows_kernel at C3, also with MIN-MAX, seq_kernel at C5),
# run on the GPU box:
#  1. the scan-mix issue-rate microbenchmark (the VALU ceiling bench.py quotes);
#  2. rocprofv3 --kernel-trace --stats over the headline bench.py command;
#  3. one --pmc pass per counter set (never combined with tracing), each under its own limit.
# Summaries: scripts/pmc_r2_summary.py -> profiles/r2_pmc_c3.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench_bitop3 > "$OUT/ubench_bitop3.jsonl" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_under_rocprof.json" 2> "$OUT/stats.err" || exit 1
echo "[stats] ok"
NORM=3 MODE=batch PODS=100000 LAUNCHES=50 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/stats_kx" -o run \
  --output-format csv -- python3 scripts/run_batch.py > "$OUT/stats_kx.log" 2>&1 || exit 1
echo "[stats_kx] ok"
pass() {
  local tag=$1 mode=$2; shift 2
  local norm=0; [ "$mode" = batch_kx ] && { norm=3; mode=batch; }
  NORM=$norm MODE=$mode PODS=100000 LAUNCHES=20 timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$tag" -o run --output-format csv \
    -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
pass b_sq batch SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit 1
pass b_sq2 batch SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS || exit 1
pass b_lds batch SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
pass b_grbm batch GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass b_fetch batch FETCH_SIZE || exit 1
pass b_write batch WRITE_SIZE || exit 1
pass k_sq batch_kx SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit 1
pass s_sq sequential SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit 1
pass s_fetch sequential FETCH_SIZE || exit 1
pass s_write sequential WRITE_SIZE || exit 1
python3 scripts/pmc_r2_summary.py "$OUT" "$OUT/r2_pmc_c3.json" > /dev/null && echo profile-r2-done
