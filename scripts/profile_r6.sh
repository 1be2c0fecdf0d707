#!/bin/bash
# Round-6 profile of the hot kernels on the GPU box (each GPU step under its own limit; stop at the first
# failure). Sections (PARTS, default "stats trace pmc"):
#  stats  rocprofv3 --kernel-trace --stats over bench.py (K = 200, the headline line) and the driver's K = 20;
#  trace  --kernel-trace --stats of each hot kernel alone (scripts/run_batch.py, C3: 5,000 nodes x 100,000
#         pods per batch): the per-pair kernel, 32 batches per launch, with the headline plugins (NodeNumber
#         w=3 DefaultNormalizeScore), the reference's w=1 list, MIN-MAX and REVERSE at w=3; generic_kernel on
#         the reference list, the headline list and NodeNumber + a DEFAULT column; C5: the auto
#         no-capacity form (pair_kernel with the commit epilogue), seq_kernel's pod blocks, one workgroup
#         (serial), and the capacity form (15 pods per node);
#  pmc    one --pmc pass per counter set (never combined with tracing).
# Summary: scripts/pmc_r6_summary.py -> $OUT/r6_pmc_c3.json (copied to profiles/; bench.py reads it for
# the counter fractions and the HBM traffic of its rooflines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/prof_r6}
PARTS=${PARTS:-"stats trace pmc"}
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { case " $PARTS " in *" $1 "*) return 0 ;; esac; return 1; }
if has stats; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
    python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_under_rocprof.json" 2> "$OUT/stats.err" || exit 1
  echo "[stats] ok"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_k20" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_k20_under_rocprof.json" 2> "$OUT/stats_k20.err" || exit 1
  echo "[stats_k20] ok"
fi
# tag mode weight norm  (environment: SPLIT, CAP, LAUNCHES)
tr() {
  local tag=$1 mode=$2 w=$3 norm=$4
  SPLIT=${SPLIT:-auto} CAP=${CAP:-0} WEIGHT=$w NORM=$norm MODE=$mode PODS=100000 LAUNCHES=${LAUNCHES:-30} \
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o run --output-format csv -- \
    python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
if has trace; then
  tr stats_multi multi 3 1 || exit 1
  tr stats_ref multi 1 0 || exit 1
  tr stats_kx multi 3 3 || exit 1
  tr stats_rev multi 3 2 || exit 1
  tr stats_generic generic 1 0 || exit 1
  tr stats_generic_hl generic 3 1 || exit 1
  tr stats_generic_col generic_col 1 0 || exit 1
  tr stats_single batch 3 1 || exit 1
  tr stats_seq_pair sequential 3 1 || exit 1
  SPLIT=blocks tr stats_seq sequential 3 1 || exit 1
  SPLIT=serial tr stats_seq_serial sequential 3 1 || exit 1
  CAP=15 LAUNCHES=5 tr stats_seq_cap sequential 1 0 || exit 1
fi
pass() {
  local tag=$1 mode=$2 w=$3 norm=$4; shift 4
  SPLIT=${SPLIT:-auto} CAP=${CAP:-0} WEIGHT=$w NORM=$norm MODE=$mode PODS=100000 LAUNCHES=${LAUNCHES:-10} \
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$tag" -o run --output-format csv -- \
    python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "[$tag] rc=$rc"; return $rc
}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
if has pmc; then
  pass m_sq multi 3 1 $SQ1 || exit 1
  pass m_fetch multi 3 1 FETCH_SIZE || exit 1
  pass m_write multi 3 1 WRITE_SIZE || exit 1
  pass r_sq multi 1 0 $SQ1 || exit 1
  pass k_sq multi 3 3 $SQ1 || exit 1
  pass v_sq multi 3 2 $SQ1 || exit 1
  pass g_sq generic 1 0 $SQ1 || exit 1
  pass gh_sq generic 3 1 $SQ1 || exit 1
  pass gc_sq generic_col 1 0 $SQ1 || exit 1
  pass gc_sq2 generic_col 1 0 $SQ2 || exit 1
  pass sp_sq sequential 3 1 $SQ1 || exit 1
  pass sp_sq2 sequential 3 1 $SQ2 || exit 1
  SPLIT=blocks pass s_sq sequential 3 1 $SQ1 || exit 1
  SPLIT=blocks pass s_sq2 sequential 3 1 $SQ2 || exit 1
  SPLIT=serial pass ss_sq sequential 3 1 $SQ1 || exit 1
  CAP=15 LAUNCHES=3 pass c_sq sequential 1 0 $SQ1 || exit 1
  CAP=15 LAUNCHES=3 pass c_sq2 sequential 1 0 $SQ2 || exit 1
  CAP=15 LAUNCHES=3 pass c_fetch sequential 1 0 FETCH_SIZE || exit 1
fi
if has pmc; then
  python3 scripts/pmc_r6_summary.py "$OUT" "$OUT/r6_pmc_c3.json" > /dev/null && echo profile-r6-done
fi
