#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats of the bench command itself (default =
# 2 streams, and --streams 1 for the isolated per-launch time), then one --pmc pass per HBM
# counter (FETCH_SIZE, WRITE_SIZE; never combined with tracing domains), plus the VALU issue-rate
# microbenchmarks. Every GPU step has its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_r1
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps ${STEPS:-50} --warmup ${WARMUP:-5} --cpu-seconds ${CPU_S:-0}"
step() {  # $1 = tag, $2.. = rocprofv3 options (before --)
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$tag" -o run --output-format csv -- python $BENCH ${MODE_ARGS:-} > "$OUT/$tag.log" 2>&1
  local rc=$?
  echo "[$tag] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 "$OUT/$tag.log" | cut -c1-200
}
# FETCH_SIZE calibration for 1 / 4 / 16 B-per-lane streaming reads (known byte counts)
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/calib" -o run --output-format csv -- ./scripts/calib_fetch > "$OUT/calib.log" 2>&1
rc=$?; echo "[calib] rc=$rc"; [ $rc -eq 0 ] || exit $rc
step stats --kernel-trace --stats
MODE_ARGS="--streams 1" step stats_1stream --kernel-trace --stats
MODE_ARGS="--streams 1" step fetch --pmc FETCH_SIZE
MODE_ARGS="--streams 1" step write --pmc WRITE_SIZE
MODE_ARGS="--mode sequential" step seq_stats --kernel-trace --stats
MODE_ARGS="--mode sequential" step seq_fetch --pmc FETCH_SIZE
MODE_ARGS="--mode sequential" step seq_write --pmc WRITE_SIZE
if [ "${UBENCH:-1}" = 1 ]; then
  timeout -k 10 200 ./scripts/ubench_valu2 > "$OUT/ubench_valu2.jsonl" || exit $?
  timeout -k 10 200 ./scripts/ubench_valu3 > "$OUT/ubench_valu3.jsonl" || exit $?
fi
echo profile-done
