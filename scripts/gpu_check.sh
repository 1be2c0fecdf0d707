#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the script stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
ok_or_stop() {  # $1 = rc, $2 = step name; test failures (rc 1) are not crashes
  local rc=$1
  echo "[$2] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $2 (rc=$rc)"; exit "$rc"; fi
}
timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
ok_or_stop $? pytest_gpu
tail -5 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok_or_stop $? smoke
tail -2 "$OUT/smoke.log"
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
ok_or_stop $? bench
tail -1 "$OUT/bench.log"
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --cpu-seconds 0 --no-check ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1
  ok_or_stop $? rocprof
  find "$OUT/prof" -name '*kernel_stats.csv' | head -3
fi
echo done
