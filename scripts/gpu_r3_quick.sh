#!/bin/bash
# Quick GPU iteration: the GPU suite (optionally a -k filter), the default bench line, the driver's
# command and a rocprofv3 --stats of the default command. Every GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r3q}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[$(date +%T)] pytest"
K=(); [ -n "${PYTEST_K:-}" ] && K=(-k "$PYTEST_K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
echo "[$(date +%T)] bench"
timeout -k 10 300 python -u bench.py --cpu-seconds 0 ${BENCH_EXTRA:-} > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -30 "$OUT/bench_default.err"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_k20.json" 2> "$OUT/bench_k20.err" || { tail -30 "$OUT/bench_k20.err"; exit 1; }
echo "[$(date +%T)] rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_under_rocprof.json" 2> "$OUT/stats.err" || exit 1
echo "[$(date +%T)] done"
