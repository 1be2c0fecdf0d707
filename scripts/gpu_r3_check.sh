#!/bin/bash
# Round-3 GPU check on the box: the GPU suite, smoke(), the default bench line and the VALU issue-rate
# microbenchmark. Every GPU step under its own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $1"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_EXTRA:-} \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
step ubench
timeout -k 10 120 ./scripts/ubench_valu_peak > "$OUT/ubench_valu_peak.jsonl" 2>&1 || { tail "$OUT/ubench_valu_peak.jsonl"; exit 1; }
tail -1 "$OUT/ubench_valu_peak.jsonl"
step bench
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -30 "$OUT/bench_default.err"; exit 1; }
step driver_cmd
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_driver_cmd.json" 2> "$OUT/bench_driver_cmd.err" || { tail -30 "$OUT/bench_driver_cmd.err"; exit 1; }
step done
