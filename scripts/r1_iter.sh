#!/bin/bash
# Iteration check: GPU parity tests, batch sweep, bench (each step time-limited; stop on failure).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="${VARIANTS:-2/0}" timeout -k 10 150 python scripts/sweep_batch.py > gpurun_out/sweep_batch.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_batch.log
timeout -k 10 240 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-400
