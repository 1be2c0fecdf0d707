#!/bin/bash
# Round-1 GPU validation: parity tests, seq/batch sweeps, bench. Each GPU step has its own limit;
# the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python scripts/sweep_seq.py > gpurun_out/sweep_seq.log 2>&1 || exit $?
VARIANTS="2/0,2/2,0/0" timeout -k 10 150 python scripts/sweep_batch.py > gpurun_out/sweep_batch.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
