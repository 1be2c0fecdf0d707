#!/bin/bash
# Parity of every batch-kernel variant (MSH_BATCH_KERNEL 3 = work queue, 2 = static direct,
# 0 = LDS-staged, 1 = compare/select) on the GPU test subset that exercises the batch path.
set -o pipefail
mkdir -p gpurun_out
for k in ${KERNELS:-3 2 0 1}; do
  MSH_BATCH_KERNEL=$k timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/pytest_k$k.log 2>&1
  rc=$?; echo "[kernel $k] rc=$rc $(tail -1 gpurun_out/pytest_k$k.log)"; [ $rc -eq 0 ] || exit $rc
done
