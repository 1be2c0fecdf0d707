set -o pipefail
mkdir -p gpurun_out
L=mini-kube-scheduler_amd
for WG in 2 1; do
  MSH_BATCH_WG_PER_CU=$WG timeout -k 10 300 python scripts/ab_libs.py $L/libminisched_hip.so $L/libminisched_hip_u16.so > gpurun_out/ab10_wg$WG.jsonl 2>/dev/null || exit $?
  echo "wg $WG"; cat gpurun_out/ab10_wg$WG.jsonl
  MSH_BATCH_WG_PER_CU=$WG PODS=400000 ROUNDS=6 timeout -k 10 300 python scripts/ab_libs.py $L/libminisched_hip.so $L/libminisched_hip_u16.so > gpurun_out/ab10b_wg$WG.jsonl 2>/dev/null || exit $?
  cat gpurun_out/ab10b_wg$WG.jsonl
done
MSH_LIBRARY=$PWD/$L/libminisched_hip_u16.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/pytest_u16.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_u16.log; exit $rc
