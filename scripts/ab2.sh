set -o pipefail
mkdir -p gpurun_out
L=mini-kube-scheduler_amd
timeout -k 10 300 python scripts/ab_libs.py $L/libminisched_hip_head.so $L/libminisched_hip.so $L/libminisched_hip_pf.so > gpurun_out/ab2.jsonl 2> gpurun_out/ab2.err || exit $?
cat gpurun_out/ab2.jsonl
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/pytest_def.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_def.log
MSH_LIBRARY=$PWD/$L/libminisched_hip_pf.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/pytest_pf.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_pf.log; exit $rc
