set -o pipefail
mkdir -p gpurun_out
L=mini-kube-scheduler_amd
timeout -k 10 300 python scripts/ab_libs.py $L/libminisched_hip.so $L/libminisched_hip_lds.so $L/libminisched_hip_diag_noload.so > gpurun_out/ab1.jsonl 2> gpurun_out/ab1.err || exit $?
cat gpurun_out/ab1.jsonl
MSH_DYN_LDS=1 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/pytest_lds.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_lds.log; exit $rc
