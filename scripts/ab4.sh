set -o pipefail
mkdir -p gpurun_out
L=mini-kube-scheduler_amd
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_all.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_all.log
timeout -k 10 300 python scripts/ab_libs.py $L/libminisched_hip_head.so $L/libminisched_hip_ulist.so $L/libminisched_hip.so > gpurun_out/ab4.jsonl 2> gpurun_out/ab4.err || exit $?
cat gpurun_out/ab4.jsonl
PODS=400000 ROUNDS=8 timeout -k 10 300 python scripts/ab_libs.py $L/libminisched_hip_head.so $L/libminisched_hip_ulist.so $L/libminisched_hip.so > gpurun_out/ab4b.jsonl 2>> gpurun_out/ab4.err || exit $?
cat gpurun_out/ab4b.jsonl
