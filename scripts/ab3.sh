set -o pipefail
mkdir -p gpurun_out
L=mini-kube-scheduler_amd
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_all.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_all.log
KERNELS="2 0" timeout -k 10 400 bash scripts/r1_variants.sh || exit $?
: > gpurun_out/podsweep.jsonl
for P in 25000 50000 100000 200000 400000 800000; do
  PODS=$P ROUNDS=8 timeout -k 10 120 python scripts/ab_libs.py $L/libminisched_hip.so >> gpurun_out/podsweep.jsonl 2>/dev/null || exit $?
done
cat gpurun_out/podsweep.jsonl
