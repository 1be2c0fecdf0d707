set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/small.jsonl
for N in 5000 100000; do for P in 64 512 4096 32768; do
  NODES=$N PODS=$P ROUNDS=6 timeout -k 10 120 python scripts/ab_libs.py mini-kube-scheduler_amd/libminisched_hip.so >> gpurun_out/small.jsonl 2>/dev/null || exit $?
done; done
cat gpurun_out/small.jsonl
