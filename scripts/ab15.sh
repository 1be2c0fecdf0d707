set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
: > gpurun_out/small2.jsonl
for N in 5000 100000; do for P in 64 512 4096 32768 100000; do
  NODES=$N PODS=$P ROUNDS=6 timeout -k 10 120 python scripts/ab_libs.py mini-kube-scheduler_amd/libminisched_hip.so >> gpurun_out/small2.jsonl 2>/dev/null || exit $?
done; done
python -c "
import json
for l in open('gpurun_out/small2.jsonl'):
    r=json.loads(l); print(r['nodes'], r['pods'], round(r['iso_us'],1), round(r['pipe_us'],1))"
