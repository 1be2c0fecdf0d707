set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/split.jsonl
for P in 4096 32768; do for SP in 1 2 4 8 16; do
  MSH_SPLIT=$SP NODES=100000 PODS=$P ROUNDS=6 timeout -k 10 120 python scripts/ab_libs.py mini-kube-scheduler_amd/libminisched_hip.so > gpurun_out/s.json 2>/dev/null || exit $?
  python -c "
import json
r=json.loads(open('gpurun_out/s.json').read()); print($P, $SP, round(r['iso_us'],1), round(r['pipe_us'],1))"
done; done
