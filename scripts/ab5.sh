set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/host_overhead.py > gpurun_out/host_overhead.jsonl 2>/dev/null || exit $?
cat gpurun_out/host_overhead.jsonl
for S in 1 2 3 4; do
  timeout -k 10 200 python bench.py --streams $S --cpu-seconds 0 --steps 400 > gpurun_out/bench_s$S.json 2>/dev/null || exit $?
  python -c "import json;b=json.load(open('gpurun_out/bench_s$S.json'));print($S, b['value'], b['ms_per_step']*1e3, b['roofline']['kernel_ms']*1e3, b['roofline']['kernel_ms_isolated']*1e3)"
done
