set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
timeout -k 10 300 python scripts/sweep_seq.py > gpurun_out/sweep_seq.jsonl 2>/dev/null || exit $?
cat gpurun_out/sweep_seq.jsonl
for i in 1 2; do timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/b$i.json 2>/dev/null || exit 1; python -c "import json;b=json.load(open('gpurun_out/b$i.json'));print(b['value']/1e12, b['ms_per_step']*1e3, b['roofline']['kernel_ms_isolated']*1e3)"; done
