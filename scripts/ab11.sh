set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
KERNELS="2 0 1" timeout -k 10 600 bash scripts/r1_variants.sh || exit $?
timeout -k 10 300 python bench.py --mode nodeshard --cpu-seconds 0 --steps 20 --warmup 2 > gpurun_out/bench_c4.json 2>/dev/null || exit $?
python -c "import json;b=json.load(open('gpurun_out/bench_c4.json'));print('c4', b['value'], b['ms_per_step'], b['roofline']['kernel_ms'], b['check'])"
