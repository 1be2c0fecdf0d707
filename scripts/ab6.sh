set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode nodeshard --cpu-seconds 0 --steps 20 --warmup 2 > gpurun_out/bench_c4.json 2>/dev/null || exit $?
python -c "import json;b=json.load(open('gpurun_out/bench_c4.json'));print('c4', b['value'], b['ms_per_step'], b['roofline']['kernel_ms'], b['check'])"
timeout -k 10 300 python bench.py --nodes 100000 --pods 1000000 --cpu-seconds 0 --steps 20 --warmup 2 > gpurun_out/bench_100k.json 2>/dev/null || exit $?
python -c "import json;b=json.load(open('gpurun_out/bench_100k.json'));print('100k batch', b['value'], b['ms_per_step'], b['roofline']['kernel_ms'], b['roofline']['kernel_ms_isolated'], b['check'])"
timeout -k 10 300 python bench.py --nodes 50000 --pods 1000000 --cpu-seconds 0 --steps 20 --warmup 2 > gpurun_out/bench_50k.json 2>/dev/null || exit $?
python -c "import json;b=json.load(open('gpurun_out/bench_50k.json'));print('50k batch', b['value'], b['ms_per_step'], b['roofline']['kernel_ms'], b['roofline']['kernel_ms_isolated'], b['check'])"
