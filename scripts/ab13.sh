set -o pipefail
mkdir -p gpurun_out
for G in 512 256 128; do for S in 2 3 4; do
  MSH_BATCH_GRID=$G timeout -k 10 200 python bench.py --streams $S --cpu-seconds 0 --steps 400 > gpurun_out/b.json 2>/dev/null || exit $?
  python -c "import json;b=json.load(open('gpurun_out/b.json'));print('grid',$G,'streams',$S, round(b['value']/1e12,2), round(b['ms_per_step']*1e3,2), round(b['roofline']['kernel_ms_isolated']*1e3,2), b['check'])"
done; done
