#!/bin/bash
# The driver's K = 20 region as the driver takes it: one timed region per fresh process, N processes;
# one line per run: us per step (wall clock of the region) and the device span per step of an
# untimed repeat. (A/B kept out: hipDeviceScheduleSpin on torch's runtime, no better than the default.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-k20os}
mkdir -p "$OUT"
for i in $(seq 1 "${N:-4}"); do
  timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/run.$i.json" 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/run.$i.json')); print(round(d['ms_per_step']*1e3,3), round(d['roofline']['region_device_ms_per_step']*1e3,3))"
done
