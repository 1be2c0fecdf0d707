#!/bin/bash
# bench.py headline (C3) under each launch mode and stream count, at the driver's K=20 and at K=200.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# STEPS / LAUNCHES / STREAMS: space-separated lists (defaults below)
for steps in ${STEPS:-20 200}; do
  for launch in ${LAUNCHES:-eager graph}; do
    for streams in ${STREAMS:-1 2 3}; do
      timeout -k 10 120 python3 bench.py --steps $steps --warmup 5 --cpu-seconds 0 --no-extras --launch $launch \
        --streams $streams > gpurun_out/sweep.tmp 2>/dev/null || { echo "bench failed: $launch $streams $steps"; exit 1; }
      python3 -c "
import json; d = json.load(open('gpurun_out/sweep.tmp'))
print(json.dumps({'steps': $steps, 'launch': '$launch', 'streams': $streams, 'ms_per_step': d['ms_per_step'],
                  'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'kernel_ms_isolated': d['roofline']['kernel_ms_isolated'],
                  'check': d['check']}))"
    done
  done
done
