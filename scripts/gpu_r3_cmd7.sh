#!/bin/bash
# Class-row persistent kernel: the full GPU suite, the K=20 region probe, the bench lines and a
# rocprofv3 --stats of the default command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3q3
timeout -k 10 120 python -u scripts/k20_probe.py 20 > gpurun_out/r3q3/k20_probe.jsonl 2>&1 || { tail gpurun_out/r3q3/k20_probe.jsonl; exit 1; }
cat gpurun_out/r3q3/k20_probe.jsonl
TAG=r3q3 bash scripts/gpu_r3_quick.sh
