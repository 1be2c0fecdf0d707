#!/bin/bash
# Build the wave-timeline A/B library (msh_kernels.hip with -DMSH_STAMPS) and its driver into
# scripts/ (never the product library), on the CPU; run scripts/stamps_run [pods] on the GPU box.
set -e
cd "$(dirname "$0")/.."
C=mini-kube-scheduler_amd/csrc
O=$(mktemp -d)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DMSH_STAMPS -x hip -c $C/msh_kernels.hip -o $O/k.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $C/msh_capi.cpp -o $O/c.o
g++ -O2 -std=c++17 -fPIC -pthread -c $C/msh_pack.cpp -o $O/p.o
hipcc --offload-arch=gfx950 -shared -fPIC $O/k.o $O/c.o $O/p.o -o scripts/libminisched_stamps.so
hipcc --offload-arch=gfx950 -O2 -Iinclude scripts/stamps_run.hip -Lscripts -lminisched_stamps \
  -Wl,-rpath,'$ORIGIN' -o scripts/stamps_run
rm -rf "$O"
