#!/bin/bash
# Build the wg_kernel phase-experiment libraries (CPU, here) into scripts/expt/ (git-ignored; never the
# product library): the product source with -DMSH_STAMPS and MSH_WG_EXPT = 0 (stamps only), 1 (no scan),
# 2 (no output stores), 4 (no table copy), 7 (none of the three); plus the driver scripts/expt/run.
# On the GPU box: for each lib, scripts/expt/run <lib> <tag> [batches per launch].
set -e
cd "$(dirname "$0")/.."
C=mini-kube-scheduler_amd/csrc
E=scripts/expt
mkdir -p $E
O=$(mktemp -d)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $C/msh_capi.cpp -o $O/c.o
g++ -O2 -std=c++17 -fPIC -pthread -c $C/msh_pack.cpp -o $O/p.o
for x in ${EXPTS:-0 1 2 4 7}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DMSH_STAMPS -DMSH_WG_EXPT=$x -x hip -c $C/msh_kernels.hip -o $O/k$x.o &
done
wait
for x in ${EXPTS:-0 1 2 4 7}; do
  hipcc --offload-arch=gfx950 -shared -fPIC $O/k$x.o $O/c.o $O/p.o -o $E/libexpt$x.so
done
hipcc -O2 -std=c++17 -Iinclude scripts/wg_expt_run.cpp -ldl -o $E/run
rm -rf "$O"
