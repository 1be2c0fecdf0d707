#!/bin/bash
# Build A/B variants of the kernel library (CPU, here) into scripts/expt/ (git-ignored; never the
# product library): one libab_<name>.so per "name=flags" argument, the product sources compiled with
# those -D flags; plus the timing driver scripts/expt/run (scripts/wg_expt_run.cpp).
#   scripts/ab_build.sh base= quad=-DMSH_WGP_QUAD=1 pipe=-DMSH_WGP_PIPE=1
# A SRC_<name>=<file> environment variable compiles <file> instead of msh_kernels.hip for that variant
# (e.g. an older revision from git show, for a before / after comparison). A name containing
# "notrack" links the C-ABI built with -DMSH_AB_NO_TRACK (no reader events after launches).
# On the GPU box: scripts/expt/run scripts/expt/libab_<name>.so <name> [batches per launch].
set -e
cd "$(dirname "$0")/.."
C=mini-kube-scheduler_amd/csrc
E=scripts/expt
mkdir -p $E
O=$(mktemp -d)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $C/msh_capi.cpp -o $O/c.o &
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DMSH_AB_NO_TRACK -c $C/msh_capi.cpp -o $O/c_notrack.o &
g++ -O2 -std=c++17 -fPIC -pthread -c $C/msh_pack.cpp -o $O/p.o &
for a in "$@"; do
  name=${a%%=*}
  flags=${a#*=}
  src_var=SRC_$name
  src=${!src_var:-$C/msh_kernels.hip}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$C $flags -x hip -c "$src" -o $O/k_$name.o &
done
wait
for a in "$@"; do
  name=${a%%=*}
  capi=$O/c.o
  case "$name" in *notrack*) capi=$O/c_notrack.o ;; esac
  hipcc --offload-arch=gfx950 -shared -fPIC $O/k_$name.o $capi $O/p.o -o $E/libab_$name.so
done
hipcc -O2 -std=c++17 -Iinclude scripts/wg_expt_run.cpp -ldl -o $E/run
rm -rf "$O"
ls -la $E
