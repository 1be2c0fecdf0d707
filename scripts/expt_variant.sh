#!/bin/bash
# Build an A/B variant of the library: the package copied to a scratch tree, a sed expression applied to
# one source file, built there, and the two shared objects copied to scripts/expt/<name>/ (loaded through
# MSH_LIBRARY by scripts/run_batch.py). Usage: scripts/expt_variant.sh <name> <csrc file> <sed expr>
set -eu
cd "$(dirname "$0")/.."
name=$1 file=$2 expr=$3
tmp=$(mktemp -d)
mkdir -p "$tmp/repo"
cp -r mini-kube-scheduler_amd include "$tmp/repo/"
rm -rf "$tmp/repo/mini-kube-scheduler_amd/build" "$tmp"/repo/mini-kube-scheduler_amd/*.so
sed -i "$expr" "$tmp/repo/mini-kube-scheduler_amd/csrc/$file"
(cd "$tmp/repo" && python3 -c "import importlib,sys; sys.path.insert(0,'.'); importlib.import_module('mini-kube-scheduler_amd.build').build(force=True)" > "$tmp/build.log" 2>&1) || { tail -20 "$tmp/build.log"; exit 1; }
mkdir -p "scripts/expt/$name"
cp "$tmp"/repo/mini-kube-scheduler_amd/libminisched_hip.so "$tmp"/repo/mini-kube-scheduler_amd/_msh_fast*.so "scripts/expt/$name/"
rm -rf "$tmp"
echo "built scripts/expt/$name"
