#!/bin/bash
# Round-4 A/B of the hot kernels' launch time (rocprofv3 --kernel-trace --stats over scripts/run_batch.py,
# C3, 30 launches each): <tag> <MODE> <NORM> <env...>; prints "tag avg_ns kernel" per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_r4
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1 mode=$2 norm=$3; shift 3
  env "$@" MODE=$mode NORM=$norm PODS=100000 LAUNCHES=30 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
    -d "$OUT/$tag" -o run --output-format csv -- python3 scripts/run_batch.py > "$OUT/$tag.log" 2>&1 || return 1
  python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, sys, pathlib
for f in pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "msh::" in r["Name"] and ("pair" in r["Name"] or "generic_kernel" in r["Name"] or "wgp" in r["Name"]):
            print(sys.argv[2], r["AverageNs"], r["Calls"], r["Name"].split("(")[0], flush=True)
PY
}
for spec in "$@"; do
  # spec: tag:mode:norm:VAR=val,VAR=val
  IFS=: read -r tag mode norm envs <<< "$spec"
  run "$tag" "$mode" "$norm" ${envs//,/ } || { echo "[$tag] failed"; exit 1; }
done
echo ab-done
