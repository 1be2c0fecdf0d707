#!/bin/bash
# Round-3 measurement on the GPU box, in order: the PMC / kernel-trace profile of the hot kernels
# (scripts/profile_r3.sh; its summary becomes profiles/r3_pmc_c3.json, which bench.py reads for
# roofline.traffic and frac_counter), smoke(), the default bench line, the driver's command, and a
# rocprofv3 --stats of the driver's command. Every GPU step under its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r3f}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $1"; }
step profile
bash scripts/profile_r3.sh > "$OUT/profile.log" 2>&1 || { tail -20 "$OUT/profile.log"; exit 1; }
cp gpurun_out/prof_r3/r3_pmc_c3.json profiles/r3_pmc_c3.json
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
step bench
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -30 "$OUT/bench_default.err"; exit 1; }
step driver_cmd
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_cmd.json" 2> "$OUT/bench_driver_cmd.err" || { tail -30 "$OUT/bench_driver_cmd.err"; exit 1; }
step rocprof_driver_cmd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_driver" -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-extras > "$OUT/bench_driver_under_rocprof.json" 2> "$OUT/stats_driver.err" || exit 1
step done
