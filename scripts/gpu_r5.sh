#!/bin/bash
# Round-5 GPU session driver: run the named steps in order, each GPU step under its own time limit,
# stopping at the first failure. Usage: TAG=x bash scripts/gpu_r5.sh step [step ...]
#   new      the tests named in $TESTS (pytest node ids / -k expression in $K)
#   parity   pytest -m gpu tests/test_gpu_parity.py
#   gpu      pytest -m gpu tests/ (the whole GPU suite)
#   bench    python bench.py (default line: K = 200)
#   quick    python bench.py --no-extras --cpu-seconds 0
#   driver   python bench.py --gpus 1 --steps 20 --warmup 5
#   stats    rocprofv3 --kernel-trace --stats over bench.py --no-extras --cpu-seconds 0
#   smoke    __graft_entry__.smoke()
#   profile  scripts/profile_r5.sh (rocprofv3 kernel stats + PMC passes -> gpurun_out/prof_r5/r5_pmc_c3.json)
#   ab       rocprofv3 --kernel-trace --stats of 32-batch C3 launches (scripts/run_batch.py) for each
#            "ENV=VAL[,ENV=VAL]:weight:norm:mode" arm in $ARMS; prints the hot kernel's average duration
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $1"; }
for s in "$@"; do
  step "$s"
  case "$s" in
    new)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v ${K:+-k "$K"} --timeout 300 --timeout-method thread \
        > "$OUT/new.log" 2>&1 || { tail -60 "$OUT/new.log"; exit 1; }
      grep -E "PASSED|FAILED|SKIPPED|passed|failed" "$OUT/new.log" | tail -40 ;;
    parity)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/parity.log" 2>&1 || { tail -40 "$OUT/parity.log"; exit 1; }
      tail -2 "$OUT/parity.log" ;;
    gpu)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=40 --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -2 "$OUT/pytest_gpu.log" ;;
    bench)
      timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
      cut -c1-600 "$OUT/bench.json" ;;
    quick)
      timeout -k 10 300 python -u bench.py --no-extras --cpu-seconds 0 > "$OUT/quick.json" 2> "$OUT/quick.err" \
        || { tail -30 "$OUT/quick.err"; exit 1; }
      cut -c1-600 "$OUT/quick.json" ;;
    driver)
      timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver.json" 2> "$OUT/driver.err" \
        || { tail -30 "$OUT/driver.err"; exit 1; }
      cut -c1-400 "$OUT/driver.json" ;;
    stats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
        python3 bench.py --no-extras --cpu-seconds 0 > "$OUT/stats_bench.json" 2> "$OUT/stats.err" || { tail -30 "$OUT/stats.err"; exit 1; }
      find "$OUT/stats" -name "*kernel_stats.csv" -exec head -12 {} \; ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { tail -30 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log" ;;
    ab)
      for arm in ${ARMS:-MSH_PAIR_PIPE=0:3:1:multi MSH_PAIR_PIPE=1:3:1:multi}; do
        IFS=: read -r envs w nm md <<< "$arm"
        tag=$(echo "$arm" | tr ':,=' '___')
        ( export $(echo "$envs" | tr ',' ' '); WEIGHT=$w NORM=$nm MODE=$md PODS=100000 LAUNCHES=${LAUNCHES:-40} \
          timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/ab/$tag" -o run --output-format csv -- \
          python3 scripts/run_batch.py > "$OUT/ab_$tag.log" 2>&1 ) || { tail -20 "$OUT/ab_$tag.log"; exit 1; }
        f=$(find "$OUT/ab/$tag" -name "*kernel_stats.csv" | head -1)
        echo "$arm $(grep -E 'pair|generic|seq_kernel' "$f" | head -1 | cut -d, -f1-5)"
      done ;;
    profile)
      timeout -k 10 1100 bash scripts/profile_r5.sh > "$OUT/profile.log" 2>&1 || { tail -30 "$OUT/profile.log"; exit 1; }
      tail -3 "$OUT/profile.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
step done
