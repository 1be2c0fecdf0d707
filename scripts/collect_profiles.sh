#!/bin/bash
# Copy the summaries of the last gpu_check.sh + profile_r1.sh call (gpurun_out/, scratch) into
# profiles/ (tracked): rocprofv3 kernel stats, PMC counter passes, bench lines, GPU test log.
set -eu
cd "$(dirname "$0")/.."
P=gpurun_out/prof_r1
python scripts/pmc_summary.py $P profiles/pmc_latest.json > /dev/null
cp $P/stats/run_kernel_stats.csv profiles/r1_kernel_stats_bench_batch.csv
cp $P/stats_1stream/run_kernel_stats.csv profiles/r1_kernel_stats_bench_batch_1stream.csv
cp $P/seq_stats/run_kernel_stats.csv profiles/r1_kernel_stats_bench_sequential.csv
cp $P/fetch/run_counter_collection.csv profiles/r1_pmc_fetch.csv
cp $P/write/run_counter_collection.csv profiles/r1_pmc_write.csv
cp $P/seq_fetch/run_counter_collection.csv profiles/r1_pmc_seq_fetch.csv
cp $P/seq_write/run_counter_collection.csv profiles/r1_pmc_seq_write.csv
cp $P/calib/run_counter_collection.csv profiles/r1_pmc_calib_fetch.csv
for t in stats:batch stats_1stream:batch_1stream seq_stats:sequential; do
  grep '^{"metric"' $P/${t%%:*}.log > profiles/r1_bench_${t##*:}_under_rocprof.json
done
grep '^{"metric"' gpurun_out/bench.log > profiles/r1_bench.json
cp gpurun_out/pytest_gpu.log profiles/r1_pytest_gpu.log
head -2 profiles/r1_kernel_stats_bench_batch_1stream.csv | tail -1
python - <<'PY'
import json
b = json.load(open("profiles/r1_bench.json")); r = b["roofline"]
print(f"value {b['value']:.4g} ms/step {b['ms_per_step']*1e3:.2f}us iso {r['kernel_ms_isolated']*1e3:.2f}us "
      f"frac {r['frac']:.3f} frac_iso {r['frac_isolated']:.3f} vs_ceiling {r['frac_vs_measured_int_ceiling']:.3f} traffic {r['traffic']}")
PY
