#!/bin/bash
# The single-batch launch at C3 (5,000 nodes x 100,000 pods, one msh_schedule_batch_device launch per batch,
# the headline list): pair_kernel at 1 / 2 / 4 slice waves per 64-pod block (msh_options.pair_slices; auto
# picks 4), rocprofv3 kernel trace, and one --pmc pass (SQ counters) of the auto form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/absingle}
mkdir -p "$OUT"
export TMPDIR=/tmp
for sl in ${SLICES:-1 2 4}; do
  PAIR_PLANES=${PLANES:-auto} PAIR_SLICES=$sl WEIGHT=3 NORM=1 MODE=${MODE:-batch} PODS=${PODS:-100000} LAUNCHES=40 timeout -k 10 120 \
    rocprofv3 --kernel-trace --stats -d "$OUT/${PLANES:-auto}_s$sl" -o run --output-format csv -- python3 scripts/run_batch.py \
    > "$OUT/${PLANES:-auto}_s$sl.log" 2>&1 || { echo "[s$sl] failed"; exit 1; }
  python3 - "$OUT/${PLANES:-auto}_s$sl" "${PLANES:-auto} slices=$sl" <<'PY'
import csv, sys, pathlib
for f in pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "pair" in r["Name"]:
            print(f"{sys.argv[2]:10s} {r['Name'].split('(')[0]:50s} avg_us={float(r['AverageNs'])/1e3:.2f} "
                  f"min_us={float(r['MinNs'])/1e3:.2f} calls={r['Calls']}")
PY
done
if [ -n "${PMC:-1}" ]; then
  PAIR_PLANES=${PLANES:-auto} WEIGHT=3 NORM=1 MODE=${MODE:-batch} PODS=${PODS:-100000} LAUNCHES=10 timeout -s KILL 120 rocprofv3 --pmc \
    SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    -d "$OUT/${PLANES:-auto}_pmc" -o run --output-format csv -- python3 scripts/run_batch.py > "$OUT/${PLANES:-auto}_pmc.log" 2>&1 || { echo "[pmc] failed"; exit 1; }
  python3 - "$OUT/${PLANES:-auto}_pmc" <<'PY'
import csv, sys, pathlib
from collections import defaultdict
acc = defaultdict(list)
for f in pathlib.Path(sys.argv[1]).rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "pair" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: sum(v) / len(v) for k, v in acc.items()})
PY
fi
