"""Per-launch HBM traffic of the hot kernels from the rocprofv3 --pmc passes of
scripts/profile_r1.sh, corrected as MI355X_MICROARCH.md's HBM section prescribes:
FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of streaming
reads (re-measured here for 4 B and 16 B per lane by scripts/calib_fetch.hip); WRITE_SIZE is exact
(checked against torch's 1.6 MB fill kernel in the same pass)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r1")
out = Path(sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_latest.json")


def per_kernel(tag):
    acc = defaultdict(list)
    for r in csv.DictReader(open(src / tag / "run_counter_collection.csv")):
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


calib = {}
for k, v in per_kernel("calib").items():
    if "stream_read" in k:
        calib[k] = (256 << 20) / v if v else None
res = {"source": str(src), "method": "FETCH_SIZE, WRITE_SIZE in separate --pmc passes; KiB*1024; "
       "FETCH x2 (gfx950 streaming-read correction, calibrated 4/16 B per lane)",
       "fetch_calibration_bytes_per_fetch_byte": calib, "kernels": {}}


def pick(d, prefix):
    """The hot kernel of a pass: the msh kernel whose name starts with `prefix`."""
    names = [k for k in d if k.startswith(prefix)]
    if len(names) != 1:
        raise SystemExit(f"expected one {prefix}* kernel, found {names}")
    return names[0]


for mode, (ft, wt, prefix, pods) in {"batch": ("fetch", "write", "void msh::ident", 100000),
                                     "sequential": ("seq_fetch", "seq_write", "void msh::seq_kernel", 100000)}.items():
    fd, wd = per_kernel(ft), per_kernel(wt)
    name = pick(fd, prefix)
    f, w = fd[name], wd[name]
    res["kernels"][mode] = {"kernel": name, "fetch_raw_bytes": f, "fetch_bytes": 2 * f, "write_bytes": w,
                            "hbm_bytes_per_launch": 2 * f + w, "nodes": 5000, "pods": pods}
# bench.py reads the batch entry (default mode)
b = res["kernels"]["batch"]
res.update({"mode": "batch", "nodes": b["nodes"], "pods": b["pods"], "hbm_bytes_per_launch": b["hbm_bytes_per_launch"]})
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
