"""Summarise scripts/profile_r2.sh (gpurun_out/prof_r2) into profiles/r2_pmc_c3.json: per-launch
counters of the hot kernels at C3 (rows_kernel, identity and MIN-MAX) and C5 (seq_kernel), with the derived figures
bench.py's roofline quotes. FETCH_SIZE / WRITE_SIZE are KiB (x 1024); WRITE_SIZE reads exact bytes
for coalesced stores (MI355X_MICROARCH.md, HBM section); FETCH_SIZE is reported raw and with the
guide's x2 correction for wide streaming reads (an upper bound here: the pod bytes are read 64 B
per wave)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r2")
out = Path(sys.argv[2] if len(sys.argv) > 2 else "profiles/r2_pmc_c3.json")
N, P = 5000, 100000


def counters(tag, prefix):
    acc, name = defaultdict(list), None
    for f in sorted((src / tag).rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not k.startswith(prefix):
                continue
            name = k.split("(")[0]
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return name, {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


res = {"source": str(src), "nodes": N, "pods": P, "kernels": {}}
for mode, prefix, tags in (("batch", "void msh::rows_kernel", ("b_sq", "b_sq2", "b_lds", "b_grbm", "b_fetch", "b_write")),
                           ("batch_minmax", "void msh::rows_kernel", ("k_sq",)),
                           ("sequential", "void msh::seq_kernel", ("s_sq", "s_fetch", "s_write"))):
    e = {"nodes": N, "pods": P, "launches_per_counter": {}}
    for t in tags:
        name, avg, cnt = counters(t, prefix)
        if name:
            e["kernel"] = name
        e.update(avg)
        e["launches_per_counter"].update(cnt)
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
        e["fetch_bytes_raw"] = e["FETCH_SIZE"] * 1024
        e["write_bytes"] = e["WRITE_SIZE"] * 1024
        e["hbm_bytes_per_launch"] = e["fetch_bytes_raw"] + e["write_bytes"]
        e["hbm_bytes_per_launch_fetch_x2"] = 2 * e["fetch_bytes_raw"] + e["write_bytes"]
    if "SQ_INSTS_VALU" in e:
        e["valu_lane_ops_per_eval"] = e["SQ_INSTS_VALU"] * 64 / (N * P)
        # the scan's modelled VALU per 8-word group and wave: rows_kernel 8 v_bitop3 + 4 ORs +
        # compare + select + move (15); with the non-match too (MIN-MAX) 38
        per_group = {"batch": 15, "batch_minmax": 38}.get(mode)
        if per_group:
            e["scan_model_share"] = (per_group / 8) * (P / 64) * (N / 32) / e["SQ_INSTS_VALU"]
    if "SQ_WAVE_CYCLES" in e:
        for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in e:
                e[k.lower() + "_frac_of_wave_cycles"] = e[k] / e["SQ_WAVE_CYCLES"]
    if "GRBM_GUI_ACTIVE" in e and "SQ_INSTS_VALU" in e:
        cyc = e["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
        e["gui_active_cycles_per_xcd"] = cyc
        e["valu_wave_instr_per_simd_cycle"] = e["SQ_INSTS_VALU"] / (1024 * cyc)
    res["kernels"][mode] = e
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
