"""Summarise scripts/pmc_valu.sh (gpurun_out/pmc_valu) for the hot kernel into a JSON file."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_valu")
out = Path(sys.argv[2] if len(sys.argv) > 2 else "profiles/r1_pmc_valu_c3.json")
vals = defaultdict(list)
kern = None
for f in sorted(src.glob("*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if not name.startswith("void msh::ident"):
            continue
        kern = name.split("(")[0]
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in vals.items()}
res = {"source": str(src), "kernel": kern, "launches_per_counter": {k: len(v) for k, v in vals.items()},
       "per_launch": avg}
n, p = 5000, 100000
if "SQ_INSTS_VALU" in avg:
    res["valu_wave_instr_per_launch"] = avg["SQ_INSTS_VALU"]
    res["valu_lane_ops_per_eval"] = avg["SQ_INSTS_VALU"] * 64 / (n * p)
    res["scan_core_share"] = (0.75 * n * p / 64) / avg["SQ_INSTS_VALU"]
if "SQ_WAIT_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
    res["wait_inst_any_frac_of_wave_cycles"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
    res["active_valu_frac_of_wave_cycles"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
if "GRBM_GUI_ACTIVE" in avg and "SQ_INSTS_VALU" in avg:
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD busy cycles = / 8
    cyc = avg["GRBM_GUI_ACTIVE"] / 8
    res["gui_active_cycles_per_xcd"] = cyc
    res["valu_wave_instr_per_simd_cycle"] = avg["SQ_INSTS_VALU"] / (1024 * cyc)
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
