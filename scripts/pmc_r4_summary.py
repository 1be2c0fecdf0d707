"""Summarise scripts/profile_r4.sh (gpurun_out/prof_r4) into profiles/r4_pmc_c3.json: per-launch
counters of the hot kernels at C3 (5,000 nodes x 100,000 pods per batch) with the derived figures
bench.py's roofline quotes.

Entries: "pair_multi" (pair_kernel, 32 batches per launch: bench.py's default submission),
"pair_minmax" (the same, MIN-MAX), "classrows_multi" (the opt-in class-row kernel, 32 batches),
"generic_ref" (generic_kernel on the reference plugin list, 32 batches), "generic_col" (generic_kernel
on NodeNumber + a DEFAULT-normalized score column, 32 batches) and "sequential" (seq_kernel at C5).
FETCH_SIZE / WRITE_SIZE are KiB (x 1024); FETCH_SIZE is reported raw and with MI355X_MICROARCH.md's x2
correction for wide streaming reads (the pod bytes are 1-byte loads: uncalibrated, an upper bound),
WRITE_SIZE as read."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r4")
out = Path(sys.argv[2] if len(sys.argv) > 2 else "profiles/r4_pmc_c3.json")
N, P = 5000, 100000
NB = 32  # batches per launch of the multi entries (MSH_BATCHES_PER_LAUNCH)
GROUPS = -(-N // 1024) * 1024 // 256  # 256-node groups of the padded table
WORDS = GROUPS * 8


def counters(tag, prefix):
    acc, name = defaultdict(list), None
    for f in sorted((src / tag).rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if prefix not in k:
                continue
            name = k.split("(")[0]
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return name, {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def stats_avg_ns(tag, prefix):
    for f in sorted((src / tag).rglob("*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if prefix in r["Name"]:
                return r["Name"].split("(")[0], float(r["AverageNs"]), int(r["Calls"])
    return None, None, None


res = {"source": str(src), "nodes": N, "pods": P, "kernels": {}, "stats": {}}
for mode, prefix, tags, nb in (
        ("pair_multi", "msh::pair", ("m_sq", "m_sq2", "m_grbm", "m_fetch", "m_write"), NB),
        ("pair_minmax", "msh::pair", ("k_sq",), NB),
        ("classrows_multi", "msh::wgp_kernel", ("c_sq",), NB),
        ("generic_ref", "msh::generic_kernel", ("g_sq", "g_grbm", "g_fetch"), NB),
        ("generic_col", "msh::generic_kernel", ("gc_sq",), NB),
        ("sequential", "msh::seq_kernel", ("s_sq",), 1)):
    e = {"nodes": N, "pods": P, "batches_per_launch": nb, "launches_per_counter": {}}
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
    elif "FETCH_SIZE" in e:
        e["fetch_bytes_raw"] = e["FETCH_SIZE"] * 1024
    if "SQ_INSTS_VALU" in e:
        e["valu_lane_ops_per_eval"] = e["SQ_INSTS_VALU"] * 64 / (N * P * nb)
        if mode.startswith("pair"):
            # the scan's model per 32-node word and 64-pod wave: v_bitop3 (X & nT) + 4 v_bitop3 for dm' and
            # half an AND3 of two words' dm' = 5.5 VALU (NONE); MIN-MAX adds one OR-accumulate of the
            # feasible non-matches (6.5)
            # (the LDS-staged form adds one v_bitop3 per group and block in NONE: 5.625; in MIN-MAX it
            # drops the OR-accumulate when group 0 settled the first non-match, MSH_PAIR_NOAX, and with
            # tolerates compaction 7 of a workgroup's 8 blocks fold X into the first compare: 4.625)
            lds = "pair_lds" in e.get("kernel", "")
            per_word = (4.625 if lds else 6.5) if mode == "pair_minmax" else (5.625 if lds else 5.5)
            e["scan_model_share"] = per_word * WORDS * (-(-P // 64)) * nb / e["SQ_INSTS_VALU"]
    if "SQ_WAVE_CYCLES" in e:
        for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in e:
                e[k.lower() + "_frac_of_wave_cycles"] = e[k] / e["SQ_WAVE_CYCLES"]
    if "GRBM_GUI_ACTIVE" in e and "SQ_INSTS_VALU" in e:
        cyc = e["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
        e["gui_active_cycles_per_xcd"] = cyc
        e["valu_wave_instr_per_simd_cycle"] = e["SQ_INSTS_VALU"] / (1024 * cyc)
    res["kernels"][mode] = e
for tag, prefix in (("stats", "msh::pair"), ("stats_k20", "msh::pair"),
                    ("stats_multi", "msh::pair"), ("stats_single", "msh::pair"),
                    ("stats_kx", "msh::pair"), ("stats_classrows", "msh::wgp_kernel"),
                    ("stats_classrows_kx", "msh::wgp_kernel"), ("stats_generic", "msh::generic_kernel"),
                    ("stats_generic_col", "msh::generic_kernel"), ("stats_seq", "msh::seq_kernel")):
    name, avg, calls = stats_avg_ns(tag, prefix)
    if name:
        res["stats"][tag] = {"kernel": name, "avg_ns": avg, "calls": calls}
out.write_text(json.dumps(res, indent=1))
print(json.dumps(res)[:2000])
