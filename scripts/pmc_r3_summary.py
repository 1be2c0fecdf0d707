"""Summarise scripts/profile_r3.sh (gpurun_out/prof_r3) into profiles/r3_pmc_c3.json: per-launch
counters of the hot kernels at C3 — the persistent class-row kernel wgp_kernel with 32 batches per
launch (bench.py's default submission, "batch_multi"), one batch per launch ("batch"), MIN-MAX
("batch_minmax", 32 batches), the generic
score pipeline ("generic") and seq_kernel at C5 ("sequential") — with the derived figures bench.py's
roofline quotes. FETCH_SIZE / WRITE_SIZE are KiB (x 1024); WRITE_SIZE reads exact bytes for
coalesced stores (MI355X_MICROARCH.md, HBM section); FETCH_SIZE is reported raw and with the guide's
x2 correction for wide streaming reads (an upper bound here)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r3")
out = Path(sys.argv[2] if len(sys.argv) > 2 else "profiles/r3_pmc_c3.json")
N, P = 5000, 100000
NB = 32  # batches per launch in the multi entries (MSH_BATCHES_PER_LAUNCH)
GROUPS = -(-N // 1024) * 1024 // 256  # 256-node groups of the padded table


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


def stats_avg_ns(tag, prefix):
    for f in sorted((src / tag).rglob("*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if r["Name"].startswith(prefix):
                return r["Name"].split("(")[0], float(r["AverageNs"]), int(r["Calls"])
    return None, None, None


res = {"source": str(src), "nodes": N, "pods": P, "kernels": {}, "stats": {}}
for mode, prefix, tags, nb in (
        ("batch_multi", "void msh::wgp_kernel", ("m_sq", "m_sq2", "m_lds", "m_grbm", "m_fetch", "m_write"), NB),
        ("batch", "void msh::wgp_kernel", ("b_sq", "b_lds", "b_fetch", "b_write"), 1),
        ("batch_minmax", "void msh::wgp_kernel", ("k_sq",), NB),
        ("generic", "msh::generic_kernel", ("g_sq", "g_fetch"), 1),
        ("sequential", "void msh::seq_kernel", ("s_sq", "s_fetch", "s_write"), 1)):
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
    if "SQ_INSTS_VALU" in e:
        e["valu_lane_ops_per_eval"] = e["SQ_INSTS_VALU"] * 64 / (N * P * nb)
        # the scan's modelled VALU per 256-node group and 64-pod wave (wgp_kernel, four groups per
        # step: 16 v_bitop3 OR3 over the 32 class-row words, two pair flags (2 v_min + 2 v_lshl_or)
        # and two address adds = 22 per four groups, 5.5; MIN-MAX adds 32 v_bitop3 for the
        # non-matches and their two flags, 58 per four groups, 14.5)
        per_group = {"batch_multi": 5.5, "batch": 5.5, "batch_minmax": 14.5}.get(mode)
        if per_group:
            e["scan_model_share"] = per_group * GROUPS * (P / 64) * nb / e["SQ_INSTS_VALU"]
    if "SQ_WAVE_CYCLES" in e:
        for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in e:
                e[k.lower() + "_frac_of_wave_cycles"] = e[k] / e["SQ_WAVE_CYCLES"]
    if "GRBM_GUI_ACTIVE" in e and "SQ_INSTS_VALU" in e:
        cyc = e["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
        e["gui_active_cycles_per_xcd"] = cyc
        e["valu_wave_instr_per_simd_cycle"] = e["SQ_INSTS_VALU"] / (1024 * cyc)
    res["kernels"][mode] = e
for tag, prefix in (("stats", "void msh::wgp_kernel"), ("stats_k20", "void msh::wgp_kernel"),
                    ("stats_single", "void msh::wgp_kernel"), ("stats_kx", "void msh::wgp_kernel"),
                    ("stats_generic", "msh::generic_kernel"), ("stats_seq", "void msh::seq_kernel")):
    name, avg, calls = stats_avg_ns(tag, prefix)
    if name:
        res["stats"][tag] = {"kernel": name, "average_ns": avg, "calls": calls}
out.write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
