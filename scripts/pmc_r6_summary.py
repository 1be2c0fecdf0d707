"""Summarise scripts/profile_r6.sh (gpurun_out/prof_r6) into profiles/r6_pmc_c3.json: per-launch counters
of the hot kernels at C3 (5,000 nodes x 100,000 pods per batch) with the derived figures bench.py's
roofline quotes.

Entries (each records its kernel, size, batch count and NodeNumber plugin entry; bench.py uses an entry
only when all of them match what it timed):
  pair_multi      the per-pair kernel, 32 batches per launch, bench.py's headline list (w=3 DEFAULT)
  pair_multi_ref  the same with the reference's own list (w=1, no normalizer)
  pair_minmax     the same, MIN-MAX w=3;  pair_reverse: REVERSE w=3
  generic_ref     generic_kernel on the reference list (w=1 NONE), 32 batches
  generic_hl      generic_kernel on the headline list (w=3 DefaultNormalizeScore: extents pass + main pass), 32 batches
  generic_col     generic_kernel on NodeNumber + a DEFAULT-normalized score column, 32 batches
  sequential_pair  C5 (headline list) without a capacity, auto: pair_kernel with the commit epilogue
  sequential      seq_kernel at C5 (headline list), pod blocks over workgroups (msh_options.seq_split blocks)
  sequential_serial  the same with msh_options.seq_split serial (one workgroup walks all pods)
  sequential_capacity  seq_kernel at C5 with a capacity of 15 pods per node (the reference list, w=1)
FETCH_SIZE / WRITE_SIZE are KiB (x 1024); FETCH_SIZE is reported raw and with MI355X_MICROARCH.md's x2
gfx950 correction (hbm_bytes_per_launch_fetch_x2 = 2 x FETCH + WRITE, what bench.py's `traffic` quotes)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r6")
out = Path(sys.argv[2] if len(sys.argv) > 2 else "profiles/r6_pmc_c3.json")
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


def tag_of(w, norm):
    return f"NodeNumber w={w} norm={norm}"


res = {"source": str(src), "nodes": N, "pods": P, "kernels": {}, "stats": {}}
for mode, prefix, tags, nb, plug in (
        ("pair_multi", "msh::pair", ("m_sq", "m_fetch", "m_write"), NB, tag_of(3, 1)),
        ("pair_multi_ref", "msh::pair", ("r_sq",), NB, tag_of(1, 0)),
        ("pair_minmax", "msh::pair", ("k_sq",), NB, tag_of(3, 3)),
        ("pair_reverse", "msh::pair", ("v_sq",), NB, tag_of(3, 2)),
        ("generic_ref", "msh::generic_kernel", ("g_sq",), NB, tag_of(1, 0)),
        ("generic_hl", "msh::generic_kernel", ("gh_sq",), NB, tag_of(3, 1)),
        ("generic_col", "msh::generic_kernel", ("gc_sq", "gc_sq2"), NB, tag_of(1, 0) + " + ScoreColumn0 w=2 norm=1"),
        ("sequential_pair", "msh::pair_kernel", ("sp_sq", "sp_sq2"), 1, tag_of(3, 1)),
        ("sequential", "msh::seq_kernel", ("s_sq", "s_sq2"), 1, tag_of(3, 1)),
        ("sequential_serial", "msh::seq_kernel", ("ss_sq",), 1, tag_of(3, 1)),
        ("sequential_capacity", "msh::seq_cap", ("c_sq", "c_sq2", "c_fetch"), 1, tag_of(1, 0) + " cap=15")):
    e = {"nodes": N, "pods": P, "batches_per_launch": nb, "plugins": plug, "launches_per_counter": {}}
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
            # the LDS-staged scan's model per 32-node word and 64-pod wave: 5.625 VALU in the identity-like
            # modes (NONE, DEFAULT), 4.625 in REVERSE / MINMAX (group 0 first, tolerates compaction)
            per_word = 4.625 if mode in ("pair_minmax", "pair_reverse") else 5.625
            e["scan_model_share"] = per_word * WORDS * (-(-P // 64)) * nb / e["SQ_INSTS_VALU"]
    if mode.startswith("sequential") and "SQ_INSTS_VALU" in e and "SQ_INSTS_SALU" in e:
        e["instructions_per_pod"] = (e["SQ_INSTS_VALU"] + e["SQ_INSTS_SALU"] + e.get("SQ_INSTS_SMEM", 0)) / P
    if "SQ_INSTS_SALU" in e and "SQ_INSTS_VALU" in e:
        e["salu_per_valu"] = e["SQ_INSTS_SALU"] / e["SQ_INSTS_VALU"]
    if "SQ_INSTS_SMEM" in e and "SQ_WAVES" in e:
        e["smem_per_wave"] = e["SQ_INSTS_SMEM"] / e["SQ_WAVES"]
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
                    ("stats_multi", "msh::pair"), ("stats_ref", "msh::pair"), ("stats_kx", "msh::pair"),
                    ("stats_rev", "msh::pair"), ("stats_single", "msh::pair"),
                    ("stats_generic", "msh::generic_kernel"), ("stats_generic_hl", "msh::generic_kernel"),
                    ("stats_generic_col", "msh::generic_kernel"),
                    ("stats_seq_pair", "msh::pair_kernel"), ("stats_seq", "msh::seq_kernel"), ("stats_seq_serial", "msh::seq_kernel"),
                    ("stats_seq_cap", "msh::seq_cap")):
    name, avg, calls = stats_avg_ns(tag, prefix)
    if name:
        res["stats"][tag] = {"kernel": name, "avg_ns": avg, "calls": calls}
out.write_text(json.dumps(res, indent=1))
print(json.dumps(res)[:2000])
