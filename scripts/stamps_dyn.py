"""Phase anatomy of the work-queue IDENT kernel (ident_dyn_kernel) from per-wave stamps
(diagnostic -DMSH_STAMPS build only; never the product library).

Stamps per wave: 0 entry, 1 first unit fetched, 2 its pods loaded + ballot, 3 its pod-pair
groups scanned (+ cross-lane reduction), 4 its tolerating-pod ulist scan done, 5 exit;
slot 6 = units this wave took, slot 7 = hardware ids. Times: s_memrealtime (100 MHz) for
wall-clock positions, s_memtime (shader clock) for phase lengths.
"""
import ctypes as C
import importlib
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
build = importlib.import_module("mini-kube-scheduler_amd.build")
os.environ["MSH_LIBRARY"] = str(build.build_diagnostic())
import torch  # noqa: E402
msh = importlib.import_module("mini-kube-scheduler_amd")
msh._native.LIB_PATH = Path(os.environ["MSH_LIBRARY"])
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
lib = msh._native.lib()
lib.msh_debug_read_stamps.argtypes = [C.c_void_p, C.c_int]
lib.msh_debug_clear_stamps.argtypes = []
NW = 16384


def pct(x):
    return {"p10": round(float(np.percentile(x, 10)), 2), "p50": round(float(np.median(x)), 2),
            "p90": round(float(np.percentile(x, 90)), 2), "max": round(float(np.max(x)), 2)}


for case in os.environ.get("CASES", "64x100000,5000x100000,5000x1000000").split(","):
    n, p = (int(v) for v in case.split("x"))
    ctx = msh.DeviceContext(0)
    u, nd, pd, pt = synth.make_soa(n, p)
    ctx.upload_nodes(u, nd)
    dev = torch.device("cuda:0")
    d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
    oi = torch.empty(p, dtype=torch.int32, device=dev)
    osc = torch.empty(p, dtype=torch.int64, device=dev)
    ost = torch.empty(p, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(), ost.data_ptr(), s)
    torch.cuda.synchronize()
    assert lib.msh_debug_clear_stamps() == 0
    ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(), ost.data_ptr(), s)
    torch.cuda.synchronize()
    buf = np.zeros(NW * 8 * 2, np.uint64)
    assert lib.msh_debug_read_stamps(buf.ctypes.data, NW) == 0
    st = buf.reshape(NW, 8, 2).astype(np.int64)
    valid = st[:, 0, 0] > 0
    st = st[valid]
    rt, cy = st[:, :, 0], st[:, :, 1]
    units = st[:, 6, 0]
    took = units > 0
    t0 = rt[:, 0].min()
    out = {"nodes": n, "pods": p, "waves": int(valid.sum()), "waves_with_units": int(took.sum()),
           "units_per_wave_hist": {int(k): int(v) for k, v in zip(*np.unique(units, return_counts=True))},
           "entry_us": pct((rt[:, 0] - t0) / 100), "exit_us": pct((rt[:, 5] - t0) / 100),
           "clock_ghz": round(float(np.median((cy[:, 5] - cy[:, 0]) / np.maximum(rt[:, 5] - rt[:, 0], 1)) / 10), 3)}
    c = cy[took]
    for a, b, name in [(0, 1, "entry_to_first_unit"), (1, 2, "pod_load"), (2, 3, "groups_scan"), (3, 4, "ulist"),
                       (4, 5, "rest_of_units")]:
        out[name + "_kcyc"] = pct((c[:, b] - c[:, a]) / 1e3)
    out["wave_life_kcyc"] = pct((cy[:, 5] - cy[:, 0]) / 1e3)
    xcc = st[:, 7, 1] & 0xF
    hw = st[:, 7, 0]
    se = (hw >> 13) & 0x7
    out["by_xcc"] = {int(x): {"waves": int((xcc == x).sum()),
                              "entry_us_p10_p50_max": [round(float(np.percentile((rt[xcc == x, 0] - t0) / 100, q)), 2)
                                                       for q in (10, 50, 100)],
                              "exit_us_p50_max": [round(float(np.percentile((rt[xcc == x, 5] - t0) / 100, q)), 2)
                                                  for q in (50, 100)],
                              "first_entry_by_se_us": [round(float((rt[(xcc == x) & (se == k), 0] - t0).min() / 100), 2)
                                                       if ((xcc == x) & (se == k)).any() else None for k in range(8)]}
                     for x in np.unique(xcc)}
    cu = (hw >> 8) & 0xF
    cukey = (xcc * 8 + se) * 16 + cu
    cu_in, cu_out, cu_x = [], [], []
    for k in np.unique(cukey):
        sel = cukey == k
        cu_in.append((rt[sel, 0].min() - t0) / 100)
        cu_out.append((rt[sel, 5].max() - t0) / 100)
        cu_x.append(int(xcc[sel][0]))
    cu_in, cu_out, cu_x = np.array(cu_in), np.array(cu_out), np.array(cu_x)
    out["cus"] = int(len(cu_in))
    out["cu_span_us"] = pct(cu_out - cu_in)
    out["cu_exit_by_xcc_min_p50_max"] = {int(x): [round(float(np.min(cu_out[cu_x == x])), 2),
                                                  round(float(np.median(cu_out[cu_x == x])), 2),
                                                  round(float(np.max(cu_out[cu_x == x])), 2)] for x in np.unique(cu_x)}
    last = np.argsort(-(rt[:, 5]))[:3]
    out["last_waves"] = [{"exit_us": float((rt[i, 5] - t0) / 100), "entry_us": float((rt[i, 0] - t0) / 100),
                          "units": int(units[i]), "life_kcyc": float((cy[i, 5] - cy[i, 0]) / 1e3)} for i in last]
    print(json.dumps(out), flush=True)
    ctx.close()
