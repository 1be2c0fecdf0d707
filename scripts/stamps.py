"""Phase anatomy of the IDENT batch kernel from per-wave stamps (diagnostic build only).

Stamps (per wave): 0 kernel entry, 1 after LDS staging barrier, 2 after pod load/ballot,
3 after the main scan groups, 4 after the tolerating-pod ulist scan, 5 exit.
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
msh._native.LIB_PATH = Path(os.environ["MSH_LIBRARY"])  # the package was imported by build above
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
lib = msh._native.lib()
lib.msh_debug_read_stamps.argtypes = [C.c_void_p, C.c_int]
NW = 16384
for n, p in [(int(x.split("x")[0]), int(x.split("x")[1])) for x in os.environ.get("CASES", "64x100000,5000x100000").split(",")]:
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
    buf = np.zeros(NW * 8 * 2, np.uint64)
    assert lib.msh_debug_read_stamps(buf.ctypes.data, NW) == 0
    st = buf.reshape(NW, 8, 2).astype(np.int64)
    valid = st[:, 0, 0] > 0
    st = st[valid]
    rt = st[:, :, 0]  # 100 MHz
    cy = st[:, :, 1]
    t0 = rt[:, 0].min()
    out = {"nodes": n, "pods": p, "waves": int(valid.sum()),
           "start_us": {"p50": float(np.median(rt[:, 0] - t0) / 100), "max": float((rt[:, 0] - t0).max() / 100)},
           "end_us": {"p50": float(np.median(rt[:, 5] - t0) / 100), "max": float((rt[:, 5] - t0).max() / 100)},
           "clock_ghz": float(np.median((cy[:, 5] - cy[:, 0]) / np.maximum(rt[:, 5] - rt[:, 0], 1)) / 10)}
    for a, b, name in [(0, 1, "staging"), (1, 2, "pod_load"), (2, 3, "main_scan"), (3, 4, "tol_scan"), (4, 5, "decode_store")]:
        d = cy[:, b] - cy[:, a]
        out[name + "_kcyc"] = {"p50": float(np.median(d) / 1e3), "p90": float(np.percentile(d, 90) / 1e3)}
    hw = st[:, 7, 0].astype(np.int64)
    xcc = st[:, 7, 1].astype(np.int64) & 0xF
    simd = (hw >> 4) & 0x3
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    end = (rt[:, 5] - t0) / 100
    dur = (cy[:, 5] - cy[:, 1]) / 1e3
    out["end_by_xcc_p50"] = [float(np.median(end[xcc == x])) if (xcc == x).any() else None for x in range(8)]
    out["dur_by_simd_p50"] = [float(np.median(dur[simd == k])) for k in range(4)]
    # waves per (xcc, se, cu, simd) slot and duration vs co-resident count
    key = ((xcc * 8 + se) * 16 + cu) * 4 + simd
    uk, cnt = np.unique(key, return_counts=True)
    out["waves_per_simd_hist"] = {int(c): int((cnt == c).sum()) for c in np.unique(cnt)}
    slowest = np.argsort(-end)[:5]
    out["slowest"] = [{"gw": int(np.nonzero(valid)[0][i]), "end_us": float(end[i]), "xcc": int(xcc[i]), "se": int(se[i]),
                       "cu": int(cu[i]), "simd": int(simd[i]), "dur_kcyc": float(dur[i])} for i in slowest]
    out["dur_kcyc_hist"] = np.histogram(dur, bins=8)[0].tolist()
    out["dur_kcyc_edges"] = [round(float(x), 1) for x in np.histogram(dur, bins=8)[1]]
    print(json.dumps(out), flush=True)
    ctx.close()
