"""Interleaved A/B of batch-kernel launch geometry in ONE process (guide §5.4 rule 24).

Times msh_schedule_batch_device on the C3 workload for each MSH_BATCH_WG_PER_CU value
(read by the launcher at every launch), round-robin, and prints median/min kernel ms.
"""
import importlib
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
if os.environ.get("MSH_LIBRARY"):
    msh._native.LIB_PATH = Path(os.environ["MSH_LIBRARY"])
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")

n = int(os.environ.get("NODES", 5000))
p = int(os.environ.get("PODS", 100000))
# variant = "<kernel>/<wg_per_cu>": kernel 0 = packed-16 IDENT, 1 = compare/select kernel; wg 0 = auto
variants = [v for v in os.environ.get("VARIANTS", "0/0,1/0,0/1,0/2,0/3,0/4").split(",")]
ctx = msh.DeviceContext(0)
u, nd, pd, pt = synth.make_soa(n, p)
ctx.upload_nodes(u, nd)
dev = torch.device("cuda:0")
d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
oi = torch.empty(p, dtype=torch.int32, device=dev)
osc = torch.empty(p, dtype=torch.int64, device=dev)
ost = torch.empty(p, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
res = {v: [] for v in variants}
for rnd in range(20):
    for v in variants:
        kern, wg = v.split("/")
        os.environ["MSH_BATCH_KERNEL"] = kern
        if wg == "0":
            os.environ.pop("MSH_BATCH_WG_PER_CU", None)
        else:
            os.environ["MSH_BATCH_WG_PER_CU"] = wg
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(),
                                      ost.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        if rnd >= 2:
            res[v].append(e0.elapsed_time(e1) / 5)
for v in variants:
    a = np.array(res[v])
    print(json.dumps({"variant": v, "nodes": n, "pods": p, "median_ms": float(np.median(a)), "min_ms": float(a.min()),
                      "evals_per_s_median": n * p / (np.median(a) * 1e-3)}))
