"""Cost of the tolerating-pod pass: the C3 batch as generated (5% of pods tolerate the
unschedulable taint) against the same batch with no tolerating pod and with every pod
tolerating, 2 streams, median per-batch us. Timing only (outputs shared)."""
import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
n, p = 5000, 100_000
ctx = msh.DeviceContext(0)
u, nd, pd, pt = synth.make_soa(n, p)
ctx.upload_nodes(u, nd)
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
s2 = torch.cuda.Stream(dev)
d_pd = torch.from_numpy(pd).to(dev)
variants = {"as_generated": pt, "none": np.zeros_like(pt), "all": np.ones_like(pt)}
d_pt = {k: torch.from_numpy(v).to(dev) for k, v in variants.items()}
oi = torch.empty(p, dtype=torch.int32, device=dev)
osc = torch.empty(p, dtype=torch.int64, device=dev)
ost = torch.empty(p, dtype=torch.int32, device=dev)
res = {k: [] for k in variants}
for rnd in range(15):
    for k in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        s2.wait_event(e0)
        for i in range(10):
            ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt[k].data_ptr(), oi.data_ptr(), osc.data_ptr(),
                                      ost.data_ptr(), (s if i % 2 == 0 else s2).cuda_stream)
        s.wait_stream(s2)
        e1.record(s)
        torch.cuda.synchronize()
        if rnd >= 2:
            res[k].append(e0.elapsed_time(e1) / 10 * 1e3)
print(json.dumps({"nodes": n, "pods": p, "ulist": int(u.sum()),
                  **{f"us[{k}]": round(float(np.median(v)), 2) for k, v in res.items()}}))
ctx.close()
