"""Minimal driver for profiling: K launches of the batched kernel on the C3 workload."""
import importlib
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
n = int(os.environ.get("NODES", 5000))
p = int(os.environ.get("PODS", 100000))
k = int(os.environ.get("LAUNCHES", 20))
mode = os.environ.get("MODE", "batch")
ctx = msh.DeviceContext(0)
norm = int(os.environ.get("NORM", 0))  # msh_normalize (3 = MINMAX: the KX kernel)
ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 1, msh.Normalize(norm))])
u, nd, pd, pt = synth.make_soa(n, p)
ctx.upload_nodes(u, nd)
dev = torch.device("cuda:0")
d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
oi = torch.empty(p, dtype=torch.int32, device=dev)
osc = torch.empty(p, dtype=torch.int64, device=dev)
ost = torch.empty(p, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(k):
    if mode == "batch":
        ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(), ost.data_ptr(), s)
    else:
        ctx.schedule_sequential_device(p, d_pd.data_ptr(), d_pt.data_ptr(), 0, oi.data_ptr(), osc.data_ptr(),
                                       ost.data_ptr(), s)
torch.cuda.synchronize()
print("ok", n, p, k, mode)
