"""Host cost of one no-capacity sequential call (C5, 5,000 x 100,000, the headline list) in the form FORM (auto |
blocks | batch: msh_schedule_batch_device for comparison): 100 calls, each after a device synchronize. Run
under rocprofv3 --hip-trace --stats to see which HIP calls the entry point makes and what each costs."""
import importlib
import os
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
form = os.environ.get("FORM", "auto")
n, p = 5000, 100_000
u, nd, pd, pt = synth.make_soa(n, p)
dev = torch.device("cuda:0")
bufs = [torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev), torch.empty(p, dtype=torch.int32, device=dev),
        torch.empty(p, dtype=torch.int64, device=dev), torch.empty(p, dtype=torch.int32, device=dev)]
s = torch.cuda.current_stream().cuda_stream
ctx = msh.DeviceContext(0, {"seq_split": "blocks"} if form == "blocks" else None)
ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 3, msh.Normalize(1))])
ctx.upload_nodes(u, nd)
ptrs = [t.data_ptr() for t in bufs]
if form == "batch":
    call = lambda: ctx.schedule_batch_device(p, *ptrs, s)
else:
    call = lambda: ctx.schedule_sequential_device(p, ptrs[0], ptrs[1], 0, *ptrs[2:], s)
ts = []
for _ in range(100):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call()
    ts.append(time.perf_counter() - t0)
torch.cuda.synchronize()
print(form, "median host call us", sorted(ts)[50] * 1e6)
