"""Minimal driver for profiling: K launches of a hot kernel on the C3 workload.

MODE=multi (bench.py's default submission: 32 independent 100k-pod batches per
msh_schedule_batches_device launch), batch (one msh_schedule_batch_device launch per batch),
sequential (C5), generic (the explicit int64 score pipeline, NodeNumber + one score column).
NORM: msh_normalize of the NodeNumber entry (3 = MINMAX)."""
import importlib
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
n = int(os.environ.get("NODES", 5000))
p = int(os.environ.get("PODS", 100000))
k = int(os.environ.get("LAUNCHES", 20))
mode = os.environ.get("MODE", "multi")
norm = int(os.environ.get("NORM", 0))
ctx = msh.DeviceContext(0)
u, nd, pd, pt = synth.make_soa(n, p)
ctx.upload_nodes(u, nd)
if mode == "generic":  # NodeNumber + one score column (weight 2, DefaultNormalizeScore)
    ctx.upload_score_column(msh.SCORE_COLUMNS[0], (np.arange(n, dtype=np.int64) * 7919) % 1000)
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, 1, msh.Normalize(norm)),
                     msh.ScorePluginConfig(msh.SCORE_COLUMNS[0], 2, msh.Normalize(1))])
else:
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, 1, msh.Normalize(norm))])
dev = torch.device("cuda:0")
nb = msh._native.BATCHES_PER_LAUNCH if mode == "multi" else 1
bufs = [(torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev), torch.empty(p, dtype=torch.int32, device=dev),
         torch.empty(p, dtype=torch.int64, device=dev), torch.empty(p, dtype=torch.int32, device=dev))
        for _ in range(nb)]
descs = ctx.batch_descs([(p, *[t.data_ptr() for t in b]) for b in bufs])
s = torch.cuda.current_stream().cuda_stream
b = bufs[0]
for _ in range(k):
    if mode == "multi":
        ctx.schedule_batches_device(descs, nb, s)
    elif mode in ("batch", "generic"):
        ctx.schedule_batch_device(p, *[t.data_ptr() for t in b], s)
    else:
        ctx.schedule_sequential_device(p, b[0].data_ptr(), b[1].data_ptr(), 0, *[t.data_ptr() for t in b[2:]], s)
torch.cuda.synchronize()
print("ok", n, p, k, mode, nb)
