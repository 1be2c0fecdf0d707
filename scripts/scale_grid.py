"""Kernel time over a grid of (nodes, pods) to separate fixed launch cost from per-pair cost."""
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
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
grid = [(64, 100_000), (1024, 100_000), (2048, 100_000), (4096, 100_000), (5000, 100_000), (8192, 100_000),
        (16384, 100_000), (5000, 25_000), (5000, 50_000), (5000, 200_000), (5000, 400_000), (5000, 1_000_000)]
kern = os.environ.get("MSH_BATCH_KERNEL", "0")
ctx = msh.DeviceContext(0)
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
for n, p in grid:
    u, nd, pd, pt = synth.make_soa(n, p)
    ctx.upload_nodes(u, nd)
    d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
    oi = torch.empty(p, dtype=torch.int32, device=dev)
    osc = torch.empty(p, dtype=torch.int64, device=dev)
    ost = torch.empty(p, dtype=torch.int32, device=dev)
    def run():
        ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(), ost.data_ptr(),
                                  s.cuda_stream)
    for _ in range(3):
        run()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s); run(); e1.record(s); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    print(json.dumps({"kernel": kern, "nodes": n, "pods": p, "ms": ms, "evals_per_s": n * p / (ms * 1e-3)}), flush=True)
