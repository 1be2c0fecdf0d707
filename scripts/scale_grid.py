"""Kernel time over a grid of (nodes, pods) to separate fixed launch cost from per-pair cost.

Each point: LAUNCHES back-to-back launches between two HIP events on the launch stream (an
event pair per launch would add its own ~3.5 us packet), median of REPS. MSH_LIBRARY selects an
A/B build (build.build_variant); TAG labels the lines.
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
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
DEFAULT_GRID = ("64x100000,1024x100000,2048x100000,5000x100000,8192x100000,16384x100000,"
                "5000x12500,5000x25000,5000x50000,5000x200000,5000x400000,5000x1000000")
grid = [tuple(int(v) for v in g.split("x")) for g in os.environ.get("GRID", DEFAULT_GRID).split(",")]
tag = os.environ.get("TAG", "default")
launches = int(os.environ.get("LAUNCHES", 20))
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
    for _ in range(int(os.environ.get("REPS", 7))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(launches):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / launches)
    ms = float(np.median(ts))
    print(json.dumps({"tag": tag, "nodes": n, "pods": p, "ms": ms, "evals_per_s": n * p / (ms * 1e-3)}), flush=True)
