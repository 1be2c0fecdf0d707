"""Isolated batch-kernel time against the batch size at 5k nodes: K launches back to back on one
stream (HIP events around them), for P from one 64-pod block to 4x C3. The small-P end is the
fixed cost of a launch (dispatch + one wave's dependency chain); the slope is the throughput.
One JSON line per (P, slices)."""
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
K = int(os.environ.get("K", 200))
N = int(os.environ.get("NODES", 5000))
SLICES = os.environ.get("SLICES", "0").split(",")
PODS = [int(x) for x in os.environ.get("PODS", "64,640,6400,25600,51200,100000,200000,400000").split(",")]
dev = torch.device("cuda:0")
u, nd = synth.make_nodes(N)[1:]
pmax = max(PODS)
pd_all, pt_all = synth._make_pods_fast(pmax, synth.SEED)[1:]
d_pd, d_pt = torch.from_numpy(pd_all).to(dev), torch.from_numpy(pt_all).to(dev)
oi = torch.empty(pmax, dtype=torch.int32, device=dev)
osc = torch.empty(pmax, dtype=torch.int64, device=dev)
ost = torch.empty(pmax, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
for sl in SLICES:
    os.environ["MSH_BITS_SLICES"] = sl
    ctx = msh.DeviceContext(0)
    ctx.upload_nodes(u, nd)
    for p in PODS:
        def run(k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(k):
                ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(),
                                          ost.data_ptr(), s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / k
        run(10)
        us = float(np.median([run(K) for _ in range(3)]))
        print(json.dumps({"nodes": N, "pods": p, "slices": sl, "us_per_launch": us,
                          "evals_per_s": N * p / (us * 1e-6)}), flush=True)
    ctx.close()
