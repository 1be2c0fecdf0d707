"""Per-pod latency of the sequential-commit kernel for MSH_SEQ_WAVES (scanning waves, read by
msh_create: one ctx per setting) in {0 = the launcher's choice, 1, 4, 16}, with and without a
capacity (CAPS)."""
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
n = int(os.environ.get("NODES", 5000))
p = int(os.environ.get("PODS", 20000))
u, nd, pd, pt = synth.make_soa(n, p)
WAVES = os.environ.get("WAVES", "0,1,4,16").split(",")
ctxs = {}
for w in WAVES:
    os.environ["MSH_SEQ_WAVES"] = w
    ctxs[w] = msh.DeviceContext(0)
    ctxs[w].upload_nodes(u, nd)
dev = torch.device("cuda:0")
d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
oi = torch.empty(p, dtype=torch.int32, device=dev)
osc = torch.empty(p, dtype=torch.int64, device=dev)
ost = torch.empty(p, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
res = {}
caps = [int(c) for c in os.environ.get("CAPS", "0").split(",")]  # max_pods_per_node (0 = reference)
for rnd in range(4):
    for cap in caps:
        for w in WAVES:
            ctx = ctxs[w]
            ctx.reset_node_pod_counts()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            ctx.schedule_sequential_device(p, d_pd.data_ptr(), d_pt.data_ptr(), cap, oi.data_ptr(), osc.data_ptr(),
                                           ost.data_ptr(), s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            if rnd:
                res.setdefault((cap, w), []).append(e0.elapsed_time(e1))
for (cap, w), t in res.items():
    ms = float(np.median(t))
    print(json.dumps({"seq_waves": w, "max_pods_per_node": cap, "nodes": n, "pods": p, "ms": ms,
                      "us_per_pod": ms * 1e3 / p, "evals_per_s": n * p / (ms * 1e-3)}))
