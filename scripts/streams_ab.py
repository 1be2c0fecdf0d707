"""A/B: K back-to-back C3 batches on one HIP stream vs alternating over S streams (independent
batches, separate output buffers). Per-launch kernel time from rocprof is not what this measures:
it reports region time / K, the steady-state rate at which batches complete."""
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
p = int(os.environ.get("PODS", 100000))
K = int(os.environ.get("K", 200))
ctx = msh.DeviceContext(0)
u, nd = synth.make_nodes(n)[1:]
ctx.upload_nodes(u, nd)
dev = torch.device("cuda:0")
pd_all, pt_all = synth._make_pods_fast(4 * p, synth.SEED)[1:]
bufs = []
for i in range(4):
    d_pd = torch.from_numpy(np.ascontiguousarray(pd_all[i * p:(i + 1) * p])).to(dev)
    d_pt = torch.from_numpy(np.ascontiguousarray(pt_all[i * p:(i + 1) * p])).to(dev)
    bufs.append((d_pd, d_pt, torch.empty(p, dtype=torch.int32, device=dev), torch.empty(p, dtype=torch.int64, device=dev),
                 torch.empty(p, dtype=torch.int32, device=dev)))
main = torch.cuda.current_stream()
streams = [main] + [torch.cuda.Stream() for _ in range(3)]


def run(ns):
    ev = torch.cuda.Event()
    ev.record(main)
    for s in streams[1:ns]:
        s.wait_event(ev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for k in range(K):
        s = streams[k % ns]
        b = bufs[k % ns]
        ctx.schedule_batch_device(p, b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), b[3].data_ptr(),
                                  b[4].data_ptr(), s.cuda_stream)
    for s in streams[1:ns]:
        e = torch.cuda.Event()
        e.record(s)
        main.wait_event(e)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K


for ns in (1, 2, 3, 1, 2, 3):
    run(ns)
    ms = float(np.median([run(ns) for _ in range(5)]))
    print(json.dumps({"streams": ns, "nodes": n, "pods": p, "ms_per_batch": ms, "evals_per_s": n * p / (ms * 1e-3)}),
          flush=True)
