"""Interleaved A/B of one launcher env knob over batch sizes, in ONE process.

ENVVAR (e.g. MSH_WAVE_RANGE) takes each of VALUES ("-" = unset) round-robin; the launcher reads
it at every launch. For each PODS size, times 10 back-to-back msh_schedule_batch_device calls on
STREAMS streams round-robin (HIP events; default 1; 2 = bench.py's pipelining) and prints the
median per-batch us per value.
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

var = os.environ.get("ENVVAR", "MSH_WAVE_RANGE")
values = os.environ.get("VALUES", "1,0").split(",")
n = int(os.environ.get("NODES", 5000))
sizes = [int(x) for x in os.environ.get("PODS", "4096,16384,65536,100000,131072").split(",")]
ctx = msh.DeviceContext(0)
u, nd, _, _ = synth.make_soa(n, 1)
ctx.upload_nodes(u, nd)
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
n_streams = int(os.environ.get("STREAMS", 1))
streams = [s] + [torch.cuda.Stream(dev) for _ in range(n_streams - 1)]
for p in sizes:
    _, _, pd, pt = synth.make_soa(1, p)
    d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
    oi = torch.empty(p, dtype=torch.int32, device=dev)
    osc = torch.empty(p, dtype=torch.int64, device=dev)
    ost = torch.empty(p, dtype=torch.int32, device=dev)
    res = {v: [] for v in values}
    for rnd in range(15):
        for v in values:
            if v == "-":
                os.environ.pop(var, None)
            else:
                os.environ[var] = v
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for x in streams[1:]:
                x.wait_event(e0)
            for k in range(10):  # the batches share outputs: timing only
                ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(),
                                          ost.data_ptr(), streams[k % n_streams].cuda_stream)
            for x in streams[1:]:
                s.wait_stream(x)
            e1.record(s)
            torch.cuda.synchronize()
            if rnd >= 2:
                res[v].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(json.dumps({"env": var, "nodes": n, "pods": p, "streams": n_streams,
                      **{f"us[{v}]": round(float(np.median(res[v])), 2) for v in values}}), flush=True)
ctx.close()
