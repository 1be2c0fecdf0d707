"""Host-buffer path rates at C3 (5,000 nodes x 100,000 pods): msh_schedule_batch with pageable
numpy buffers (staged) and with page-locked ones (msh_host_alloc), outputs written by the kernel
straight into page-locked memory (default) or DMA'd from device scratch (MSH_HOST_IO=dma), wall
time per synchronous call. Also the host cost of one msh_schedule_batch_device call from Python
(submission only, no synchronisation) against the device's per-batch time. One JSON line each."""
import importlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
n, p = 5000, 100_000
u, nd, pd, pt = synth.make_soa(n, p)
hpd, hpt = msh.pinned_empty(p, np.int8), msh.pinned_empty(p, np.uint8)
hpd[:], hpt[:] = pd, pt
pin_out = (msh.pinned_empty(p, np.int32), msh.pinned_empty(p, np.int64), msh.pinned_empty(p, np.int32))
page_out = (np.empty(p, np.int32), np.empty(p, np.int64), np.empty(p, np.int32))
for io, sync in (("zc", "stream"), ("zc2", "stream"), ("zc", "poll"), ("zc2", "poll"), ("dma", "stream")):
    os.environ["MSH_HOST_IO"] = io
    os.environ["MSH_HOST_SYNC"] = sync
    ctx = msh.DeviceContext(0)
    ctx.upload_nodes(u, nd)
    for name, args, out in (("pageable", (pd, pt), page_out), ("pinned", (hpd, hpt), pin_out)):
        for _ in range(5):
            ctx.schedule_batch(*args, out=out)
        ts = []
        for _ in range(100):
            t0 = time.perf_counter()
            ctx.schedule_batch(*args, out=out)
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts))
        print(json.dumps({"path": name, "io": io, "sync": sync, "nodes": n, "pods": p, "us_per_batch_median": med * 1e6,
                          "us_per_batch_min": min(ts) * 1e6, "pods_per_s": p / med, "evals_per_s": n * p / med}),
              flush=True)
    ctx.close()

# submission cost of the device-resident entry point from Python (ctypes) vs device time
os.environ.pop("MSH_HOST_IO", None)
os.environ.pop("MSH_HOST_SYNC", None)
ctx = msh.DeviceContext(0)
ctx.upload_nodes(u, nd)
dev = torch.device("cuda:0")
d = [torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev), torch.empty(p, dtype=torch.int32, device=dev),
     torch.empty(p, dtype=torch.int64, device=dev), torch.empty(p, dtype=torch.int32, device=dev)]
ptrs = [t.data_ptr() for t in d]
s = torch.cuda.current_stream().cuda_stream
for K in (20, 200):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.schedule_batch_device(p, *ptrs, s)
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"what": "msh_schedule_batch_device from Python", "K": K, "host_submit_us_per_call": (t1 - t0) / K * 1e6,
                      "device_us_per_batch": e0.elapsed_time(e1) / K * 1e3, "wall_us_per_batch": (t2 - t0) / K * 1e6}),
          flush=True)
