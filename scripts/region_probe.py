"""Where the driver's K = 20 region goes (bench.py's timed region, one launch of 20 C3 batches): host time
of the msh_schedule_batches_device call, then the wait in torch.cuda.synchronize(), against the kernel's
own duration (msh_timing_begin events). Medians over R repeats. Prints one JSON line.
Usage: python scripts/region_probe.py [R] [idle seconds before each region]"""
import ctypes
import importlib
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 200
K = 20
n, p = 5000, 100_000
dev = torch.device("cuda:0")
ctx = msh.DeviceContext(0)
ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 3, msh.Normalize(1))])
u, nd = synth.make_nodes(n)[1:]
ctx.upload_nodes(u, nd)
pd_all, pt_all = synth._make_pods_fast(p * K, synth.SEED)[1:]
bufs = []
for i in range(K):
    pd, pt = pd_all[i * p:(i + 1) * p], pt_all[i * p:(i + 1) * p]
    bufs.append([torch.from_numpy(np.ascontiguousarray(pd)).to(dev), torch.from_numpy(np.ascontiguousarray(pt)).to(dev),
                 torch.empty(p, dtype=torch.int32, device=dev), torch.empty(p, dtype=torch.int64, device=dev),
                 torch.empty(p, dtype=torch.int32, device=dev)])
descs = ctx.batch_descs([(p, *[t.data_ptr() for t in b]) for b in bufs])
addr = ctypes.addressof(descs)
fast, handle = ctx._fast, ctx._hv()
sh = torch.cuda.current_stream(dev).cuda_stream
for _ in range(10):
    fast.schedule_batches_device(handle, K, addr, sh or None)
torch.cuda.synchronize()
call, wait, region = [], [], []
# SYNC=stream: wait for the launch stream only (torch.cuda.current_stream().synchronize()), to separate the
# device-wide synchronize's own cost from the launch's completion latency
sync = torch.cuda.current_stream(dev).synchronize if __import__("os").environ.get("SYNC") == "stream" else torch.cuda.synchronize
gap = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # seconds of host idle before each region
for _ in range(R):
    torch.cuda.synchronize()
    if gap:
        time.sleep(gap)
    t0 = time.perf_counter()
    fast.schedule_batches_device(handle, K, addr, sh or None)
    t1 = time.perf_counter()
    sync()
    t2 = time.perf_counter()
    call.append(t1 - t0)
    wait.append(t2 - t1)
    region.append(t2 - t0)
ctx.timing_begin(R)
for _ in range(R):
    fast.schedule_batches_device(handle, K, addr, sh or None)
n_t, tot, _ = ctx.timing_end()
torch.cuda.synchronize()
med = lambda xs: float(np.median(xs)) * 1e6
pct = lambda xs, q: float(np.percentile(xs, q)) * 1e6
print(json.dumps({"batches_per_launch": K, "repeats": R, "host_call_us": med(call), "sync_wait_us": med(wait),
                  "region_us": med(region), "kernel_us": tot / max(n_t, 1) * 1e3,
                  "region_minus_kernel_us": med(region) - tot / max(n_t, 1) * 1e3,
                  "region_us_p10_p90_max": [pct(region, 10), pct(region, 90), max(region) * 1e6],
                  "region_us_first10": [round(x * 1e6, 1) for x in region[:10]]}))
