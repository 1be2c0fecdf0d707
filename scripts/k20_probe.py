"""Where a K=20 bench region goes (the driver's command: 20 C3 batches, one launch of 20): host-side
timestamps around each call of the timed region and the device-side spans (the region's events, the
kernel's own start / stop from msh_timing_*). One JSON line per repetition."""
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
K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
ctx = msh.DeviceContext(0)
u, nd = synth.make_nodes(5000)[1:]
ctx.upload_nodes(u, nd)
p = 100_000
G = msh._native.BATCHES_PER_LAUNCH
pd_all, pt_all = synth._make_pods_fast(p * G, synth.SEED)[1:]
bufs = []
for i in range(G):
    pd, pt = pd_all[i * p:(i + 1) * p], pt_all[i * p:(i + 1) * p]
    bufs.append([torch.from_numpy(np.ascontiguousarray(pd)).to(dev), torch.from_numpy(np.ascontiguousarray(pt)).to(dev),
                 torch.empty(p, dtype=torch.int32, device=dev), torch.empty(p, dtype=torch.int64, device=dev),
                 torch.empty(p, dtype=torch.int32, device=dev)])
descs = ctx.batch_descs([(p, *[t.data_ptr() for t in b]) for b in bufs])
import ctypes
addr = ctypes.addressof(descs)
fast, h = ctx._fast, ctx._hv()
stream = torch.cuda.current_stream(dev)
sh = stream.cuda_stream


def submit(k):
    for i0 in range(0, k, G):
        rc = fast.schedule_batches_device(h, min(G, k - i0), addr, sh or None)
        assert rc == 0


submit(5)
torch.cuda.synchronize()
r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for e in (r0, r1):
    e.record(stream)
torch.cuda.synchronize()
for rep in range(8):
    torch.cuda.synchronize()
    time.sleep(0.001)
    ctx.timing_begin(4)
    t0 = time.perf_counter()
    r0.record(stream)
    t1 = time.perf_counter()
    submit(K)
    t2 = time.perf_counter()
    r1.record(stream)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    n, tot, mx = ctx.timing_end()
    us = lambda a, b: round((b - a) * 1e6, 2)
    print(json.dumps({"K": K, "rep": rep, "host_total_us": us(t0, t4), "record_r0_us": us(t0, t1), "submit_us": us(t1, t2),
                      "record_r1_us": us(t2, t3), "sync_us": us(t3, t4), "device_region_us": round(r0.elapsed_time(r1) * 1e3, 2),
                      "kernel_us": round(tot * 1e3, 2), "launches": n}), flush=True)
# the same without the events in the region (host clock only)
for rep in range(4):
    torch.cuda.synchronize()
    time.sleep(0.001)
    t0 = time.perf_counter()
    submit(K)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"K": K, "rep": rep, "no_events": True, "submit_us": round((t1 - t0) * 1e6, 2),
                      "host_total_us": round((t2 - t0) * 1e6, 2)}), flush=True)
ctx.close()
