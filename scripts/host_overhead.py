"""Host-side cost per step of the bench loop (is the C3 step launch-bound?)."""
import ctypes as C
import importlib
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
N = msh._native
dev = torch.device("cuda:0")
ctx = msh.DeviceContext(0)
u, nd, pd, pt = synth.make_soa(5000, 100000)
ctx.upload_nodes(u, nd)
d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
oi = torch.empty(100000, dtype=torch.int32, device=dev)
osc = torch.empty(100000, dtype=torch.int64, device=dev)
ost = torch.empty(100000, dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream()
s = stream.cuda_stream
args = (d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(), ost.data_ptr(), s)
lib, h = N.lib(), ctx.handle
K = 2000


def host_us(fn, k=K):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / k * 1e6, (t2 - t0) / k * 1e6


out = {}
n = C.c_int32()
out["ctypes_num_nodes"] = host_us(lambda: lib.msh_num_nodes(h, C.byref(n)))
ev = torch.cuda.Event(enable_timing=True)
out["torch_event_record"] = host_us(lambda: ev.record(stream))
out["wrapper_p64"] = host_us(lambda: ctx.schedule_batch_device(64, *args))
out["raw_ctypes_p64"] = host_us(lambda: lib.msh_schedule_batch_device(h, 64, *args))
out["wrapper_p100k"] = host_us(lambda: ctx.schedule_batch_device(100000, *args), 500)
out["raw_ctypes_p100k"] = host_us(lambda: lib.msh_schedule_batch_device(h, 100000, *args), 500)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def with_events():
    e0.record(stream)
    ctx.schedule_batch_device(100000, *args)
    e1.record(stream)


out["wrapper_p100k_2events"] = host_us(with_events, 500)
for k, v in out.items():
    print(json.dumps({"what": k, "host_us_per_call": round(v[0], 2), "wall_us_per_call": round(v[1], 2)}))
