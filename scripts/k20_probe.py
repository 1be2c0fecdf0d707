"""Where the time of a short timed region goes (the driver runs bench.py --steps 20 --warmup 5):
host time after each launch of the C3 batch on 2 streams, the HIP-event time of the region, and
the wall time to the final synchronize. Several repetitions, one JSON line each."""
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
if os.environ.get("SPIN"):  # A/B: completion waits spin instead of yielding / sleeping
    import ctypes
    import importlib.util as _u
    _hip = ctypes.CDLL(str(Path(_u.find_spec("torch").submodule_search_locations[0]) / "lib" / "libamdhip64.so"),
                       mode=ctypes.RTLD_GLOBAL)
    print(json.dumps({"hipSetDeviceFlags(spin)": _hip.hipSetDeviceFlags(int(os.environ["SPIN"]))}), flush=True)
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
K = int(os.environ.get("K", 20))
NS = int(os.environ.get("STREAMS", 2))
dev = torch.device("cuda:0")
ctx = msh.DeviceContext(0)
u, nd = synth.make_nodes(5000)[1:]
ctx.upload_nodes(u, nd)
p = 100_000
pd_all, pt_all = synth._make_pods_fast(p * NS, synth.SEED)[1:]
main = torch.cuda.current_stream()
streams = [main] + [torch.cuda.Stream() for _ in range(NS - 1)]
bufs = []
for i in range(NS):
    b = [torch.from_numpy(np.ascontiguousarray(pd_all[i * p:(i + 1) * p])).to(dev),
         torch.from_numpy(np.ascontiguousarray(pt_all[i * p:(i + 1) * p])).to(dev),
         torch.empty(p, dtype=torch.int32, device=dev), torch.empty(p, dtype=torch.int64, device=dev),
         torch.empty(p, dtype=torch.int32, device=dev)]
    bufs.append(b)
fn, h = ctx._fast.schedule_batch_device, ctx._hv()
args = [(h, p, *[t.data_ptr() for t in b], st.cuda_stream or None) for b, st in zip(bufs, streams)]


r0, r1, ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), torch.cuda.Event()
jevs = [torch.cuda.Event() for _ in streams[1:]]
for e in [r0, r1, ev] + jevs:
    e.record(main)


def region(k):
    torch.cuda.synchronize()
    t = [time.perf_counter()]
    r0.record(main)
    ev.record(main)
    for st in streams[1:]:
        st.wait_event(ev)
    t.append(time.perf_counter())
    for i in range(k):
        fn(*args[i % NS])
        t.append(time.perf_counter())
    for st, e in zip(streams[1:], jevs):
        e.record(st)
        main.wait_event(e)
    r1.record(main)
    t.append(time.perf_counter())
    torch.cuda.synchronize()
    t.append(time.perf_counter())
    us = np.diff(np.array(t)) * 1e6
    return {"k": k, "streams": NS, "wall_us": (t[-1] - t[0]) * 1e6, "event_us": r0.elapsed_time(r1) * 1e3,
            "fork_us": us[0], "launch_us": [round(x, 2) for x in us[1:1 + k]], "join_us": us[1 + k],
            "sync_us": us[2 + k]}


for i in range(5):
    fn(*args[0])
torch.cuda.synchronize()
for rep in range(6):
    print(json.dumps(region(K)), flush=True)
    time.sleep(0.01 if rep % 2 else 0)
