"""C5 without a capacity (5,000 nodes x 100,000 pods, the headline list), each no-capacity form timed three
ways on one box: msh_timing events per launch (what bench.py's kernel_ms uses), the wall clock of R
back-to-back launches between two synchronizes (per launch), and torch events around the same R launches.
Prints one JSON line per form and method. Usage: python3 scripts/c5_timing.py [R]"""
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
R = int(sys.argv[1]) if len(sys.argv) > 1 else 200
n, p = 5000, 100_000
u, nd, pd, pt = synth.make_soa(n, p)
dev = torch.device("cuda:0")
bufs = [torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev), torch.empty(p, dtype=torch.int32, device=dev),
        torch.empty(p, dtype=torch.int64, device=dev), torch.empty(p, dtype=torch.int32, device=dev)]
s = torch.cuda.current_stream().cuda_stream
for form in ("auto", "blocks", "auto", "blocks"):
    ctx = msh.DeviceContext(0, None if form == "auto" else {"seq_split": form})
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, 3, msh.Normalize(1))])
    ctx.upload_nodes(u, nd)
    seq = lambda: ctx.schedule_sequential_device(p, bufs[0].data_ptr(), bufs[1].data_ptr(), 0,
                                                 *[t.data_ptr() for t in bufs[2:]], s)
    for _ in range(10):
        seq()
    torch.cuda.synchronize()
    ctx.timing_begin(R)
    for _ in range(R):
        seq()
    nt, tot, mx = ctx.timing_end()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(R):
        seq()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / R
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(R):
        seq()
    e1.record()
    torch.cuda.synchronize()
    seq_span = e0.elapsed_time(e1) / R * 1e3
    e0.record()
    for _ in range(R):
        ctx.schedule_batch_device(p, *[t.data_ptr() for t in bufs], s)
    e1.record()
    torch.cuda.synchronize()
    batch_span = e0.elapsed_time(e1) / R * 1e3
    hc = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        seq()
        hc.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    hb = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.schedule_batch_device(p, *[t.data_ptr() for t in bufs], s)
        hb.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    print(json.dumps({"form": form, "host_call_us_seq": sorted(hc)[25] * 1e6, "host_call_us_batch": sorted(hb)[25] * 1e6, "events_us": tot / max(nt, 1) * 1e3, "events_max_us": mx * 1e3,
                      "wall_us_per_launch": wall * 1e6, "torch_events_us_per_launch": seq_span,
                      "batch_torch_events_us_per_launch": batch_span}),
          flush=True)
    ctx.close()
