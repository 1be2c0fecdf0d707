"""A/B of seq_kernel at C5 (5,000 nodes x 100,000 pods, bench.py's snapshot, the headline plugin list):
per-launch kernel time (msh_timing_begin / _end, the kernel-trace interval) of the pod-block form for every
msh_options.seq_pod_waves value, the one-workgroup serial form, and the capacity form (15 pods per node,
the reference list; counts reset before each launch). Each variant is checked against the batch result
(or, with a capacity, against tests/closed_form.closed_form_capacity). One JSON line per variant."""
from __future__ import annotations

import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
from closed_form import closed_form_capacity, closed_form_modes  # noqa: E402

n, p = 5000, 100_000
u, nd, pd, pt = synth.make_soa(n, p)
dev = torch.device("cuda:0")
d = [torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev), torch.empty(p, dtype=torch.int32, device=dev),
     torch.empty(p, dtype=torch.int64, device=dev), torch.empty(p, dtype=torch.int32, device=dev)]
s = torch.cuda.current_stream().cuda_stream
R = int(sys.argv[1]) if len(sys.argv) > 1 else 20


def run(name, options, w, norm, cap, reps):
    ctx = msh.DeviceContext(0, options)
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, w, msh.Normalize(norm))])
    ctx.upload_nodes(u, nd)
    launch = lambda: ctx.schedule_sequential_device(p, d[0].data_ptr(), d[1].data_ptr(), cap, *[t.data_ptr() for t in d[2:]], s)
    launch()
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        if cap:
            ctx.reset_node_pod_counts()
        ctx.timing_begin(1)
        launch()
        k, tot, _ = ctx.timing_end()
        times.append(tot / max(k, 1))
    got = tuple(t.cpu().numpy() for t in d[2:])
    want = closed_form_capacity(u, nd, pd, pt, w, cap)[:3] if cap else closed_form_modes(u, nd, pd, pt, w, norm)
    ok = all((g == x).all() for g, x in zip(got, want))
    print(json.dumps({"variant": name, "us_avg": 1e3 * float(np.mean(times)), "us_min": 1e3 * float(np.min(times)),
                      "launches": reps, "check": "ok" if ok else "MISMATCH"}), flush=True)
    ctx.close()


for pw in (1, 2, 4, 8):
    run(f"blocks_pod_waves_{pw}", {"seq_pod_waves": pw}, 3, 1, 0, R)
run("serial", {"seq_split": "serial"}, 3, 1, 0, 3)
run("capacity15", None, 1, 0, 15, 3)
