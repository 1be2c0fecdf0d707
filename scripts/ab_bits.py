"""A/B of the bit-sliced batch kernel's slice count (MSH_BITS_SLICES, read at msh_create; 0 = the
launcher's choice): per-batch time over K back-to-back launches on 1 and 2 HIP streams, several
BASELINE shapes and normalize modes. Outputs of every variant are compared with the default's
(bit-exact). One JSON line per (config, slices, streams). The packed-16 kernels this replaced
were measured against it in profiles/ab/r2_ab_bits_vs_legacy.jsonl."""
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
dev = torch.device("cuda:0")
K = int(os.environ.get("K", 100))
CONFIGS = [  # nodes, pods, normalize, weight
    (5000, 100_000, 0, 1), (5000, 100_000, 1, 3), (5000, 100_000, 3, 1), (1000, 10_000, 0, 1),
    (5000, 800_000, 0, 1), (100_000, 1_000_000, 0, 1), (100_000, 512, 0, 1), (20_000, 4096, 2, 1),
]
if os.environ.get("CONFIGS"):
    CONFIGS = [tuple(int(x) for x in c.split(":")) for c in os.environ["CONFIGS"].split(",")]
SLICES = [s for s in os.environ.get("SLICES", "0").split(",")]


def make_ctx(kernel, slices, n, norm, weight):
    os.environ["MSH_BITS_SLICES"] = slices
    ctx = msh.DeviceContext(0)
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, weight, msh.Normalize(norm))])
    u, nd = synth.make_nodes(n)[1:]
    ctx.upload_nodes(u, nd)
    return ctx


def timed(ctx, bufs, p, ns, streams):
    main = streams[0]
    ev = torch.cuda.Event()
    ev.record(main)
    for s in streams[1:ns]:
        s.wait_event(ev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for k in range(K):
        b = bufs[k % ns]
        ctx.schedule_batch_device(p, b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), b[3].data_ptr(),
                                  b[4].data_ptr(), streams[k % ns].cuda_stream)
    for s in streams[1:ns]:
        e = torch.cuda.Event()
        e.record(s)
        main.wait_event(e)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K


streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(1)]
for n, p, norm, weight in CONFIGS:
    pd_all, pt_all = synth._make_pods_fast(2 * p, synth.SEED)[1:]
    bufs = []
    for i in range(2):
        bufs.append((torch.from_numpy(np.ascontiguousarray(pd_all[i * p:(i + 1) * p])).to(dev),
                     torch.from_numpy(np.ascontiguousarray(pt_all[i * p:(i + 1) * p])).to(dev),
                     torch.empty(p, dtype=torch.int32, device=dev), torch.empty(p, dtype=torch.int64, device=dev),
                     torch.empty(p, dtype=torch.int32, device=dev)))
    outs = {}
    for kernel, sl in [("bits", "0")] + [("bits", s) for s in SLICES if s != "0"]:
        ctx = make_ctx(kernel, sl, n, norm, weight)
        for ns in (1, 2):
            timed(ctx, bufs, p, ns, streams)
            ms = float(np.median([timed(ctx, bufs, p, ns, streams) for _ in range(5)]))
            print(json.dumps({"kernel": kernel, "slices": sl, "nodes": n, "pods": p, "normalize": norm, "weight": weight,
                              "streams": ns, "ms_per_batch": ms, "evals_per_s": n * p / (ms * 1e-3)}), flush=True)
        torch.cuda.synchronize()
        outs[(kernel, sl)] = tuple(t.cpu().numpy() for t in bufs[0][2:])
        ctx.close()
    ref = outs[("bits", "0")]
    for key, o in outs.items():
        same = all((a == b).all() for a, b in zip(o, ref))
        print(json.dumps({"check": "same outputs as the default slices", "kernel": key[0], "slices": key[1], "nodes": n,
                          "pods": p, "normalize": norm, "ok": bool(same)}), flush=True)
