"""End-to-end rates around the device path at C3 (5,000 nodes, 100,000 pods per batch).

* host_buffers: msh_schedule_batch on host numpy arrays: the 2 B/pod inputs go to the device
  and the 16 B/pod outputs come back over PCIe every batch (the PCIe-inclusive rate that
  DESIGN.md quotes beside bench.py's HBM-resident `value`).
* loop: SchedulingLoop.schedule_once over a freshly filled activeQ of 100,000 informer pod
  objects: queue drain, node-cache check, host-buffer device call, ErrorFunc requeue of the
  failures, Permit/Bind hand-off of the placements (Python host side, §8 f1-f3).
Prints one JSON line per measurement. Not part of bench.py's contract.
"""
import importlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
L = importlib.import_module("mini-kube-scheduler_amd.loop")
S = importlib.import_module("mini-kube-scheduler_amd.scheduler")

N_NODES, P = 5000, 100_000
u, nd, pd, pt = synth.make_soa(N_NODES, P)

ctx = msh.DeviceContext(0)
ctx.upload_nodes(u, nd)
for _ in range(3):
    ctx.schedule_batch(pd, pt)
K = 30
t0 = time.perf_counter()
for _ in range(K):
    ctx.schedule_batch(pd, pt)
dt = (time.perf_counter() - t0) / K
print(json.dumps({"what": "host_buffers (msh_schedule_batch, PCIe in and out)", "nodes": N_NODES, "pods": P,
                  "us_per_batch": dt * 1e6, "pods_per_s": P / dt, "evals_per_s": N_NODES * P / dt}), flush=True)

TOL = [{"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"}]
nodes = [{"metadata": {"name": f"node{i}"}, "spec": {"unschedulable": bool(u_)}}
         for i, u_ in zip(range(N_NODES), u)]


def pods(k):
    out = []
    for j in range(P):
        d = int(pd[j])
        name = f"pod{k}-{j}{d}" if d >= 0 else f"pod{k}-{j}-x"
        out.append({"metadata": {"name": name, "namespace": "default"},
                    "spec": {"tolerations": TOL if pt[j] else []}})
    return out


class Clock:
    t = 1000.0

    def __call__(self):
        return self.t


clock = Clock()
loop = L.SchedulingLoop(S.Scheduler(ctx=ctx), clock=clock, max_batch=P, bind=lambda pod, node: None)
for n in nodes:
    loop.on_node_add(n)
rows = []
for k in range(4):
    batch = pods(k)
    t_add = time.perf_counter()
    loop.on_pods_add(batch)
    t0 = time.perf_counter()
    r = loop.schedule_once()
    t1 = time.perf_counter()
    clock.t += 20.0  # every Permit wait (<= 9 s) falls due: the next cycle binds them
    rows.append({"add_s": t0 - t_add, "cycle_s": t1 - t0, "pods": len(r), **r.counts()})
best = min(rows[1:], key=lambda x: x["cycle_s"])
print(json.dumps({"what": "loop (SchedulingLoop.schedule_once: drain + device + requeue + Permit hand-off)",
                  "nodes": N_NODES, "pods": best["pods"], "cycle_ms": best["cycle_s"] * 1e3,
                  "pods_per_s": best["pods"] / best["cycle_s"], "informer_add_ms": best["add_s"] * 1e3,
                  "counts": {k: best[k] for k in ("placed", "fit_error", "score_error")}}), flush=True)
loop.close()
