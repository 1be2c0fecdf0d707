"""Rates of the widened §8 rows on the device side (f2 node-table deltas, f4 result export).

* f2: msh_patch_nodes for k changed nodes (a cordon flip: Spec.Unschedulable toggled, List order
  unchanged) against a full msh_upload_nodes of the table, at 5k and 100k nodes. Both are
  synchronous (they return with the table re-prepared), so host wall time is the cost.
* f4: msh_export_results (the per-pair filter verdict, raw and final score matrices the
  simulator's result store turns into annotations), pairs/s into host buffers.
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


def timed(fn, k):
    fn()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return (time.perf_counter() - t0) / k


ctx = msh.DeviceContext(0)
for n in (5000, 100_000):
    u, nd, pd, pt = synth.make_soa(n, 1000)
    ctx.upload_nodes(u, nd)
    full = timed(lambda: ctx.upload_nodes(u, nd), 50)
    rng = np.random.default_rng(n)
    for k in (1, 64, 1024):
        idx = rng.choice(n, k, replace=False).astype(np.int32)
        flip = [(1 - u[idx]).astype(np.uint8), u[idx].astype(np.uint8)]
        state = [0]

        def patch():
            ctx.patch_nodes(idx, flip[state[0]], nd[idx])
            state[0] ^= 1

        t = timed(patch, 50)
        print(json.dumps({"row": "f2 msh_patch_nodes", "nodes": n, "changed": k, "us": t * 1e6,
                          "full_upload_us": full * 1e6}), flush=True)

u, nd, pd, pt = synth.make_soa(5000, 1000)
ctx.upload_nodes(u, nd)
t = timed(lambda: ctx.export_results(pd, pt), 5)
pairs = 5000 * 1000
print(json.dumps({"row": "f4 msh_export_results", "nodes": 5000, "pods": 1000, "ms": t * 1e3,
                  "pairs_per_s": pairs / t, "bytes_to_host": pairs * 17}), flush=True)
ctx.close()
