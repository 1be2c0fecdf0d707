"""Interleaved A/B of libminisched_hip.so build variants in ONE process (guide rule 24).

Usage: python scripts/ab_libs.py <lib.so> [<lib.so> ...]   (first = reference for the outputs)

Each variant is loaded as its own ctypes handle (its own code object and context), gets the
same C3 node table and pod batch, and is timed round-robin: `LAUNCHES` back-to-back launches
on one stream (isolated per-launch time) and the same number alternating over two streams
(pipelined). Outputs of every variant are compared with the first library's; a variant tagged
`diag` in its file name is a timing diagnostic whose outputs are not checked.
Prints one JSON line per variant. Tuning tool only: never part of the product path.
"""
import ctypes as C
import importlib
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")

n = int(os.environ.get("NODES", 5000))
p = int(os.environ.get("PODS", 100000))
rounds = int(os.environ.get("ROUNDS", 12))
launches = int(os.environ.get("LAUNCHES", 20))
libs = [Path(a) for a in sys.argv[1:]]
assert libs, "give at least one library"

u, nd, pd, pt = synth.make_soa(n, p)
dev = torch.device("cuda:0")
d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


class Variant:
    def __init__(self, path: Path):
        self.path = path
        self.lib = C.CDLL(str(path))
        self.ctx = C.c_void_p()
        assert self.lib.msh_create(0, C.byref(self.ctx)) == 0, "msh_create"
        rc = self.lib.msh_upload_nodes(self.ctx, C.c_int32(n), u.ctypes.data_as(C.c_void_p),
                                       nd.ctypes.data_as(C.c_void_p))
        assert rc == 0, f"upload {rc}"
        # two output sets (one per stream)
        self.out = [(torch.empty(p, dtype=torch.int32, device=dev), torch.empty(p, dtype=torch.int64, device=dev),
                     torch.empty(p, dtype=torch.int32, device=dev)) for _ in range(2)]
        self.iso, self.pipe = [], []

    def launch(self, k: int, stream):
        oi, osc, ost = self.out[k]
        rc = self.lib.msh_schedule_batch_device(
            self.ctx, C.c_int32(p), C.c_void_p(d_pd.data_ptr()), C.c_void_p(d_pt.data_ptr()),
            C.c_void_p(oi.data_ptr()), C.c_void_p(osc.data_ptr()), C.c_void_p(ost.data_ptr()),
            C.c_void_p(stream.cuda_stream))
        assert rc == 0, f"{self.path.name}: schedule rc={rc}"


vs = [Variant(pth) for pth in libs]
main = torch.cuda.current_stream()
for rnd in range(rounds):
    for v in vs:
        # isolated: back to back on one stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(streams[0]):
            e0.record()
            for _ in range(launches):
                v.launch(0, streams[0])
            e1.record()
        torch.cuda.synchronize()
        # pipelined: alternate two streams forked from / joined into streams[0]
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record(streams[0])
        streams[1].wait_event(f0)
        for i in range(launches):
            v.launch(i & 1, streams[i & 1])
        j = torch.cuda.Event()
        j.record(streams[1])
        streams[0].wait_event(j)
        f1.record(streams[0])
        torch.cuda.synchronize()
        if rnd >= 2:
            v.iso.append(e0.elapsed_time(e1) / launches)
            v.pipe.append(f0.elapsed_time(f1) / launches)

ref = [t.cpu() for t in vs[0].out[0]]
for v in vs:
    ok = None
    if "diag" not in v.path.name:
        ok = all(torch.equal(a.cpu(), b) for k in range(2) for a, b in zip(v.out[k], ref))
    iso, pipe = np.median(v.iso), np.median(v.pipe)
    print(json.dumps({"lib": v.path.name, "nodes": n, "pods": p, "iso_us": iso * 1e3, "pipe_us": pipe * 1e3,
                      "iso_min_us": float(np.min(v.iso)) * 1e3, "pipe_min_us": float(np.min(v.pipe)) * 1e3,
                      "evals_per_s_pipe": n * p / (pipe * 1e-3), "same_outputs": ok}), flush=True)
