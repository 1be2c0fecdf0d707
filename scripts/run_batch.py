"""Minimal driver for profiling: K launches of a hot kernel on the C3 workload (5,000 nodes x 100,000
pods per batch, bench.py's synthetic snapshot).

MODE
  multi        bench.py's default submission: 32 independent batches per msh_schedule_batches_device
               launch (the per-pair kernel)
  batch        one msh_schedule_batch_device launch per batch
  generic      generic_kernel (explicit int64 score per pair) on the reference plugin list, 32 batches
               per launch (MSH_BATCH_KERNEL=generic is set here)
  generic_col  generic_kernel on NodeNumber + ScoreColumn0 (weight 2, DefaultNormalizeScore), 32 batches
               per launch (bench.py's generic.nodenumber_plus_default_column)
  generic_2col generic_kernel's general form: NodeNumber + a DEFAULT and a MIN-MAX column, 32 batches per launch
  generic_w64  generic_kernel's 64-bit form: NodeNumber + ScoreColumn0 over the whole int32 range (COLNORM:
               the column's normalizer), 32 batches per launch
  sequential   C5: no capacity, auto: the per-pair kernel with the commit epilogue (SPLIT=blocks: seq_kernel's
               64-pod blocks; SPLIT=serial: the whole batch in one workgroup, in order; CAP=k: a capacity of k
               pods per node, the counts reset before every launch)
NORM / WEIGHT: msh_normalize and weight of the NodeNumber entry (bench.py's headline: WEIGHT=3 NORM=1).
NB: batches per launch in the multi-batch modes (default 32).
Kernel overrides go to msh_create_ex as msh_options (the library reads no environment variable)."""
import importlib
import os
import sys
from pathlib import Path

import numpy as np

mode = os.environ.get("MODE", "multi")
options = {}
if mode == "generic":
    options["batch_kernel"] = "generic"
if os.environ.get("SPLIT", "auto") in ("serial", "blocks"):
    options["seq_split"] = os.environ["SPLIT"]
if os.environ.get("PAIR_PLANES"):
    options["pair_planes"] = os.environ["PAIR_PLANES"]  # msh_options.pair_planes: auto, sgpr, lds
if os.environ.get("PAIR_SLICES"):
    options["pair_slices"] = int(os.environ["PAIR_SLICES"])  # msh_options.pair_slices: 1, 2, 4 slice waves per block
if os.environ.get("SEQ_WAVES"):
    options["seq_waves"] = os.environ["SEQ_WAVES"]  # msh_options.seq_waves: 1, 4, 15, 16 scanning waves
cap = int(os.environ.get("CAP", 0))

import torch  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
msh = importlib.import_module("mini-kube-scheduler_amd")
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
n = int(os.environ.get("NODES", 5000))
p = int(os.environ.get("PODS", 100000))
k = int(os.environ.get("LAUNCHES", 20))
norm = int(os.environ.get("NORM", 0))
weight = int(os.environ.get("WEIGHT", 1))
ctx = msh.DeviceContext(0, options or None)
u, nd, pd, pt = synth.make_soa(n, p)
ctx.upload_nodes(u, nd)
if mode == "generic_col":
    ctx.upload_score_column(msh.SCORE_COLUMNS[0], (np.arange(n, dtype=np.int64) * 7919) % 1000 - 300)
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, 1, msh.Normalize(norm)),
                     msh.ScorePluginConfig(msh.SCORE_COLUMNS[0], 2, msh.Normalize(1))])
elif mode == "generic_2col":
    # two normalizing columns of small range: generic_kernel's general form (a runtime column count)
    ctx.upload_score_column(msh.SCORE_COLUMNS[0], (np.arange(n, dtype=np.int64) * 7919) % 1000 - 300)
    ctx.upload_score_column(msh.SCORE_COLUMNS[1], (np.arange(n, dtype=np.int64) * 104729) % 101)
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, 1, msh.Normalize(norm)),
                     msh.ScorePluginConfig(msh.SCORE_COLUMNS[0], 2, msh.Normalize(1)),
                     msh.ScorePluginConfig(msh.SCORE_COLUMNS[1], 1, msh.Normalize(3))])
elif mode == "generic_w64":
    # a column over the whole int32 range: no 32-bit bound, generic_kernel's 64-bit general form
    ctx.upload_score_column(msh.SCORE_COLUMNS[0], ((np.arange(n, dtype=np.int64) * 2654435761) % (1 << 32)) - (1 << 31))
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, 1, msh.Normalize(norm)),
                     msh.ScorePluginConfig(msh.SCORE_COLUMNS[0], 1, msh.Normalize(int(os.environ.get("COLNORM", 0))))])
else:
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, weight, msh.Normalize(norm))])
dev = torch.device("cuda:0")
nb = int(os.environ.get("NB", msh._native.BATCHES_PER_LAUNCH)) if mode in ("multi", "generic", "generic_col", "generic_w64", "generic_2col") else 1
bufs = [(torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev), torch.empty(p, dtype=torch.int32, device=dev),
         torch.empty(p, dtype=torch.int64, device=dev), torch.empty(p, dtype=torch.int32, device=dev))
        for _ in range(nb)]
descs = ctx.batch_descs([(p, *[t.data_ptr() for t in b]) for b in bufs])
s = torch.cuda.current_stream().cuda_stream
b = bufs[0]
for _ in range(k):
    if nb > 1:
        ctx.schedule_batches_device(descs, nb, s)
    elif mode == "batch":
        ctx.schedule_batch_device(p, *[t.data_ptr() for t in b], s)
    else:
        if cap:
            ctx.reset_node_pod_counts()
        ctx.schedule_sequential_device(p, b[0].data_ptr(), b[1].data_ptr(), cap, *[t.data_ptr() for t in b[2:]], s)
torch.cuda.synchronize()
print("ok", n, p, k, mode, nb, os.environ.get("MSH_BATCH_KERNEL", "pair"), f"NodeNumber w={weight} norm={norm}")
