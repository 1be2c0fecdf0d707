"""Experiment: can two ranks of the library's own RCCL communicator share one GPU (msh_comm_init with
world 2 from two processes on cuda:0)? If RCCL allows it, the node-sharded path of msh_schedule_nodeshard
runs a real two-rank all-reduce on the one-GPU box. Prints one JSON line; never part of the suite."""
from __future__ import annotations

import importlib
import json
import sys
from pathlib import Path

import numpy as np
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def worker(rank, world, q_id, q_out):
    try:
        sys.path.insert(0, str(ROOT))
        msh = importlib.import_module("mini-kube-scheduler_amd")
        D = importlib.import_module("mini-kube-scheduler_amd.distributed")
        if rank == 0:
            cid = msh.DeviceContext.comm_unique_id()
            for _ in range(world - 1):
                q_id.put(cid)
        else:
            cid = q_id.get(timeout=30)
        rng = np.random.default_rng(7)
        n, p = 6000, 20_000
        u = (rng.random(n) < 0.3).astype(np.uint8)
        nd = rng.integers(-1, 10, n).astype(np.int8)
        pd = rng.integers(-1, 10, p).astype(np.int8)
        pt = (rng.random(p) < 0.2).astype(np.uint8)
        lo, hi = D.shard_range(n, world, rank)
        with msh.DeviceContext(0) as ctx:
            ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 2, msh.Normalize(3))])
            ctx.upload_nodes(u[lo:hi], nd[lo:hi])
            ctx.comm_init(cid, world, rank)
            got = ctx.schedule_nodeshard(pd, pt, lo)
            q_out.put((rank, "ok", [a.tolist() for a in got]))
    except Exception as e:
        q_out.put((rank, "error", repr(e)))


def main():
    world = 2
    ctx = mp.get_context("spawn")
    q_id, q_out = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, q_id, q_out)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = {}
    try:
        for _ in range(world):
            r, st, val = q_out.get(timeout=90)
            res[r] = (st, val)
    except Exception as e:
        res["timeout"] = repr(e)
    for pr in procs:
        pr.join(timeout=10)
        if pr.is_alive():
            pr.kill()
    out = {"world": world, "status": {str(k): v[0] for k, v in res.items() if k != "timeout"}}
    if all(k in res and res[k][0] == "ok" for k in range(world)):
        sys.path.insert(0, str(ROOT))
        oracle = importlib.import_module("oracle.oracle")
        rng = np.random.default_rng(7)
        n, p = 6000, 20_000
        u = (rng.random(n) < 0.3).astype(np.uint8)
        nd = rng.integers(-1, 10, n).astype(np.int8)
        pd = rng.integers(-1, 10, p).astype(np.int8)
        pt = (rng.random(p) < 0.2).astype(np.uint8)
        want = oracle.c_schedule_batch(u, nd, pd, pt, oracle.PluginSet(weights=[2], normalize=[3]), threads=8)
        out["bit_exact_vs_oracle"] = all(all(np.array_equal(np.array(g), w) for g, w in zip(res[r][1], want[:3]))
                                         for r in range(world))
    else:
        out["detail"] = {str(k): (v if k == "timeout" else v[1]) for k, v in res.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
