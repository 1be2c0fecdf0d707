"""RCCL on the device: the collectives the N > 1 paths issue, run through the "nccl" (RCCL) process
group on the one-GPU box at world size 1.

A one-GPU box cannot host two RCCL ranks, and distributed.py skips its collectives at world size 1 (an
all-reduce over one rank is the identity). So this test calls dist.all_reduce itself, on the same device
buffers, dtypes, ops and stream scopes that the N > 1 paths use:

* NodeShardedScheduler (BASELINE C4 shape): int32 keys from msh_shard_keys_device, all_reduce MAX on a
  busy non-default stream, then msh_decode_keys_device on that stream;
* GenericNodeShardedScheduler: int64 extents MAX, int64 totals MAX and int32 indices MIN between its five
  launches;
* PodShardedScheduler.merge_node_counts: int32 node counts SUM;
* bench.py's max-over-ranks timing: a float64 all_reduce MAX, and dist.barrier().

Every decision is compared with the oracle (oracle/msh_oracle.c, the restatement of
minisched/minisched.go:115-199, 304-325). The check is that RCCL initialises on MI355X under this image's
environment and that each collective leaves its buffer intact and ordered on the stream the kernels run on.
It says nothing about cross-GPU bandwidth; that comes from the driver's 8-GPU SCALE run.
"""
from __future__ import annotations

import importlib
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(port, out_q):
    try:
        import torch
        import torch.distributed as dist
        sys.path.insert(0, str(ROOT))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        msh = importlib.import_module("mini-kube-scheduler_amd")
        D = importlib.import_module("mini-kube-scheduler_amd.distributed")
        oracle = importlib.import_module("oracle.oracle")
        res = {"backend": dist.get_backend()}
        rng = np.random.default_rng(20261018)
        n, p = 5000, 20_000
        u = (rng.random(n) < 0.3).astype(np.uint8)
        nd = rng.integers(-1, 10, n).astype(np.int8)
        pd = rng.integers(-1, 10, p).astype(np.int8)
        pt = (rng.random(p) < 0.2).astype(np.uint8)
        d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
        side = torch.cuda.Stream(dev)
        busy = torch.randn(4096, 4096, device=dev)

        def same(got, want):
            return all(bool((np.asarray(g) == np.asarray(x)).all()) for g, x in zip(got, want[:3]))

        # ---- node-shard keys: int32 MAX between the keys kernel and the decode, on a busy side stream
        for norm in (0, 2):  # NONE (identity keys), MINMAX (non-match keys)
            ctx = msh.DeviceContext(0)
            ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                            [msh.ScorePluginConfig(msh.NODE_NUMBER, 2, msh.Normalize(norm))])
            ctx.upload_nodes(u, nd)
            keys = torch.empty(ctx.shard_keys_len(p), dtype=torch.int32, device=dev)
            oi = torch.empty(p, dtype=torch.int32, device=dev)
            osc = torch.empty(p, dtype=torch.int64, device=dev)
            ost = torch.empty(p, dtype=torch.int32, device=dev)
            with torch.cuda.stream(side):
                for _ in range(4):
                    busy = busy @ busy * 1e-3  # keep the stream busy so a mis-ordered reduce would show
                ctx.shard_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), 0, keys.data_ptr(), side.cuda_stream)
                before = keys.clone()
                dist.all_reduce(keys, op=dist.ReduceOp.MAX)
                ctx.decode_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), keys.data_ptr(), oi.data_ptr(),
                                       osc.data_ptr(), ost.data_ptr(), side.cuda_stream)
            torch.cuda.synchronize()
            ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=["NodeNumber"], score=["NodeNumber"],
                                  weights=[2], normalize=[norm])
            want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=16)
            res[f"keys_norm{norm}"] = bool(torch.equal(before, keys)) and same(
                (oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy()), want)
            ctx.close()

        # ---- the generic pipeline: int64 MAX (extents, totals) and int32 MIN (indices)
        col = rng.integers(-(1 << 31), (1 << 31) + 1, n)
        score = [msh.NODE_NUMBER, "ScoreColumn0"]
        ctx = msh.DeviceContext(0)
        ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                        [msh.ScorePluginConfig(msh.NODE_NUMBER, 3, msh.Normalize(1)),
                         msh.ScorePluginConfig("ScoreColumn0", 5, msh.Normalize(2))])
        ctx.upload_nodes(u, nd)
        ctx.upload_score_column("ScoreColumn0", col)
        n_ext = ctx.generic_ext_len(p)
        ext = torch.empty(max(n_ext, 1), dtype=torch.int64, device=dev)
        tot = torch.empty(p, dtype=torch.int64, device=dev)
        idx = torch.empty(p, dtype=torch.int32, device=dev)
        oi = torch.empty(p, dtype=torch.int32, device=dev)
        osc = torch.empty(p, dtype=torch.int64, device=dev)
        ost = torch.empty(p, dtype=torch.int32, device=dev)
        with torch.cuda.stream(side):
            ctx.generic_extents_device(p, d_pd.data_ptr(), d_pt.data_ptr(), ext.data_ptr(), side.cuda_stream)
            dist.all_reduce(ext, op=dist.ReduceOp.MAX)
            ctx.generic_best_device(p, d_pd.data_ptr(), d_pt.data_ptr(), ext.data_ptr(), 0, tot.data_ptr(),
                                    idx.data_ptr(), side.cuda_stream)
            mt = tot.clone()
            dist.all_reduce(mt, op=dist.ReduceOp.MAX)
            ctx.generic_candidates_device(p, tot.data_ptr(), mt.data_ptr(), idx.data_ptr(), side.cuda_stream)
            dist.all_reduce(idx, op=dist.ReduceOp.MIN)
            ctx.generic_decode_device(p, d_pd.data_ptr(), mt.data_ptr(), idx.data_ptr(), oi.data_ptr(),
                                      osc.data_ptr(), ost.data_ptr(), side.cuda_stream)
        torch.cuda.synchronize()
        ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=["NodeNumber"], score=score,
                              weights=[3, 5], normalize=[1, 2])
        want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=16, cols={0: col})
        res["generic"] = bool(n_ext > 0) and same((oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy()), want)
        ctx.close()

        # ---- sequential node counts: int32 SUM (merge_node_counts' collective)
        ctx = msh.DeviceContext(0)
        ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 1)])
        sched = D.PodShardedScheduler(ctx, u, nd, 1, 0)
        ctx.reset_node_pod_counts()
        ctx.schedule_sequential(pd, pt, 0)
        counts = torch.from_numpy(ctx.node_pod_counts()).to(dev)
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
        ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=["NodeNumber"], score=["NodeNumber"],
                              weights=[1], normalize=[0])
        want = oracle.c_schedule_sequential(u, nd, pd, pt, ps, 0)
        res["counts"] = bool((counts.cpu().numpy() == want[3]).all())
        ctx.close()
        del sched

        # ---- bench.py's max-over-ranks timing and its barrier
        t = torch.tensor([1.5, 2.25, 3.0], dtype=torch.float64, device=dev)
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res["timing"] = t.cpu().tolist() == [1.5, 2.25, 3.0]
        dist.destroy_process_group()
        out_q.put(res)
    except Exception as e:  # report, do not hang the parent
        out_q.put({"error": repr(e)})


def test_rccl_world1_collectives(msh, oracle):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_worker, args=(_free_port(), q))
    proc.start()
    try:
        res = q.get(timeout=100)
    finally:
        proc.join(timeout=20)
        if proc.is_alive():
            proc.kill()
            proc.join()
    assert "error" not in res, res
    assert res["backend"] == "nccl", res
    assert all(res[k] for k in ("keys_norm0", "keys_norm2", "generic", "counts", "timing")), res
