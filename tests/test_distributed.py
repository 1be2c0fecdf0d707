"""Multi-process (gloo, world_size 2 and 3) tests of the N>1 paths, on CPU.

The device kernels cannot run here, so each rank's per-shard results are produced on that rank's
node slice by a numpy restatement of the C-ABI contract (test infrastructure):
* msh_shard_keys_device (reference plugins): per pod the first feasible match and first feasible
  non-match of the slice, as 0x7FFFFFFF - global_idx (ABI v7 layout: 2p int32 keys);
* msh_generic_extents_device / msh_generic_best_device / _candidates / _decode (any plugin list):
  per pod the extents of the normalizing plugins over the slice, then its best (total, global index).
What is tested is the product's sharding arithmetic and collectives (merge_shard_keys_ = all_reduce
MAX; GenericNodeShardedScheduler's MAX / MAX / MIN all-reduces): the merged results must equal the
unsharded oracle's answer exactly. The GPU side of the same contracts is
tests/test_gpu_parity.py::test_node_shards_merge and tests/test_distributed_gpu.py.
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

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _case(seed, n, p):
    rng = np.random.default_rng(seed)
    u = (rng.random(n) < 0.4).astype(np.uint8)
    nd = rng.integers(-1, 10, n).astype(np.int8)
    pd = rng.integers(-1, 10, p).astype(np.int8)
    pt = (rng.random(p) < 0.3).astype(np.uint8)
    return u, nd, pd, pt


def _shard_keys_oracle(dist_mod, u, nd, pd, pt, lo, hi):
    """Per-shard keys exactly as msh_shard_keys_device defines them (ABI v7) for NONE normalize: p
    first feasible match keys, then p first feasible node keys, both per pod (REVERSE / MINMAX put the
    first feasible NON-match in the second slot; the decode below reads either form)."""
    us, ns = u[lo:hi], nd[lo:hi]
    p = len(pd)
    fm = np.full(p, -1, np.int64)
    fx = np.full(p, -1, np.int64)
    for j in range(p):
        feas = np.ones(hi - lo, bool) if pt[j] else (us == 0)
        m = feas & (ns == pd[j]) & (pd[j] >= 0)
        x = feas
        if m.any():
            fm[j] = lo + int(np.argmax(m))
        if x.any():
            fx[j] = lo + int(np.argmax(x))
    return np.concatenate([dist_mod.encode_key(fm), dist_mod.encode_key(fx)])


def _worker(rank, world, port, seed, n, p, out_q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = importlib.import_module("mini-kube-scheduler_amd.distributed")
    O = importlib.import_module("oracle.oracle")
    u, nd, pd, pt = _case(seed, n, p)
    lo, hi = D.shard_range(n, world, rank)
    keys = torch.from_numpy(_shard_keys_oracle(D, u, nd, pd, pt, lo, hi))
    D.merge_shard_keys_(keys)
    k = keys.numpy()
    assert keys.dtype == torch.int32 and len(k) == 2 * p
    im, ix = D.decode_key(k[:p]), D.decode_key(k[p:])
    ia = np.where(im < 0, ix, np.where(ix < 0, im, np.minimum(im, ix)))  # first feasible node
    # decode exactly as decode_pod (NONE mode, reference plugin set)
    idx = np.where(ia < 0, -1, np.where(pd < 0, -1, np.where(im >= 0, im, ia)))
    status = np.where(ia < 0, 1, np.where(pd < 0, 2, 0))
    score = np.where((status == 0) & (im >= 0), 10, 0)
    # pod sharding: every rank schedules its slice; gather reassembles the batch
    plo, phi = D.shard_range(p, world, rank)
    gi, gs, gst, _ = O.c_schedule_batch(u, nd, pd[plo:phi], pt[plo:phi])
    parts = [None] * world
    dist.all_gather_object(parts, (plo, gi.tolist()))
    if rank == 0:
        pod_idx = np.concatenate([np.array(x[1], np.int64) for x in sorted(parts)])
        out_q.put((idx, score, status, pod_idx))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_node_and_pod_sharding_gloo(oracle, world):
    n, p, seed = 777, 300, 41 + world
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seed, n, p, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    idx, score, status, pod_idx = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    u, nd, pd, pt = _case(seed, n, p)
    wi, ws, wst, _ = oracle.c_schedule_batch(u, nd, pd, pt)
    assert (idx == wi).all() and (score == ws).all() and (status == wst).all()
    assert (pod_idx == wi).all()


def test_shard_range_covers_everything():
    D = importlib.import_module("mini-kube-scheduler_amd.distributed")
    for total in (0, 1, 7, 100_000, 1_000_003):
        for world in (1, 2, 3, 8):
            spans = [D.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_key_encoding_roundtrip():
    D = importlib.import_module("mini-kube-scheduler_amd.distributed")
    g = np.array([-1, 0, 1, 12345, 2**31 - 2])
    assert (D.decode_key(D.encode_key(g)) == g).all()
    assert D.encode_key(np.array([3]))[0] > D.encode_key(np.array([4]))[0]  # MAX = lowest index


def _worker_minmax(rank, world, port, seed, n, p, out_q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = importlib.import_module("mini-kube-scheduler_amd.distributed")
    u, nd, pd, pt = _case(seed, n, p)
    lo, hi = D.shard_range(n, world, rank)
    keys = torch.from_numpy(_shard_keys_oracle(D, u, nd, pd, pt, lo, hi))
    D.merge_shard_keys_(keys)
    if rank == 0:
        k = keys.numpy()
        assert keys.dtype == torch.int32 and len(k) == 2 * p
        out_q.put((D.decode_key(k[:p]), D.decode_key(k[p:])))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_node_sharding_minmax_keys_gloo(oracle, world):
    """Per-pod slot-1 keys (MINMAX): after the MAX merge, decode_pod's rule for mode 3 gives the
    unsharded oracle's answer (weight 1)."""
    n, p, seed = 555, 200, 7 + world
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_minmax, args=(r, world, port, seed, n, p, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    im, ix = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    u, nd, pd, pt = _case(seed, n, p)
    ia = np.where(im < 0, ix, np.where(ix < 0, im, np.minimum(im, ix)))  # first feasible of any class
    idx = np.where(ia < 0, -1, np.where(pd < 0, -1, np.where(im >= 0, im, ix)))
    status = np.where(ia < 0, 1, np.where(pd < 0, 2, 0))
    score = np.where((status == 0) & (im >= 0) & (ix >= 0), 100, 0)
    ps = oracle.PluginSet(normalize=[3])
    wi, ws, wst, _ = oracle.c_schedule_batch(u, nd, pd, pt, ps)
    assert (idx == wi).all() and (score == ws).all() and (status == wst).all()


# ---- node-sharded generic pipeline (any plugin list) ----
INT64_MIN, INT64_MAX, INT32_MAX = -(1 << 63), (1 << 63) - 1, (1 << 31) - 1


def _wrap64(v: int) -> int:
    return (v + (1 << 63)) % (1 << 64) - (1 << 63)


def _go_div(a: int, b: int) -> int:  # Go / C integer division: truncates toward zero
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _normalize(raw: int, mode: int, mx: int, mn: int) -> int:
    if mode == 1:
        m = max(mx, 0)
        return raw if m == 0 else _go_div(100 * raw, m)
    if mode == 2:
        m = max(mx, 0)
        return 100 if m == 0 else 100 - _go_div(100 * raw, m)
    if mode == 3:
        return 0 if mx == mn else _go_div((raw - mn) * 100, mx - mn)
    return raw


class _ShardCtx:
    """numpy restatement of the msh_generic_* contract on one node slice (test infrastructure):
    filter [NodeUnschedulable], prescore [NodeNumber], score = `plugins` [(name, weight, mode)]."""

    def __init__(self, u, nd, cols, plugins):
        self.u, self.nd, self.cols, self.plugins = u, nd, cols, plugins
        self.ncol = sum(1 for nm, _, _ in plugins if nm != "NodeNumber")

    @staticmethod
    def _arr(ptr, n, ctype):
        import ctypes
        return np.ctypeslib.as_array((ctype * n).from_address(ptr)) if n else np.zeros(0)

    def _raw(self, name, j_digit):
        if name == "NodeNumber":
            return np.where((self.nd == j_digit) & (j_digit >= 0), 10, 0).astype(np.int64)
        return self.cols[int(name[-1])].astype(np.int64)

    def _feas(self, tol):
        return np.ones(len(self.u), bool) if tol else (self.u == 0)

    def generic_ext_len(self, p):
        return 2 * (1 + self.ncol) * p if any(m for _, _, m in self.plugins) else 0

    def generic_extents_device(self, p, pdp, ptp, extp, h):
        import ctypes
        pd, pt = self._arr(pdp, p, ctypes.c_int8), self._arr(ptp, p, ctypes.c_uint8)
        ext = self._arr(extp, self.generic_ext_len(p), ctypes.c_int64)
        for j in range(p):
            f = self._feas(pt[j])
            e = 1
            for name, _, _ in self.plugins:
                slot = 0 if name == "NodeNumber" else e
                e += name != "NodeNumber"
                r = self._raw(name, pd[j])[f]
                ext[2 * slot * p + j] = int(r.max()) if r.size else INT64_MIN
                ext[(2 * slot + 1) * p + j] = -int(r.min()) if r.size else -INT64_MAX
            for slot in range(1 + self.ncol):  # slots of plugins not in the list stay empty
                if "NodeNumber" not in [nm for nm, _, _ in self.plugins] and slot == 0:
                    ext[j] = INT64_MIN
                    ext[p + j] = -INT64_MAX

    def generic_best_device(self, p, pdp, ptp, extp, lo, totp, idxp, h):
        import ctypes
        pd, pt = self._arr(pdp, p, ctypes.c_int8), self._arr(ptp, p, ctypes.c_uint8)
        n_ext = self.generic_ext_len(p)
        ext = self._arr(extp, n_ext, ctypes.c_int64) if n_ext else None
        tot, idx = self._arr(totp, p, ctypes.c_int64), self._arr(idxp, p, ctypes.c_int32)
        for j in range(p):
            f = np.flatnonzero(self._feas(pt[j]))
            best, bi = None, None
            for i in f:
                t, e = 0, 1
                for name, w, mode in self.plugins:
                    slot = 0 if name == "NodeNumber" else e
                    e += name != "NodeNumber"
                    raw = int(self._raw(name, pd[j])[i])
                    if mode:
                        raw = _normalize(raw, mode, int(ext[2 * slot * p + j]), -int(ext[(2 * slot + 1) * p + j]))
                    t = _wrap64(t + raw * w)
                if best is None or t > best:
                    best, bi = t, i
            tot[j] = best if best is not None else INT64_MIN
            idx[j] = lo + bi if bi is not None else INT32_MAX

    def generic_candidates_device(self, p, ltp, mtp, idxp, h):
        import ctypes
        lt, mt = self._arr(ltp, p, ctypes.c_int64), self._arr(mtp, p, ctypes.c_int64)
        idx = self._arr(idxp, p, ctypes.c_int32)
        idx[(idx != INT32_MAX) & (lt != mt)] = INT32_MAX

    def generic_decode_device(self, p, pdp, mtp, mip, oip, osp, ostp, h):
        import ctypes
        pd = self._arr(pdp, p, ctypes.c_int8)
        mt, mi = self._arr(mtp, p, ctypes.c_int64), self._arr(mip, p, ctypes.c_int32)
        oi, ost = self._arr(oip, p, ctypes.c_int32), self._arr(ostp, p, ctypes.c_int32)
        os_ = self._arr(osp, p, ctypes.c_int64)
        nn = any(nm == "NodeNumber" for nm, _, _ in self.plugins)
        st = np.where(mi == INT32_MAX, 1, np.where(nn & (pd < 0), 2, 0))
        ost[:] = st
        oi[:] = np.where(st == 0, mi, -1)
        os_[:] = np.where(st == 0, mt, 0)


GENERIC_PLUGINS = [
    [("NodeNumber", 3, 3), ("ScoreColumn0", 2, 3)],   # min-max on both
    [("NodeNumber", 1, 1), ("ScoreColumn1", 5, 1)],   # DefaultNormalizeScore
    [("ScoreColumn0", 1, 2), ("NodeNumber", 7, 0)],   # reverse column + raw NodeNumber
    [("ScoreColumn2", 1, 0)],                          # no normalizer: no extent merge
]


def _generic_case(seed, n, p):
    u, nd, pd, pt = _case(seed, n, p)
    rng = np.random.default_rng(seed + 1)
    cols = {0: rng.integers(-50, 51, n), 1: rng.integers(0, 4, n) * 9, 2: rng.integers(-3, 4, n)}
    return u, nd, pd, pt, cols


def _worker_generic(rank, world, port, seed, n, p, li, out_q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D = importlib.import_module("mini-kube-scheduler_amd.distributed")
        u, nd, pd, pt, cols = _generic_case(seed, n, p)
        lo, hi = D.shard_range(n, world, rank)

        class Ctx(_ShardCtx):  # the product's uploads of the slice land here
            def __init__(self):
                pass

            def upload_nodes(self, us, nds):
                self.u, self.nd = us, nds

            def upload_score_column(self, name, col):
                self.cols[int(name[-1])] = col

        ctx = Ctx()
        ctx.cols, ctx.plugins = {}, GENERIC_PLUGINS[li]
        ctx.ncol = sum(1 for nm, _, _ in ctx.plugins if nm != "NodeNumber")
        sched = D.GenericNodeShardedScheduler(ctx, u, nd, world, rank,
                                              columns={f"ScoreColumn{k}": c for k, c in cols.items()})
        assert (sched.shard.lo, sched.shard.hi) == (lo, hi)
        t_pd, t_pt = torch.from_numpy(pd), torch.from_numpy(pt)
        oi, osc, ost = torch.empty(p, dtype=torch.int32), torch.empty(p, dtype=torch.int64), torch.empty(p, dtype=torch.int32)
        sched.schedule(t_pd, t_pt, oi, osc, ost)
        if rank == 0:
            out_q.put((oi.numpy().copy(), osc.numpy().copy(), ost.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("li", range(len(GENERIC_PLUGINS)))
def test_generic_node_sharding_gloo(oracle, world, li):
    """GenericNodeShardedScheduler over gloo: extents merged by MAX (mins negated), bests by MAX total
    then MIN global index; equals the unsharded oracle (RunScorePlugins over the whole table) for
    min-max, DefaultNormalizeScore, reverse and raw plugin lists with score columns."""
    n, p, seed = 333, 120, 17 * world + li
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_generic, args=(r, world, port, seed, n, p, li, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    gi, gs, gst = q.get(timeout=180)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    u, nd, pd, pt, cols = _generic_case(seed, n, p)
    pl = GENERIC_PLUGINS[li]
    ps = oracle.PluginSet(score=[nm for nm, _, _ in pl], weights=[w for _, w, _ in pl],
                          normalize=[m for _, _, m in pl],
                          prescore=["NodeNumber"] if any(nm == "NodeNumber" for nm, _, _ in pl) else [])
    wi, ws, wst, _ = oracle.c_schedule_batch(u, nd, pd, pt, ps, cols=cols)
    assert (gi == wi).all() and (gs == ws).all() and (gst == wst).all()
