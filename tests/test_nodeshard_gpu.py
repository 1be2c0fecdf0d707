"""Node sharding with the merge inside the library (ABI v8), vs the oracle over the whole table.

The reference schedules each pod against the whole List-order node list and keeps the first maximum
(minisched/minisched.go:40, :115-199, :304-325). Split into contiguous slices, the shards' first maxima
merge back into it; ABI v8 does that merge inside libminisched_hip.so, in the two shapes a scheduler
process takes (verdict r5, next #1):

* msh_group_*: one process driving several shard ctxs (on the one-GPU box: several ctxs on device 0, the
  peer mapping trivially local). BASELINE C4's shape at its own size, 100,000 nodes over 8 shards x
  1,000,000 pods, against the oracle; score-column lists with every normalizer (the generic form: extents
  merged by MAX and read back by every shard, then the first maximum over the shards' bests), an empty
  shard, error cases.
* msh_comm_* + msh_schedule_nodeshard(_device): one process per GPU with an RCCL communicator in the ctx.
  A one-GPU box hosts a world of one: the communicator is created through the C-ABI (ncclGetUniqueId,
  ncclCommInitRank inside the library) and every all-reduce of the path runs on it, in a spawned process
  so that an RCCL hang cannot stall the suite. World > 1 needs one GPU per rank (the driver's 8-GPU
  node); its reduction is the same MAX / MIN the group merge and the gloo protocol tests check.
"""
from __future__ import annotations

import importlib
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

from closed_form import closed_form_modes

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _shards(n, world):
    return [(n * r // world, n * (r + 1) // world) for r in range(world)]


def _case(seed, n, p, p_unsched=0.3, p_tol=0.2):
    rng = np.random.default_rng(seed)
    u = (rng.random(n) < p_unsched).astype(np.uint8)
    nd = rng.integers(-1, 10, n).astype(np.int8)
    nd[: n // 2][nd[: n // 2] == 5] = 6  # digit 5 only in the second half: matches in later shards
    pd = rng.integers(-1, 10, p).astype(np.int8)
    pt = (rng.random(p) < p_tol).astype(np.uint8)
    return rng, u, nd, pd, pt


def _same(got, want, what):
    for name, g, w in zip(("idx", "score", "status"), got, want[:3]):
        bad = np.flatnonzero(np.asarray(g) != np.asarray(w))
        assert bad.size == 0, f"{what}: {name} differs at {bad[:5]}: got {np.asarray(g)[bad[:5]]} want {np.asarray(w)[bad[:5]]}"


def _set(ctx, msh, plugins):
    pre = ["NodeNumber"] if any(nm == "NodeNumber" for nm, _, _ in plugins) else []
    ctx.set_plugins(["NodeUnschedulable"], pre, [msh.ScorePluginConfig(nm, w, msh.Normalize(m)) for nm, w, m in plugins])


def _ps(oracle, plugins):
    pre = ["NodeNumber"] if any(nm == "NodeNumber" for nm, _, _ in plugins) else []
    return oracle.PluginSet(filters=["NodeUnschedulable"], prescore=pre, score=[nm for nm, _, _ in plugins],
                            weights=[w for _, w, _ in plugins], normalize=[m for _, _, m in plugins])


def _group(msh, plugins, u, nd, cuts, cols=None):
    ctxs = []
    for lo, hi in cuts:
        c = msh.DeviceContext(0)
        _set(c, msh, plugins)
        c.upload_nodes(u[lo:hi], nd[lo:hi])
        for k, col in (cols or {}).items():
            c.upload_score_column(f"ScoreColumn{k}", np.ascontiguousarray(col[lo:hi]))
        ctxs.append(c)
    return ctxs, msh.DeviceGroup(ctxs)


def _close(ctxs, g):
    g.close()
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("plugins", [[("NodeNumber", 1, 0)], [("NodeNumber", 3, 1)], [("NodeNumber", 3, 3)]],
                         ids=["reference", "w3-default", "w3-minmax"])
def test_group_c4_eight_shards(msh, oracle, synth, plugins):
    """BASELINE C4 at its own size through msh_group_schedule_batch: 100,000 nodes in 8 List-order
    slices (8 ctxs), 1,000,000 pods; the library merges the shards' keys on the home device. The
    reference list against the oracle over the whole table (all 10^11 pairs); the w = 3 lists against
    the closed form (every pod) and the oracle (the first 100,000 pods)."""
    n, p = 100_000, 1_000_000
    u, nd = synth.make_nodes(n)[1:]
    pd, pt = synth._make_pods_fast(p, synth.SEED + 4)[1:]
    ctxs, g = _group(msh, plugins, u, nd, _shards(n, 8))
    try:
        got = g.schedule_batch(pd, pt)
    finally:
        _close(ctxs, g)
    (_, w, m), = plugins
    _same(got, closed_form_modes(u, nd, pd, pt, w, m), f"C4 group {plugins} vs closed form")
    sub = slice(None) if plugins == [("NodeNumber", 1, 0)] else slice(0, 100_000)
    want = oracle.c_schedule_batch(u, nd, pd[sub], pt[sub], _ps(oracle, plugins), threads=16)
    _same(tuple(x[sub] for x in got), want, f"C4 group {plugins} vs oracle")


GROUP_LISTS = [
    [("NodeNumber", 2, 2)],                                                  # REVERSE: the non-match keys
    [("NodeNumber", 1, 0), ("ScoreColumn0", 2, 1)],                          # generic, one DEFAULT column
    [("ScoreColumn1", 3, 3), ("NodeNumber", 1, 1), ("ScoreColumn0", 1, 0)],  # MIN-MAX column + node-only sum
    [("ScoreColumn0", 1 << 32, 2), ("ScoreColumn1", 5, 3)],                   # two normalizers, 64-bit totals
    [("ScoreColumn0", 7, 0)],                                                # no normalizer: no extents merge
]


@pytest.mark.parametrize("lst", range(len(GROUP_LISTS)))
def test_group_plugin_lists(msh, oracle, lst):
    """Every key layout and the generic form through the group, on uneven slices with an empty shard
    in the middle, against the oracle over the whole table."""
    plugins = GROUP_LISTS[lst]
    rng, u, nd, pd, pt = _case(40 + lst, 7000, 6000)
    cols = {0: rng.integers(-(1 << 31), (1 << 31) + 1, 7000), 1: rng.integers(0, 9, 7000) * 17}
    cuts = [(0, 1500), (1500, 1500), (1500, 4100), (4100, 7000)]
    ctxs, g = _group(msh, plugins, u, nd, cuts, cols)
    try:
        got = g.schedule_batch(pd, pt)
        got2 = g.schedule_batch(pd[:777], pt[:777], scores=False)  # a smaller batch, scores not copied
    finally:
        _close(ctxs, g)
    want = oracle.c_schedule_batch(u, nd, pd, pt, _ps(oracle, plugins), cols=cols, threads=8)
    _same(got, want, f"group {plugins}")
    assert got2[1] is None
    _same((got2[0], want[1][:777], got2[2]), tuple(x[:777] for x in want), f"group {plugins} p=777")


def test_group_errors(msh):
    """A shard without nodes or with other plugin lists is MSH_ERR_STATE at the call; a ctx twice is
    MSH_ERR_INVALID at msh_group_create."""
    N = msh._native
    a, b = msh.DeviceContext(0), msh.DeviceContext(0)
    try:
        with pytest.raises(msh.MshError) as e:
            msh.DeviceGroup([a, a])
        assert e.value.code == N.MSH_ERR_INVALID
        a.upload_nodes(np.zeros(10, np.uint8), np.zeros(10, np.int8))
        g = msh.DeviceGroup([a, b])
        pd, pt = np.zeros(5, np.int8), np.zeros(5, np.uint8)
        with pytest.raises(msh.MshError, match="no node table") as e:
            g.schedule_batch(pd, pt)
        assert e.value.code == N.MSH_ERR_STATE
        b.upload_nodes(np.zeros(10, np.uint8), np.ones(10, np.int8))
        b.set_plugins(["NodeUnschedulable"], ["NodeNumber"], [msh.ScorePluginConfig("NodeNumber", 2)])
        with pytest.raises(msh.MshError, match="other plugin lists"):
            g.schedule_batch(pd, pt)
        a.set_plugins(["NodeUnschedulable"], ["NodeNumber"], [msh.ScorePluginConfig("NodeNumber", 2)])
        idx, score, status = g.schedule_batch(pd, pt)  # pod digit 0: node 0 of shard a, score 20
        assert (idx == 0).all() and (score == 20).all() and (status == 0).all()
        g.close()
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("plugins", [[("NodeNumber", 1, 0)], [("NodeNumber", 2, 3)],
                                     [("NodeNumber", 1, 1), ("ScoreColumn0", 3, 2)]],
                         ids=["reference", "minmax", "generic"])
def test_nodeshard_without_comm(msh, oracle, plugins):
    """msh_schedule_nodeshard(_device) on a ctx without a communicator is a world of one: the whole
    table on one shard gives msh_schedule_batch's decisions; a slice with node_base reports global
    indices (base + local), the host and device forms alike, launches on two streams in turn."""
    torch = pytest.importorskip("torch")
    rng, u, nd, pd, pt = _case(77, 5000, 20_000)
    cols = {0: rng.integers(-1000, 1000, 5000)}
    want = oracle.c_schedule_batch(u, nd, pd, pt, _ps(oracle, plugins), cols=cols, threads=8)
    dev = torch.device("cuda:0")
    with msh.DeviceContext(0) as ctx:
        _set(ctx, msh, plugins)
        ctx.upload_nodes(u, nd)
        ctx.upload_score_column("ScoreColumn0", cols[0])
        assert ctx.comm_info() == (0, 0)
        _same(ctx.schedule_nodeshard(pd, pt, 0), want, "host, whole table")
        d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
        outs = [[torch.full((len(pd),), -7, dtype=dt, device=dev) for dt in (torch.int32, torch.int64, torch.int32)]
                for _ in range(2)]
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        torch.cuda.synchronize()
        for o, st in zip(outs, streams):
            ctx.schedule_nodeshard_device(len(pd), d_pd.data_ptr(), d_pt.data_ptr(), 0, *[t.data_ptr() for t in o],
                                          st.cuda_stream)
        torch.cuda.synchronize()
        for o in outs:
            _same([t.cpu().numpy() for t in o], want, "device, whole table")
        # a slice at node_base 123,456: the shard's own first maximum, as a global index
        lo, hi = 1000, 3000
        ctx.upload_nodes(u[lo:hi], nd[lo:hi])
        ctx.upload_score_column("ScoreColumn0", np.ascontiguousarray(cols[0][lo:hi]))
        part = oracle.c_schedule_batch(u[lo:hi], nd[lo:hi], pd, pt, _ps(oracle, plugins), cols={0: cols[0][lo:hi]},
                                       threads=8)
        gi, gs, gst = ctx.schedule_nodeshard(pd, pt, 123_456)
        placed = part[2] == 0
        assert (gi[placed] == part[0][placed] + 123_456).all() and (gi[~placed] == -1).all()
        _same((gi, gs, gst), (np.where(placed, part[0] + 123_456, -1), part[1], part[2]), "slice at node_base")
        with pytest.raises(msh.MshError, match="node_base"):
            ctx.schedule_nodeshard(pd, pt, -1)


def _comm_worker(out_q):
    try:
        import torch
        sys.path.insert(0, str(ROOT))
        sys.path.insert(0, str(ROOT / "tests"))
        msh = importlib.import_module("mini-kube-scheduler_amd")
        oracle = importlib.import_module("oracle.oracle")
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        res = {}
        rng, u, nd, pd, pt = _case(2026, 5000, 50_000)
        cols = {0: rng.integers(-(1 << 31), (1 << 31) + 1, 5000)}
        comm_id = msh.DeviceContext.comm_unique_id()
        res["id_len"] = len(comm_id)
        for name, plugins in (("reference", [("NodeNumber", 1, 0)]), ("minmax", [("NodeNumber", 3, 3)]),
                              ("generic", [("NodeNumber", 3, 1), ("ScoreColumn0", 5, 2)])):
            with msh.DeviceContext(0) as ctx:
                _set(ctx, msh, plugins)
                ctx.upload_nodes(u, nd)
                ctx.upload_score_column("ScoreColumn0", cols[0])
                ctx.comm_init(msh.DeviceContext.comm_unique_id(), 1, 0)  # ncclCommInitRank in the library
                res[f"{name}_info"] = ctx.comm_info()
                want = oracle.c_schedule_batch(u, nd, pd, pt, _ps(oracle, plugins), cols=cols, threads=16)
                host = ctx.schedule_nodeshard(pd, pt, 0)
                # the device form on a busy side stream: the all-reduces must stay ordered on it
                side = torch.cuda.Stream(dev)
                d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
                out = [torch.full((len(pd),), -7, dtype=dt, device=dev) for dt in (torch.int32, torch.int64, torch.int32)]
                busy = torch.randn(3000, 3000, device=dev)
                torch.cuda.synchronize()
                with torch.cuda.stream(side):
                    for _ in range(6):
                        busy = busy @ busy * 1e-3
                ctx.schedule_nodeshard_device(len(pd), d_pd.data_ptr(), d_pt.data_ptr(), 0, *[t.data_ptr() for t in out],
                                              side.cuda_stream)
                torch.cuda.synchronize()
                dv = [t.cpu().numpy() for t in out]
                res[name] = all(bool((np.asarray(g) == np.asarray(w)).all()) for g, w in zip(host, want[:3])) and \
                    all(bool((g == w).all()) for g, w in zip(dv, want[:3]))
                try:
                    ctx.comm_init(comm_id, 1, 0)
                    res[f"{name}_reinit"] = "accepted"
                except msh.MshError as e:
                    res[f"{name}_reinit"] = e.code
        out_q.put(res)
    except Exception as e:  # report, do not hang the parent
        out_q.put({"error": repr(e)})


def test_comm_world1_through_the_abi(msh, oracle):
    """An RCCL communicator created and used entirely through the C-ABI (msh_comm_unique_id,
    msh_comm_init, msh_schedule_nodeshard / _device): at world 1 every all-reduce of the path (keys
    MAX; the generic form's extents MAX, totals MAX, indices MIN) runs on it; decisions vs the oracle,
    host and device forms; a second msh_comm_init on the ctx is MSH_ERR_STATE."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_comm_worker, args=(q,))
    proc.start()
    try:
        res = q.get(timeout=100)
    finally:
        proc.join(timeout=20)
        if proc.is_alive():
            proc.kill()
            proc.join()
    assert "error" not in res, res
    assert res["id_len"] == msh._native.COMM_ID_BYTES
    for name in ("reference", "minmax", "generic"):
        assert res[f"{name}_info"] == (1, 0), res
        assert res[name] is True, res
        assert res[f"{name}_reinit"] == msh._native.MSH_ERR_STATE, res
