"""GPU parity: the gfx950 path (through the C-ABI) vs the CPU oracle, bit-exact.

Every test here calls libminisched_hip.so on cuda:0 and compares idx / score / status with
oracle/msh_oracle.c (the restatement of minisched/minisched.go:115-199,304-325) on the same
seeded inputs; large sizes additionally against the independent closed form.
"""
from __future__ import annotations

import importlib
import itertools
import json
from pathlib import Path

import numpy as np
import pytest

from closed_form import closed_form

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def _rand_case(rng, n, p, p_unsched=0.3, p_tol=0.2, p_nd_node=0.1, p_nd_pod=0.1):
    unsched = (rng.random(n) < p_unsched).astype(np.uint8)
    nd = rng.integers(0, 10, n).astype(np.int8)
    nd[rng.random(n) < p_nd_node] = -1
    pd = rng.integers(0, 10, p).astype(np.int8)
    pd[rng.random(p) < p_nd_pod] = -1
    pt = (rng.random(p) < p_tol).astype(np.uint8)
    return unsched, nd, pd, pt


def _plugins(oracle, filters, prescore, score, weight=1, norm=0):
    return oracle.PluginSet(filters=list(filters), prescore=list(prescore), score=list(score),
                            weights=[weight] * len(score), normalize=[norm] * len(score))


def _set(ctx, msh, ps):
    ctx.set_plugins(ps.filters, ps.prescore,
                    [msh.ScorePluginConfig(s, w, msh.Normalize(m)) for s, w, m in zip(ps.score, ps.weights, ps.normalize)])


def _pair_opts(spec):
    """msh_options for the pair kernel from a spec "planes[-noax|-axlast]" (planes: sgpr, lds or auto;
    noax / axlast: group 0 scanned first and the non-match / feasible reduction dropped where it settled
    it, or never — else auto: the first for REVERSE / MINMAX, the second for the identity-like modes)."""
    parts = spec.split("-")
    return {"pair_planes": parts[0], "pair_noax": "noax" if "noax" in parts else "axlast" if "axlast" in parts else "auto"}


def _assert_same(got, want, what=""):
    gi, gs, gst = got
    wi, ws, wst = want[:3]
    bad = np.nonzero((gi != wi) | (gs != ws) | (gst != wst))[0]
    assert bad.size == 0, (f"{what}: {bad.size} pods differ; first {bad[:5]}: got "
                           f"{[(int(gi[b]), int(gs[b]), int(gst[b])) for b in bad[:5]]} want "
                           f"{[(int(wi[b]), int(ws[b]), int(wst[b])) for b in bad[:5]]}")


def test_scenario_golden(msh, gpu_ctx):
    """sched.go:70-143: the reference's only known answer."""
    fx = json.loads((GOLDEN / "scenario.json").read_text())
    sched = msh.Scheduler(ctx=gpu_ctx)
    for phase in fx["phases"]:
        res = sched.schedule_batch([{"metadata": {"name": p["name"]}, "spec": {"tolerations": p.get("tolerations", [])}}
                                    for p in fx["pods"]],
                                   [{"metadata": {"name": n["name"]}, "spec": {"unschedulable": n["unschedulable"]}}
                                    for n in phase["nodes"]])
        for r, want in zip(res, phase["expect"]):
            assert r.outcome.name == want["outcome"]
            assert r.node_name == want.get("node")
            assert sorted(r.unschedulable_plugins) == sorted(want.get("unschedulable_plugins", []))


def test_golden_fixtures(msh, gpu_ctx, oracle):
    for path in sorted(GOLDEN.glob("case_*.json")):
        fx = json.loads(path.read_text())
        ps = oracle.PluginSet(**fx["plugins"])
        _set(gpu_ctx, msh, ps)
        gpu_ctx.upload_nodes(np.array(fx["unsched"], np.uint8), np.array(fx["node_digit"], np.int8))
        got = gpu_ctx.schedule_batch(np.array(fx["pod_digit"], np.int8), np.array(fx["pod_tol"], np.uint8))
        want = (np.array(fx["idx"], np.int32), np.array(fx["score"], np.int64), np.array(fx["status"], np.int32))
        _assert_same(got, want, path.name)


PLUGIN_COMBOS = [
    (["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"]),   # the reference
    ([], ["NodeNumber"], ["NodeNumber"]),
    (["NodeUnschedulable"], [], ["NodeNumber"]),               # score without prescore state
    (["NodeUnschedulable"], ["NodeNumber"], []),
    ([], [], []),
]


@pytest.mark.parametrize("combo", range(len(PLUGIN_COMBOS)))
@pytest.mark.parametrize("norm", [0, 1, 2, 3])
@pytest.mark.parametrize("weight", [1, 3, 1 << 32])
def test_plugin_sets_random(msh, gpu_ctx, oracle, combo, norm, weight):
    rng = np.random.default_rng(1000 * combo + 10 * norm + (weight % 97))
    f, pre, s = PLUGIN_COMBOS[combo]
    ps = _plugins(oracle, f, pre, s, weight, norm)
    _set(gpu_ctx, msh, ps)
    for n, p in [(1, 5), (70, 300), (1000, 2000)]:
        u, nd, pd, pt = _rand_case(rng, n, p)
        gpu_ctx.upload_nodes(u, nd)
        got = gpu_ctx.schedule_batch(pd, pt)
        want = oracle.c_schedule_batch(u, nd, pd, pt, ps)
        _assert_same(got, want, f"combo={combo} norm={norm} w={weight} n={n} p={p}")


@pytest.mark.parametrize("n", [0, 1, 5, 63, 64, 65, 1023, 1024, 1025, 5000, 16384, 16385, 21504, 21505, 40000,
                               64512, 64513, 70000, 140000])
def test_node_sizes(msh, gpu_ctx, oracle, n):
    """Empty / ragged / boundary node tables: 32-node words, 256-node groups, 1,024-node prep
    blocks, and slice splits of the group range (bits_slices) at several table sizes."""
    rng = np.random.default_rng(n)
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = _rand_case(rng, n, 777)
    gpu_ctx.upload_nodes(u, nd)
    got = gpu_ctx.schedule_batch(pd, pt)
    _assert_same(got, oracle.c_schedule_batch(u, nd, pd, pt, ps), f"n={n}")
    _assert_same(got, closed_form(u, nd, pd, pt), f"closed form n={n}")


@pytest.mark.parametrize("n_only", [0, 1, 63, 64, 255, 256, 257, 511, 512, 1023, 1024, 1800])
def test_tolerating_list_blocks(msh, gpu_ctx, oracle, n_only):
    """The tolerating pods' pass reads the class-1-only node list (ulist) in sentinel-padded
    256-entry blocks with no bounds check: list lengths at and around the block and table-padding
    boundaries, with every tolerating pod's only match the LAST listed node, the first, or none."""
    rng = np.random.default_rng(4242 + n_only)
    n = 2048
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    u = np.zeros(n, np.uint8)
    u[n - n_only:] = 1                       # the list = the last n_only nodes
    nd = np.full(n, 9, np.int8)              # feasible nodes never match digits 0..8
    nd[n - n_only:] = rng.integers(0, 9, n_only).astype(np.int8)
    if n_only:
        nd[n - 1] = 3                        # the last listed node: the only '3' -> list tail
        nd[n - n_only] = 5 if n_only > 1 else 3
        nd[n - n_only + 1:n - 1][nd[n - n_only + 1:n - 1] == 5] = 6
        nd[n - n_only + 1:n - 1][nd[n - n_only + 1:n - 1] == 3] = 4
    p = 4096
    pd = rng.integers(0, 10, p).astype(np.int8)
    pt = (rng.random(p) < 0.5).astype(np.uint8)
    gpu_ctx.upload_nodes(u, nd)
    got = gpu_ctx.schedule_batch(pd, pt)
    _assert_same(got, oracle.c_schedule_batch(u, nd, pd, pt, ps), f"ulist={n_only}")
    _assert_same(got, closed_form(u, nd, pd, pt), f"closed form ulist={n_only}")
    if n_only:
        tol3 = (pt == 1) & (pd == 3)
        assert (got[0][tol3] == n - 1).all()


@pytest.mark.parametrize("norm", [0, 2, 3])
def test_multitile_normalize(msh, gpu_ctx, oracle, norm):
    rng = np.random.default_rng(77 + norm)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 2, norm)
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = _rand_case(rng, 33000, 3000, p_unsched=0.9)
    gpu_ctx.upload_nodes(u, nd)
    _assert_same(gpu_ctx.schedule_batch(pd, pt), oracle.c_schedule_batch(u, nd, pd, pt, ps), f"norm={norm}")


@pytest.mark.parametrize("p", [0, 1, 2, 63, 64, 65, 1000, 4097, 250_000])
def test_pod_sizes(msh, gpu_ctx, oracle, p):
    """Empty / ragged pod batches, including windows that end mid-group."""
    rng = np.random.default_rng(p + 5)
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = _rand_case(rng, 300, p)
    gpu_ctx.upload_nodes(u, nd)
    got = gpu_ctx.schedule_batch(pd, pt)
    _assert_same(got, oracle.c_schedule_batch(u, nd, pd, pt, ps), f"p={p}")


def test_all_unschedulable_and_tolerations(msh, gpu_ctx, oracle):
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    n = 500
    u = np.ones(n, np.uint8)
    nd = (np.arange(n) % 10).astype(np.int8)
    pd = (np.arange(200) % 11 - 1).astype(np.int8)
    pt = (np.arange(200) % 3 == 0).astype(np.uint8)
    gpu_ctx.upload_nodes(u, nd)
    got = gpu_ctx.schedule_batch(pd, pt)
    want = oracle.c_schedule_batch(u, nd, pd, pt, ps)
    _assert_same(got, want, "all unschedulable")
    assert (got[2][pt == 0] == 1).all()  # FitError for non-tolerating pods


def test_c2_full(msh, gpu_ctx, oracle, synth):
    """BASELINE config C2: 1k nodes x 10k pods, plus a 100%-unschedulable block."""
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = synth.make_soa(1000, 10_000)
    gpu_ctx.upload_nodes(u, nd)
    _assert_same(gpu_ctx.schedule_batch(pd, pt), oracle.c_schedule_batch(u, nd, pd, pt, ps), "C2")
    u2 = np.ones_like(u)
    gpu_ctx.upload_nodes(u2, nd)
    _assert_same(gpu_ctx.schedule_batch(pd, pt), oracle.c_schedule_batch(u2, nd, pd, pt, ps), "C2 all-unsched")


def test_c3_full_and_weight3(msh, gpu_ctx, oracle, synth):
    """BASELINE config C3: 5k nodes x 100k pods; weight 3 must place identically."""
    u, nd, pd, pt = synth.make_soa(5000, 100_000)
    ps1 = oracle.PluginSet()
    _set(gpu_ctx, msh, ps1)
    gpu_ctx.upload_nodes(u, nd)
    got1 = gpu_ctx.schedule_batch(pd, pt)
    _assert_same(got1, oracle.c_schedule_batch(u, nd, pd, pt, ps1, threads=8), "C3")
    _assert_same(got1, closed_form(u, nd, pd, pt), "C3 closed form")
    ps3 = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 3, 0)
    _set(gpu_ctx, msh, ps3)
    got3 = gpu_ctx.schedule_batch(pd, pt)
    assert (got3[0] == got1[0]).all() and (got3[2] == got1[2]).all()
    assert (got3[1] == 3 * got1[1]).all()


def test_c4_full_size_batch_and_shards(msh, gpu_ctx, synth):
    """BASELINE config C4 at full size on one device: 100k nodes x 1M pods, checked through the
    independent closed form (the scalar oracle would need minutes). Both the whole-table batch
    (multi-tile work-queue kernel) and the 8-way node-sharded path (per-shard int32 keys,
    element-wise MAX, device decode), with pods also permuted: every pod's decision must move
    with it (pods are independent)."""
    torch = pytest.importorskip("torch")
    u, nd, pd, pt = synth.make_soa(100_000, 1_000_000)
    want = closed_form(u, nd, pd, pt)
    gpu_ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 1)])
    gpu_ctx.upload_nodes(u, nd)
    _assert_same(gpu_ctx.schedule_batch(pd, pt), want, "C4 batch")
    perm = np.random.default_rng(5).permutation(len(pd))
    got_p = gpu_ctx.schedule_batch(np.ascontiguousarray(pd[perm]), np.ascontiguousarray(pt[perm]))
    _assert_same(got_p, tuple(w[perm] for w in want), "C4 permuted pods")

    dev = torch.device("cuda:0")
    d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
    p = len(pd)
    D = importlib.import_module("mini-kube-scheduler_amd.distributed")
    for world in (1, 8):  # 1: one 100k-node shard (multi-tile keys); 8: 12.5k-node shards
        merged, ctxs = None, []
        for r in range(world):
            lo, hi = D.shard_range(len(u), world, r)
            c = msh.DeviceContext(0)
            c.upload_nodes(u[lo:hi], nd[lo:hi])
            keys = torch.empty(c.shard_keys_len(p), dtype=torch.int32, device=dev)
            c.shard_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), lo, keys.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)
            merged = keys if merged is None else torch.maximum(merged, keys)
            ctxs.append(c)
        oi = torch.empty(p, dtype=torch.int32, device=dev)
        osc = torch.empty(p, dtype=torch.int64, device=dev)
        ost = torch.empty(p, dtype=torch.int32, device=dev)
        ctxs[0].decode_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), merged.data_ptr(), oi.data_ptr(),
                                   osc.data_ptr(), ost.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        _assert_same((oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy()), want, f"C4 {world} shards")
        for c in ctxs:
            c.close()


SEQ_CASES = ([("0", n) for n in (1, 70, 1000, 5000, 8192, 8193, 12289, 32768, 40000)]
             + [("1", 70), ("1", 8192), ("4", 1000), ("4", 8193), ("4", 32768), ("16", 1000), ("16", 40000),
                ("1", 12289)])


@pytest.mark.parametrize("max_pods", [0, 1, 3])
@pytest.mark.parametrize("seq_waves,n", SEQ_CASES)
def test_sequential(msh, oracle, n, max_pods, seq_waves):
    """Sequential commit against the oracle's serial loop, node counts included; one scanning wave
    up to 8,192 nodes, four up to 32,768, then 15 (+ finalizer) / 16 (msh_options.seq_waves, read once by
    msh_create_ex, forces a count; one too small for the table is raised: the last case). Auto at every
    table size, each forced count at the sizes around its limits."""
    rng = np.random.default_rng(n + max_pods)
    ps = oracle.PluginSet()
    u, nd, pd, pt = _rand_case(rng, n, 3001)  # not a multiple of the 4 pods one wave decides per step
    with msh.DeviceContext(0, {"seq_waves": seq_waves}) as ctx:
        _set(ctx, msh, ps)
        ctx.upload_nodes(u, nd)
        got = ctx.schedule_sequential(pd, pt, max_pods)
        want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, max_pods)
        _assert_same(got, (want_i, want_s, want_st), f"seq n={n} max={max_pods} waves={seq_waves}")
        assert (ctx.node_pod_counts() == want_counts).all()
        if max_pods == 0:
            ctx.reset_node_pod_counts()
            _assert_same(got, ctx.schedule_batch(pd, pt), "seq == batch")


@pytest.mark.parametrize("norm", [0, 1, 2, 3])
@pytest.mark.parametrize("split", ["auto", "blocks", "serial"])
@pytest.mark.parametrize("seq_waves,n", [("1", 1000), ("4", 8193), ("16", 40000)])
def test_sequential_pod_blocks(msh, oracle, seq_waves, n, split, norm):
    """Without a capacity no commit feeds a later decision. Auto (msh_options.seq_split 0) runs the per-pair
    batch kernel with the commit epilogue (every placed pod's count added to a count replica, tables up to
    32,768 nodes); "blocks" the sequential kernel's 64-pod blocks of consecutive pods, one workgroup each;
    "serial" one workgroup walking every pod in order (the 40,000-node table stays in one workgroup in
    every form). All give the serial loop's placements and node counts, for batch sizes around the
    64-pod block edges, in every normalize mode, with counts carried over between calls."""
    rng = np.random.default_rng(n + 77)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 2, norm)
    p = 20_000 if n < 10_000 else 6_000  # (the oracle's serial loop is n x p)
    u, nd, pd, pt = _rand_case(rng, n, p, p_unsched=0.2, p_tol=0.1)
    with msh.DeviceContext(0, {"seq_waves": seq_waves, "seq_split": split}) as ctx:
        _set(ctx, msh, ps)
        ctx.upload_nodes(u, nd)
        cuts = [0, 1, 64, 65, 191, p // 2 - 1, p]
        parts = [ctx.schedule_sequential(pd[a:b], pt[a:b], 0) for a, b in zip(cuts, cuts[1:])]
        want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, 0)
        _assert_same(tuple(np.concatenate(x) for x in zip(*parts)), (want_i, want_s, want_st),
                     f"seq blocks split={split} waves={seq_waves} n={n}")
        assert (ctx.node_pod_counts() == want_counts).all()
    with pytest.raises(msh.MshError, match="seq_split"):
        msh.DeviceContext(0, {"seq_split": 7})


@pytest.mark.parametrize("pod_waves", [1, 2, 4, 8])
@pytest.mark.parametrize("norm", [0, 1, 3])
def test_sequential_pod_waves(msh, oracle, pod_waves, norm):
    """Pod-block workgroups of the one-scanning-wave form (tables up to 8,192 nodes, no capacity) shared by
    1, 2, 4 or 8 pod waves (msh_options.seq_pod_waves; 1 is the automatic choice): each wave holds the
    whole table and walks 64 / waves consecutive pods in order, the waves add their commits to the
    workgroup's LDS counts, flushed to the device count replicas at the end. Ragged batches (the last
    block's trailing waves get no pod), counts carried over calls, vs the oracle's serial loop."""
    rng = np.random.default_rng(31 * pod_waves + norm)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 2, norm)
    u, nd, pd, pt = _rand_case(rng, 3000, 20_037, p_unsched=0.2, p_tol=0.1)
    with msh.DeviceContext(0, {"seq_pod_waves": pod_waves, "seq_split": "blocks"}) as ctx:
        _set(ctx, msh, ps)
        ctx.upload_nodes(u, nd)
        cuts = [0, 1, 64, 65, 70, 191, 10_000, 20_037]
        parts = [ctx.schedule_sequential(pd[a:b], pt[a:b], 0) for a, b in zip(cuts, cuts[1:])]
        want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, 0)
        _assert_same(tuple(np.concatenate(x) for x in zip(*parts)), (want_i, want_s, want_st),
                     f"pod waves={pod_waves} norm={norm}")
        assert (ctx.node_pod_counts() == want_counts).all()


def test_sequential_count_replicas(msh, oracle):
    """Pod-block launches add their commits to count replicas; the next one-workgroup launch (here a
    capacity launch, which reads the counts) and msh_node_pod_counts fold them first. Blocks, a small
    serial batch, blocks again, then a capacity batch, against the oracle's serial loop with a capacity
    no earlier batch reaches (so it acts only on the last); the ctx held a table too large for pod
    blocks (one count array) before, so the upload reallocates the counts with their replicas."""
    rng = np.random.default_rng(99)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 1, 0)
    u, nd, pd, pt = _rand_case(rng, 2000, 31_000, p_unsched=0.2, p_tol=0.1)
    cuts = [0, 10_000, 10_040, 30_000, 31_000]
    pre = oracle.c_schedule_sequential(u, nd, pd[:30_000], pt[:30_000], ps, 0)[3]
    cap = int(pre.max()) + 3
    want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, cap)
    with msh.DeviceContext(0) as ctx:
        _set(ctx, msh, ps)
        # a table past the pod-block limit first (one count array), then this one (the replicas)
        ub, ndb = _rand_case(rng, 40_000, 10)[:2]
        ctx.upload_nodes(ub, ndb)
        ctx.schedule_sequential(pd[:300], pt[:300], 0)
        ctx.upload_nodes(u, nd)
        parts = [ctx.schedule_sequential(pd[a:b], pt[a:b], cap if b == 31_000 else 0)
                 for a, b in zip(cuts, cuts[1:])]
        _assert_same(tuple(np.concatenate(x) for x in zip(*parts)), (want_i, want_s, want_st), "replicas")
        assert (ctx.node_pod_counts() == want_counts).all()
        assert want_counts.max() == cap  # the capacity did act on the last batch


def test_sequential_pod_blocks_two_streams(msh, oracle):
    """Two pod-block sequential launches of one ctx on two streams, back to back (their blocks add to
    the same device counts): each batch's placements and the summed node counts equal the serial
    loop's."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(4242)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 3, 1)
    u, nd, pd, pt = _rand_case(rng, 3000, 50_000, p_unsched=0.2, p_tol=0.1)
    halves = [(pd[:20_000], pt[:20_000]), (pd[20_000:], pt[20_000:])]
    with msh.DeviceContext(0) as ctx:
        _set(ctx, msh, ps)
        ctx.upload_nodes(u, nd)
        bufs = [_dev_batch(torch, dev, a, b) for a, b in halves]
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        torch.cuda.synchronize()
        for t, st in zip(bufs, streams):
            ctx.schedule_sequential_device(len(t[0]), t[0].data_ptr(), t[1].data_ptr(), 0, t[2].data_ptr(),
                                           t[3].data_ptr(), t[4].data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, 0)
        got = tuple(np.concatenate([t[i].cpu().numpy() for t in bufs]) for i in (2, 3, 4))
        _assert_same(got, (want_i, want_s, want_st), "two streams")
        assert (ctx.node_pod_counts() == want_counts).all()


@pytest.mark.parametrize("seq_waves", ["1", "16"])
@pytest.mark.parametrize("norm", [0, 1, 2, 3])
@pytest.mark.parametrize("combo", range(len(PLUGIN_COMBOS)))
def test_sequential_plugin_sets(msh, oracle, combo, norm, seq_waves):
    """Sequential commit for every plugin-list combination and normalize mode (the KX decode
    included), at 1 and 16 scanning waves (4 in test_sequential), with and without a capacity, on
    tables where whole pod classes have no feasible node (FitError) and pods without a digit (score
    error)."""
    rng = np.random.default_rng(500 + 10 * combo + norm)
    f, pre, sc = PLUGIN_COMBOS[combo]
    ps = _plugins(oracle, f, pre, sc, 3, norm)
    with msh.DeviceContext(0, {"seq_waves": seq_waves}) as ctx:
        _set(ctx, msh, ps)
        for n, p_unsched in ((300, 1.0), (300, 0.0), (2000, 0.5)):
            u, nd, pd, pt = _rand_case(rng, n, 1001, p_unsched=p_unsched, p_tol=0.3)
            ctx.upload_nodes(u, nd)
            for cap in (0, 2):
                ctx.reset_node_pod_counts()
                got = ctx.schedule_sequential(pd, pt, cap)
                want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, cap)
                what = f"combo={combo} norm={norm} waves={seq_waves} n={n} unsched={p_unsched} cap={cap}"
                _assert_same(got, (want_i, want_s, want_st), what)
                assert (ctx.node_pod_counts() == want_counts).all(), what


@pytest.mark.parametrize("norm", [0, 3])
def test_empty_node_table(msh, gpu_ctx, oracle, norm):
    """A cluster without nodes (the reference's List returns none, minisched.go:40): every pod is a
    FitError in the batch, multi-batch and sequential entry points, with and without a capacity, and no
    node count exists; then a one-node table on the same ctx schedules again."""
    rng = np.random.default_rng(40 + norm)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 3, norm)
    _set(gpu_ctx, msh, ps)
    u0, nd0 = np.zeros(0, np.uint8), np.zeros(0, np.int8)
    pd, pt = _rand_case(rng, 1, 700)[2:]
    gpu_ctx.upload_nodes(u0, nd0)
    want = oracle.c_schedule_batch(u0, nd0, pd, pt, ps)
    assert (want[2] == 1).all()
    _assert_same(gpu_ctx.schedule_batch(pd, pt), want, "empty table batch")
    for cap in (0, 3):
        _assert_same(gpu_ctx.schedule_sequential(pd, pt, cap), want, f"empty table seq cap={cap}")
    assert gpu_ctx.node_pod_counts().size == 0
    u1, nd1 = np.zeros(1, np.uint8), np.array([int(pd[0]) if pd[0] >= 0 else 4], np.int8)
    gpu_ctx.upload_nodes(u1, nd1)
    for cap in (0, 3):
        gpu_ctx.reset_node_pod_counts()
        got = gpu_ctx.schedule_sequential(pd, pt, cap)
        wi, ws, wst, wc = oracle.c_schedule_sequential(u1, nd1, pd, pt, ps, cap)
        _assert_same(got, (wi, ws, wst), f"one-node table seq cap={cap}")
        assert (gpu_ctx.node_pod_counts() == wc).all()


@pytest.mark.parametrize("norm", [0, 1, 2, 3])
def test_sequential_capacity_fills(msh, gpu_ctx, oracle, norm):
    """The capacity form decides 4 pods per step against the step's starting state and resolves them in
    order: a pod whose match, non-match or class fallback an earlier pod of the step fills is decided
    again, and counts of several pods of one step on one node add up. Capacities 1 and 2 fill nodes
    inside nearly every step; runs of pods with one digit land on one node; tiny tables run out of
    nodes (FitError mid-batch); batch sizes are not multiples of 4 or 64; the counts carry over into a
    second call. Against the oracle's serial loop, in every normalize mode."""
    rng = np.random.default_rng(1700 + norm)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 3, norm)
    _set(gpu_ctx, msh, ps)
    for n in (1, 33, 64, 500, 8192, 12289, 16384, 24577, 32768):  # one wave up to 32,768 nodes (16 words per lane)
        u, nd, pd, pt = _rand_case(rng, n, 2003, p_unsched=0.3, p_tol=0.3)
        pd[100:400] = pd[100]  # a run of one digit
        for cap in (1, 2, 4, 15):
            gpu_ctx.upload_nodes(u, nd)  # zeroes the counts
            a = gpu_ctx.schedule_sequential(pd[:999], pt[:999], cap)
            b = gpu_ctx.schedule_sequential(pd[999:], pt[999:], cap)
            want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, cap)
            what = f"capacity fills norm={norm} n={n} cap={cap}"
            _assert_same(tuple(np.concatenate([x, y]) for x, y in zip(a, b)), (want_i, want_s, want_st), what)
            assert (gpu_ctx.node_pod_counts() == want_counts).all(), what


@pytest.mark.parametrize("norm", [0, 3])
def test_sequential_large_tables(msh, gpu_ctx, oracle, norm):
    """Tables far past the round-1 cap of 12,288 nodes: 300,000 nodes (15 scanning waves x 10 words
    per lane) without a capacity, 200,000 with one; counts carried over between calls; one node past
    each register limit is MSH_ERR_UNSUPPORTED, never a silent truncation."""
    rng = np.random.default_rng(300 + norm)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 1, norm)
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = _rand_case(rng, 300_000, 1500, p_unsched=0.3)
    nd[: 250_000][nd[: 250_000] == 7] = 8  # digit 7 only near the end: late first matches
    gpu_ctx.upload_nodes(u, nd)
    got = gpu_ctx.schedule_sequential(pd, pt, 0)
    want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, 0)
    _assert_same(got, (want_i, want_s, want_st), "seq 300k")
    assert (gpu_ctx.node_pod_counts() == want_counts).all()
    u2, nd2 = u[:200_000], nd[:200_000]
    gpu_ctx.upload_nodes(u2, nd2)
    a = gpu_ctx.schedule_sequential(pd[:700], pt[:700], 2)
    b = gpu_ctx.schedule_sequential(pd[700:], pt[700:], 2)  # continues from the carried counts
    want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u2, nd2, pd, pt, ps, 2)
    _assert_same(tuple(np.concatenate([x, y]) for x, y in zip(a, b)), (want_i, want_s, want_st), "seq cap 200k")
    assert (gpu_ctx.node_pod_counts() == want_counts).all()
    for n, cap in ((368_641, 0), (262_145, 1)):
        gpu_ctx.upload_nodes(np.zeros(n, np.uint8), np.zeros(n, np.int8))
        with pytest.raises(msh.MshError) as ei:
            gpu_ctx.schedule_sequential(pd[:10], pt[:10], cap)
        assert ei.value.code == msh._native.MSH_ERR_UNSUPPORTED
    gpu_ctx.upload_nodes(np.zeros(368_640, np.uint8), np.zeros(368_640, np.int8))
    got = gpu_ctx.schedule_sequential(pd[:50], pt[:50], 0)
    _assert_same(got, closed_form(np.zeros(368_640, np.uint8), np.zeros(368_640, np.int8), pd[:50], pt[:50])
                 if norm == 0 else oracle.c_schedule_batch(np.zeros(368_640, np.uint8), np.zeros(368_640, np.int8),
                                                           pd[:50], pt[:50], ps), "seq at the limit")


@pytest.mark.parametrize("norm,weight,cap", [(0, 1, 0), (3, 3, 0), (0, 1, 15)])
def test_c5_full_size_vs_oracle(msh, gpu_ctx, oracle, synth, norm, weight, cap):
    """BASELINE C5 at its own size: 5,000 nodes x 100,000 pods committed one at a time (the
    reference's strictly sequential loop, minisched/minisched.go:28-30,32-113), bench.py's synthetic
    snapshot, against the oracle's serial loop: idx / score / status of every pod and the per-node
    commit counts. NONE (the reference) and MIN-MAX at weight 3; and a capacity of 15 pods per node,
    which fills every digit's matching nodes (500 x 15 = 7,500 slots against ~10,000 pods per digit),
    so that later pods of a digit fall back to the first feasible non-full node."""
    u, nd, pd, pt = synth.make_soa(5000, 100_000)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], weight, norm)
    _set(gpu_ctx, msh, ps)
    gpu_ctx.upload_nodes(u, nd)  # zeroes the commit counts
    got = gpu_ctx.schedule_sequential(pd, pt, cap)
    want_i, want_s, want_st, want_counts = oracle.c_schedule_sequential(u, nd, pd, pt, ps, cap)
    _assert_same(got, (want_i, want_s, want_st), f"C5 norm={norm} w={weight} cap={cap}")
    counts = gpu_ctx.node_pod_counts()
    assert (counts == want_counts).all()
    assert counts.sum() == (want_st == 0).sum()
    if cap:
        assert counts.max() == cap


def test_sequential_commit_callback(msh, gpu_ctx, oracle):
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = _rand_case(np.random.default_rng(3), 200, 500)
    gpu_ctx.upload_nodes(u, nd)
    seen = []
    idx, _, status = gpu_ctx.schedule_sequential(pd, pt, 0, on_commit=lambda j, i, s: seen.append((j, i)))
    assert seen == [(j, int(idx[j])) for j in range(len(pd)) if status[j] == 0]


@pytest.mark.parametrize("norm", [0, 1, 2, 3])
def test_node_shards_merge(msh, gpu_ctx, oracle, norm):
    """Node-sharded mode: per-shard keys, element-wise MAX, device decode == unsharded."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(11 + norm)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 1, norm)
    u, nd, pd, pt = _rand_case(rng, 9000, 4000)
    want = oracle.c_schedule_batch(u, nd, pd, pt, ps)
    dev = torch.device("cuda:0")
    d_pd = torch.from_numpy(pd).to(dev)
    d_pt = torch.from_numpy(pt).to(dev)
    p = len(pd)
    bounds = [0, 1234, 5000, 5001, 9000]
    ctxs, merged = [], None
    for a, b in zip(bounds[:-1], bounds[1:]):
        c = msh.DeviceContext(0)
        _set(c, msh, ps)
        c.upload_nodes(u[a:b], nd[a:b])
        klen = c.shard_keys_len(p)
        # ABI v7: per pod, the first feasible match and the first feasible non-match (8 B per pod)
        assert klen == 2 * p and not c.keys_slot1_is_any()
        keys = torch.full((klen,), -7, dtype=torch.int32, device=dev)  # every entry must be written
        c.shard_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), a, keys.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
        assert int(keys.min()) >= 0
        merged = keys if merged is None else torch.maximum(merged, keys)
        ctxs.append(c)
    oi = torch.empty(p, dtype=torch.int32, device=dev)
    osc = torch.empty(p, dtype=torch.int64, device=dev)
    ost = torch.empty(p, dtype=torch.int32, device=dev)
    ctxs[0].decode_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), merged.data_ptr(), oi.data_ptr(),
                               osc.data_ptr(), ost.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    _assert_same((oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy()), want, f"shards norm={norm}")
    for c in ctxs:
        c.close()


def test_determinism_device_entry(msh, gpu_ctx, oracle, synth):
    torch = pytest.importorskip("torch")
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = synth.make_soa(5000, 50_000)
    gpu_ctx.upload_nodes(u, nd)
    dev = torch.device("cuda:0")
    d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
    outs = []
    for _ in range(3):
        oi = torch.empty(len(pd), dtype=torch.int32, device=dev)
        osc = torch.empty(len(pd), dtype=torch.int64, device=dev)
        ost = torch.empty(len(pd), dtype=torch.int32, device=dev)
        gpu_ctx.schedule_batch_device(len(pd), d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(),
                                      ost.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append((oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy()))
    for o in outs[1:]:
        _assert_same(o, outs[0], "repeat")
    _assert_same(outs[0], oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8), "device entry")


@pytest.mark.parametrize("n,norm", [(5000, 0), (100_000, 0), (100_000, 3), (20_000, 2)])
def test_pipelined_streams(msh, gpu_ctx, oracle, n, norm):
    """Independent batches in flight on several HIP streams of ONE ctx, as bench.py pipelines them,
    in the identity and the KX modes, at several slice counts: every batch gets the oracle's
    answer (no per-ctx scratch is shared between launches)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(n + norm)
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 1, norm)
    _set(gpu_ctx, msh, ps)
    u, nd, _, _ = _rand_case(rng, n, 1, p_unsched=0.2, p_tol=0.3)
    gpu_ctx.upload_nodes(u, nd)
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    batches, outs = [], []
    for k in range(6):
        _, _, pd, pt = _rand_case(rng, 1, 3000 + 500 * k, p_tol=0.3)
        batches.append((pd, pt))
        d = (torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev))
        o = (torch.empty(len(pd), dtype=torch.int32, device=dev), torch.empty(len(pd), dtype=torch.int64, device=dev),
             torch.empty(len(pd), dtype=torch.int32, device=dev))
        outs.append((d, o))
    torch.cuda.synchronize()
    for k, ((d_pd, d_pt), (oi, osc, ost)) in enumerate(outs):
        gpu_ctx.schedule_batch_device(len(d_pd), d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(),
                                      ost.data_ptr(), streams[k % 3].cuda_stream)
    torch.cuda.synchronize()
    for (pd, pt), (_, (oi, osc, ost)) in zip(batches, outs):
        want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
        _assert_same((oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy()), want, f"n={n} norm={norm}")


@pytest.mark.parametrize("norm", [0, 3])
def test_scores_optional(msh, gpu_ctx, oracle, synth, norm):
    """out_score = NULL (ABI v4) through every entry point that takes it: idx and status as with
    scores, nothing written where the scores would go (device entry points keep a sentinel-filled
    buffer untouched)."""
    torch = pytest.importorskip("torch")
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 2, norm)
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = synth.make_soa(5000, 50_000)
    gpu_ctx.upload_nodes(u, nd)
    want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
    p = len(pd)

    def same2(got, what):
        assert got[1] is None
        assert (got[0] == want[0]).all() and (got[2] == want[2]).all(), what

    same2(gpu_ctx.schedule_batch(pd, pt, scores=False), "pageable")
    hpd, hpt = msh.pinned_empty(p, np.int8), msh.pinned_empty(p, np.uint8)
    hpd[:], hpt[:] = pd, pt
    outs = (msh.pinned_empty(p, np.int32), None, msh.pinned_empty(p, np.int32))
    same2(gpu_ctx.schedule_batch(hpd, hpt, out=outs, scores=False), "pinned")
    dev = torch.device("cuda:0")
    d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
    oi, ost = torch.empty(p, dtype=torch.int32, device=dev), torch.empty(p, dtype=torch.int32, device=dev)
    gpu_ctx.schedule_batch_device(p, d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), 0, ost.data_ptr())
    torch.cuda.synchronize()
    same2((oi.cpu().numpy(), None, ost.cpu().numpy()), "device batch")
    gpu_ctx.reset_node_pod_counts()
    gpu_ctx.schedule_sequential_device(p, d_pd.data_ptr(), d_pt.data_ptr(), 0, oi.data_ptr(), 0, ost.data_ptr())
    torch.cuda.synchronize()
    same2((oi.cpu().numpy(), None, ost.cpu().numpy()), "device sequential")
    klen = gpu_ctx.shard_keys_len(p)
    keys = torch.zeros(klen, dtype=torch.int32, device=dev)
    gpu_ctx.shard_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), 0, keys.data_ptr())
    gpu_ctx.decode_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), keys.data_ptr(), oi.data_ptr(), 0,
                               ost.data_ptr())
    torch.cuda.synchronize()
    same2((oi.cpu().numpy(), None, ost.cpu().numpy()), "shard keys + decode")


@pytest.mark.parametrize("change", ["patch", "upload"])
def test_table_change_while_batches_in_flight(msh, gpu_ctx, oracle, change):
    """msh_patch_nodes / msh_upload_nodes while batches of the same ctx queued on another stream
    still read the tables: the rebuild is ordered after the ctx's own launches in flight (one event
    per caller stream), so the queued batches see the old table and later ones the new."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(77)
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    n = 20_000
    u, nd, _, _ = _rand_case(rng, n, 1, p_unsched=0.2)
    gpu_ctx.upload_nodes(u, nd)
    dev = torch.device("cuda:0")
    side = torch.cuda.Stream(dev)
    _, _, pd, pt = _rand_case(rng, 1, 200_000, p_tol=0.3)
    d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
    old = [(torch.empty(len(pd), dtype=torch.int32, device=dev), torch.empty(len(pd), dtype=torch.int64, device=dev),
            torch.empty(len(pd), dtype=torch.int32, device=dev)) for _ in range(4)]
    torch.cuda.synchronize()
    for oi, osc, ost in old:  # queued, not waited for
        gpu_ctx.schedule_batch_device(len(pd), d_pd.data_ptr(), d_pt.data_ptr(), oi.data_ptr(), osc.data_ptr(),
                                      ost.data_ptr(), side.cuda_stream)
    u2, nd2 = u.copy(), nd.copy()
    idx = rng.choice(n, 6000, replace=False).astype(np.int32)
    u2[idx] ^= 1
    nd2[idx[:3000]] = rng.integers(-1, 10, 3000).astype(np.int8)
    if change == "patch":
        gpu_ctx.patch_nodes(idx, u2[idx], nd2[idx])
    else:
        gpu_ctx.upload_nodes(u2, nd2)
    new = gpu_ctx.schedule_batch(pd, pt)
    torch.cuda.synchronize()
    want_old = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
    for oi, osc, ost in old:
        _assert_same((oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy()), want_old, f"{change}: queued batch")
    _assert_same(new, oracle.c_schedule_batch(u2, nd2, pd, pt, ps, threads=8), f"{change}: after the change")


@pytest.mark.parametrize("change", ["patch", "upload", "reset_counts"])
def test_table_change_does_not_wait_for_other_ctx(msh, oracle, change):
    """A table change of ctx A waits for A's own launches only (verdict r2 #3): ctx B has ~10 ms of
    C4-size batches queued on its own stream; A's one-node cordon flip (the f2 informer Update path,
    eventhandler.go:45-65), re-upload or count reset returns while B's batches are still running. A's
    batch queued before the change sees the old table, A's batch after it the new one, and B's
    outputs are all bit-exact vs the oracle."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(91)
    dev = torch.device("cuda:0")
    ua, nda, _, _ = _rand_case(rng, 5000, 1, p_unsched=0.2)
    ub, ndb, _, _ = _rand_case(rng, 100_000, 1, p_unsched=0.1)
    _, _, pd, pt = _rand_case(rng, 1, 100_000, p_tol=0.2)
    _, _, pdb, ptb = _rand_case(rng, 1, 1_000_000, p_tol=0.05)
    with msh.DeviceContext(0) as A, msh.DeviceContext(0) as B:
        A.upload_nodes(ua, nda)
        B.upload_nodes(ub, ndb)
        sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        a_old = _dev_batch(torch, dev, pd, pt)
        b_bufs = [_dev_batch(torch, dev, pdb, ptb) for _ in range(2)]
        done_b = torch.cuda.Event()
        torch.cuda.synchronize()
        for k in range(36):  # ~275 us each on one MI355X: ~10 ms queued on B's stream
            t = b_bufs[k % 2]
            B.schedule_batch_device(len(pdb), t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(),
                                    t[4].data_ptr(), sb.cuda_stream)
        done_b.record(sb)
        A.schedule_batch_device(len(pd), *[x.data_ptr() for x in a_old], sa.cuda_stream)
        u2, nd2 = ua.copy(), nda.copy()
        u2[17] ^= 1
        if change == "patch":
            A.patch_nodes(np.array([17], np.int32), u2[17:18], nd2[17:18])
        elif change == "upload":
            A.upload_nodes(u2, nd2)
        else:
            A.reset_node_pod_counts()
            u2 = ua
        b_running = not done_b.query()
        a_new = A.schedule_batch(pd, pt)
        torch.cuda.synchronize()
        assert b_running, f"{change} on ctx A waited for ctx B's queued batches"
        _assert_same([a_old[i].cpu().numpy() for i in (2, 3, 4)], oracle.c_schedule_batch(ua, nda, pd, pt),
                     f"{change}: A before")
        _assert_same(a_new, oracle.c_schedule_batch(u2, nd2, pd, pt), f"{change}: A after")
        want_b = closed_form(ub, ndb, pdb, ptb)
        for t in b_bufs:
            _assert_same([t[i].cpu().numpy() for i in (2, 3, 4)], want_b, f"{change}: B")


def test_maximum_node_table(msh, gpu_ctx, synth):
    """The largest table a ctx accepts (2^24 - 2 nodes, 261 compute tiles) against the closed
    form, with matches placed only in the last tile for some digits; one node more is
    MSH_ERR_INVALID, never a silent truncation."""
    n = 0xFFFFFE
    rng = np.random.default_rng(24)
    u = (rng.random(n) < 0.5).astype(np.uint8)
    nd = np.full(n, 9, np.int8)
    nd[-3000:] = rng.integers(0, 9, 3000).astype(np.int8)   # digits 0..8 only near the end
    pd = rng.integers(-1, 10, 512).astype(np.int8)
    pt = (rng.random(512) < 0.3).astype(np.uint8)
    gpu_ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 1)])
    gpu_ctx.upload_nodes(u, nd)
    got = gpu_ctx.schedule_batch(pd, pt)
    _assert_same(got, closed_form(u, nd, pd, pt), "max table")
    placed = (got[2] == 0) & (pd >= 0) & (pd <= 8)
    assert placed.any() and (got[0][placed] >= n - 3000).all()
    with pytest.raises(msh.MshError):
        gpu_ctx.upload_nodes(np.zeros(n + 1, np.uint8), np.zeros(n + 1, np.int8))
    gpu_ctx.upload_nodes(u[:10], nd[:10])  # the ctx stays usable after the rejected upload
    _assert_same(gpu_ctx.schedule_batch(pd, pt), closed_form(u[:10], nd[:10], pd, pt), "after reject")


@pytest.mark.parametrize("slices", ["1", "2", "4"])
@pytest.mark.parametrize("n", [20_000, 70_000])
def test_pair_slices(msh, oracle, n, slices):
    """Few pods against a large table: SLICES waves of pair_kernel share each 64-pod block, each
    scanning a range of 256-node groups, firsts merged by min in LDS. Every slice count
    (msh_options.pair_slices, read once by msh_create_ex) against the oracle, for the batch and the shard-key
    entry points, in the identity-like and the non-match (MINMAX) modes."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(n + int(slices))
    u, nd, pd, pt = _rand_case(rng, n, 1537, p_unsched=0.2, p_tol=0.3)
    nd[: n // 2][nd[: n // 2] == 3] = 4  # digit 3 only in the second half: late first matches
    dev = torch.device("cuda:0")
    d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
    p = len(pd)
    with msh.DeviceContext(0, {"pair_slices": slices}) as ctx:
        for norm in (0, 3):
            ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 1, norm)
            _set(ctx, msh, ps)
            ctx.upload_nodes(u, nd)
            want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
            _assert_same(ctx.schedule_batch(pd, pt), want, f"slices={slices} n={n} norm={norm}")
            keys = torch.empty(ctx.shard_keys_len(p), dtype=torch.int32, device=dev)
            ctx.shard_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), 0, keys.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
            oi = torch.empty(p, dtype=torch.int32, device=dev)
            osc = torch.empty(p, dtype=torch.int64, device=dev)
            ost = torch.empty(p, dtype=torch.int32, device=dev)
            ctx.decode_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), keys.data_ptr(), oi.data_ptr(),
                                   osc.data_ptr(), ost.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            _assert_same((oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy()), want,
                         f"keys slices={slices} n={n} norm={norm}")


@pytest.mark.parametrize("p", [1, 2, 3, 63, 64, 65, 127, 128, 129, 1000, 8191, 65_535, 65_536, 65_537, 100_003,
                               131_073, 300_001, 1_000_003])
def test_ragged_pod_blocks(msh, gpu_ctx, oracle, p):
    """Pod counts on either side of the 64-pod block and of the slice-count cuts (one block per
    workgroup; 4, 2 and 1 slice waves as the batch grows), against the oracle."""
    rng = np.random.default_rng(p)
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = _rand_case(rng, 5000, p, p_unsched=0.25, p_tol=0.3)
    gpu_ctx.upload_nodes(u, nd)
    want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
    _assert_same(gpu_ctx.schedule_batch(pd, pt), want, f"p={p}")


@pytest.mark.parametrize("norm", [0, 3])
def test_host_buffer_paths(msh, gpu_ctx, oracle, synth, norm):
    """msh_schedule_batch / msh_schedule_sequential with page-locked buffers (zero-copy: the
    kernel writes the caller's outputs over PCIe) and with pageable ones (staged), mixed, and a
    batch large enough for the threaded copy-out: identical to the oracle every time."""
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 3, norm)
    _set(gpu_ctx, msh, ps)
    u, nd, pd, pt = synth.make_soa(5000, 100_000)
    gpu_ctx.upload_nodes(u, nd)
    want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
    p = len(pd)
    hpd, hpt = msh.pinned_empty(p, np.int8), msh.pinned_empty(p, np.uint8)
    hpd[:], hpt[:] = pd, pt
    outs = (msh.pinned_empty(p, np.int32), msh.pinned_empty(p, np.int64), msh.pinned_empty(p, np.int32))
    for o in outs:
        o.fill(-7)
    got = gpu_ctx.schedule_batch(hpd, hpt, out=outs)
    assert all(g is o for g, o in zip(got, outs))
    _assert_same(got, want, "pinned in / pinned out")
    _assert_same(gpu_ctx.schedule_batch(pd, pt), want, "pageable in / pageable out")
    _assert_same(gpu_ctx.schedule_batch(hpd, hpt), want, "pinned in / pageable out")
    for o in outs:
        o.fill(-7)
    _assert_same(gpu_ctx.schedule_batch(pd, pt, out=outs), want, "pageable in / pinned out")
    # ragged batch sizes through the staged and the zero-copy input paths
    for q in (2 * 16384 + 7, 3 * 16384 + 100, 99_937):
        _assert_same(gpu_ctx.schedule_batch(pd[:q], pt[:q]), tuple(w[:q] for w in want[:3]), f"pageable {q}")
        _assert_same(gpu_ctx.schedule_batch(hpd[:q], hpt[:q]), tuple(w[:q] for w in want[:3]), f"pinned in {q}")
    gpu_ctx.reset_node_pod_counts()
    for o in outs:
        o.fill(-7)
    got = gpu_ctx.schedule_sequential(hpd[:20_000], hpt[:20_000], 0, out=outs)
    _assert_same(tuple(g[:20_000] for g in got), tuple(w[:20_000] for w in want[:3]), "sequential pinned")
    assert (outs[0][20_000:] == -7).all()  # nothing written past p


def test_async_host_batches(msh, gpu_ctx, oracle):
    """msh_schedule_batch_async + msh_wait (ABI v5): six batches in page-locked buffers submitted
    back to back (the fifth and sixth wait for the ring's oldest: MSH_ASYNC_DEPTH = 4), waited
    out of order; every batch bit-exact vs the oracle. Pageable buffers are rejected, an unknown
    ticket is MSH_ERR_INVALID, an empty batch gets a ticket, and a synchronous call completes all."""
    rng = np.random.default_rng(606)
    ps = oracle.PluginSet()
    _set(gpu_ctx, msh, ps)
    u, nd, _, _ = _rand_case(rng, 5000, 1, p_unsched=0.2)
    gpu_ctx.upload_nodes(u, nd)
    sets = []
    for k in range(6):
        _, _, pd, pt = _rand_case(rng, 1, [100_000, 1, 64, 4097, 99_999, 0][k], p_tol=0.1)
        hpd, hpt = msh.pinned_empty(len(pd), np.int8), msh.pinned_empty(len(pd), np.uint8)
        hpd[:], hpt[:] = pd, pt
        outs = (msh.pinned_empty(len(pd), np.int32), msh.pinned_empty(len(pd), np.int64),
                msh.pinned_empty(len(pd), np.int32))
        for o in outs:
            o.fill(-7)
        sets.append((pd, pt, hpd, hpt, outs))
    tickets = [gpu_ctx.schedule_batch_async(hpd, hpt, outs) for _, _, hpd, hpt, outs in sets]
    assert tickets == list(range(tickets[0], tickets[0] + 6))
    for k in (3, 0, 5, 1, 4, 2):
        gpu_ctx.wait(tickets[k])
        pd, pt, _, _, outs = sets[k]
        _assert_same(outs, oracle.c_schedule_batch(u, nd, pd, pt, ps), f"async batch {k}")
    with pytest.raises(msh.MshError):
        gpu_ctx.wait(tickets[-1] + 1)
    with pytest.raises(msh.MshError):
        gpu_ctx.wait(0)
    pd, pt = sets[0][0], sets[0][1]
    with pytest.raises(msh.MshError):  # pageable buffers
        gpu_ctx.schedule_batch_async(pd, pt, (np.empty(len(pd), np.int32), np.empty(len(pd), np.int64),
                                              np.empty(len(pd), np.int32)))
    _, _, hpd, hpt, outs = sets[3]
    t = gpu_ctx.schedule_batch_async(hpd, hpt, outs, scores=False)  # out_score = NULL
    gpu_ctx.schedule_batch(sets[0][0], sets[0][1])  # a synchronous call drains the ctx's stream
    gpu_ctx.wait(t)  # already complete
    pd3, pt3 = sets[3][0], sets[3][1]
    want = oracle.c_schedule_batch(u, nd, pd3, pt3, ps)
    assert (outs[0] == want[0]).all() and (outs[2] == want[2]).all()


def _dev_batch(torch, dev, pd, pt, scores=True):
    return [torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev),
            torch.full((len(pd),), -7, dtype=torch.int32, device=dev),
            torch.full((len(pd),), -7, dtype=torch.int64, device=dev) if scores else None,
            torch.full((len(pd),), -7, dtype=torch.int32, device=dev)]


def _desc(t):
    return (len(t[0]), t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr() if t[3] is not None else 0,
            t[4].data_ptr())


@pytest.mark.parametrize("norm", [0, 1, 2, 3])
@pytest.mark.parametrize("nb", [1, 3, 8, 9, 17, 32, 33, 70])
def test_multi_batch_launch(msh, gpu_ctx, oracle, norm, nb):
    """msh_schedule_batches_device (ABI v5): nb independent batches, up to 32 per launch, ragged pod
    counts (empty and one-pod batches among them), some without scores; every batch bit-exact vs
    the oracle, and nothing written past a batch's end."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(77 * nb + norm)
    sizes = ([0, 1, 64, 65, 255, 257, 100_003, 5000, 333, 4096, 1, 2, 700, 64, 128, 129, 999] * 5)[:nb]
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 3, norm)
    _set(gpu_ctx, msh, ps)
    u, nd, _, _ = _rand_case(rng, 5000, 1)
    gpu_ctx.upload_nodes(u, nd)
    cases = []
    for k, p in enumerate(sizes):
        _, _, pd, pt = _rand_case(rng, 1, p)
        t = _dev_batch(torch, dev, pd, pt, scores=(k % 3 != 2))
        pad = torch.full((8,), -7, dtype=torch.int32, device=dev)  # canary behind nothing: outputs sized p
        cases.append((pd, pt, t, pad))
    descs = gpu_ctx.batch_descs([_desc(c[2]) for c in cases])
    stream = torch.cuda.current_stream().cuda_stream
    gpu_ctx.schedule_batches_device(descs, stream=stream)
    torch.cuda.synchronize()
    for k, (pd, pt, t, _) in enumerate(cases):
        want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
        gi, gst = t[2].cpu().numpy(), t[4].cpu().numpy()
        gs = t[3].cpu().numpy() if t[3] is not None else want[1]
        _assert_same((gi, gs, gst), want, f"batch {k} of {nb} (p={len(pd)}) norm={norm}")
    # a second submission on the same descriptors gives the same outputs (buffers reused)
    for _, _, t, _ in cases:
        t[2].fill_(-7)
    gpu_ctx.schedule_batches_device(descs, stream=stream)
    torch.cuda.synchronize()
    for k, (pd, pt, t, _) in enumerate(cases):
        assert (t[2].cpu().numpy() == oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)[0]).all(), k


@pytest.mark.parametrize("n,norm", [(5000, 0), (5000, 3), (8192, 1), (40_000, 2)])
def test_multi_batch_full_launch(msh, oracle, n, norm):
    """A full multi-batch launch (32 batches of ~100k pods, ragged, empty and one-pod batches among them)
    on the per-pair kernel with its planes staged in LDS (auto: the launch fills the chip; 4-wave
    workgroups up to 32,768 nodes, 16-wave ones above) and with scalar-loaded planes; every batch
    bit-exact vs the oracle."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(4242 + n + norm)
    # 32 batches of ~100k pods; at 40,000 nodes ~20k (still 10,000 waves: the 16-wave form's launch)
    f = 1 if n <= 8192 else 5
    sizes = [x // f for x in [100_000, 99_937, 100_003, 64, 0, 1, 99_999, 98_304] + [100_000 - 7 * k for k in range(24)]]
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 2, norm)
    u, nd, _, _ = _rand_case(rng, n, 1)
    pods = [_rand_case(rng, 1, p)[2:] for p in sizes]
    wants = [oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=16) for pd, pt in pods]
    for planes in ("auto", "sgpr"):
        with msh.DeviceContext(0, {"pair_planes": planes}) as ctx:
            _set(ctx, msh, ps)
            ctx.upload_nodes(u, nd)
            bufs = [_dev_batch(torch, dev, pd, pt, scores=(k % 5 != 4)) for k, (pd, pt) in enumerate(pods)]
            ctx.schedule_batches_device(ctx.batch_descs([_desc(t) for t in bufs]),
                                        stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            for k, (t, want) in enumerate(zip(bufs, wants)):
                gi, gst = t[2].cpu().numpy(), t[4].cpu().numpy()
                gs = t[3].cpu().numpy() if t[3] is not None else want[1]
                _assert_same((gi, gs, gst), want, f"{planes} batch {k} (p={len(pods[k][0])}) n={n} norm={norm}")


@pytest.mark.parametrize("noax", ["auto", "flip"])
@pytest.mark.parametrize("norm", [0, 1, 2, 3])
@pytest.mark.parametrize("n", [7000, 40_000])
def test_multi_batch_launch_lds(msh, oracle, n, norm, noax):
    """The LDS-staged pair kernel forced on small ragged multi-batch launches (pair_planes lds): each
    built instance — 4-wave workgroups (7,000 nodes) and 16-wave ones (40,000), identity-like and
    REVERSE / MINMAX — in every normalize mode, with group 0 scanned first and last (pair_noax auto
    and the other value); workgroups whose blocks end inside or before a batch, empty and one-pod batches,
    NULL scores."""
    torch = pytest.importorskip("torch")
    kx = norm in (2, 3)
    opts = _pair_opts("lds" + ("" if noax == "auto" else ("-axlast" if kx else "-noax")))
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(99 * n + norm)
    sizes = [0, 1, 64, 65, 255, 257, 20_003, 5000, 333, 4096, 1, 2, 700, 64, 128, 1025, 999] * 2
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 3, norm)
    u, nd, _, _ = _rand_case(rng, n, 1)
    pods = [_rand_case(rng, 1, p)[2:] for p in sizes]
    with msh.DeviceContext(0, opts) as ctx:
        _set(ctx, msh, ps)
        ctx.upload_nodes(u, nd)
        bufs = [_dev_batch(torch, dev, pd, pt, scores=(k % 4 != 3)) for k, (pd, pt) in enumerate(pods)]
        ctx.schedule_batches_device(ctx.batch_descs([_desc(t) for t in bufs]),
                                    stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for k, (t, (pd, pt)) in enumerate(zip(bufs, pods)):
            want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
            gi, gst = t[2].cpu().numpy(), t[4].cpu().numpy()
            gs = t[3].cpu().numpy() if t[3] is not None else want[1]
            _assert_same((gi, gs, gst), want, f"lds batch {k} (p={len(pd)}) n={n} norm={norm} noax={noax}")


def test_multi_batch_invalid(msh, gpu_ctx):
    """Bad descriptors are rejected before any launch (MSH_ERR_INVALID), and nb = 0 is a no-op."""
    N = msh._native
    fast = gpu_ctx._fast
    assert fast.schedule_batches_device(gpu_ctx._hv(), 0, None, None) == 0
    assert fast.schedule_batches_device(gpu_ctx._hv(), 2, None, None) == N.MSH_ERR_INVALID
    assert fast.schedule_batches_device(gpu_ctx._hv(), -1, None, None) == N.MSH_ERR_INVALID
    bad = gpu_ctx.batch_descs([(-1, 1, 1, 1, 0, 1)])
    with pytest.raises(msh.MshError):
        gpu_ctx.schedule_batches_device(bad)
    bad = gpu_ctx.batch_descs([(10, 1, 0, 1, 0, 1)])  # null pod_tol
    with pytest.raises(msh.MshError):
        gpu_ctx.schedule_batches_device(bad)


@pytest.mark.parametrize("planes", ["auto", "sgpr", "lds", "lds-noax", "lds-axlast"])
@pytest.mark.parametrize("n", [1000, 8192, 8193, 20_000, 32_768, 70_000, 106_496, 106_497])
def test_pair_kernel_late_matches(msh, oracle, n, planes):
    """pair_kernel re-reads the first group with a hit from memory when it lies above the lowest group
    of the wave's range (kept in registers): digit 3 only in the second half of the table makes those
    pods' first matches late. Batch, multi-batch and shard-key entry points, NONE and MINMAX, on tables
    with and without a padded top group."""
    torch = pytest.importorskip("torch")
    opts = _pair_opts(planes)  # lds: 4-wave workgroups up to 32,768 nodes, 16-wave up to
    # 106,496 (106,497 falls back to scalar-loaded planes); auto (3,000 pods: the slice kernel): planes
    # staged in LDS up to 32,768 nodes, scalar loads above
    rng = np.random.default_rng(n + 4)
    u, nd, pd, pt = _rand_case(rng, n, 3000, p_unsched=0.2, p_tol=0.3)
    nd[: n // 2][nd[: n // 2] == 3] = 4
    dev = torch.device("cuda:0")
    p = len(pd)
    with msh.DeviceContext(0, opts) as ctx:
        for norm in (0, 3):
            ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], 1, norm)
            _set(ctx, msh, ps)
            ctx.upload_nodes(u, nd)
            want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
            _assert_same(ctx.schedule_batch(pd, pt), want, f"pair n={n} norm={norm}")
            halves = [_dev_batch(torch, dev, pd[: p // 3], pt[: p // 3]), _dev_batch(torch, dev, pd[p // 3:], pt[p // 3:])]
            descs = ctx.batch_descs([_desc(t) for t in halves])
            ctx.schedule_batches_device(descs, stream=torch.cuda.current_stream().cuda_stream)
            t0, t1 = halves
            keys = torch.empty(ctx.shard_keys_len(p), dtype=torch.int32, device=dev)
            d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
            ctx.shard_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), 0, keys.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
            out = _dev_batch(torch, dev, pd, pt)
            ctx.decode_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), keys.data_ptr(), out[2].data_ptr(),
                                   out[3].data_ptr(), out[4].data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            got = [np.concatenate([t0[i].cpu().numpy(), t1[i].cpu().numpy()]) for i in (2, 3, 4)]
            _assert_same(got, want, f"multi n={n} norm={norm}")
            _assert_same([out[i].cpu().numpy() for i in (2, 3, 4)], want, f"keys n={n} norm={norm}")


@pytest.mark.parametrize("planes,slices", [("auto", 0), ("auto", 1), ("auto", 2), ("auto", 4),
                                           ("sgpr", 0), ("sgpr", 1), ("sgpr", 2), ("sgpr", 4), ("lds", 0),
                                           ("lds-noax", 0), ("lds-axlast", 0)])
@pytest.mark.parametrize("n", [1000, 5000, 20_000])
def test_pair_kernel_late_feasible(msh, oracle, n, planes, slices):
    """The identity-like modes take a pod's first feasible node from the scalar unit's per-group
    feasibility (V & ~X, V): with the first 60% of the table unschedulable and digit 7 only there,
    a non-tolerating pod of digit 7 has no feasible match and its first feasible node lies far above
    the lowest group of every slice; tolerating pods match early. NONE, DEFAULT, no NodeNumber score,
    MINMAX; batch and shard keys; every slice count."""
    torch = pytest.importorskip("torch")
    opts = {**_pair_opts(planes), "pair_slices": slices}  # "lds": the LDS-staged form at any launch size
    rng = np.random.default_rng(n + slices)
    u, nd, pd, pt = _rand_case(rng, n, 2000, p_unsched=0.0, p_tol=0.2)
    cut = int(n * 0.6)
    u[:cut] = 1
    nd[cut:][nd[cut:] == 7] = 8
    pd[: 600] = 7
    dev = torch.device("cuda:0")
    p = len(pd)
    lists = [(["NodeNumber"], 1, 0), (["NodeNumber"], 2, 1), ([], 1, 0), (["NodeNumber"], 1, 3)]
    with msh.DeviceContext(0, opts) as ctx:
        for score, w, norm in lists:
            ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], score, w, norm)
            _set(ctx, msh, ps)
            ctx.upload_nodes(u, nd)
            want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8)
            _assert_same(ctx.schedule_batch(pd, pt), want, f"late-feasible n={n} {score} norm={norm}")
            keys = torch.empty(ctx.shard_keys_len(p), dtype=torch.int32, device=dev)
            d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
            st = torch.cuda.current_stream().cuda_stream
            ctx.shard_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), 0, keys.data_ptr(), st)
            out = _dev_batch(torch, dev, pd, pt)
            ctx.decode_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), keys.data_ptr(), out[2].data_ptr(),
                                   out[3].data_ptr(), out[4].data_ptr(), st)
            torch.cuda.synchronize()
            _assert_same([out[i].cpu().numpy() for i in (2, 3, 4)], want, f"late-feasible keys n={n} norm={norm}")


@pytest.mark.parametrize("kernel", ["pair", "generic"])
def test_batch_kernel_ab(msh, oracle, kernel):
    """The default per-pair kernel and generic_kernel (msh_options.batch_kernel generic, read once by
    msh_create_ex: explicit int64 totals for the reference list) place identically at C3 size, multi-batch
    included; a value outside the field's set is rejected at msh_create_ex."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    u, nd, pd, pt = _rand_case(rng, 5000, 100_000, p_unsched=0.1, p_tol=0.05)
    dev = torch.device("cuda:0")
    with msh.DeviceContext(0, {"batch_kernel": kernel}) as ctx:
        ctx.upload_nodes(u, nd)
        want = oracle.c_schedule_batch(u, nd, pd, pt, threads=8)
        _assert_same(ctx.schedule_batch(pd, pt), want, kernel)
        ts = [_dev_batch(torch, dev, pd, pt) for _ in range(3)]
        ctx.schedule_batches_device(ctx.batch_descs([_desc(t) for t in ts]),
                                    stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for t in ts:
            _assert_same([t[i].cpu().numpy() for i in (2, 3, 4)], want, f"{kernel} multi")
    with pytest.raises(msh.MshError, match="batch_kernel"):
        msh.DeviceContext(0, {"batch_kernel": 2})


# ---- the generic score pipeline (score-column plugins; north_star stages 1-5 with explicit int64 scores)

GENERIC_LISTS = [
    ["ScoreColumn0"],
    ["NodeNumber", "ScoreColumn0"],
    ["ScoreColumn1", "NodeNumber", "ScoreColumn0"],
    ["ScoreColumn0", "ScoreColumn1", "ScoreColumn2", "ScoreColumn3", "NodeNumber"],
]


def _cols(rng, n):
    return {0: rng.integers(-(1 << 31), (1 << 31) + 1, n), 1: rng.integers(0, 5, n) * 11,
            2: np.full(n, 7), 3: rng.integers(-3, 3, n)}


@pytest.mark.parametrize("lst", range(len(GENERIC_LISTS)))
@pytest.mark.parametrize("norm", [0, 1, 2, 3])
def test_generic_pipeline_score_columns(msh, gpu_ctx, oracle, lst, norm):
    """Score lists with score-column plugins run on generic_kernel: per pair an explicit int64
    total (weight x NormalizeScore(raw) summed, Go int64 wrap), per-plugin extents by shuffle + LDS
    reduction, wave-shuffle argmax; bit-exact vs the oracle's RunScorePlugins restatement for
    tables across tile boundaries, ragged pod blocks, weights up to 2^32, tied / negative columns."""
    rng = np.random.default_rng(31 * lst + norm)
    names = GENERIC_LISTS[lst]
    weights = [int(w) for w in rng.choice([1, 3, 1 << 32], len(names))]
    modes = [norm if k % 2 == 0 else (norm + k) % 4 for k in range(len(names))]
    pre = ["NodeNumber"] if "NodeNumber" in names else []
    ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=pre, score=names, weights=weights, normalize=modes)
    gpu_ctx.set_plugins(ps.filters, ps.prescore, [msh.ScorePluginConfig(s, w, msh.Normalize(m))
                                                  for s, w, m in zip(names, weights, modes)])
    for n, p in [(1, 7), (70, 300), (1025, 1000), (5000, 4097), (20_000, 513)]:
        u, nd, pd, pt = _rand_case(rng, n, p, p_unsched=0.3, p_tol=0.2)
        cols = _cols(rng, n)
        gpu_ctx.upload_nodes(u, nd)
        for k in range(4):
            gpu_ctx.upload_score_column(f"ScoreColumn{k}", cols[k])
        got = gpu_ctx.schedule_batch(pd, pt)
        want = oracle.c_schedule_batch(u, nd, pd, pt, ps, cols=cols)
        _assert_same(got, want, f"generic {names} modes={modes} n={n} p={p}")


W32_LISTS = [
    # (name, weight, normalize) per score plugin; small weights and columns 1..3 (|raw| <= 44): every
    # feasible total fits 31 bits, so generic_kernel runs its 32-bit keys
    [("NodeNumber", 2, 0)],
    [("NodeNumber", 3, 1)],
    [("NodeNumber", 1, 0), ("ScoreColumn1", 2, 1)],           # one DEFAULT column (no min-max offset)
    [("NodeNumber", 2, 3), ("ScoreColumn1", 3, 3)],           # one MIN-MAX column
    [("ScoreColumn1", 1, 2), ("NodeNumber", 1, 0)],           # one REVERSE column
    [("NodeNumber", 1, 1), ("ScoreColumn3", 5, 0)],           # a column without a normalizer (node-only sum)
    [("ScoreColumn2", 2, 0), ("ScoreColumn1", 1, 3), ("ScoreColumn3", 3, 0), ("NodeNumber", 4, 2)],
    [("ScoreColumn1", 1, 1), ("ScoreColumn3", 1, 3)],         # two normalizing columns: the general form
    [("NodeNumber", 200_000, 1)],  # weight x 100 >= 2^24: NodeNumber's key by the select, not base + bit x delta
]


@pytest.mark.parametrize("lst", range(len(W32_LISTS)))
def test_generic_small_totals(msh, gpu_ctx, oracle, lst):
    """generic_kernel's 32-bit keys (the host bounds every feasible total below 2^31 - 1 from the weights,
    the modes and the uploaded columns' range) and, for two normalizing columns, its general 64-bit form:
    every instance family (no column, one DEFAULT / MIN-MAX / REVERSE column, a node-only sum) on tables
    of one and several LDS tiles, few and many pods (slice waves), against the oracle."""
    rng = np.random.default_rng(700 + lst)
    pl = W32_LISTS[lst]
    names = [nm for nm, _, _ in pl]
    pre = ["NodeNumber"] if "NodeNumber" in names else []
    ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=pre, score=names,
                          weights=[w for _, w, _ in pl], normalize=[m for _, _, m in pl])
    gpu_ctx.set_plugins(ps.filters, ps.prescore, [msh.ScorePluginConfig(nm, w, msh.Normalize(m)) for nm, w, m in pl])
    for n, p in [(1, 7), (70, 300), (1025, 1000), (5000, 20_000), (33_000, 513)]:
        u, nd, pd, pt = _rand_case(rng, n, p, p_unsched=0.3, p_tol=0.2)
        cols = _cols(rng, n)
        gpu_ctx.upload_nodes(u, nd)
        for k in range(4):
            gpu_ctx.upload_score_column(f"ScoreColumn{k}", cols[k])
        _assert_same(gpu_ctx.schedule_batch(pd, pt), oracle.c_schedule_batch(u, nd, pd, pt, ps, cols=cols),
                     f"w32 {pl} n={n} p={p}")


W32_EDGES = [
    # (plugins, column ranges) at the edges of generic_kernel's 32-bit keys: a DEFAULT and a
    # REVERSE column at weight 2^23 - 1 (the largest __mul24 operand, totals near 2^31; the REVERSE weight
    # is negated in the kernel); a MIN-MAX column at 2^23 - 1; a NONE column whose weight x max|raw| is just
    # below 2^31 - 2 (32-bit keys) and just above it (the 64-bit fallback); the same NONE column beside a
    # DEFAULT column at weight 2^23 (past the 24-bit operand limit: 64-bit keys)
    ([("ScoreColumn1", (1 << 23) - 1, 1), ("ScoreColumn2", (1 << 23) - 1, 2)], {1: (0, 45), 2: (-3, 40)}),
    ([("ScoreColumn1", (1 << 23) - 1, 3), ("NodeNumber", 7, 0)], {1: (-1000, 1000)}),
    ([("ScoreColumn3", ((1 << 31) - 2) // 1000, 0)], {3: (-1000, 1001)}),
    ([("ScoreColumn3", ((1 << 31) - 2) // 1000 + 1, 0)], {3: (-1000, 1001)}),
    ([("ScoreColumn3", 3, 0), ("ScoreColumn1", 1 << 23, 1)], {1: (0, 50), 3: (-1000, 1001)}),
]


@pytest.mark.parametrize("case", range(len(W32_EDGES)))
def test_generic_key_width_edges(msh, gpu_ctx, oracle, case):
    """generic_kernel at the edges of its 32-bit key instances (totals near +-(2^31 - 2), the signed 24-bit
    multiply at its largest operands) and just past them (the 64-bit form), each against the oracle."""
    rng = np.random.default_rng(2300 + case)
    pl, ranges = W32_EDGES[case]
    names = [nm for nm, _, _ in pl]
    pre = ["NodeNumber"] if "NodeNumber" in names else []
    ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=pre, score=names,
                          weights=[w for _, w, _ in pl], normalize=[m for _, _, m in pl])
    gpu_ctx.set_plugins(ps.filters, ps.prescore, [msh.ScorePluginConfig(nm, w, msh.Normalize(m)) for nm, w, m in pl])
    for n, p in [(70, 300), (5000, 20_000), (33_000, 513)]:
        u, nd, pd, pt = _rand_case(rng, n, p, p_unsched=0.3, p_tol=0.2)
        cols = {k: rng.integers(lo, hi, n) for k, (lo, hi) in ranges.items()}
        for k, (lo, hi) in ranges.items():
            cols[k][rng.integers(0, n)] = hi - 1  # the range's top is present
        gpu_ctx.upload_nodes(u, nd)
        for k, col in cols.items():
            gpu_ctx.upload_score_column(f"ScoreColumn{k}", col)
        _assert_same(gpu_ctx.schedule_batch(pd, pt), oracle.c_schedule_batch(u, nd, pd, pt, ps, cols=cols, threads=8),
                     f"edge {pl} n={n} p={p}")


@pytest.mark.parametrize("lst", [0, 1, 3])
def test_generic_nn_key_select(msh, oracle, lst):
    """msh_options.gen_nnkey select (read once by msh_create_ex): NodeNumber's key by the compare and select instead of
    the compare-free base + bit x delta, on the 32-bit lists, at C3 size and on a multi-tile table."""
    rng = np.random.default_rng(900 + lst)
    pl = W32_LISTS[lst]
    names = [nm for nm, _, _ in pl]
    ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=["NodeNumber"], score=names,
                          weights=[w for _, w, _ in pl], normalize=[m for _, _, m in pl])
    with msh.DeviceContext(0, {"gen_nnkey": "select"}) as ctx:
        ctx.set_plugins(ps.filters, ps.prescore, [msh.ScorePluginConfig(nm, w, msh.Normalize(m)) for nm, w, m in pl])
        for n, p in [(5000, 100_000), (33_000, 700)]:
            u, nd, pd, pt = _rand_case(rng, n, p, p_unsched=0.3, p_tol=0.2)
            cols = _cols(rng, n)
            ctx.upload_nodes(u, nd)
            for k in range(4):
                ctx.upload_score_column(f"ScoreColumn{k}", cols[k])
            _assert_same(ctx.schedule_batch(pd, pt), oracle.c_schedule_batch(u, nd, pd, pt, ps, cols=cols, threads=8),
                         f"select {pl} n={n} p={p}")
    with pytest.raises(msh.MshError, match="gen_nnkey"):
        msh.DeviceContext(0, {"gen_nnkey": 2})


@pytest.mark.parametrize("f53", ["f53", "u64"])
def test_generic_f53_bounds(msh, oracle, f53):
    """8-byte keys as doubles (msh_options.gen_keys auto, the default) when the host bounds the totals below 2^53, else
    uint64_t keys: a column over the whole int32 range at weight 2^21 (bound 2^52: doubles) and 2^22 (2^53:
    uint64_t), with NodeNumber DEFAULT and a DEFAULT column beside it; two normalizing columns (the general
    form) below and past the bound; on one- and multi-tile tables; and the same lists on the uint64_t keys
    throughout (gen_keys u64)."""
    rng = np.random.default_rng(53)
    lists = [[("ScoreColumn0", 1 << 21, 0), ("NodeNumber", 1, 1)],
             [("ScoreColumn0", 1 << 22, 0), ("NodeNumber", 3, 0)],
             [("ScoreColumn0", 7, 1), ("NodeNumber", 2, 3), ("ScoreColumn1", 1 << 20, 0)],
             [("ScoreColumn0", 1, 2)],
             # two normalizing columns (the general form): below and past the 2^53 bound
             [("ScoreColumn0", 3, 1), ("ScoreColumn1", 2, 3), ("NodeNumber", 1, 2)],
             [("ScoreColumn1", 1 << 31, 1), ("NodeNumber", 5, 0), ("ScoreColumn0", 1, 2)]]
    with msh.DeviceContext(0, {"gen_keys": f53}) as ctx:
        for pl in lists:
            names = [nm for nm, _, _ in pl]
            pre = ["NodeNumber"] if "NodeNumber" in names else []
            ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=pre, score=names,
                                  weights=[w for _, w, _ in pl], normalize=[m for _, _, m in pl])
            ctx.set_plugins(ps.filters, ps.prescore, [msh.ScorePluginConfig(nm, w, msh.Normalize(m)) for nm, w, m in pl])
            for n, p in [(700, 3000), (20_000, 2000)]:
                u, nd, pd, pt = _rand_case(rng, n, p, p_unsched=0.3, p_tol=0.2)
                cols = {0: rng.integers(-(1 << 31), (1 << 31) + 1, n), 1: rng.integers(-(1 << 31), (1 << 31) + 1, n),
                        2: np.zeros(n, np.int64), 3: np.zeros(n, np.int64)}
                ctx.upload_nodes(u, nd)
                for k in range(2):
                    ctx.upload_score_column(f"ScoreColumn{k}", cols[k])
                _assert_same(ctx.schedule_batch(pd, pt), oracle.c_schedule_batch(u, nd, pd, pt, ps, cols=cols, threads=8),
                             f"f53={f53} {pl} n={n}")
    with pytest.raises(msh.MshError, match="gen_keys"):
        msh.DeviceContext(0, {"gen_keys": 2})


def test_generic_int64_min_totals(msh, gpu_ctx, oracle):
    """64-bit totals equal to INT64_MIN (weight 2^32 x raw -2^31): such a pair's key collides with the
    infeasible key 0, so a pod whose every feasible total is INT64_MIN takes its first feasible node
    (selectHost's scan with strict '>' keeps the first of equal maxima); nodes with a larger total win."""
    rng = np.random.default_rng(64)
    n, p = 3000, 2000
    u, nd, pd, pt = _rand_case(rng, n, p, p_unsched=0.4, p_tol=0.3)
    ps = oracle.PluginSet(filters=["NodeUnschedulable"], prescore=[], score=["ScoreColumn0"], weights=[1 << 32],
                          normalize=[0])
    gpu_ctx.set_plugins(ps.filters, ps.prescore, [msh.ScorePluginConfig("ScoreColumn0", 1 << 32)])
    gpu_ctx.upload_nodes(u, nd)
    for col in (np.full(n, -(1 << 31), np.int64), np.where(np.arange(n) % 997 == 5, -3, -(1 << 31)).astype(np.int64)):
        gpu_ctx.upload_score_column("ScoreColumn0", col)
        got = gpu_ctx.schedule_batch(pd, pt)
        _assert_same(got, oracle.c_schedule_batch(u, nd, pd, pt, ps, cols={0: col}), "INT64_MIN totals")
    assert (got[1][got[2] == 0] != np.iinfo(np.int64).min).any()


def test_generic_pipeline_entry_points_and_errors(msh, oracle):
    """The generic pipeline through the multi-batch and async entry points; a column not uploaded
    since the last node upload is MSH_ERR_STATE; bad column uploads are MSH_ERR_INVALID; shard keys,
    sequential mode and the export reject score-column lists (MSH_ERR_UNSUPPORTED)."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(12)
    u, nd, pd, pt = _rand_case(rng, 3000, 2000)
    cols = _cols(rng, 3000)
    ps = oracle.PluginSet(score=["NodeNumber", "ScoreColumn2", "ScoreColumn0"], weights=[5, 1, 2], normalize=[1, 0, 3])
    with msh.DeviceContext(0) as ctx:
        ctx.set_plugins(ps.filters, ps.prescore, [msh.ScorePluginConfig(s, w, msh.Normalize(m))
                                                  for s, w, m in zip(ps.score, ps.weights, ps.normalize)])
        ctx.upload_nodes(u, nd)
        ctx.upload_score_column("ScoreColumn0", cols[0])
        with pytest.raises(msh.MshError, match="MSH_ERR_STATE"):  # ScoreColumn2 missing
            ctx.schedule_batch(pd, pt)
        ctx.upload_score_column("ScoreColumn2", cols[2])
        want = oracle.c_schedule_batch(u, nd, pd, pt, ps, cols=cols)
        _assert_same(ctx.schedule_batch(pd, pt), want, "generic host path")
        ts = [_dev_batch(torch, dev, pd, pt) for _ in range(3)]
        ctx.schedule_batches_device(ctx.batch_descs([_desc(t) for t in ts]),
                                    stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for t in ts:
            _assert_same([t[i].cpu().numpy() for i in (2, 3, 4)], want, "generic multi-batch")
        hpd, hpt = msh.pinned_empty(len(pd), np.int8), msh.pinned_empty(len(pd), np.uint8)
        hpd[:], hpt[:] = pd, pt
        outs = (msh.pinned_empty(len(pd), np.int32), msh.pinned_empty(len(pd), np.int64),
                msh.pinned_empty(len(pd), np.int32))
        ctx.wait(ctx.schedule_batch_async(hpd, hpt, outs))
        _assert_same(outs, want, "generic async")
        with pytest.raises(msh.MshError, match="MSH_ERR_INVALID"):
            ctx.upload_score_column("ScoreColumn1", np.zeros(2999, np.int64))
        bad = np.zeros(3000, np.int64)
        bad[5] = (1 << 31) + 1
        with pytest.raises(msh.MshError, match="MSH_ERR_INVALID"):
            ctx.upload_score_column("ScoreColumn1", bad)
        with pytest.raises(msh.MshError, match="MSH_ERR_UNSUPPORTED"):
            ctx.schedule_sequential(pd, pt)
        with pytest.raises(msh.MshError, match="MSH_ERR_UNSUPPORTED"):
            ctx.export_results(pd[:5], pt[:5])
        d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
        keys = torch.empty(2 * len(pd), dtype=torch.int32, device=dev)
        with pytest.raises(msh.MshError, match="MSH_ERR_UNSUPPORTED"):
            ctx.shard_keys_device(len(pd), d_pd.data_ptr(), d_pt.data_ptr(), 0, keys.data_ptr(), 0)
        ctx.upload_nodes(u, nd)  # drops the columns
        with pytest.raises(msh.MshError, match="MSH_ERR_STATE"):
            ctx.schedule_batch(pd, pt)


@pytest.mark.parametrize("combo", range(len(PLUGIN_COMBOS)))
@pytest.mark.parametrize("norm", [0, 1, 2, 3])
def test_generic_kernel_cross_checks_bitmap_kernel(msh, oracle, combo, norm):
    """msh_options.batch_kernel generic runs the reference plugin lists on generic_kernel too (explicit
    int64 scores, real NormalizeScore over the feasible list) instead of the bitmap kernel's closed
    forms: both place identically, and both equal the oracle (BASELINE C2 size, weight 3)."""
    rng = np.random.default_rng(500 + 10 * combo + norm)
    f, pre, s = PLUGIN_COMBOS[combo]
    ps = _plugins(oracle, f, pre, s, 3, norm)
    u, nd, pd, pt = _rand_case(rng, 1000, 10_000, p_unsched=0.3, p_tol=0.1)
    with msh.DeviceContext(0, {"batch_kernel": "generic"}) as ctx:
        _set(ctx, msh, ps)
        ctx.upload_nodes(u, nd)
        _assert_same(ctx.schedule_batch(pd, pt), oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=8),
                     f"generic combo={combo} norm={norm}")


# ---- BASELINE C3 in full on the per-pair kernels, against the oracle (verdict r3, next #3) ----
def _c3_cols(n):
    rng = np.random.default_rng(0xC3)
    return {0: rng.integers(-(1 << 31), (1 << 31) + 1, n), 1: rng.integers(0, 7, n) * 13}


@pytest.mark.parametrize("kernel", ["pair", "pair-sgpr", "generic"])
def test_c3_reference_list_vs_oracle(msh, oracle, synth, kernel):
    """5,000 nodes x 100,000 pods (BASELINE C3, the headline workload), the reference plugin list,
    weight 1, no normalizer, through the batch and the 32-batch entry points of the per-pair kernel
    (pair_kernel, the headline) and of generic_kernel (explicit int64 scores, batch_kernel generic):
    bit-exact vs oracle.c_schedule_batch (the restatement of minisched.go:115-199,304-325)."""
    torch = pytest.importorskip("torch")
    opts = {**_pair_opts(kernel.split("-")[1] if "-" in kernel else "auto"), "batch_kernel": kernel.split("-")[0]}
    kernel = kernel.split("-")[0]
    u, nd, pd, pt = synth.make_soa(5000, 100_000)
    want = oracle.c_schedule_batch(u, nd, pd, pt, oracle.PluginSet(), threads=16)
    dev = torch.device("cuda:0")
    with msh.DeviceContext(0, opts) as ctx:
        ctx.upload_nodes(u, nd)
        _assert_same(ctx.schedule_batch(pd, pt), want, f"C3 {kernel}")
        # 12 batches: enough waves for the launcher's LDS-staged pair kernel (bench.py's 32-batch launch)
        ts = [_dev_batch(torch, dev, pd, pt) for _ in range(12)]
        ctx.schedule_batches_device(ctx.batch_descs([_desc(t) for t in ts]), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for t in ts:
            _assert_same([t[i].cpu().numpy() for i in (2, 3, 4)], want, f"C3 {kernel} multi")


@pytest.mark.parametrize("norm,weight", [(3, 3), (1, 2)])
def test_c3_score_column_vs_oracle(msh, gpu_ctx, oracle, synth, norm, weight):
    """C3 in full on generic_kernel with NodeNumber + ScoreColumn0 (columns spanning [-2^31, 2^31]),
    both normalized (MIN-MAX at weight 3, DefaultNormalizeScore at weight 2): the per-pair division
    by the pod's exact reciprocal, the first maximum over int64 totals, bit-exact vs the oracle."""
    u, nd, pd, pt = synth.make_soa(5000, 100_000)
    cols = _c3_cols(5000)
    ps = oracle.PluginSet(score=["NodeNumber", "ScoreColumn0"], weights=[weight, weight], normalize=[norm, norm])
    want = oracle.c_schedule_batch(u, nd, pd, pt, ps, cols=cols, threads=16)
    gpu_ctx.set_plugins(ps.filters, ps.prescore, [msh.ScorePluginConfig(s, w, msh.Normalize(m))
                                                  for s, w, m in zip(ps.score, ps.weights, ps.normalize)])
    gpu_ctx.upload_nodes(u, nd)
    gpu_ctx.upload_score_column("ScoreColumn0", cols[0])
    _assert_same(gpu_ctx.schedule_batch(pd, pt), want, f"C3 column norm={norm} w={weight}")
    gpu_ctx.set_plugins(["NodeUnschedulable"], ["NodeNumber"], [msh.ScorePluginConfig("NodeNumber")])


# ---- the exact headline launch of bench.py, against the oracle (verdict r5, next #2) ----
@pytest.mark.parametrize("weight,norm", [(3, 1), (3, 3), (3, 2), (1, 0)],
                         ids=["headline-w3-default", "w3-minmax", "w3-reverse", "reference-w1"])
def test_headline_launch_vs_oracle(msh, oracle, synth, weight, norm):
    """bench.py's timed step at N = 1, reproduced: the C3 snapshot (synth.make_nodes(5000)), 32 distinct
    100,000-pod batches cut from one synthetic pod stream exactly as bench.py cuts them for rank 0, all
    32 in ONE msh_schedule_batches_device call (the launch shape that selects
    pair_lds_kernel<false, false, 4> for the identity-like modes and <false, true, 4> for REVERSE /
    MINMAX); every batch's idx / score / status bit-exact vs oracle.c_schedule_batch over the whole table
    (minisched.go:115-199, 304-325). The headline list (NodeNumber w=3 DefaultNormalizeScore), the two
    other normalizers bench.py times beside it, and the reference's own w=1 list."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda:0")
    G, p = msh._native.BATCHES_PER_LAUNCH, 100_000
    u, nd = synth.make_nodes(5000)[1:]
    pd_all, pt_all = synth._make_pods_fast(p * G, synth.SEED)[1:]
    pods = [(np.ascontiguousarray(pd_all[i * p:(i + 1) * p]), np.ascontiguousarray(pt_all[i * p:(i + 1) * p]))
            for i in range(G)]
    ps = _plugins(oracle, ["NodeUnschedulable"], ["NodeNumber"], ["NodeNumber"], weight, norm)
    with msh.DeviceContext(0) as ctx:
        _set(ctx, msh, ps)
        ctx.upload_nodes(u, nd)
        bufs = [_dev_batch(torch, dev, pd, pt) for pd, pt in pods]
        ctx.schedule_batches_device(ctx.batch_descs([_desc(t) for t in bufs]),
                                    stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = [[t[i].cpu().numpy() for i in (2, 3, 4)] for t in bufs]
    for k, (pd, pt) in enumerate(pods):
        _assert_same(got[k], oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=16), f"headline batch {k} w={weight} norm={norm}")
