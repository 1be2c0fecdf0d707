"""Host side around the device path: scheduling queue (§8 f1), node cache (§8 f2),
Permit/Bind (§8 f3) and the batched loop. CPU tests use the oracle-backed OracleCtx;
the `gpu` tests drive the same event streams through the real device and compare."""
from __future__ import annotations

import importlib
import random

import numpy as np
import pytest

from oracle import oracle as O
from tests.oracle_ctx import OracleCtx

Q = importlib.import_module("mini-kube-scheduler_amd.queue")
NC = importlib.import_module("mini-kube-scheduler_amd.nodecache")
B = importlib.import_module("mini-kube-scheduler_amd.binder")
L = importlib.import_module("mini-kube-scheduler_amd.loop")
S = importlib.import_module("mini-kube-scheduler_amd.scheduler")
N = importlib.import_module("mini-kube-scheduler_amd._native")

TOL = O.Toleration(key="node.kubernetes.io/unschedulable", operator="Exists", effect="NoSchedule")


class Clock:
    def __init__(self, t: float = 1000.0):
        self.t = t

    def __call__(self) -> float:
        return self.t

    def advance(self, dt: float) -> None:
        self.t += dt


@pytest.fixture(autouse=True)
def _built(msh):
    """The packer (host code in libminisched_hip.so) must be built."""
    return msh


def make_loop(ctx=None, clock=None, **kw):
    clock = clock or Clock()
    sched = S.Scheduler(ctx=ctx or OracleCtx())
    return L.SchedulingLoop(sched, clock=clock, **kw), clock


# ---------------------------------------------------------------- queue (f1) --
def test_backoff_durations():
    # queue.go:219-235: 1s doubling, capped at 10s; attempts 0 and 1 both give 1s
    assert [Q.calculate_backoff_duration(a) for a in range(7)] == [1, 1, 2, 4, 8, 10, 10]


def test_events_to_register_matches_initialize():
    m = Q.events_to_register()
    nu = Q.ClusterEvent(Q.NODE, Q.ActionType.ADD | Q.ActionType.UPDATE_NODE_TAINT)
    nn = Q.ClusterEvent(Q.NODE, Q.ActionType.ADD)
    # NodeNumber's event registered under NodeUnschedulable's name (initialize.go:153-154)
    assert m == {nu: frozenset({"NodeUnschedulable"}), nn: frozenset({"NodeUnschedulable"})}
    g = Q.unioned_gvks(m)
    assert g == {Q.NODE: Q.ActionType.ADD | Q.ActionType.UPDATE_NODE_TAINT}
    # the informer registers Add and Update handlers, not Delete (eventhandler.go:39-57)
    assert g[Q.NODE] & Q.ActionType.ADD and g[Q.NODE] & Q.ActionType.UPDATE
    assert not g[Q.NODE] & Q.ActionType.DELETE


def test_fifo_batch_drain_across_chunks():
    q = Q.SchedulingQueue(clock=Clock())
    q.add_many([O.Pod(f"a{i}") for i in range(5)])
    q.add_soa([f"b{i}" for i in range(7)], np.arange(7) % 10, np.zeros(7, np.uint8))
    q.add(O.Pod("c1", (TOL,)))
    assert q.active_len() == 13
    b1 = q.next_batch(3)
    assert b1.names == ["a0", "a1", "a2"]
    b2 = q.next_batch(6)
    assert b2.names == ["a3", "a4", "b0", "b1", "b2", "b3"]
    assert list(b2.digit) == [3, 4, 0, 1, 2, 3]
    b3 = q.next_batch(100)
    assert b3.names == ["b4", "b5", "b6", "c1"]
    assert list(b3.tolerates) == [0, 0, 0, 1] and b3.digit[-1] == 1
    assert q.active_len() == 0 and len(q.next_batch(10)) == 0
    assert q.next_pod() is None


def test_move_semantics_match_podMatchesEvent_and_backoff():
    clk = Clock()
    q = Q.SchedulingQueue(clock=clk)
    ids = q.add_many([O.Pod("p1"), O.Pod("p2"), O.Pod("p3")])
    q.next_batch(3)
    q.add_unschedulable(ids[0], {"NodeUnschedulable"})    # FitError diagnosis
    q.add_unschedulable(ids[1], None)                     # score error: nil set
    q.add_unschedulable(ids[2], {"SomeOtherPlugin"})      # not registered for any event
    assert list(q.unschedulable_ids()) == list(ids)
    # within the 1 s backoff: matching pods go to podBackoffQ (queue.go:75-79)
    clk.advance(0.5)
    assert q.move_all_to_active_or_backoff_queue(Q.NODE_ADD) == 2
    assert q.backoff_ids() == [ids[0], ids[1]] and q.active_len() == 0
    assert list(q.unschedulable_ids()) == [ids[2]]
    # reference never flushes podBackoffQ; the extension does once the backoff expired
    assert q.flush_backoff_completed() == 0
    clk.advance(0.6)
    assert q.flush_backoff_completed() == 2 and q.active_len() == 2
    # p3 only moves on a wildcard event
    assert q.move_all_to_active_or_backoff_queue(Q.NODE_UPDATE) == 0
    assert q.move_all_to_active_or_backoff_queue(Q.WILDCARD_EVENT) == 1
    assert q.next_batch(5).names == ["p1", "p2", "p3"]


def test_node_update_matches_taint_bit_and_delete_does_not():
    clk = Clock()
    q = Q.SchedulingQueue(clock=clk)
    i = q.add(O.Pod("p1"))
    q.next_batch(1)
    q.add_unschedulable(i, {"NodeUnschedulable"})
    clk.advance(2)
    assert q.move_all_to_active_or_backoff_queue(Q.NODE_DELETE) == 0
    # Update (all four update bits) & (Add|UpdateNodeTaint) != 0
    assert q.move_all_to_active_or_backoff_queue(Q.NODE_UPDATE) == 1
    assert q.active_len() == 1


def test_add_unschedulable_refreshes_timestamp_and_dedupes_by_key():
    clk = Clock()
    q = Q.SchedulingQueue(clock=clk)
    i = q.add(O.Pod("p1", namespace="ns"))
    assert q.id_of("p1", "ns") == i
    q.add_unschedulable(i, {"NodeUnschedulable"})
    t0 = q.timestamp(i)
    clk.advance(0.9)
    q.add_unschedulable(i, {"NodeUnschedulable"})        # add-or-update, new timestamp
    assert q.timestamp(i) == t0 + 0.9
    assert list(q.unschedulable_ids()) == [i]
    clk.advance(0.5)                                     # 0.5 s after the refresh: backing off
    q.move_all_to_active_or_backoff_queue(Q.NODE_ADD)
    assert q.backoff_ids() == [i]
    assert q.unschedulable_plugins(i) == frozenset({"NodeUnschedulable"})


def test_queue_stubs_raise_like_reference():
    q = Q.SchedulingQueue()
    with pytest.raises(NotImplementedError):
        q.update(None, None)
    with pytest.raises(NotImplementedError):
        q.delete(None)


# ----------------------------------------------------------- node cache (f2) --
def test_node_cache_order_matches_packer(msh):
    rng = random.Random(7)
    names = sorted({f"node-{rng.randrange(10**6)}{rng.choice(['', 'x', 'é', 'Z'])}" for _ in range(500)})
    rng.shuffle(names)
    nodes = [O.Node(n, rng.random() < 0.3) for n in names]
    cache = NC.NodeCache(nodes)
    table = msh.pack_nodes(nodes)
    assert cache.names == table.names
    assert np.array_equal(cache.unsched, table.unsched)
    assert np.array_equal(cache.digit, table.digit)


def test_node_cache_sync_upload_vs_patch():
    ctx = OracleCtx()
    cache = NC.NodeCache([O.Node("n3"), O.Node("n1"), O.Node("n2", True)])
    assert cache.sync(ctx) == "upload" and ctx.calls[-1] == ("upload", 3)
    assert cache.sync(ctx) == "clean"
    cache.update(O.Node("n1"), O.Node("n1", True))
    cache.update(O.Node("n2", True), O.Node("n2", False))
    cache.update(O.Node("n3"), O.Node("n3"))              # no-op update
    assert cache.sync(ctx) == "patch" and ctx.calls[-1] == ("patch", [0, 1])
    assert list(ctx.unsched) == [1, 0, 0]
    cache.add(O.Node("n0"))
    cache.update(O.Node("n3"), O.Node("n3", True))
    assert cache.sync(ctx) == "upload"
    assert cache.names == ["n0", "n1", "n2", "n3"] and list(ctx.unsched) == [0, 1, 0, 1]
    cache.delete("n1")
    assert cache.sync(ctx) == "upload" and list(ctx.digit) == [0, 2, 3]
    with pytest.raises(KeyError):
        cache.delete("n1")
    with pytest.raises(ValueError):
        cache.add(O.Node(""))


def test_name_digit():
    assert [NC.name_digit(s) for s in ["a0", "a9", "a", "9a", "é", "x1é", "7"]] == [0, 9, -1, -1, -1, -1, 7]


# -------------------------------------------------------------- binder (f3) --
def test_permit_delays_and_bind_order():
    clk = Clock()
    bound = []
    b = B.PermitBinder(lambda i, n: bound.append((i, n)), clock=clk)
    b.submit(np.array([10, 11, 12]), ["node3", "nodeX", "node0"], np.array([3, -1, 0]))
    out = b.poll()           # nodeX (no digit: allowed at once) and node0 (0 s timer)
    assert list(out.bound_ids) == [11, 12] and bound == [(11, "nodeX"), (12, "node0")]
    assert b.waiting() == 1
    clk.advance(2.9)
    assert len(b.poll().bound_ids) == 0
    clk.advance(0.1)
    out = b.poll()
    assert list(out.bound_ids) == [10] and out.bound_nodes == ["node3"] and b.waiting() == 0


def test_permit_timeout_rejects_and_bind_errors_fail():
    clk = Clock()

    def bind(i, n):
        if i == 2:
            raise RuntimeError("conflict")

    b = B.PermitBinder(bind, clock=clk, permit_timeout_s=5.0)
    b.submit(np.array([1, 2, 3]), ["n7", "n1", "n4"], np.array([7, 1, 4]))
    clk.advance(10)
    out = b.poll()
    assert list(out.bound_ids) == [3]
    assert sorted(out.failed_ids.tolist()) == [1, 2]
    assert any("timeout" in r for r in out.failed_reasons) and any("conflict" in r for r in out.failed_reasons)


# -------------------------------------------------------------- loop (host) --
def scenario_steps(loop, clock):
    """sched.go:70-143: pod1 against node0..node8 (all unschedulable), then node10 added."""
    for i in range(9):
        loop.on_node_add(O.Node(f"node{i}", True))
    loop.on_pod_add(O.Pod("pod1"))
    r1 = loop.schedule_once()
    clock.advance(3.0)                           # the scenario sleeps before creating node10
    loop.on_node_add(O.Node("node10"))
    r2 = loop.schedule_once()
    r3 = loop.schedule_once()                    # Permit for node10 (digit 0): 0 s wait -> bind
    return r1, r2, r3


def check_scenario(loop, r1, r2, r3):
    assert r1.counts() == {"placed": 0, "fit_error": 1, "score_error": 0}
    assert r1.results(frozenset({"NodeUnschedulable"}))[0].outcome.name == "FIT_ERROR"
    assert r2.counts()["placed"] == 1 and r2.node_names[r2.node_index[0]] == "node10"
    assert r2.sync == "upload"
    assert list(r3.bind.bound_ids) == [loop.queue.id_of("pod1", "default")]
    assert r3.bind.bound_nodes == ["node10"]
    assert loop.queue.active_len() == 0 and len(loop.queue.unschedulable_ids()) == 0


def test_loop_reference_scenario_host():
    loop, clock = make_loop()
    check_scenario(loop, *scenario_steps(loop, clock))


def test_loop_requeue_rules_host():
    loop, clock = make_loop()
    loop.on_pod_add(O.Pod("pod-a1"))                           # no nodes: FitError, empty diagnosis
    assert loop.on_pod_add({"metadata": {"name": "bound1"}, "spec": {"nodeName": "n1"}}) is None
    r = loop.schedule_once()
    assert len(r) == 1 and r.counts()["fit_error"] == 1
    pid = loop.queue.id_of("pod-a1", "default")
    assert loop.queue.unschedulable_plugins(pid) == frozenset()
    # a pod whose name has no digit suffix: PreScore error -> nil set (minisched.go:61-67)
    clock.advance(5)
    loop.on_node_add(O.Node("n1"))
    loop.on_pod_add(O.Pod("pod-x"))
    r = loop.schedule_once()
    by_name = dict(zip(r.names, r.status.tolist()))
    assert by_name == {"pod-a1": N.MSH_PLACED, "pod-x": N.MSH_SCORE_ERROR}
    assert loop.queue.unschedulable_plugins(loop.queue.id_of("pod-x", "default")) == frozenset()


def test_loop_node_event_inside_backoff_strands_pod_host():
    """Reference behaviour: a matching event inside the 1 s backoff moves the pod to
    podBackoffQ, which nothing flushes (queue.go:75-79, :136-140)."""
    loop, clock = make_loop()
    loop.on_node_add(O.Node("node0", True))
    loop.on_pod_add(O.Pod("pod1"))
    loop.schedule_once()
    clock.advance(0.5)
    loop.on_node_add(O.Node("node10"))
    pid = loop.queue.id_of("pod1", "default")
    assert loop.queue.backoff_ids() == [pid]
    assert len(loop.schedule_once()) == 0
    clock.advance(1.0)
    assert loop.queue.flush_backoff_completed() == 1      # the explicit extension
    r = loop.schedule_once()
    assert r.node_names[r.node_index[0]] == "node10"


def random_event_stream(seed: int, steps: int = 40):
    rng = random.Random(seed)
    events = []
    live: dict[str, bool] = {}
    pod_no = 0
    for _ in range(steps):
        k = rng.random()
        if k < 0.35:
            for _ in range(rng.randrange(1, 40)):
                pod_no += 1
                suffix = rng.choice([str(rng.randrange(10)), str(rng.randrange(10)), "x"])
                tol = (TOL,) if rng.random() < 0.2 else ()
                events.append(("pod", O.Pod(f"p{pod_no}-{suffix}", tol)))
        elif k < 0.55 or not live:
            for _ in range(rng.randrange(1, 6)):
                name = f"node-{rng.randrange(300)}{rng.choice(['', 'a'])}"
                u = rng.random() < 0.6
                events.append(("node_add", O.Node(name, u)))
                live[name] = u
        elif k < 0.75:
            name = rng.choice(sorted(live))
            u = not live[name]
            events.append(("node_update", O.Node(name, live[name]), O.Node(name, u)))
            live[name] = u
        elif k < 0.82:
            name = rng.choice(sorted(live))
            events.append(("node_delete", name))
            del live[name]
        elif k < 0.9:
            events.append(("tick", rng.choice([0.3, 1.5, 4.0])))
        else:
            events.append(("cycle", rng.choice([None, 7])))
    events.append(("cycle", None))
    return events


def drive(loop, clock, events):
    trace = []
    for ev in events:
        kind = ev[0]
        if kind == "pod":
            loop.on_pod_add(ev[1])
        elif kind == "node_add":
            loop.on_node_add(ev[1])
        elif kind == "node_update":
            loop.on_node_update(ev[1], ev[2])
        elif kind == "node_delete":
            loop.on_node_delete(ev[1])
        elif kind == "tick":
            clock.advance(ev[1])
        else:
            r = loop.schedule_once(ev[1])
            trace.append((r.names, r.node_index.tolist(), r.score.tolist(), r.status.tolist(),
                          sorted(r.bind.bound_ids.tolist())))
    q = loop.queue
    trace.append(("final", q.active_len(), q.backoff_ids(), q.unschedulable_ids().tolist()))
    return trace


def test_loop_random_stream_bookkeeping_host():
    """Every drained pod ends up bound, waiting in Permit, or in one of the queues."""
    loop, clock = make_loop()
    trace = drive(loop, clock, random_event_stream(3, 80))
    seen = sum(len(t[0]) for t in trace[:-1])
    assert seen > 0
    clock.advance(20)
    loop.poll_binder()
    assert loop.binder.waiting() == 0


# ------------------------------------------------------------------ GPU ------
@pytest.mark.gpu
def test_loop_reference_scenario_gpu(gpu_ctx):
    loop, clock = make_loop(ctx=gpu_ctx)
    check_scenario(loop, *scenario_steps(loop, clock))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_loop_random_stream_gpu_vs_oracle(gpu_ctx, seed):
    """Same informer/event stream through the device loop and the oracle loop: identical
    decisions per cycle, identical bindings and identical final queue state. Exercises
    msh_patch_nodes (cordon/uncordon updates) and re-uploads (adds / deletes)."""
    events = random_event_stream(seed, 120)
    lg, cg = make_loop(ctx=gpu_ctx)
    lo, co = make_loop()
    assert drive(lg, cg, events) == drive(lo, co, events)


@pytest.mark.gpu
def test_node_cache_cordon_flip_between_batches_gpu(gpu_ctx, oracle):
    """The informer path the Go binding runs (go/minisched/gpusched NodeSnapshot.Sync, verdict r3 #6):
    nodes arrive through the Add handler (one upload), a cordon flip between two batches through the
    Update handler reaches the device as a patch (msh_patch_nodes), not a re-upload, and the second
    batch sees it; an Add then forces one upload. Every batch bit-exact vs the oracle on the cache's
    List-order columns. The Go test of the same sequence: TestNodeSnapshotCordonFlipBetweenBatches."""
    gpu_ctx.set_plugins(["NodeUnschedulable"], ["NodeNumber"], [S.ScorePluginConfig("NodeNumber")])
    rng = random.Random(0x5eed)
    nodes = [O.Node(f"node{i}", rng.random() < 0.1) for i in range(2000)]
    rng.shuffle(nodes)
    pd = np.array([rng.randrange(-1, 10) for _ in range(4000)], np.int8)
    pt = np.array([rng.random() < 0.05 for _ in range(4000)], np.uint8)
    cache = NC.NodeCache()
    for n in nodes:
        cache.add(n)

    def check():
        got = gpu_ctx.schedule_batch(pd, pt)
        want = oracle.c_schedule_batch(cache.unsched, cache.digit, pd, pt)
        assert all((g == w).all() for g, w in zip(got, want[:3]))

    assert cache.sync(gpu_ctx) == "upload"
    check()
    assert cache.sync(gpu_ctx) == "clean"
    first_ok = next(i for i in range(len(cache)) if cache.unsched[i] == 0)
    first_cordoned = next(i for i in range(len(cache)) if cache.unsched[i] == 1)
    for i in (first_ok, first_cordoned):
        name, u = cache.names[i], bool(cache.unsched[i])
        cache.update(O.Node(name, u), O.Node(name, not u))
    assert cache.sync(gpu_ctx) == "patch"
    check()
    cache.add(O.Node("node0000"))
    assert cache.sync(gpu_ctx) == "upload"
    check()
