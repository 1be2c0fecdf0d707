"""The oracle pinned before it is trusted: scenario known answer, fixtures, closed form."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest

from closed_form import closed_form

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_scenario_known_answer(oracle):
    """sched.go:70-143 — the reference's only end-to-end known answer."""
    fx = json.loads((GOLDEN / "scenario.json").read_text())
    oo = oracle.ObjectOracle()
    names = {0: "PLACED", 1: "FIT_ERROR", 2: "SCORE_ERROR"}
    for ph in fx["phases"]:
        res = oo.schedule([oracle.Pod(p["name"]) for p in fx["pods"]],
                          [oracle.Node(n["name"], n["unschedulable"]) for n in ph["nodes"]])
        for r, e in zip(res, ph["expect"]):
            assert names[r.status] == e["outcome"]
            assert r.node == e.get("node")
            assert sorted(r.unschedulable_plugins) == sorted(e.get("unschedulable_plugins", []))


@pytest.mark.parametrize("path", sorted(GOLDEN.glob("case_*.json")), ids=lambda p: p.stem)
def test_fixture_both_restatements(oracle, path):
    fx = json.loads(path.read_text())
    ps = oracle.PluginSet(**fx["plugins"])
    # C restatement on the SoA columns
    i, s, st, _ = oracle.c_schedule_batch(np.array(fx["unsched"], np.uint8), np.array(fx["node_digit"], np.int8),
                                          np.array(fx["pod_digit"], np.int8), np.array(fx["pod_tol"], np.uint8), ps)
    assert i.tolist() == fx["idx"] and s.tolist() == fx["score"] and st.tolist() == fx["status"]
    # object restatement on names / tolerations
    T = oracle.Toleration
    pods = [oracle.Pod(p["name"], tuple(T(**t) for t in p["tolerations"])) for p in fx["pods"]]
    nodes = [oracle.Node(n["name"], n["unschedulable"]) for n in fx["nodes"]]
    res = oracle.ObjectOracle(ps).schedule(pods, nodes)
    assert [r.node for r in res] == fx["node"]
    assert [r.score for r in res] == fx["score"]
    assert [sorted(r.unschedulable_plugins) for r in res] == fx["unschedulable_plugins"]


@pytest.mark.parametrize("seed", range(6))
def test_c_oracle_vs_closed_form(oracle, seed):
    rng = np.random.default_rng(seed)
    n, p = int(rng.integers(0, 700)), int(rng.integers(1, 900))
    u = (rng.random(n) < rng.random()).astype(np.uint8)
    nd = rng.integers(-1, 10, n).astype(np.int8)
    pd = rng.integers(-1, 10, p).astype(np.int8)
    pt = (rng.random(p) < 0.3).astype(np.uint8)
    w = int(rng.integers(1, 5))
    got = oracle.c_schedule_batch(u, nd, pd, pt, oracle.PluginSet(weights=[w]))
    want = closed_form(u, nd, pd, pt, w)
    for g, e in zip(got[:3], want):
        assert (g == e).all()


def test_omp_matches_scalar(oracle, synth):
    u, nd, pd, pt = synth.make_soa(1000, 20_000)
    a = oracle.c_schedule_batch(u, nd, pd, pt)
    b = oracle.c_schedule_batch(u, nd, pd, pt, threads=4)
    for x, y in zip(a[:3], b[:3]):
        assert (x == y).all()


def test_sequential_without_capacity_equals_batch(oracle, synth):
    u, nd, pd, pt = synth.make_soa(300, 3000)
    a = oracle.c_schedule_batch(u, nd, pd, pt)
    i, s, st, counts = oracle.c_schedule_sequential(u, nd, pd, pt)
    assert (a[0] == i).all() and (a[1] == s).all() and (a[2] == st).all()
    assert counts.sum() == (st == 0).sum()


def test_sequential_capacity_spreads(oracle):
    u = np.zeros(20, np.uint8)
    nd = (np.arange(20) % 10).astype(np.int8)
    pd = np.full(50, 3, np.int8)
    pt = np.zeros(50, np.uint8)
    i, s, st, counts = oracle.c_schedule_sequential(u, nd, pd, pt, max_pods=2)
    assert counts.max() <= 2 and (st == 0).sum() == 40 and (st == 1).sum() == 10


def test_norm_in_loop_quirk_is_identity_for_nodenumber(oracle, synth):
    """minisched.go:178-183 calls NormalizeScore inside the node loop; NodeNumber has none
    (nodenumber.go:98-100), so the quirk cannot change the reference plugin set's results."""
    u, nd, pd, pt = synth.make_soa(200, 500)
    a = oracle.c_schedule_batch(u, nd, pd, pt, norm_in_loop=False)
    b = oracle.c_schedule_batch(u, nd, pd, pt, norm_in_loop=True)
    for x, y in zip(a[:3], b[:3]):
        assert (x == y).all()


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("weight", [1, 3])
def test_closed_form_modes_matches_oracle(oracle, mode, weight):
    """The per-class closed form bench.py checks its extra configs with (tests/closed_form.py)
    agrees with the oracle's real normalizers on random tables, empty ones included."""
    from closed_form import closed_form_modes
    rng = np.random.default_rng(10 * mode + weight)
    for n in (0, 1, 37, 300):
        u = (rng.random(n) < 0.4).astype(np.uint8)
        nd = rng.integers(-1, 10, n).astype(np.int8)
        pd = rng.integers(-1, 10, 400).astype(np.int8)
        pt = (rng.random(400) < 0.3).astype(np.uint8)
        want = oracle.c_schedule_batch(u, nd, pd, pt, oracle.PluginSet(weights=[weight], normalize=[mode]))
        got = closed_form_modes(u, nd, pd, pt, weight, mode)
        assert all((a == b).all() for a, b in zip(got, want[:3]))


@pytest.mark.parametrize("seed", range(6))
def test_score_columns_both_restatements(oracle, seed):
    """Score-column plugins (the generic pipeline's build extension: Score = a host-given int64 per
    node): the C restatement and the object restatement agree for NodeNumber + two columns, every
    normalize mode, weights up to 2^32 (Go int64 totals wrap), negative and tied column values."""
    rng = np.random.default_rng(seed)
    n, p = int(rng.integers(1, 60)), 40
    names = [f"node{i}" for i in range(n)]
    nodes = oracle.list_order([oracle.Node(x, bool(rng.random() < 0.3)) for x in names])
    unsched = np.array([nd.unschedulable for nd in nodes], np.uint8)
    digit = np.array([oracle.atoi_last_byte(nd.name) for nd in nodes], np.int8)
    cols = {0: rng.integers(-(1 << 31), 1 << 31, n), 1: rng.integers(0, 4, n) * 7}  # List order
    T = oracle.Toleration
    pods = [oracle.Pod(f"pod{j}" + ("x" if rng.random() < 0.1 else ""),
                       (T("node.kubernetes.io/unschedulable", "Exists", "", "NoSchedule"),) if rng.random() < 0.2 else ())
            for j in range(p)]
    pd = np.array([oracle.atoi_last_byte(x.name) for x in pods], np.int8)
    pt = np.array([oracle.pod_tolerates_unschedulable(x) for x in pods], np.uint8)
    for modes in ([0, 0, 0], [1, 2, 3], [3, 3, 1], [2, 0, 3]):
        for weights in ([1, 1, 1], [3, 1 << 32, 7]):
            ps = oracle.PluginSet(score=["NodeNumber", "ScoreColumn0", "ScoreColumn1"], weights=weights,
                                  normalize=modes)
            ci, cs, cst, _ = oracle.c_schedule_batch(unsched, digit, pd, pt, ps, cols=cols)
            oo = oracle.ObjectOracle(ps, columns={f"ScoreColumn{k}": {nd.name: int(v[i]) for i, nd in enumerate(nodes)}
                                                  for k, v in cols.items()})
            res = oo.schedule(pods, nodes)
            assert [r.index for r in res] == ci.tolist(), (modes, weights)
            assert [r.score for r in res] == cs.tolist(), (modes, weights)
            assert [r.status for r in res] == cst.tolist(), (modes, weights)


def test_capacity_closed_form_matches_oracle_serial_loop():
    """tests/closed_form.closed_form_capacity (bench.py's checker of the capacity form of C5) against the
    oracle's serial loop (oracle_schedule_sequential: minisched.go:28-30 with the capacity filter) on
    random tables with unschedulable nodes, digit-less names and tolerating pods, counts included."""
    import importlib
    import numpy as np
    from closed_form import closed_form_capacity
    importlib.import_module("oracle.build").build_oracle()
    O = importlib.import_module("oracle.oracle")
    rng = np.random.default_rng(15)
    for n, p, cap in [(1, 10, 1), (300, 4000, 3), (1000, 20_000, 7), (50, 3000, 2), (2000, 5000, 0), (64, 64, 64)]:
        u = (rng.random(n) < 0.3).astype(np.uint8)
        nd = rng.integers(-1, 10, n).astype(np.int8)
        pd = rng.integers(-1, 10, p).astype(np.int8)
        pt = (rng.random(p) < 0.2).astype(np.uint8)
        got = closed_form_capacity(u, nd, pd, pt, 1, cap)
        want = O.c_schedule_sequential(u, nd, pd, pt, O.PluginSet(), cap)
        assert all((g == w).all() for g, w in zip(got, want)), (n, p, cap)
