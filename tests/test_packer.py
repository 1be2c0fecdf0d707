"""Snapshot packer (host C++ in libminisched_hip.so) vs the object-level restatement.

List order = byte-wise name order (minisched.go:40, etcd key order); digits = strconv.Atoi of
the last byte (nodenumber.go:51-52, :81-83); tolerates = upstream TolerationsTolerateTaint
with the unschedulable taint. No GPU needed (host-only entry points).
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("path", sorted(GOLDEN.glob("case_*.json")), ids=lambda p: p.stem)
def test_pack_matches_fixture(msh, path):
    fx = json.loads(path.read_text())
    nt = msh.pack_nodes([{"metadata": {"name": n["name"]}, "spec": {"unschedulable": n["unschedulable"]}}
                         for n in fx["nodes"]])
    assert nt.names == fx["list_order"]
    assert nt.unsched.tolist() == fx["unsched"]
    assert nt.digit.tolist() == fx["node_digit"]
    pt = msh.pack_pods([{"metadata": {"name": p["name"]}, "spec": {"tolerations": p["tolerations"]}}
                        for p in fx["pods"]])
    assert pt.digit.tolist() == fx["pod_digit"]
    assert pt.tolerates.tolist() == fx["pod_tol"]


def test_byte_order_not_numeric(msh):
    nt = msh.pack_nodes([{"metadata": {"name": f"node{i}"}} for i in (2, 10, 1, 100, 0)])
    assert nt.names == ["node0", "node1", "node10", "node100", "node2"]
    assert nt.order.tolist() == [4, 2, 1, 3, 0]


def test_utf8_and_prefix_order(msh, oracle):
    names = ["nodé9", "node", "node0", "nodea", "Node1", "nodeÿ", "no"]
    nt = msh.pack_nodes([{"metadata": {"name": n}} for n in names])
    assert nt.names == [n.name for n in oracle.list_order([oracle.Node(n) for n in names])]
    assert nt.digit.tolist() == [oracle.atoi_last_byte(n) for n in nt.names]


def test_rejects_empty_and_duplicate_names(msh):
    with pytest.raises(msh.MshError):
        msh.pack_nodes([{"metadata": {"name": ""}}])
    with pytest.raises(msh.MshError):
        msh.pack_nodes([{"metadata": {"name": "a1"}}, {"metadata": {"name": "a1"}}])
    with pytest.raises(msh.MshError):
        msh.pack_pods([{"metadata": {"name": ""}}])


@pytest.mark.parametrize("tol,want", [
    ({"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"}, 1),
    ({"key": "node.kubernetes.io/unschedulable", "operator": "Equal", "value": "", "effect": "NoSchedule"}, 1),
    ({"key": "node.kubernetes.io/unschedulable"}, 1),                      # empty op == Equal, any effect
    ({"key": "node.kubernetes.io/unschedulable", "operator": "Equal", "value": "true"}, 0),
    ({"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoExecute"}, 0),
    ({"operator": "Exists"}, 1),                                            # wildcard
    ({"key": "x", "operator": "Exists"}, 0),
    ({"key": "node.kubernetes.io/unschedulable", "operator": "Lt"}, 0),    # unknown operator
])
def test_toleration_rules(msh, oracle, tol, want):
    pt = msh.pack_pods([{"metadata": {"name": "p1"}, "spec": {"tolerations": [tol]}}])
    assert int(pt.tolerates[0]) == want
    t = oracle.Toleration(tol.get("key", ""), tol.get("operator", ""), tol.get("value", ""), tol.get("effect", ""))
    assert int(oracle.tolerates_taint(t)) == want


def test_random_names_vs_object_oracle(msh, oracle):
    rng = np.random.default_rng(7)
    alphabet = list("abz09-.+Z")
    names = sorted({"".join(rng.choice(alphabet, int(rng.integers(1, 8)))) for _ in range(400)})
    rng.shuffle(names)
    nt = msh.pack_nodes([{"metadata": {"name": n}, "spec": {"unschedulable": bool(i % 3 == 0)}}
                         for i, n in enumerate(names)])
    objs = oracle.list_order([oracle.Node(n, i % 3 == 0) for i, n in enumerate(names)])
    assert nt.names == [o.name for o in objs]
    assert nt.unsched.tolist() == [int(o.unschedulable) for o in objs]


def test_large_pod_batch_split_over_threads(msh, oracle):
    """msh_pack_pods splits batches of 16,384+ pods over host threads: a 50,003-pod batch with
    random suffixes and every toleration shape, against the object oracle pod by pod; an invalid
    offset in the last part is still rejected."""
    rng = np.random.default_rng(11)
    alphabet = list("abz09-.+Z7")
    shapes = [{"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"},
              {"key": "node.kubernetes.io/unschedulable", "operator": "Equal", "value": "true"},
              {"operator": "Exists"}, {"key": "x", "operator": "Exists"},
              {"key": "node.kubernetes.io/unschedulable", "effect": "NoExecute"}]
    pods, want_d, want_t = [], [], []
    for j in range(50_003):
        name = f"p{j}" + "".join(rng.choice(alphabet, int(rng.integers(0, 3))))
        tols = [shapes[int(k)] for k in rng.integers(0, len(shapes), int(rng.integers(0, 3)))]
        pods.append({"metadata": {"name": name}, "spec": {"tolerations": tols}})
        want_d.append(oracle.atoi_last_byte(name))
        want_t.append(int(any(oracle.tolerates_taint(oracle.Toleration(t.get("key", ""), t.get("operator", ""),
                                                                        t.get("value", ""), t.get("effect", "")))
                              for t in tols)))
    pt = msh.pack_pods(pods)
    assert pt.digit.tolist() == want_d
    assert pt.tolerates.tolist() == want_t
    pods[-1]["metadata"]["name"] = ""
    with pytest.raises(msh.MshError):
        msh.pack_pods(pods)
