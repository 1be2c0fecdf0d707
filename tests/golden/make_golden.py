"""Generate the golden fixtures under tests/golden/ (committed; re-run to regenerate).

Pinning: scenario.json holds the reference's only known answer (sched.go:70-143 — nine
unschedulable nodes node0..node8 + pod1 -> FitError{NodeUnschedulable}; after node10 is
created -> pod1 bound to node10). The expectations in it are written from the reference,
not computed; this script asserts the object-level oracle reproduces them.

case_*.json: edge-case vectors computed by the object-level oracle (oracle/oracle.py,
ObjectOracle), each cross-checked against the C restatement (oracle/msh_oracle.c) and, for
the reference plugin set, the independent closed form (tests/closed_form.py). A fixture is
data only: inputs (names, flags, tolerations, SoA columns) and expected outputs.

Usage: python tests/golden/make_golden.py   (needs oracle/build/libmsh_oracle.so: make -C oracle)
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(HERE.parent))

from oracle import oracle as O  # noqa: E402
from closed_form import closed_form  # noqa: E402

STATUS_NAME = {O.PLACED: "PLACED", O.FIT_ERROR: "FIT_ERROR", O.SCORE_ERROR: "SCORE_ERROR"}


def scenario():
    nodes9 = [{"name": f"node{i}", "unschedulable": True} for i in range(9)]
    fx = {
        "source": "/root/reference/sched.go:70-143 (scenario) and README.md:13-64",
        "note": "expectations written from the reference's scenario, not computed",
        "pods": [{"name": "pod1", "tolerations": []}],
        "phases": [
            {"nodes": nodes9,
             "expect": [{"outcome": "FIT_ERROR", "unschedulable_plugins": ["NodeUnschedulable"]}]},
            {"nodes": nodes9 + [{"name": "node10", "unschedulable": False}],
             "expect": [{"outcome": "PLACED", "node": "node10"}]},
        ],
    }
    # pin the object oracle on it
    oo = O.ObjectOracle()
    for ph in fx["phases"]:
        res = oo.schedule([O.Pod("pod1")], [O.Node(n["name"], n["unschedulable"]) for n in ph["nodes"]])
        exp = ph["expect"][0]
        assert STATUS_NAME[res[0].status] == exp["outcome"], (res, exp)
        assert res[0].node == exp.get("node"), (res, exp)
        assert sorted(res[0].unschedulable_plugins) == sorted(exp.get("unschedulable_plugins", []))
    return fx


def _tol_dict(t: O.Toleration):
    return {"key": t.key, "operator": t.operator, "value": t.value, "effect": t.effect}


def case(name, nodes, pods, plugins: O.PluginSet | None = None):
    plugins = plugins or O.PluginSet()
    oo = O.ObjectOracle(plugins)
    ordered = O.list_order(nodes)
    res = oo.schedule(pods, nodes)
    unsched = np.array([1 if n.unschedulable else 0 for n in ordered], np.uint8)
    nd = np.array([O.atoi_last_byte(n.name) for n in ordered], np.int8)
    pd = np.array([O.atoi_last_byte(p.name) for p in pods], np.int8)
    pt = np.array([1 if O.pod_tolerates_unschedulable(p) else 0 for p in pods], np.uint8)
    idx = np.array([r.index for r in res], np.int32)
    score = np.array([r.score for r in res], np.int64)
    status = np.array([r.status for r in res], np.int32)
    ci, cs, cst, _ = O.c_schedule_batch(unsched, nd, pd, pt, plugins)
    assert (ci == idx).all() and (cs == score).all() and (cst == status).all(), name
    if (plugins.filters == ["NodeUnschedulable"] and plugins.prescore == ["NodeNumber"]
            and plugins.score == ["NodeNumber"] and plugins.normalize == [O.NORM_NONE]):
        fi, fs, fst = closed_form(unsched, nd, pd, pt, plugins.weights[0])
        assert (fi == idx).all() and (fs == score).all() and (fst == status).all(), name
    fx = {
        "name": name,
        "plugins": {"filters": plugins.filters, "prescore": plugins.prescore, "score": plugins.score,
                    "weights": plugins.weights, "normalize": plugins.normalize},
        "nodes": [{"name": n.name, "unschedulable": n.unschedulable} for n in nodes],
        "pods": [{"name": p.name, "tolerations": [_tol_dict(t) for t in p.tolerations]} for p in pods],
        "list_order": [n.name for n in ordered],
        "unsched": unsched.tolist(), "node_digit": nd.tolist(),
        "pod_digit": pd.tolist(), "pod_tol": pt.tolist(),
        "idx": idx.tolist(), "score": score.tolist(), "status": status.tolist(),
        "node": [r.node for r in res],
        "unschedulable_plugins": [sorted(r.unschedulable_plugins) for r in res],
    }
    (HERE / f"case_{name}.json").write_text(json.dumps(fx, indent=1) + "\n")


def main():
    (HERE / "scenario.json").write_text(json.dumps(scenario(), indent=1) + "\n")

    rng = np.random.default_rng(0x6D696E69)
    T = O.Toleration
    tol_variants = [
        (),
        (T("node.kubernetes.io/unschedulable", "Exists", "", "NoSchedule"),),
        (T("node.kubernetes.io/unschedulable", "Equal", "", "NoSchedule"),),   # Equal, empty value: tolerates
        (T("node.kubernetes.io/unschedulable", "", "", ""),),                  # empty op == Equal, any effect
        (T("node.kubernetes.io/unschedulable", "Equal", "true", "NoSchedule"),),  # non-empty value: no
        (T("node.kubernetes.io/unschedulable", "Exists", "", "NoExecute"),),   # wrong effect: no
        (T("", "Exists", "", ""),),                                            # tolerate everything
        (T("other-key", "Exists", "", "NoSchedule"),),                         # wrong key: no
        (T("node.kubernetes.io/unschedulable", "Gt", "", "NoSchedule"),),      # unknown operator: no
        (T("a", "Exists", "", ""), T("", "Exists", "", "NoSchedule")),         # second one matches
    ]

    # 1. README variant + byte-order ties (node1 < node10 < node100 < node2 ...)
    nodes = [O.Node(f"node{i}", i % 7 == 3) for i in range(120)]
    pods = [O.Pod(f"pod{j}") for j in range(12)] + [O.Pod("web-x"), O.Pod("pod-+"), O.Pod("pod-")]
    case("list_order_ties", nodes, pods)

    # 2. non-digit node suffixes and names ending in '+'/'-'
    nodes = [O.Node(nm, u) for nm, u in [("worker-a", False), ("node7", True), ("node-", False), ("node+", False),
                                          ("gpu-node-9", False), ("z9", False), ("a9", True), ("m7", False)]]
    pods = [O.Pod(n) for n in ("pod9", "pod7", "pod1", "podx", "p9")]
    case("nondigit_suffix", nodes, pods)

    # 3. tolerations (every ToleratesTaint branch) against mostly unschedulable nodes
    nodes = [O.Node(f"n{i}", i != 5) for i in range(10)]
    pods = [O.Pod(f"pod{k}", tol_variants[k % len(tol_variants)]) for k in range(30)]
    case("tolerations", nodes, pods)

    # 4. all nodes unschedulable (FitError) / no nodes at all
    case("all_unschedulable", [O.Node(f"node{i}", True) for i in range(9)],
         [O.Pod("pod1"), O.Pod("pod2", tol_variants[1]), O.Pod("podz")])
    case("no_nodes", [], [O.Pod("pod1"), O.Pod("pod2", tol_variants[6])])

    # 5. random mixed cluster
    nodes = [O.Node(f"node{int(x)}" if rng.random() > 0.1 else f"node{int(x)}-q", bool(rng.random() < 0.3))
             for x in rng.choice(10_000, 300, replace=False)]
    pods = [O.Pod(f"pod{j}" if rng.random() > 0.05 else f"pod{j}x",
                  tol_variants[int(rng.integers(0, len(tol_variants)))] if rng.random() < 0.3 else ())
            for j in range(500)]
    case("random_mixed", nodes, pods)

    # 6. build extensions: weights and normalize modes, other plugin lists
    for norm in (O.NORM_DEFAULT, O.NORM_DEFAULT_REVERSE, O.NORM_MINMAX):
        case(f"normalize_{norm}", nodes, pods, O.PluginSet(weights=[3], normalize=[norm]))
    case("weight_7", nodes, pods, O.PluginSet(weights=[7]))
    case("no_filter", nodes, pods, O.PluginSet(filters=[]))
    case("score_without_prescore", nodes, pods, O.PluginSet(prescore=[]))
    case("no_score", nodes, pods, O.PluginSet(score=[], weights=[], normalize=[]))
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
