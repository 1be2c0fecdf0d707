"""Result store (§8 f4): the store semantics against the cases of
scheduler/plugin/resultstore/store_test.go, and the device's per-pair export against the oracle."""
from __future__ import annotations

import importlib
import json

import numpy as np
import pytest

from oracle import oracle as O

RS = importlib.import_module("mini-kube-scheduler_amd.resultstore")
S = importlib.import_module("mini-kube-scheduler_amd.scheduler")
N = importlib.import_module("mini-kube-scheduler_amd._native")
FW = importlib.import_module("mini-kube-scheduler_amd.framework")


def data(store, ns="default", pod="pod1"):
    return store.results[RS.new_key(ns, pod)]


# store_test.go TestStore_AddFilterResult (:17-135)
def test_add_filter_result():
    s = RS.ResultStore()
    s.add_filter_result("default", "pod1", "node1", "plugin1", RS.PASSED_FILTER_MESSAGE)
    s.add_filter_result("default", "pod1", "node1", "plugin2", RS.PASSED_FILTER_MESSAGE)
    s.add_filter_result("default", "pod1", "node0", "plugin1", "filter failed")
    assert data(s) == {"score": {}, "finalscore": {},
                       "filter": {"node1": {"plugin1": "passed", "plugin2": "passed"},
                                  "node0": {"plugin1": "filter failed"}}}


# TestStore_AddScoreResult (:137-284): final = score * weight, written by AddScoreResult too
def test_add_score_result_applies_weight():
    s = RS.ResultStore({"plugin1": 2})
    s.add_score_result("default", "pod1", "node1", "plugin1", 10)
    assert data(s) == {"filter": {}, "score": {"node1": {"plugin1": "10"}},
                       "finalscore": {"node1": {"plugin1": "20"}}}
    s2 = RS.ResultStore({"plugin2": 2})
    s2.results[RS.new_key("default", "pod1")] = {"filter": {}, "score": {"node1": {"plugin1": "10"}},
                                                  "finalscore": {"node1": {"plugin1": "30"}}}
    s2.add_score_result("default", "pod1", "node1", "plugin2", 10)
    assert data(s2)["score"] == {"node1": {"plugin1": "10", "plugin2": "10"}}
    assert data(s2)["finalscore"] == {"node1": {"plugin1": "30", "plugin2": "20"}}


# TestStore_AddNormalizedScoreResult (:286-403) and the zero weight of an unknown plugin
def test_add_normalized_score_result():
    s = RS.ResultStore({"plugin1": 2})
    s.add_normalized_score_result("default", "pod1", "node1", "plugin1", 10)
    assert data(s) == {"filter": {}, "score": {}, "finalscore": {"node1": {"plugin1": "20"}}}
    s.add_normalized_score_result("default", "pod1", "node1", "unknown", 10)
    assert data(s)["finalscore"]["node1"]["unknown"] == "0"


# TestStore_addSchedulingResultToPod (:405-600): annotation values are json.Marshal output
def test_annotations_json():
    s = RS.ResultStore({"plugin1": 2})
    for node in ("node1", "node0"):
        s.add_filter_result("default", "pod1", node, "plugin1", RS.PASSED_FILTER_MESSAGE)
        s.add_score_result("default", "pod1", node, "plugin1", 10)
    a = s.annotations("default", "pod1")
    assert a[RS.FILTER_RESULT_ANNOTATION_KEY] == '{"node0":{"plugin1":"passed"},"node1":{"plugin1":"passed"}}'
    assert a[RS.SCORE_RESULT_ANNOTATION_KEY] == '{"node0":{"plugin1":"10"},"node1":{"plugin1":"10"}}'
    assert a[RS.FINAL_SCORE_RESULT_ANNOTATION_KEY] == '{"node0":{"plugin1":"20"},"node1":{"plugin1":"20"}}'
    s2 = RS.ResultStore()
    s2.add_filter_result("default", "pod1", "node0", "plugin1", RS.PASSED_FILTER_MESSAGE)
    a2 = s2.annotations("default", "pod1")
    assert a2[RS.SCORE_RESULT_ANNOTATION_KEY] == "{}" and a2[RS.FINAL_SCORE_RESULT_ANNOTATION_KEY] == "{}"
    assert s2.annotations("default", "nope") is None
    assert RS.go_json({"a<b": {"x": "&"}}) == '{"a\\u003cb":{"x":"\\u0026"}}'


def expected_export(unsched, ndig, pdig, ptol, plugins: O.PluginSet):
    """Per-pair filter / raw / final from the oracle's plugin rules and normalizers."""
    p, n = len(pdig), len(unsched)
    has_nu = "NodeUnschedulable" in plugins.filters
    has_nn = "NodeNumber" in plugins.score
    pre = "NodeNumber" in plugins.prescore
    mode = plugins.normalize[0] if has_nn else 0
    w = plugins.weights[0] if has_nn else 1
    filt = np.zeros((p, n), np.uint8)
    raw = np.full((p, n), N.MSH_EXPORT_NONE, np.int64)
    fin = np.full((p, n), N.MSH_EXPORT_NONE, np.int64)
    for j in range(p):
        feas = [not (has_nu and unsched[i] and not ptol[j]) for i in range(n)]
        filt[j] = feas
        fl = [i for i in range(n) if feas[i]]
        if not fl or not has_nn or not pre or pdig[j] < 0:
            continue
        r = [10 if ndig[i] == pdig[j] else 0 for i in fl]
        o = O.normalize(mode, r)
        for k, i in enumerate(fl):
            raw[j, i] = r[k]
            fin[j, i] = o[k] * w
    return filt, raw, fin


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("weight", [1, 3])
def test_export_matches_oracle_and_decisions(gpu_ctx, synth, mode, weight):
    n, p = 333, 64
    rng = np.random.default_rng(mode * 10 + weight)
    unsched = (rng.random(n) < 0.5).astype(np.uint8)
    ndig = rng.integers(-1, 10, n).astype(np.int8)
    pdig = rng.integers(-1, 10, p).astype(np.int8)
    ptol = (rng.random(p) < 0.3).astype(np.uint8)
    pdig[:3] = [5, 5, -1]
    ptol[:3] = [0, 1, 0]
    unsched[:] = np.where(np.arange(n) % 7 == 0, 1, unsched)
    cfg = [S.ScorePluginConfig("NodeNumber", weight, FW.Normalize(mode))]
    gpu_ctx.set_plugins(["NodeUnschedulable"], ["NodeNumber"], cfg)
    gpu_ctx.upload_nodes(unsched, ndig)
    filt, raw, fin = gpu_ctx.export_results(pdig, ptol)
    plugins = O.PluginSet(weights=[weight], normalize=[mode])
    ef, er, eo = expected_export(unsched, ndig, pdig, ptol, plugins)
    assert np.array_equal(filt, ef) and np.array_equal(raw, er) and np.array_equal(fin, eo)
    # selectHost over the exported final scores (first max) is the device decision
    idx, score, status = gpu_ctx.schedule_batch(pdig, ptol)
    for j in range(p):
        if status[j] == N.MSH_PLACED:
            row = np.where(fin[j] == N.MSH_EXPORT_NONE, np.iinfo(np.int64).min, fin[j])
            assert int(np.argmax(row)) == idx[j] and row[idx[j]] == score[j]
        else:
            assert (raw[j] == N.MSH_EXPORT_NONE).all()


@pytest.mark.gpu
def test_record_batch_scenario_annotations(gpu_ctx, msh):
    """sched.go scenario phase 2: pod1 against node0..node8 (cordoned) + node10."""
    nodes = [O.Node(f"node{i}", True) for i in range(9)] + [O.Node("node10")]
    table = msh.pack_nodes(nodes)
    pods = msh.pack_pods([O.Pod("pod1")])
    gpu_ctx.set_plugins(["NodeUnschedulable"], ["NodeNumber"], [S.ScorePluginConfig("NodeNumber")])
    gpu_ctx.upload_nodes(table.unsched, table.digit)
    store = RS.ResultStore({"NodeNumber": 1})
    store.record_batch(gpu_ctx, table.names, pods.names, pods.digit, pods.tolerates,
                       ["NodeUnschedulable"], ["NodeNumber"])
    a = store.annotations("default", "pod1")
    filt = json.loads(a[RS.FILTER_RESULT_ANNOTATION_KEY])
    assert filt["node10"] == {"NodeUnschedulable": "passed"}
    assert all(filt[f"node{i}"] == {"NodeUnschedulable": RS.ERR_REASON_UNSCHEDULABLE} for i in range(9))
    assert a[RS.SCORE_RESULT_ANNOTATION_KEY] == '{"node10":{"NodeNumber":"0"}}'
    assert a[RS.FINAL_SCORE_RESULT_ANNOTATION_KEY] == '{"node10":{"NodeNumber":"0"}}'
