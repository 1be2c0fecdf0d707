"""Per-plugin filter / score / final-score results as simulator pod annotations.

Mirrors scheduler/plugin/resultstore/store.go: per pod ("namespace/name") three maps
node -> plugin -> string, written as JSON into the annotations named in
scheduler/plugin/annotation/annotation.go:5-9. The wrapped plugins record (plugins.go:278-325):
* Filter:  "passed", or the failing status message (NodeUnschedulable: "node(s) were
  unschedulable", k8s.io/kubernetes v1.22.0 plugins/nodeunschedulable ErrReasonUnschedulable);
* Score:   the raw score, and final = raw * weight (store.go:188-205);
* NormalizeScore: final = normalized * weight, overwriting (store.go:207-229).
applyWeightOnScore reads the weight from a map, so an unknown plugin gets weight 0
(store.go:231-234).

`record_batch` fills the store for a whole batch from the device's per-pair matrices
(msh_export_results) instead of one callback per (pod, node, plugin).
"""
from __future__ import annotations

import json
from typing import Mapping, Sequence

import numpy as np

from . import _native as N
from .framework import NODE_NUMBER, NODE_UNSCHEDULABLE

FILTER_RESULT_ANNOTATION_KEY = "scheduler-simulator/filter-result"
SCORE_RESULT_ANNOTATION_KEY = "scheduler-simulator/score-result"
FINAL_SCORE_RESULT_ANNOTATION_KEY = "scheduler-simulator/finalscore-result"
PASSED_FILTER_MESSAGE = "passed"
ERR_REASON_UNSCHEDULABLE = "node(s) were unschedulable"


def go_json(obj) -> str:
    """encoding/json.Marshal of map[string]map[string]string: keys sorted (byte order equals
    code-point order for UTF-8), no whitespace, and Go's HTML-safe escapes."""
    s = json.dumps(obj, ensure_ascii=False, separators=(",", ":"), sort_keys=True)
    return (s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
            .replace("\u2028", "\\u2028").replace("\u2029", "\\u2029"))


def new_key(namespace: str, pod_name: str) -> str:
    return f"{namespace}/{pod_name}"   # store.go:66-69


def _new_data() -> dict[str, dict]:
    return {"score": {}, "finalscore": {}, "filter": {}}


class ResultStore:
    def __init__(self, score_plugin_weight: Mapping[str, int] | None = None):
        self.results: dict[str, dict[str, dict]] = {}
        self.score_plugin_weight = dict(score_plugin_weight or {})

    def _data(self, namespace: str, pod: str) -> dict[str, dict]:
        return self.results.setdefault(new_key(namespace, pod), _new_data())

    def add_filter_result(self, namespace: str, pod: str, node: str, plugin: str, reason: str) -> None:
        self._data(namespace, pod)["filter"].setdefault(node, {})[plugin] = reason

    def add_score_result(self, namespace: str, pod: str, node: str, plugin: str, score: int) -> None:
        self._data(namespace, pod)["score"].setdefault(node, {})[plugin] = str(int(score))
        self.add_normalized_score_result(namespace, pod, node, plugin, score)

    def add_normalized_score_result(self, namespace: str, pod: str, node: str, plugin: str,
                                    normalized: int) -> None:
        final = self.apply_weight_on_score(plugin, normalized)
        self._data(namespace, pod)["finalscore"].setdefault(node, {})[plugin] = str(final)

    def apply_weight_on_score(self, plugin: str, score: int) -> int:
        return int(score) * int(self.score_plugin_weight.get(plugin, 0))

    def delete_data(self, key: str) -> None:
        self.results.pop(key, None)

    def annotations(self, namespace: str, pod: str) -> dict[str, str] | None:
        """The three annotations addSchedulingResultToPod writes (store.go:83-135), or None
        when nothing was recorded for the pod."""
        d = self.results.get(new_key(namespace, pod))
        if d is None:
            return None
        return {FILTER_RESULT_ANNOTATION_KEY: go_json(d["filter"]),
                SCORE_RESULT_ANNOTATION_KEY: go_json(d["score"]),
                FINAL_SCORE_RESULT_ANNOTATION_KEY: go_json(d["finalscore"])}

    def record_batch(self, ctx, node_names: Sequence[str], pod_names: Sequence[str],
                     pod_digit: np.ndarray, pod_tol: np.ndarray, filter_plugins: Sequence[str],
                     score_plugins: Sequence[str], namespaces: Sequence[str] | str = "default") -> None:
        """Record what the wrapped plugins would for every (pod, node) of a batch.

        `ctx` holds the node table (List order, `node_names`) and the plugin set; the final
        score comes from the device (normalize mode and weight applied there), so the store's
        weight map is only used by the per-call add_* methods."""
        filt, raw, fin = ctx.export_results(pod_digit, pod_tol)
        node_names = list(node_names)
        nn = np.asarray(node_names, dtype=object)
        has_nu = NODE_UNSCHEDULABLE in filter_plugins
        has_nn = NODE_NUMBER in score_plugins
        for j, pod in enumerate(pod_names):
            ns = namespaces if isinstance(namespaces, str) else namespaces[j]
            d = self._data(ns, pod)
            if has_nu:
                for i, name in enumerate(node_names):
                    d["filter"].setdefault(name, {})[NODE_UNSCHEDULABLE] = (
                        PASSED_FILTER_MESSAGE if filt[j, i] else ERR_REASON_UNSCHEDULABLE)
            if has_nn:
                rec = np.nonzero(raw[j] != N.MSH_EXPORT_NONE)[0]
                for i in rec:
                    name = nn[i]
                    d["score"].setdefault(name, {})[NODE_NUMBER] = str(int(raw[j, i]))
                    d["finalscore"].setdefault(name, {})[NODE_NUMBER] = str(int(fin[j, i]))
