"""Independent closed-form checker (NOT reference code, NOT the oracle's loop structure).

For the reference plugin set (filter NodeUnschedulable, prescore+score NodeNumber, weight w,
no normalize, first-max tie-break) the outcome per pod is:
  - no feasible node                       -> FIT_ERROR
  - pod name suffix not a digit            -> SCORE_ERROR (NodeNumber has no PreScore state)
  - else the first feasible node (List order) whose suffix digit equals the pod's, score 10*w;
    if none, the first feasible node, score 0.
Vectorised over pods by (digit, tolerates) class: it must never be used as the kernel
(SURVEY.md §7 hazard "degenerate closed form"), only as a cross-check.
"""
from __future__ import annotations

import numpy as np


def closed_form(unsched, node_digit, pod_digit, pod_tol, weight: int = 1):
    unsched = np.asarray(unsched, bool)
    node_digit = np.asarray(node_digit, np.int16)
    p = len(pod_digit)
    idx = np.full(p, -1, np.int32)
    score = np.zeros(p, np.int64)
    status = np.zeros(p, np.int32)
    n = len(unsched)
    for tol in (0, 1):
        feas = np.ones(n, bool) if tol else ~unsched
        first_feas = int(np.argmax(feas)) if feas.any() else -1
        for d in range(-1, 10):
            sel = (np.asarray(pod_tol) == tol) & (np.asarray(pod_digit) == d)
            if not sel.any():
                continue
            if first_feas < 0:
                status[sel] = 1
                continue
            if d < 0:
                status[sel] = 2
                continue
            m = feas & (node_digit == d)
            if m.any():
                idx[sel] = int(np.argmax(m))
                score[sel] = 10 * weight
            else:
                idx[sel] = first_feas
    return idx, score, status


def closed_form_modes(unsched, node_digit, pod_digit, pod_tol, weight: int = 1, mode: int = 0):
    """The same, for every NormalizeScore mode of the C-ABI (msh_normalize) with the reference
    filter / prescore / score lists and weight w. Per (tolerates, digit) class: the first feasible
    node, the first feasible digit match (raw 10) and the first feasible non-match (raw 0); over a
    2-level raw list the normalised winner and its score are (build extensions):
      NONE     match ? (match, 10w) : (first feasible, 0)
      DEFAULT  match ? (match, 100w) : (first feasible, 0)          DefaultNormalizeScore
      REVERSE  non-match ? (non-match, 100w) : (first feasible, 0)  DefaultNormalizeScore reverse
      MINMAX   match ? (match, non-match ? 100w : 0) : (first feasible, 0)"""
    unsched = np.asarray(unsched, bool)
    node_digit = np.asarray(node_digit, np.int16)
    pod_digit, pod_tol = np.asarray(pod_digit), np.asarray(pod_tol)
    p, n = len(pod_digit), len(unsched)
    idx = np.full(p, -1, np.int32)
    score = np.zeros(p, np.int64)
    status = np.zeros(p, np.int32)
    first = lambda m: int(np.argmax(m)) if m.any() else -1
    for tol in (0, 1):
        feas = np.ones(n, bool) if tol else ~unsched
        ia = first(feas)
        for d in range(-1, 10):
            sel = (pod_tol == tol) & (pod_digit == d)
            if not sel.any():
                continue
            if ia < 0:
                status[sel] = 1
                continue
            if d < 0:
                status[sel] = 2
                continue
            im = first(feas & (node_digit == d))
            ix = first(feas & (node_digit != d))
            if mode in (0, 1):
                idx[sel], score[sel] = (im, (10 if mode == 0 else 100) * weight) if im >= 0 else (ia, 0)
            elif mode == 2:
                idx[sel], score[sel] = (ix, 100 * weight) if ix >= 0 else (ia, 0)
            else:
                idx[sel], score[sel] = (im, 100 * weight if ix >= 0 else 0) if im >= 0 else (ia, 0)
    return idx, score, status


def _trunc_div(a: np.ndarray, b) -> np.ndarray:
    """Go / C integer division (truncates toward zero), int64 arrays."""
    q = np.abs(a) // np.abs(b)
    return np.where((a >= 0) == (np.asarray(b) >= 0), q, -q)


def direct_plugins(unsched, node_digit, pod_digit, pod_tol, plugins, cols=None, has_nu: bool = True,
                   nn_prescore: bool = True):
    """Direct per-pod evaluation of any plugin list over the whole node list, vectorised over the
    nodes (a second, independent statement of RunFilterPlugins + RunScorePlugins + first-max
    selectHost, not the oracle's code): `plugins` = [(name, weight, mode)], name "NodeNumber" or
    "ScoreColumnK" (cols[K] the int64 per-node scores). Go int64 arithmetic (wrapping), normalize
    modes as msh_normalize. For sampled checks of the generic pipeline at full size."""
    unsched = np.asarray(unsched, bool)
    node_digit = np.asarray(node_digit, np.int64)
    p = len(pod_digit)
    idx = np.full(p, -1, np.int32)
    score = np.zeros(p, np.int64)
    status = np.zeros(p, np.int32)
    nn = any(nm == "NodeNumber" for nm, _, _ in plugins)
    with np.errstate(over="ignore"):
        for j in range(p):
            feas = np.ones(len(unsched), bool) if (pod_tol[j] or not has_nu) else ~unsched
            f = np.flatnonzero(feas)
            if f.size == 0:
                status[j] = 1
                continue
            if nn and (not nn_prescore or not 0 <= pod_digit[j] <= 9):
                status[j] = 2
                continue
            tot = np.zeros(f.size, np.int64)
            for name, w, mode in plugins:
                if name == "NodeNumber":
                    raw = np.where(node_digit[f] == pod_digit[j], 10, 0).astype(np.int64)
                else:
                    raw = np.asarray(cols[int(name[-1])], np.int64)[f]
                if mode in (1, 2):
                    m = max(int(raw.max()), 0)
                    if m == 0:
                        raw = raw if mode == 1 else np.full(f.size, 100, np.int64)
                    else:
                        raw = _trunc_div(100 * raw, m)
                        raw = raw if mode == 1 else 100 - raw
                elif mode == 3:
                    mx, mn = int(raw.max()), int(raw.min())
                    raw = np.zeros(f.size, np.int64) if mx == mn else _trunc_div((raw - mn) * 100, mx - mn)
                tot = tot + raw * np.int64(w) if w < (1 << 63) else tot
            b = int(np.argmax(tot))  # the first maximum
            idx[j], score[j] = f[b], tot[b]
    return idx, score, status


def closed_form_capacity(unsched, node_digit, pod_digit, pod_tol, weight: int = 1, cap: int = 0, counts=None):
    """The reference plugin set (NONE, weight w) in sequential-commit order with a capacity: a node that
    holds `cap` pods is infeasible for every later pod (the build's capacity filter). Per pod, in order:
    the first feasible non-full node whose digit matches, else the first feasible non-full node; FitError
    when every feasible node is full (or none is feasible); the NodeNumber score error for a pod without
    a digit. Each (tolerates, digit) list and each tolerates list keeps a pointer to its first non-full
    node, which only moves forward (counts only grow): O(P + N) overall, not the oracle's O(P x N) loop.
    Returns (idx, score, status, counts)."""
    unsched = np.asarray(unsched, bool)
    node_digit = np.asarray(node_digit, np.int16)
    pod_digit, pod_tol = np.asarray(pod_digit), np.asarray(pod_tol)
    n, p = len(unsched), len(pod_digit)
    counts = np.zeros(n, np.int64) if counts is None else np.array(counts, np.int64)
    feas = {0: np.flatnonzero(~unsched), 1: np.arange(n)}
    match = {(t, d): f[node_digit[f] == d] for t, f in feas.items() for d in range(10)}
    ptr = {}
    idx = np.full(p, -1, np.int32)
    score = np.zeros(p, np.int64)
    status = np.zeros(p, np.int32)
    full = (lambda i: counts[i] >= cap) if cap > 0 else (lambda i: False)

    def first(key, lst):
        k = ptr.get(key, 0)
        while k < len(lst) and full(lst[k]):
            k += 1
        ptr[key] = k
        return int(lst[k]) if k < len(lst) else -1

    for j in range(p):
        t, d = int(pod_tol[j] != 0), int(pod_digit[j])
        ia = first(("f", t), feas[t])
        if ia < 0:
            status[j] = 1
            continue
        if not 0 <= d <= 9:
            status[j] = 2
            continue
        im = first(("m", t, d), match[(t, d)])
        idx[j], score[j] = (im, 10 * weight) if im >= 0 else (ia, 0)
        counts[idx[j]] += 1
    return idx, score, status, counts.astype(np.int32)
