"""Seeded synthetic clusters (SURVEY.md §8d / BASELINE.md workloads).

splitmix64 with seed 0x6d696e69 ("mini"). Nodes are named "node%d" and delivered in List
order (byte-wise sorted names, the apiserver LIST order of minisched/minisched.go:40);
Spec.Unschedulable ~ Bernoulli(0.10), with at least one schedulable node forced per digit
class. Pods are "pod%d"; 1% get a non-digit suffix ("pod%d-x"); 5% tolerate
node.kubernetes.io/unschedulable (op Exists, effect NoSchedule).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SEED = 0x6D696E69
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, n: int, stream: int = 0) -> np.ndarray:
    """n splitmix64 outputs for (seed, stream) as uint64."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed + stream * 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF)
        z = base + (np.arange(1, n + 1, dtype=np.uint64) * _GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, n: int, stream: int) -> np.ndarray:
    return (splitmix64(seed, n, stream) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


@dataclass
class Cluster:
    node_names: list[str]     # List order
    unsched: np.ndarray       # uint8, List order
    node_digit: np.ndarray    # int8, List order
    pod_names: list[str]
    pod_digit: np.ndarray     # int8
    pod_tol: np.ndarray       # uint8


def list_order_names(n: int) -> list[str]:
    return sorted((f"node{i}" for i in range(n)), key=lambda s: s.encode())


def make_nodes(n: int, seed: int = SEED, p_unsched: float = 0.10, all_unsched: bool = False):
    names = list_order_names(n)
    u = uniform(seed, n, 1) < p_unsched
    if all_unsched:
        u[:] = True
    elif n:
        # force one schedulable node per digit class (the first of each class in List order)
        seen = set()
        for k, nm in enumerate(names):
            d = nm[-1]
            if d not in seen:
                seen.add(d)
                u[k] = False
    digit = np.array([ord(nm[-1]) - 48 if nm[-1].isdigit() else -1 for nm in names], np.int8)
    return names, u.astype(np.uint8), digit


def make_pods(p: int, seed: int = SEED, p_nondigit: float = 0.01, p_tol: float = 0.05):
    nd = uniform(seed, p, 2) < p_nondigit
    tl = uniform(seed, p, 3) < p_tol
    names = [f"pod{j}-x" if nd[j] else f"pod{j}" for j in range(p)]
    digit = np.where(nd, -1, np.arange(p) % 10).astype(np.int8)
    return names, digit, tl.astype(np.uint8)


def make_cluster(n: int, p: int, seed: int = SEED, **kw) -> Cluster:
    node_names, unsched, node_digit = make_nodes(n, seed, **{k: v for k, v in kw.items() if k in ("p_unsched", "all_unsched")})
    pod_names, pod_digit, pod_tol = make_pods(p, seed, **{k: v for k, v in kw.items() if k in ("p_nondigit", "p_tol")})
    return Cluster(node_names, unsched, node_digit, pod_names, pod_digit, pod_tol)


def make_soa(n: int, p: int, seed: int = SEED):
    """Fast SoA-only workload for large sizes (no name strings): same distributions.

    Node digits follow the List order of "node%d" names, computed without building strings
    for n <= 10**6 via the sorted name list when n is small, else by the same sort."""
    _, unsched, node_digit = make_nodes(n, seed)
    _, pod_digit, pod_tol = make_pods(p, seed) if p <= 200_000 else _make_pods_fast(p, seed)
    return unsched, node_digit, pod_digit, pod_tol


def _make_pods_fast(p: int, seed: int):
    nd = uniform(seed, p, 2) < 0.01
    tl = uniform(seed, p, 3) < 0.05
    digit = np.where(nd, -1, np.arange(p) % 10).astype(np.int8)
    return None, digit, tl.astype(np.uint8)
