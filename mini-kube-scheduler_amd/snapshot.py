"""Snapshot packer: v1.Node / v1.Pod objects -> SoA tables for the device path.

Replaces, once per batch, the decoding the reference repeats on every cycle: the node LIST
in etcd key order (minisched/minisched.go:40), the name-suffix digit (nodenumber.go:51-52,
:81-83) and the pod's unschedulable-taint toleration (upstream NodeUnschedulable.Filter).
The packing itself runs in native code (msh_pack_nodes / msh_pack_pods in
libminisched_hip.so); this module only flattens Python objects into byte blobs.

Objects may be dataclass-like (`.name`, `.unschedulable`, `.tolerations`) or k8s-shaped
dicts ({"metadata": {"name": ...}, "spec": {"unschedulable": ..., "tolerations": [...]}}).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Any, Iterable, Mapping, Sequence

import numpy as np

from . import _native as N


def _get(obj: Any, *path: str, default=None):
    cur = obj
    for p in path:
        if cur is None:
            return default
        if isinstance(cur, dict):
            cur = cur.get(p)
        else:
            cur = getattr(cur, p, None)
    return default if cur is None else cur


def node_name(n: Any) -> str:
    return n.name if hasattr(n, "name") else _get(n, "metadata", "name", default="")


def node_unschedulable(n: Any) -> bool:
    if hasattr(n, "unschedulable"):
        return bool(n.unschedulable)
    return bool(_get(n, "spec", "unschedulable", default=False))


def pod_name(p: Any) -> str:
    return p.name if hasattr(p, "name") else _get(p, "metadata", "name", default="")


def pod_tolerations(p: Any) -> list:
    if hasattr(p, "tolerations"):
        return list(p.tolerations or ())
    return list(_get(p, "spec", "tolerations", default=[]) or [])


def _tol_field(t: Any, *names: str) -> str:
    for nm in names:
        v = t.get(nm) if isinstance(t, dict) else getattr(t, nm, None)
        if v:
            return str(v)
    return ""


def _blob(names: Sequence[str]) -> tuple[bytes, np.ndarray]:
    enc = [s.encode("utf-8") for s in names]
    off = np.zeros(len(enc) + 1, np.int64)
    if enc:
        off[1:] = np.cumsum([len(b) for b in enc])
    return b"".join(enc), off


@dataclass
class NodeTable:
    """Node SoA in List order. `order[k]` = input index of the k-th node."""
    names: list[str]          # in List order
    unsched: np.ndarray       # uint8
    digit: np.ndarray         # int8, -1 = suffix not '0'..'9'
    order: np.ndarray         # int32

    def __len__(self) -> int:
        return len(self.names)


@dataclass
class PodTable:
    names: list[str]
    digit: np.ndarray         # int8
    tolerates: np.ndarray     # uint8

    def __len__(self) -> int:
        return len(self.names)


def pack_nodes(nodes: Iterable[Any]) -> NodeTable:
    nodes = list(nodes)
    names = [node_name(n) for n in nodes]
    uns = np.array([1 if node_unschedulable(n) else 0 for n in nodes], np.uint8)
    blob, off = _blob(names)
    n = len(names)
    order = np.empty(n, np.int32)
    out_u = np.empty(n, np.uint8)
    out_d = np.empty(n, np.int8)
    N.check(N.lib().msh_pack_nodes(n, blob, N.ptr(off), N.ptr(uns), N.ptr(order), N.ptr(out_u), N.ptr(out_d)))
    return NodeTable([names[i] for i in order], out_u, out_d, order)


def pod_fields(pods: Sequence[Any]) -> tuple[list[str], list[str], list[Sequence[Any]]]:
    """(names, namespaces, tolerations) of pod objects in one pass. k8s-shaped dicts take a
    direct path (the informer's common case); anything else goes through the accessors."""
    names, spaces, tols = [], [], []
    for p in pods:
        if type(p) is dict:
            md = p.get("metadata") or {}
            names.append(md.get("name") or "")
            spaces.append(md.get("namespace") or p.get("namespace") or "")
            tols.append((p.get("spec") or {}).get("tolerations") or ())
        else:
            names.append(pod_name(p))
            spaces.append(pod_namespace(p))
            tols.append(pod_tolerations(p))
    return names, spaces, tols


def pod_namespace(p: Any) -> str:
    if isinstance(p, Mapping):
        return (p.get("metadata") or {}).get("namespace", "") or p.get("namespace", "") or ""
    md = getattr(p, "metadata", None)
    ns = getattr(md, "namespace", None) if md is not None else None
    return ns if ns is not None else getattr(p, "namespace", "") or ""


def pack_pods(pods: Iterable[Any], fields: tuple[list[str], list[str], list[Sequence[Any]]] | None = None) -> PodTable:
    """`fields`: pod_fields(pods) when the caller already has them."""
    pods = list(pods)
    names, _, tol_lists = fields if fields is not None else pod_fields(pods)
    blob, off = _blob(names)
    tols_flat: list[N.Toleration] = []
    keep: list[bytes] = []  # keep encoded strings alive for the call
    tol_off = np.zeros(len(pods) + 1, np.int64)
    for j, tl in enumerate(tol_lists):
        for t in tl:
            fields = [_tol_field(t, "key"), _tol_field(t, "operator", "op"), _tol_field(t, "value"),
                      _tol_field(t, "effect")]
            enc = [f.encode("utf-8") for f in fields]
            keep.extend(enc)
            tols_flat.append(N.Toleration(*enc))
        tol_off[j + 1] = len(tols_flat)
    arr = (N.Toleration * max(len(tols_flat), 1))(*tols_flat)
    p = len(names)
    digit = np.empty(p, np.int8)
    tol = np.empty(p, np.uint8)
    N.check(N.lib().msh_pack_pods(p, blob, N.ptr(off), C.cast(arr, C.POINTER(N.Toleration)),
                                  N.ptr(tol_off), N.ptr(digit), N.ptr(tol)))
    return PodTable(names, digit, tol)
