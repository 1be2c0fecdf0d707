"""Incremental node snapshot: informer deltas -> List-order SoA on the device.

The reference LISTs every node from the API server on every scheduling cycle
(minisched/minisched.go:40) and re-derives each plugin input from the objects. Here a node
cache receives the informer's Add / Update / Delete callbacks (eventhandler.go:37-57) and
keeps the two device columns (Spec.Unschedulable, name-suffix digit) in List order, i.e.
ascending byte order of the name (etcd key order of /registry/minions/<name>). Python's str
order is code-point order, which equals UTF-8 byte order, so `bisect` over the names gives
the same order msh_pack_nodes produces.

Device synchronisation (`sync`) is O(delta) when the List order did not change (only
field updates: msh_patch_nodes scatters the changed entries) and one msh_upload_nodes of
2 B/node otherwise (adds / deletes shift every later index).
"""
from __future__ import annotations

import bisect
from typing import Any

import numpy as np

from .snapshot import node_name, node_unschedulable


def name_digit(name: str) -> int:
    """Last byte of the name as '0'..'9' -> 0..9, else -1 (nodenumber.go:81-87 Atoi of the
    last byte; a multi-byte UTF-8 tail is never a digit)."""
    b = name.encode("utf-8")
    return b[-1] - 48 if b and 48 <= b[-1] <= 57 else -1


class NodeCache:
    """The node table in List order, maintained from informer events."""

    def __init__(self, nodes: Any = ()):
        self.names: list[str] = []
        self._unsched = np.zeros(0, np.uint8)
        self._digit = np.zeros(0, np.int8)
        self._structural = True               # List order changed since the last sync
        self._patched: dict[str, None] = {}   # names updated in place since the last sync
        self.version = 0                      # bumps on every change
        for n in nodes:
            self.add(n)

    def __len__(self) -> int:
        return len(self.names)

    def __contains__(self, name: str) -> bool:
        i = bisect.bisect_left(self.names, name)
        return i < len(self.names) and self.names[i] == name

    @property
    def unsched(self) -> np.ndarray:
        return self._unsched

    @property
    def digit(self) -> np.ndarray:
        return self._digit

    def index(self, name: str) -> int:
        i = bisect.bisect_left(self.names, name)
        if i == len(self.names) or self.names[i] != name:
            raise KeyError(name)
        return i

    # ---- informer callbacks ---------------------------------------------------
    def add(self, node: Any) -> None:
        """Node Add. An Add for a name already present is applied as an Update."""
        name = node_name(node)
        if not name:
            raise ValueError("node with empty name")
        u = 1 if node_unschedulable(node) else 0
        i = bisect.bisect_left(self.names, name)
        if i < len(self.names) and self.names[i] == name:
            self._set(i, name, u)
            return
        self.names.insert(i, name)
        self._unsched = np.insert(self._unsched, i, np.uint8(u))
        self._digit = np.insert(self._digit, i, np.int8(name_digit(name)))
        self._structural = True
        self.version += 1

    def update(self, old: Any, new: Any) -> None:
        """Node Update. Names are immutable in Kubernetes; a renamed object is delete + add."""
        on, nn = node_name(old), node_name(new)
        if on != nn:
            self.delete(old)
            self.add(new)
            return
        i = self.index(nn)
        self._set(i, nn, 1 if node_unschedulable(new) else 0)

    def delete(self, node: Any) -> None:
        """Node Delete (accepts a node object or a name)."""
        name = node if isinstance(node, str) else node_name(node)
        i = self.index(name)
        del self.names[i]
        self._unsched = np.delete(self._unsched, i)
        self._digit = np.delete(self._digit, i)
        self._patched.pop(name, None)
        self._structural = True
        self.version += 1

    def _set(self, i: int, name: str, u: int) -> None:
        if self._unsched[i] != u:
            self._unsched[i] = u
            self._patched[name] = None
            self.version += 1

    # ---- device ---------------------------------------------------------------
    def dirty(self) -> bool:
        return self._structural or bool(self._patched)

    def sync(self, ctx) -> str:
        """Bring `ctx`'s device table up to date. Returns "upload", "patch" or "clean"."""
        if self._structural:
            ctx.upload_nodes(self._unsched, self._digit)
            self._structural = False
            self._patched.clear()
            return "upload"
        if self._patched:
            idx = np.array([self.index(n) for n in self._patched], np.int32)
            ctx.patch_nodes(idx, self._unsched[idx], self._digit[idx])
            self._patched.clear()
            return "patch"
        return "clean"

    def mark_stale(self) -> None:
        """Force a full upload on the next sync (e.g. a new device context)."""
        self._structural = True
