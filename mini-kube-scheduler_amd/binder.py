"""Permit / WaitOnPermit / Bind for batched placements.

What happens to a pod after selectHost in the reference (minisched/minisched.go:89-112):
* RunPermitPlugins (:201-236) calls NodeNumber.Permit (nodenumber.go:102-119): if the
  chosen node's name ends in a digit d, the pod waits and a timer Allows it after d seconds,
  with a 10 s plugin timeout that Rejects it (waitingpod.go NewWaitingPod); a node name
  without a digit suffix is allowed at once.
* WaitOnPermit (:239-261) blocks until the signal; a Reject is routed to ErrorFunc.
* Bind (:263-277) posts a v1.Binding; a failure is routed to ErrorFunc.
Both failure paths call ErrorFunc with scheduleOne's `err`, which is nil there (the permit and
bind errors are only logged), so the pod is requeued with no UnschedulablePlugins
(minisched.go:94-97, :101-105 and :283-298).

Here the waits are deadlines on an injectable clock, grouped per (batch, delay), so a batch of
100k placements costs a handful of numpy groups rather than 100k goroutines/timers. The
reference's race, where a 0 s timer can fire before the WaitingPod is registered
(GetWaitingPod returns nil and Allow dereferences it), cannot happen: a deadline exists
before it can be observed.
"""
from __future__ import annotations

import heapq
import time
from dataclasses import dataclass, field
from typing import Callable, Sequence

import numpy as np

PERMIT_TIMEOUT_S = 10.0   # nodenumber.go:117


@dataclass
class BindOutcome:
    """What one poll() resolved: pods bound, and pods to requeue (permit reject or bind error)."""
    bound_ids: np.ndarray = field(default_factory=lambda: np.empty(0, np.int64))
    bound_nodes: list[str] = field(default_factory=list)
    failed_ids: np.ndarray = field(default_factory=lambda: np.empty(0, np.int64))
    failed_reasons: list[str] = field(default_factory=list)


def permit_delay_s(node_digit: np.ndarray) -> np.ndarray:
    """NodeNumber.Permit wait per placement: the node's suffix digit in seconds, or 0 (allowed
    without waiting) for a node whose name does not end in a digit (nodenumber.go:103-109)."""
    d = np.asarray(node_digit, np.int64)
    return np.where(d >= 0, d, 0).astype(np.float64)


class PermitBinder:
    """Deadline-driven Permit + Bind for placed pods.

    `bind(pod_id, node_name)` performs the Binding; raising marks that pod failed."""

    def __init__(self, bind: Callable[[int, str], None] | None = None,
                 clock: Callable[[], float] = time.monotonic,
                 permit_timeout_s: float = PERMIT_TIMEOUT_S, permit_enabled: bool = True):
        self.bind = bind
        self.clock = clock
        self.permit_timeout_s = permit_timeout_s
        self.permit_enabled = permit_enabled
        self._heap: list[tuple[float, int, bool, np.ndarray, list[str]]] = []
        self._seq = 0
        self._waiting = 0

    def waiting(self) -> int:
        """Pods that passed selectHost and have not been bound or rejected yet."""
        return self._waiting

    def submit(self, ids: np.ndarray, node_names: Sequence[str], node_digit: np.ndarray) -> None:
        """RunPermitPlugins for a batch of placements made now."""
        ids = np.asarray(ids, np.int64)
        if not len(ids):
            return
        now = self.clock()
        if self.permit_enabled:
            delay = permit_delay_s(node_digit)
        else:
            delay = np.zeros(len(ids))
        # Allow at now+delay unless the plugin timeout comes first (then Reject at the timeout).
        allowed = delay < self.permit_timeout_s
        due = now + np.where(allowed, delay, self.permit_timeout_s)
        names = list(node_names)
        for t in np.unique(due):
            for ok in (True, False):
                sel = np.nonzero((due == t) & (allowed == ok))[0]
                if len(sel):
                    heapq.heappush(self._heap, (float(t), self._seq, ok, ids[sel], [names[k] for k in sel]))
                    self._seq += 1
        self._waiting += len(ids)

    def next_deadline(self) -> float | None:
        return self._heap[0][0] if self._heap else None

    def poll(self) -> BindOutcome:
        """Resolve every wait whose deadline has passed, in deadline order."""
        now = self.clock()
        b_ids: list[np.ndarray] = []
        b_nodes: list[str] = []
        f_ids: list[int] = []
        f_why: list[str] = []
        while self._heap and self._heap[0][0] <= now:
            _, _, ok, ids, nodes = heapq.heappop(self._heap)
            self._waiting -= len(ids)
            if not ok:
                f_ids.extend(int(i) for i in ids)
                f_why.extend(["rejected due to timeout after waiting "
                              f"{self.permit_timeout_s:g}s at plugin NodeNumber"] * len(ids))
                continue
            if self.bind is None:
                b_ids.append(ids)
                b_nodes.extend(nodes)
                continue
            keep = np.ones(len(ids), bool)
            for k, (i, n) in enumerate(zip(ids, nodes)):
                try:
                    self.bind(int(i), n)
                except Exception as e:  # noqa: BLE001 - any Binding failure requeues the pod
                    keep[k] = False
                    f_ids.append(int(i))
                    f_why.append(f"bind: {e}")
            b_ids.append(ids[keep])
            b_nodes.extend(n for n, k in zip(nodes, keep) if k)
        return BindOutcome(np.concatenate(b_ids) if b_ids else np.empty(0, np.int64), b_nodes,
                           np.array(f_ids, np.int64), f_why)
