"""Batched scheduling loop: informer events in, placements and requeues out.

The reference runs scheduleOne in a loop (minisched/minisched.go:28-113): NextPod, LIST
nodes, filter, prescore, score, selectHost, Permit, then WaitOnPermit + Bind in a goroutine,
with ErrorFunc requeueing failures. SchedulingLoop.schedule_once does the same for a whole
batch: it drains up to `max_batch` pods from activeQ (queue.SchedulingQueue, §8 f1), brings the
device node table up to date from the informer cache (nodecache.NodeCache, §8 f2), runs the
device path once (msh_schedule_batch), hands placements to Permit/Bind (binder.PermitBinder,
§8 f3) and routes FIT_ERROR / SCORE_ERROR through ErrorFunc's rules:

* FitError  -> UnschedulablePlugins = the filter plugins that rejected a node
  (RunFilterPlugins diagnosis, :127-147): {NodeUnschedulable} when there is at least one node,
  empty when the node list is empty.
* Any other failure (PreScore / Score error, Permit reject, Bind error) -> ErrorFunc gets
  scheduleOne's nil `err`, so the set is empty (:61-75, :94-106).

Because the two plugins on the path read no placement-dependent state (NodeInfo is rebuilt
per cycle, :126), scheduling a batch against one snapshot gives each pod the decision the
reference would give it against that same snapshot. The informer handlers
(eventhandler.go:14-90) are the on_* methods; they are applied between batches.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Any, Callable, Iterable

import numpy as np

from . import _native as N
from .binder import BindOutcome, PermitBinder
from .framework import NODE_NUMBER, NODE_UNSCHEDULABLE, Outcome, ScheduleResult
from .nodecache import NodeCache
from .queue import (NODE_ADD, NODE_DELETE, NODE_UPDATE, NODE, ActionType, SchedulingQueue,
                    events_to_register, unioned_gvks)
from .snapshot import _get
from .scheduler import Scheduler


def assigned_pod(pod: Any) -> bool:
    """eventhandler.go:80-82: len(pod.Spec.NodeName) != 0."""
    nn = getattr(pod, "node_name", None)
    if nn is None:
        nn = _get(pod, "spec", "nodeName", default="")
    return bool(nn)


@dataclass
class CycleReport:
    """One schedule_once: the drained pods and the device's decision for each."""
    ids: np.ndarray        # queue pod ids, drain order
    names: list[str]
    node_index: np.ndarray # int32, -1 unless placed
    score: np.ndarray      # int64
    status: np.ndarray     # int32 msh_status
    node_names: tuple[str, ...]  # List-order names of the snapshot used (a copy)
    sync: str              # node table sync: "upload" / "patch" / "clean"
    bind: BindOutcome      # Permit/Bind resolutions that became due during this cycle

    def __len__(self) -> int:
        return len(self.ids)

    def counts(self) -> dict[str, int]:
        return {"placed": int(np.sum(self.status == N.MSH_PLACED)),
                "fit_error": int(np.sum(self.status == N.MSH_FIT_ERROR)),
                "score_error": int(np.sum(self.status == N.MSH_SCORE_ERROR))}

    def results(self, unschedulable_plugins: frozenset[str] = frozenset()) -> list[ScheduleResult]:
        out = []
        for j, name in enumerate(self.names):
            st = int(self.status[j])
            if st == N.MSH_PLACED:
                i = int(self.node_index[j])
                out.append(ScheduleResult(name, Outcome.PLACED, self.node_names[i], i, int(self.score[j])))
            elif st == N.MSH_FIT_ERROR:
                out.append(ScheduleResult(name, Outcome.FIT_ERROR, unschedulable_plugins=unschedulable_plugins))
            else:
                out.append(ScheduleResult(name, Outcome.SCORE_ERROR))
        return out


class SchedulingLoop:
    """Queue + node cache + device path + Permit/Bind, one batch per cycle."""

    def __init__(self, scheduler: Scheduler | None = None, *, max_batch: int = 1 << 16,
                 clock: Callable[[], float] = time.monotonic,
                 bind: Callable[[int, str], None] | None = None,
                 permit: bool | None = None):
        self.scheduler = scheduler or Scheduler()
        self.ctx = self.scheduler.ctx
        if max_batch < 1:
            raise ValueError("max_batch < 1")
        self.max_batch = max_batch
        self.clock = clock
        score_names = [c.name for c in self.scheduler.score_plugins]
        self.cluster_event_map = events_to_register(self.scheduler.filter_plugins, score_names)
        self.gvk = unioned_gvks(self.cluster_event_map)
        self.queue = SchedulingQueue(self.cluster_event_map, clock=clock)
        self.cache = NodeCache()
        # permitPlugins = [NodeNumber] in the reference (initialize.go:124-131)
        self.binder = PermitBinder(bind, clock=clock,
                                   permit_enabled=(NODE_NUMBER in score_names) if permit is None else permit)
        self._fit_mask = self.queue.plugins_mask(self._fit_plugins(nonempty=True))

    def close(self) -> None:
        self.scheduler.close()

    def _fit_plugins(self, nonempty: bool) -> frozenset[str]:
        if nonempty and NODE_UNSCHEDULABLE in self.scheduler.filter_plugins:
            return frozenset([NODE_UNSCHEDULABLE])
        return frozenset()

    # ---- informer handlers (eventhandler.go) -----------------------------------
    def on_pod_add(self, pod: Any) -> int | None:
        """addPodToSchedulingQueue for unassigned pods (:20-35, :84-90)."""
        if assigned_pod(pod):
            return None
        return self.queue.add(pod)

    def on_pods_add(self, pods: Iterable[Any]) -> np.ndarray:
        return self.queue.add_many([p for p in pods if not assigned_pod(p)])

    def _node_event(self, action: ActionType, event) -> None:
        # A handler exists only for the actions some plugin registered (eventhandler.go:37-57).
        if self.gvk.get(NODE, ActionType(0)) & action:
            self.queue.move_all_to_active_or_backoff_queue(event)

    def on_node_add(self, node: Any) -> None:
        self.cache.add(node)
        self._node_event(ActionType.ADD, NODE_ADD)

    def on_node_update(self, old: Any, new: Any) -> None:
        self.cache.update(old, new)
        self._node_event(ActionType.UPDATE, NODE_UPDATE)

    def on_node_delete(self, node: Any) -> None:
        self.cache.delete(node)
        self._node_event(ActionType.DELETE, NODE_DELETE)

    # ---- the cycle ---------------------------------------------------------------
    def error_func(self, ids: np.ndarray, status: np.ndarray) -> None:
        """ErrorFunc (minisched.go:283-298) for a batch, in drain order."""
        if not len(ids):
            return
        fit = status == N.MSH_FIT_ERROR
        fit_mask = self._fit_mask if len(self.cache) > 0 else 0
        masks = np.where(fit, np.uint64(fit_mask), np.uint64(0)).astype(np.uint64)
        self.queue.add_unschedulable(ids, masks)

    def schedule_once(self, max_pods: int | None = None) -> CycleReport:
        """One batched scheduling cycle. Returns what was decided; placements are handed to
        Permit/Bind, failures are requeued."""
        bind = self.poll_binder()
        batch = self.queue.next_batch(self.max_batch if max_pods is None else max_pods)
        sync = self.cache.sync(self.ctx)
        # the report keeps a snapshot of the List-order names: NodeCache.add / delete change the
        # live list in place, and node_index must keep naming this cycle's nodes
        names = tuple(self.cache.names)
        if not len(batch):
            return CycleReport(batch.ids, [], np.empty(0, np.int32), np.empty(0, np.int64),
                               np.empty(0, np.int32), names, sync, bind)
        idx, score, status = self.ctx.schedule_batch(batch.digit, batch.tolerates)
        placed = status == N.MSH_PLACED
        self.error_func(batch.ids[~placed], status[~placed])
        if placed.any():
            node_idx = idx[placed]
            self.binder.submit(batch.ids[placed], [names[i] for i in node_idx], self.cache.digit[node_idx])
        return CycleReport(batch.ids, batch.names, idx, score, status, names, sync, bind)

    def poll_binder(self) -> BindOutcome:
        """Resolve due Permit waits; rejected / failed binds go back through ErrorFunc."""
        out = self.binder.poll()
        if len(out.failed_ids):
            self.queue.add_unschedulable(out.failed_ids, None)
        return out

    def run_until_idle(self, max_cycles: int = 1 << 20) -> list[CycleReport]:
        """schedule_once until activeQ is empty (pods left in unschedulableQ / backoffQ stay)."""
        reports = []
        for _ in range(max_cycles):
            if self.queue.active_len() == 0:
                break
            reports.append(self.schedule_once())
        return reports
