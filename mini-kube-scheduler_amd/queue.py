"""Scheduling queue with batch drain: the pod source in front of the device path.

Mirrors minisched/queue/queue.go (SchedulingQueue) and the requeue half of the scheduling
cycle (Scheduler.ErrorFunc, minisched/minisched.go:283-298), with one change of shape: instead
of NextPod() handing out one pod per cycle (queue.go:84-92, a busy-wait), `next_batch()` drains
up to B pods from the head of activeQ in FIFO order and returns them as the SoA columns
msh_schedule_batch consumes (pod digit, tolerates-unschedulable). Pods are packed once, on Add.

Semantics kept from the reference:
* Add appends to activeQ (queue.go:35-43); a second Add of the same pod appends it again.
* AddUnschedulable refreshes the timestamp and adds-or-updates unschedulableQ, keyed by
  "name_namespace" (queue.go:95-107, keyFunc :152-154).
* MoveAllToActiveOrBackoffQueue moves every unschedulable pod whose UnschedulablePlugins is
  empty, or that matches the event through clusterEventMap (podMatchesEvent, :167-190), to
  podBackoffQ if its backoff has not expired (isPodBackingoff, :205-209) else to activeQ
  (:54-81).
* Backoff = 1 s doubled per attempt, capped at 10 s (calculateBackoffDuration, :219-235).
  ErrorFunc builds a fresh QueuedPodInfo (minisched.go:284-286), so Attempts is always 0 and
  the backoff is always 1 s; `attempts` is kept per pod for callers that count.
* podBackoffQ is never flushed by the reference (flushBackoffQCompleted panics, :136-140);
  `flush_backoff_completed()` is an explicit extension the caller must invoke.

The one deliberate determinism choice: the reference ranges over the unschedulableQ Go map,
so the order in which moved pods re-enter activeQ is random. Here it is the order of their
latest AddUnschedulable, which is one of the orders the reference can produce.

Cluster events and their registration (initialize.go:142-176) follow k8s.io/kubernetes
v1.22.0 (go.mod:51), pkg/scheduler/framework/types.go: ActionType bits and
ClusterEvent.IsWildCard; plugins/nodeunschedulable EventsToRegister = {Node, Add|UpdateNodeTaint}.
"""
from __future__ import annotations

import enum
import time
from dataclasses import dataclass
from typing import Any, Callable, Iterable, Mapping, Sequence

import numpy as np

from .framework import NODE_NUMBER, NODE_UNSCHEDULABLE
from .snapshot import pack_pods, pod_fields

WILDCARD = "*"
NODE = "Node"
POD = "Pod"

POD_INITIAL_BACKOFF_S = 1.0   # queue.go:213
POD_MAX_BACKOFF_S = 10.0      # queue.go:214


class ActionType(enum.IntFlag):
    """framework.ActionType (k8s v1.22 types.go)."""
    ADD = 1
    DELETE = 2
    UPDATE_NODE_ALLOCATABLE = 4
    UPDATE_NODE_LABEL = 8
    UPDATE_NODE_TAINT = 16
    UPDATE_NODE_CONDITION = 32
    ALL = 63
    UPDATE = 4 | 8 | 16 | 32


@dataclass(frozen=True)
class ClusterEvent:
    """framework.ClusterEvent. Registered events carry no label; the ones the event handlers
    raise do (eventhandler.go:40-52), so they never collide as map keys."""
    resource: str
    action: ActionType
    label: str = ""

    def is_wildcard(self) -> bool:
        return self.resource == WILDCARD and self.action == ActionType.ALL


# What the informer handlers raise (eventhandler.go:37-57).
NODE_ADD = ClusterEvent(NODE, ActionType.ADD, "NodeAdd")
NODE_UPDATE = ClusterEvent(NODE, ActionType.UPDATE, "NodeUpdate")
NODE_DELETE = ClusterEvent(NODE, ActionType.DELETE, "NodeDelete")
WILDCARD_EVENT = ClusterEvent(WILDCARD, ActionType.ALL, "WildCardEvent")

# EnqueueExtensions.EventsToRegister of the two plugins on the path.
PLUGIN_EVENTS: dict[str, tuple[ClusterEvent, ...]] = {
    # k8s v1.22 plugins/nodeunschedulable/node_unschedulable.go
    NODE_UNSCHEDULABLE: (ClusterEvent(NODE, ActionType.ADD | ActionType.UPDATE_NODE_TAINT),),
    # minisched/plugins/score/nodenumber/nodenumber.go:66-70
    NODE_NUMBER: (ClusterEvent(NODE, ActionType.ADD),),
}


def events_to_register(filter_plugins: Sequence[str] = (NODE_UNSCHEDULABLE,),
                       score_plugins: Sequence[str] = (NODE_NUMBER,)) -> dict[ClusterEvent, frozenset[str]]:
    """clusterEventMap as initialize.go:142-156 builds it.

    Reference quirk kept: NodeNumber's events are registered under NodeUnschedulable's name
    (initialize.go:153-154), so a pod that failed only on NodeNumber would never be matched
    by name; with this plugin set that cannot happen (score failures requeue with an empty
    set, minisched.go:70-75)."""
    emap: dict[ClusterEvent, set[str]] = {}
    registrant = NODE_UNSCHEDULABLE

    def register(name: str, evts: Iterable[ClusterEvent]) -> None:
        for e in evts:
            emap.setdefault(e, set()).add(name)

    if NODE_UNSCHEDULABLE in filter_plugins:
        register(registrant, PLUGIN_EVENTS[NODE_UNSCHEDULABLE])
    if NODE_NUMBER in score_plugins:
        register(registrant, PLUGIN_EVENTS[NODE_NUMBER])
    return {e: frozenset(s) for e, s in emap.items()}


def unioned_gvks(cluster_event_map: Mapping[ClusterEvent, Any]) -> dict[str, ActionType]:
    """initialize.go:168-176: per resource, the OR of every registered action."""
    out: dict[str, ActionType] = {}
    for e in cluster_event_map:
        out[e.resource] = out.get(e.resource, ActionType(0)) | e.action
    return out


def calculate_backoff_duration(attempts: int) -> float:
    """queue.go:219-235 (seconds)."""
    d = POD_INITIAL_BACKOFF_S
    for _ in range(1, attempts):
        if d > POD_MAX_BACKOFF_S - d:
            return POD_MAX_BACKOFF_S
        d += d
    return d


@dataclass
class PodBatch:
    """A FIFO drain of activeQ, ready for msh_schedule_batch."""
    ids: np.ndarray        # int64 queue-internal pod ids
    names: list[str]
    digit: np.ndarray      # int8, -1 = name suffix not a digit
    tolerates: np.ndarray  # uint8

    def __len__(self) -> int:
        return len(self.ids)


class _Column:
    """Growable 1-D numpy column."""

    def __init__(self, dtype, fill=0):
        self.a = np.full(64, fill, dtype)
        self.fill = fill

    def ensure(self, n: int) -> None:
        if n > len(self.a):
            b = np.full(max(n, 2 * len(self.a)), self.fill, self.a.dtype)
            b[:len(self.a)] = self.a
            self.a = b


class SchedulingQueue:
    """activeQ / podBackoffQ / unschedulableQ over a SoA pod table.

    `clock` returns seconds (monotonic by default); tests inject a fake one."""

    def __init__(self, cluster_event_map: Mapping[ClusterEvent, frozenset[str]] | None = None,
                 clock: Callable[[], float] = time.monotonic):
        self.cluster_event_map = dict(events_to_register() if cluster_event_map is None else cluster_event_map)
        self.clock = clock
        # plugin name -> bit of the per-pod UnschedulablePlugins mask
        self._plugin_bit: dict[str, int] = {}
        for names in self.cluster_event_map.values():
            for nm in sorted(names):
                self._bit(nm)
        # pod table (id = first-Add order of the key)
        self._key_to_id: dict[str, int] = {}
        self.keys: list[str] = []
        self.names: list[str] = []
        self.objs: list[Any] = []
        self._digit = _Column(np.int8, -1)
        self._tol = _Column(np.uint8)
        self._ts = _Column(np.float64)          # QueuedPodInfo.Timestamp
        self._t0 = _Column(np.float64)          # InitialAttemptTimestamp
        self._attempts = _Column(np.int32)
        self._plugins = _Column(np.uint64)      # UnschedulablePlugins bitmask
        self._in_unsched = _Column(np.bool_)
        self._unsched_seq = _Column(np.int64, -1)
        self._seq = 0
        # activeQ / podBackoffQ: FIFO of id chunks
        self._active: list[np.ndarray] = []
        self._active_head = 0
        self._active_len = 0
        self._backoff: list[int] = []

    # ---- plugin-name bit mask ------------------------------------------------
    def _bit(self, name: str) -> int:
        b = self._plugin_bit.get(name)
        if b is None:
            if len(self._plugin_bit) >= 64:
                raise ValueError("more than 64 distinct plugin names")
            b = self._plugin_bit[name] = 1 << len(self._plugin_bit)
        return b

    def plugins_mask(self, names: Iterable[str] | None) -> int:
        m = 0
        for nm in names or ():
            m |= self._bit(nm)
        return m

    def plugin_names(self, mask: int) -> frozenset[str]:
        return frozenset(n for n, b in self._plugin_bit.items() if mask & b)

    # ---- pod table -----------------------------------------------------------
    @staticmethod
    def key_of(name: str, namespace: str = "") -> str:
        return f"{name}_{namespace}"     # keyFunc, queue.go:152-154

    def _intern(self, keys: Sequence[str], names: Sequence[str], objs: Sequence[Any],
                digit: np.ndarray, tol: np.ndarray) -> np.ndarray:
        ids = np.empty(len(keys), np.int64)
        now = self.clock()
        for j, k in enumerate(keys):
            i = self._key_to_id.get(k)
            if i is None:
                i = self._key_to_id[k] = len(self.keys)
                self.keys.append(k)
                self.names.append(names[j])
                self.objs.append(objs[j])
            else:                            # re-Add: the newest object wins
                self.names[i] = names[j]
                self.objs[i] = objs[j]
            ids[j] = i
        n = len(self.keys)
        for col in (self._digit, self._tol, self._ts, self._t0, self._attempts, self._plugins,
                    self._in_unsched, self._unsched_seq):
            col.ensure(n)
        self._digit.a[ids] = digit
        self._tol.a[ids] = tol
        # newQueuedPodInfo (queue.go:156-165) for the fresh activeQ entry. A pod that also sits in
        # unschedulableQ keeps that entry's UnschedulablePlugins and Timestamp: upstream Add appends
        # a NEW QueuedPodInfo and leaves the map entry (and what MoveAll / backoff read) alone.
        fresh = ids[~self._in_unsched.a[ids].astype(bool)]
        self._ts.a[fresh] = now
        self._t0.a[fresh] = now
        self._attempts.a[fresh] = 0
        self._plugins.a[fresh] = 0
        return ids

    def _push_active(self, ids: np.ndarray) -> None:
        if len(ids):
            self._active.append(np.asarray(ids, np.int64))
            self._active_len += len(ids)

    # ---- reference API -------------------------------------------------------
    def add(self, pod: Any) -> int:
        """queue.go:35-43 for one pod object (anything snapshot.pod_name understands)."""
        return int(self.add_many([pod])[0])

    def add_many(self, pods: Iterable[Any]) -> np.ndarray:
        """Add for a list of pod objects, packed once (one msh_pack_pods call)."""
        pods = list(pods)
        fields = pod_fields(pods)
        table = pack_pods(pods, fields)
        keys = [f"{n}_{ns}" for n, ns in zip(fields[0], fields[1])]  # keyFunc, queue.go:152-154
        ids = self._intern(keys, table.names, pods, table.digit, table.tolerates)
        self._push_active(ids)
        return ids

    def add_soa(self, names: Sequence[str], digit: np.ndarray, tolerates: np.ndarray,
                namespace: str = "") -> np.ndarray:
        """Add for already-packed pods (bench / bulk ingestion): digit int8, tolerates uint8."""
        digit = np.ascontiguousarray(digit, np.int8)
        tolerates = np.ascontiguousarray(tolerates, np.uint8)
        if not (len(names) == len(digit) == len(tolerates)):
            raise ValueError("names / digit / tolerates length mismatch")
        keys = [self.key_of(n, namespace) for n in names]
        ids = self._intern(keys, list(names), [None] * len(names), digit, tolerates)
        self._push_active(ids)
        return ids

    def next_pod(self) -> Any | None:
        """NextPod (queue.go:84-92) without the busy-wait: None when activeQ is empty."""
        b = self.next_batch(1)
        if not len(b):
            return None
        i = int(b.ids[0])
        return self.objs[i] if self.objs[i] is not None else self.names[i]

    def next_batch(self, max_pods: int) -> PodBatch:
        """Pop up to `max_pods` pods from the head of activeQ, in FIFO order."""
        if max_pods < 0:
            raise ValueError("max_pods < 0")
        take: list[np.ndarray] = []
        need = min(max_pods, self._active_len)
        while need > 0:
            chunk = self._active[0]
            avail = len(chunk) - self._active_head
            k = min(avail, need)
            take.append(chunk[self._active_head:self._active_head + k])
            need -= k
            self._active_len -= k
            if k == avail:
                self._active.pop(0)
                self._active_head = 0
            else:
                self._active_head += k
        ids = np.concatenate(take) if take else np.empty(0, np.int64)
        return PodBatch(ids, [self.names[i] for i in ids], self._digit.a[ids].copy(),
                        self._tol.a[ids].copy())

    def add_unschedulable(self, ids: np.ndarray | Sequence[int] | int,
                          unschedulable_plugins: Iterable[str] | np.ndarray | int | None = None) -> None:
        """AddUnschedulable (queue.go:95-107) for one pod id or many. The plugin set is either
        one set for all (names or a mask) or a per-pod uint64 mask array."""
        ids = np.atleast_1d(np.asarray(ids, np.int64))
        if isinstance(unschedulable_plugins, np.ndarray):
            masks = np.asarray(unschedulable_plugins, np.uint64)
            if masks.shape != ids.shape:
                raise ValueError("per-pod plugin masks must match ids")
        elif isinstance(unschedulable_plugins, (int, np.integer)):
            masks = np.uint64(unschedulable_plugins)
        else:
            masks = np.uint64(self.plugins_mask(unschedulable_plugins))
        self._plugins.a[ids] = masks
        self._ts.a[ids] = self.clock()         # "Refresh the timestamp"
        self._in_unsched.a[ids] = True
        n = len(ids)
        self._unsched_seq.a[ids] = np.arange(self._seq, self._seq + n)
        self._seq += n

    def _matches(self, masks: np.ndarray, event: ClusterEvent) -> np.ndarray:
        """podMatchesEvent (queue.go:167-190) over many pods."""
        if event.is_wildcard():
            return np.ones(len(masks), bool)
        hit = np.zeros(len(masks), bool)
        for evt, names in self.cluster_event_map.items():
            if evt.is_wildcard() or (evt.resource == event.resource and (evt.action & event.action) != 0):
                hit |= (masks & np.uint64(self.plugins_mask(names))) != 0
        return hit

    def move_all_to_active_or_backoff_queue(self, event: ClusterEvent) -> int:
        """queue.go:54-81. Returns how many pods left unschedulableQ."""
        ids = np.nonzero(self._in_unsched.a[:len(self.keys)])[0]
        if not len(ids):
            return 0
        ids = ids[np.argsort(self._unsched_seq.a[ids], kind="stable")]
        masks = self._plugins.a[ids]
        move = (masks == 0) | self._matches(masks, event)
        ids = ids[move]
        backoff_s = np.array([calculate_backoff_duration(int(a)) for a in self._attempts.a[ids]])
        backing_off = self._ts.a[ids] + backoff_s > self.clock()
        self._backoff.extend(int(i) for i in ids[backing_off])
        self._push_active(ids[~backing_off])
        self._in_unsched.a[ids] = False
        return len(ids)

    def flush_backoff_completed(self) -> int:
        """Extension: what flushBackoffQCompleted (queue.go:136-140, unimplemented in the
        reference) describes. Moves pods whose backoff expired from podBackoffQ to activeQ."""
        if not self._backoff:
            return 0
        now = self.clock()
        done, keep = [], []
        for i in self._backoff:
            t = self._ts.a[i] + calculate_backoff_duration(int(self._attempts.a[i]))
            (keep if t > now else done).append(i)
        self._backoff = keep
        self._push_active(np.array(done, np.int64))
        return len(done)

    def update(self, old_pod: Any, new_pod: Any) -> None:
        raise NotImplementedError("SchedulingQueue.Update is not implemented in the reference (queue.go:109-113)")

    def delete(self, pod: Any) -> None:
        raise NotImplementedError("SchedulingQueue.Delete is not implemented in the reference (queue.go:115-119)")

    # ---- introspection -------------------------------------------------------
    def active_len(self) -> int:
        return self._active_len

    def backoff_ids(self) -> list[int]:
        return list(self._backoff)

    def unschedulable_ids(self) -> np.ndarray:
        ids = np.nonzero(self._in_unsched.a[:len(self.keys)])[0]
        return ids[np.argsort(self._unsched_seq.a[ids], kind="stable")]

    def unschedulable_plugins(self, pod_id: int) -> frozenset[str]:
        return self.plugin_names(int(self._plugins.a[pod_id]))

    def timestamp(self, pod_id: int) -> float:
        return float(self._ts.a[pod_id])

    def id_of(self, name: str, namespace: str = "") -> int:
        return self._key_to_id[self.key_of(name, namespace)]

