"""mini-kube-scheduler_amd — MI355X (gfx950) batched scheduling core for mini-kube-scheduler.

The reference's per-pod filter -> prescore -> score -> selectHost loop
(minisched/minisched.go:32-87) runs here as a batched pods x nodes evaluation in
hand-written HIP kernels behind the C-ABI in include/minisched_hip.h (libminisched_hip.so).

Import with `importlib.import_module("mini-kube-scheduler_amd")` (the directory name is not
a Python identifier).
"""
from . import _native
from ._native import MshError, device_count
from .framework import (MAX_NODE_SCORE, NODE_NUMBER, NODE_UNSCHEDULABLE, SCORE_COLUMNS, Code, NodeScore, Normalize,
                        Outcome, ScheduleResult)
from .scheduler import DeviceContext, DeviceGroup, Scheduler, ScorePluginConfig, pinned_empty
from .snapshot import NodeTable, PodTable, pack_nodes, pack_pods
from .queue import (ActionType, ClusterEvent, PodBatch, SchedulingQueue, calculate_backoff_duration,
                    events_to_register)
from .nodecache import NodeCache
from .binder import PermitBinder
from .loop import CycleReport, SchedulingLoop
from .resultstore import ResultStore

__all__ = [
    "MAX_NODE_SCORE", "NODE_NUMBER", "NODE_UNSCHEDULABLE", "Code", "NodeScore", "Normalize", "Outcome",
    "ScheduleResult", "DeviceContext", "DeviceGroup", "Scheduler", "ScorePluginConfig", "pinned_empty", "NodeTable", "PodTable",
    "pack_nodes", "pack_pods", "MshError", "device_count", "_native",
    "ActionType", "ClusterEvent", "PodBatch", "SchedulingQueue", "calculate_backoff_duration",
    "events_to_register", "NodeCache", "PermitBinder", "CycleReport", "SchedulingLoop",
    "ResultStore",
]
