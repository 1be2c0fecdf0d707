"""Host-side mirrors of the upstream framework types the hot path exchanges.

Reference: k8s.io/kubernetes@v1.22.0 pkg/scheduler/framework (interface.go, types.go,
cycle_state.go) as used by minisched/minisched.go:37,118-199,283-298. Only what the batched
path needs to report results the way the reference does is restated here: status codes,
the scored node, and the FitError diagnosis routed by ErrorFunc.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field

MAX_NODE_SCORE = 100  # framework.MaxNodeScore

# Plugin names (framework.Plugin.Name()) the device path implements.
NODE_UNSCHEDULABLE = "NodeUnschedulable"  # upstream nodeunschedulable.Name
NODE_NUMBER = "NodeNumber"                # minisched/plugins/score/nodenumber/nodenumber.go:31
# Score-column plugins (build extension, generic pipeline): Score(pod, node) = a per-node int64 the
# host computed (DeviceContext.upload_score_column); names "ScoreColumn0" .. "ScoreColumn3"
SCORE_COLUMNS = tuple(f"ScoreColumn{k}" for k in range(4))

# The taint NodeUnschedulable.Filter tolerates against (upstream v1.22.0).
TAINT_NODE_UNSCHEDULABLE = "node.kubernetes.io/unschedulable"
TAINT_EFFECT_NO_SCHEDULE = "NoSchedule"


class Code(enum.IntEnum):
    """framework.Code (interface.go, v1.22.0)."""
    Success = 0
    Error = 1
    Unschedulable = 2
    UnschedulableAndUnresolvable = 3
    Wait = 4
    Skip = 5


class Outcome(enum.IntEnum):
    """Per-pod outcome of one scheduling cycle's selection part (minisched.go:50-87)."""
    PLACED = 0       # selectHost returned a node
    FIT_ERROR = 1    # RunFilterPlugins -> *framework.FitError
    SCORE_ERROR = 2  # RunScorePlugins returned a non-success status


class Normalize(enum.IntEnum):
    """Per-score-plugin NormalizeScore stage (NONE == reference NodeNumber)."""
    NONE = 0
    DEFAULT = 1          # helper.DefaultNormalizeScore(MaxNodeScore, false, ...)
    DEFAULT_REVERSE = 2  # helper.DefaultNormalizeScore(MaxNodeScore, true, ...)
    MINMAX = 3           # build extension


@dataclass(frozen=True)
class NodeScore:
    """framework.NodeScore."""
    name: str
    score: int


@dataclass
class ScheduleResult:
    """What scheduleOne's selection part produces for one pod.

    PLACED: `node_name`/`node_index`/`score` are set (the name handed to Permit/Bind,
    minisched.go:89-112). FIT_ERROR: `unschedulable_plugins` is the FitError diagnosis
    ErrorFunc copies into QueuedPodInfo.UnschedulablePlugins (minisched.go:287-289).
    SCORE_ERROR: ErrorFunc is called with the filter's nil error, so the plugin set is
    empty (minisched.go:70-75).
    """
    pod: str
    outcome: Outcome
    node_name: str | None = None
    node_index: int = -1
    score: int = 0
    unschedulable_plugins: frozenset[str] = field(default_factory=frozenset)

    @property
    def placed(self) -> bool:
        return self.outcome == Outcome.PLACED
