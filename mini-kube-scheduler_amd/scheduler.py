"""Host-side mirror of minisched.Scheduler's selection path, driving the gfx950 device path.

Reference (shopetan/mini-kube-scheduler, Go):
  Scheduler struct + plugin lists   minisched/initialize.go:18-29, :80-123
  scheduleOne (selection part)      minisched/minisched.go:32-87
  RunFilterPlugins / RunPreScorePlugins / RunScorePlugins / selectHost
                                    minisched/minisched.go:115-199, :304-325
  ErrorFunc routing                 minisched/minisched.go:283-298

`DeviceContext` wraps one msh_ctx (one GPU). `Scheduler` keeps the reference's plugin
configuration by plugin *name* (framework.Plugin.Name()), maps the names the device path
implements to device ids, and schedules a whole batch of pods in one call. Unknown plugin
names raise MshError(MSH_ERR_UNSUPPORTED): there is no silent host fallback.
"""
from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass
from typing import Any, Callable, Iterable, Sequence

import numpy as np

from . import _native as N
from .framework import (NODE_NUMBER, NODE_UNSCHEDULABLE, SCORE_COLUMNS, Normalize, Outcome, ScheduleResult)
from .snapshot import NodeTable, PodTable, pack_nodes, pack_pods

FILTER_IDS = {NODE_UNSCHEDULABLE: N.MSH_PLUGIN_NODE_UNSCHEDULABLE}
SCORE_IDS = {NODE_NUMBER: N.MSH_PLUGIN_NODE_NUMBER,
             **{name: N.MSH_PLUGIN_SCORE_COLUMN0 + k for k, name in enumerate(SCORE_COLUMNS)}}
# Only NodeNumber implements PreScore (nodenumber.go:50-64); a score column has none, so naming one in
# the prescore list is MSH_ERR_UNSUPPORTED here exactly as in msh_set_plugins_ex.
PRESCORE_IDS = {NODE_NUMBER: N.MSH_PLUGIN_NODE_NUMBER}


@dataclass(frozen=True)
class ScorePluginConfig:
    name: str
    weight: int = 1
    normalize: Normalize = Normalize.NONE


def pinned_empty(shape, dtype) -> np.ndarray:
    """A numpy array over page-locked host memory (msh_host_alloc): pod columns and outputs in
    such arrays take the zero-copy path of msh_schedule_batch / msh_schedule_sequential. The
    memory is freed (msh_host_free) when the array and every view of it are gone."""
    dt = np.dtype(dtype)
    nbytes = max(int(np.prod(shape, dtype=np.int64)) * dt.itemsize, 1)
    lib = N.lib()
    ptr = C.c_void_p()
    N.check(lib.msh_host_alloc(nbytes, C.byref(ptr)))
    raw = (C.c_uint8 * nbytes).from_address(ptr.value)
    weakref.finalize(raw, lib.msh_host_free, ptr)
    return np.frombuffer(raw, np.uint8, count=int(np.prod(shape, dtype=np.int64)) * dt.itemsize).view(dt).reshape(shape)


def _same_len(what: str, *arrays) -> int:
    n = len(arrays[0])
    if any(len(a) != n for a in arrays[1:]):
        raise ValueError(f"{what}: column length mismatch {[len(a) for a in arrays]}")
    return n


def _ids(names: Sequence[str], table: dict, what: str) -> np.ndarray:
    out = []
    for n in names:
        if n not in table:
            raise N.MshError(N.MSH_ERR_UNSUPPORTED, f"{what} plugin {n!r} has no device implementation")
        out.append(table[n])
    return np.array(out, np.int32)


class DeviceContext:
    """One msh_ctx bound to one HIP device.

    `options` (tests and A/B measurement only): msh_options overrides for msh_create_ex, e.g.
    {"batch_kernel": "generic", "seq_waves": 16, "seq_split": "serial"} (names in _native.OPTION_NAMES,
    ints as they are; a value outside a field's set is MSH_ERR_INVALID from the library)."""

    def __init__(self, device: int = 0, options: dict | None = None):
        self._lib = N.lib()
        self._fast = N.fast()
        h = C.c_void_p()
        opts = N.make_options(options)
        if opts is None:
            rc = self._lib.msh_create(device, C.byref(h))
        else:
            rc = self._lib.msh_create_ex(device, C.byref(opts), C.byref(h))
        if rc != N.MSH_OK:
            raw = self._lib.msh_last_error(None)
            raise N.MshError(rc, raw.decode() if raw else "")
        self.handle = h
        self.device = device
        self.n_nodes = 0

    # -- lifecycle --
    def close(self) -> None:
        if self.handle:
            self._lib.msh_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int) -> None:
        N.check(rc, self.handle)

    def _hv(self):
        """The ctx handle as an int for the fast-call module (None once closed: MSH_ERR_INVALID)."""
        return self.handle.value if self.handle else None

    # -- configuration --
    def set_plugins(self, filters: Sequence[str], prescore: Sequence[str],
                    score: Sequence[ScorePluginConfig]) -> None:
        f = _ids(filters, FILTER_IDS, "filter")
        pre = _ids(prescore, PRESCORE_IDS, "prescore")
        s = _ids([c.name for c in score], SCORE_IDS, "score")
        w = np.array([int(c.weight) for c in score], np.int64)
        nm = np.array([int(c.normalize) for c in score], np.int32)
        self._check(self._lib.msh_set_plugins_ex(self.handle, N.ptr(f), len(f), N.ptr(pre), len(pre),
                                                 N.ptr(s), N.ptr(w), N.ptr(nm), len(s)))

    def upload_nodes(self, unsched: np.ndarray, digit: np.ndarray) -> None:
        unsched = np.ascontiguousarray(unsched, np.uint8)
        digit = np.ascontiguousarray(digit, np.int8)
        n = _same_len("upload_nodes", unsched, digit)
        self._check(self._lib.msh_upload_nodes(self.handle, n, N.ptr(unsched), N.ptr(digit)))
        self.n_nodes = len(unsched)

    def upload_score_column(self, name: str, scores: np.ndarray) -> None:
        """msh_upload_score_column: the per-node int64 scores (List order) of score-column plugin
        `name` ("ScoreColumn0".."ScoreColumn3")."""
        if name not in SCORE_COLUMNS:
            raise ValueError(f"{name!r} is not a score-column plugin")
        scores = np.ascontiguousarray(scores, np.int64)
        self._check(self._lib.msh_upload_score_column(self.handle, SCORE_IDS[name], len(scores), N.ptr(scores)))

    def patch_nodes(self, idx: np.ndarray, unsched: np.ndarray, digit: np.ndarray) -> None:
        """In-place update of table entries (List order unchanged): msh_patch_nodes."""
        idx = np.ascontiguousarray(idx, np.int32)
        unsched = np.ascontiguousarray(unsched, np.uint8)
        digit = np.ascontiguousarray(digit, np.int8)
        if not (len(idx) == len(unsched) == len(digit)):
            raise ValueError("idx / unsched / digit length mismatch")
        self._check(self._lib.msh_patch_nodes(self.handle, len(idx), N.ptr(idx), N.ptr(unsched), N.ptr(digit)))

    def export_results(self, pod_digit: np.ndarray, pod_tol: np.ndarray):
        """Per-pair plugin results [p, n]: (filter uint8, raw score int64, final score int64);
        scores are N.MSH_EXPORT_NONE where none is recorded (msh_export_results)."""
        pod_digit = np.ascontiguousarray(pod_digit, np.int8)
        pod_tol = np.ascontiguousarray(pod_tol, np.uint8)
        p, n = _same_len("export_results", pod_digit, pod_tol), int(self.n_nodes)
        filt = np.empty((p, n), np.uint8)
        raw = np.empty((p, n), np.int64)
        fin = np.empty((p, n), np.int64)
        self._check(self._lib.msh_export_results(self.handle, p, N.ptr(pod_digit), N.ptr(pod_tol),
                                                 N.ptr(filt), N.ptr(raw), N.ptr(fin)))
        return filt, raw, fin

    # -- host-buffer entry points --
    @staticmethod
    def _outputs(p: int, out, scores: bool = True):
        if out is None:
            return np.empty(p, np.int32), (np.empty(p, np.int64) if scores else None), np.empty(p, np.int32)
        idx, score, status = out
        if not scores:
            score = None
        for a, dt in ((idx, np.int32), (score, np.int64), (status, np.int32)):
            if a is None and dt is np.int64:
                continue
            if a.dtype != dt or len(a) < p or not a.flags["C_CONTIGUOUS"]:
                raise ValueError("out: (int32 idx, int64 score or None, int32 status), C-contiguous, >= p entries")
        return idx, score, status

    def schedule_batch(self, pod_digit: np.ndarray, pod_tol: np.ndarray, out=None, scores: bool = True):
        """msh_schedule_batch. `out` = (idx, score, status) arrays to fill (e.g. pinned_empty ones:
        with page-locked columns and outputs the call copies nothing on the host). scores=False
        (or out with score None): scores are not written and (idx, None, status) comes back."""
        pod_digit = np.ascontiguousarray(pod_digit, np.int8)
        pod_tol = np.ascontiguousarray(pod_tol, np.uint8)
        p = _same_len("schedule_batch", pod_digit, pod_tol)
        idx, score, status = self._outputs(p, out, scores)
        rc = self._fast.schedule_batch_host(self._hv(), pod_digit, pod_tol, idx, score, status)
        if rc:
            self._check(rc)
        return idx, score, status

    def schedule_batch_async(self, pod_digit: np.ndarray, pod_tol: np.ndarray, out, scores: bool = True) -> int:
        """msh_schedule_batch_async: page-locked columns and outputs (pinned_empty arrays) only; returns
        the ticket. The outputs are valid after wait(ticket); keep every array alive and untouched
        until then."""
        p = _same_len("schedule_batch_async", pod_digit, pod_tol)
        idx, score, status = self._outputs(p, out, scores)
        rc, ticket = self._fast.schedule_batch_host_async(self._hv(), pod_digit, pod_tol, idx, score, status)
        if rc:
            self._check(rc)
        return ticket

    def wait(self, ticket: int) -> None:
        """msh_wait: batch `ticket` of schedule_batch_async (and every earlier one) has completed."""
        rc = self._fast.wait(self._hv(), int(ticket))
        if rc:
            self._check(rc)

    def timing_begin(self, max_launches: int) -> None:
        """msh_timing_begin: the next hot-kernel launches of this ctx (from this thread) record their
        own start / stop (the kernel-trace interval)."""
        self._check(self._lib.msh_timing_begin(self.handle, int(max_launches)))

    def timing_end(self) -> tuple[int, float, float]:
        """msh_timing_end: (launches timed, summed ms, longest ms)."""
        n, tot, mx = C.c_int32(), C.c_double(), C.c_double()
        self._check(self._lib.msh_timing_end(self.handle, C.byref(n), C.byref(tot), C.byref(mx)))
        return n.value, tot.value, mx.value

    def schedule_sequential(self, pod_digit: np.ndarray, pod_tol: np.ndarray, max_pods_per_node: int = 0,
                            on_commit: Callable[[int, int, int], None] | None = None, out=None):
        pod_digit = np.ascontiguousarray(pod_digit, np.int8)
        pod_tol = np.ascontiguousarray(pod_tol, np.uint8)
        p = _same_len("schedule_sequential", pod_digit, pod_tol)
        idx, score, status = self._outputs(p, out)
        cb = N.COMMIT_CB(lambda _u, j, i, s: on_commit(j, i, s)) if on_commit else N.COMMIT_CB()
        self._check(self._lib.msh_schedule_sequential(self.handle, p, N.ptr(pod_digit), N.ptr(pod_tol),
                                                      int(max_pods_per_node), N.ptr(idx), N.ptr(score),
                                                      N.ptr(status), cb, None))
        return idx, score, status

    def node_pod_counts(self) -> np.ndarray:
        out = np.zeros(self.n_nodes, np.int32)
        self._check(self._lib.msh_node_pod_counts(self.handle, N.ptr(out) if self.n_nodes else None))
        return out

    def reset_node_pod_counts(self) -> None:
        self._check(self._lib.msh_reset_node_pod_counts(self.handle))

    # -- device-resident entry points (integer device addresses, hipStream_t as int) --
    # The per-batch device entry points go through the CPython fast-call module (csrc/msh_pyfast.c):
    # ctypes argument conversion cost ~0.9 us per call next to a ~2.6 us launch.
    def schedule_batch_device(self, p: int, d_pod_digit: int, d_pod_tol: int, d_idx: int, d_score: int,
                              d_status: int, stream: int = 0) -> None:
        rc = self._fast.schedule_batch_device(self._hv(), p, d_pod_digit, d_pod_tol, d_idx, d_score,
                                              d_status, stream or None)
        if rc:
            self._check(rc)

    @staticmethod
    def batch_descs(batches: Sequence[tuple]) -> "C.Array":
        """An msh_batch array for schedule_batches_device from (p, d_pod_digit, d_pod_tol, d_idx,
        d_score or 0, d_status) tuples of device addresses; build it once and reuse it."""
        arr = (N.Batch * len(batches))()
        for i, (p, pd, pt, oi, os_, ost) in enumerate(batches):
            arr[i] = N.Batch(int(p), 0, pd, pt, oi, os_ or None, ost)
        return arr

    def schedule_batches_device(self, descs, nb: int | None = None, stream: int = 0) -> None:
        """msh_schedule_batches_device over an msh_batch array (batch_descs): up to
        N.BATCHES_PER_LAUNCH batches per kernel launch, asynchronous on `stream`."""
        nb = len(descs) if nb is None else nb
        rc = self._fast.schedule_batches_device(self._hv(), nb, C.addressof(descs), stream or None)
        if rc:
            self._check(rc)

    def schedule_sequential_device(self, p: int, d_pod_digit: int, d_pod_tol: int, max_pods_per_node: int,
                                   d_idx: int, d_score: int, d_status: int, stream: int = 0) -> None:
        rc = self._fast.schedule_sequential_device(self._hv(), p, d_pod_digit, d_pod_tol,
                                                   int(max_pods_per_node), d_idx, d_score, d_status, stream or None)
        if rc:
            self._check(rc)

    def shard_keys_len(self, p: int) -> int:
        """int32 entries msh_shard_keys_device writes for p pods: 2p (ABI v7)."""
        v = C.c_int32(0)
        self._check(self._lib.msh_shard_keys_len(self.handle, int(p), C.byref(v)))
        return int(v.value)

    def shard_keys_device(self, p: int, d_pod_digit: int, d_pod_tol: int, node_base: int, d_keys: int,
                          stream: int = 0) -> None:
        rc = self._fast.shard_keys_device(self._hv(), p, d_pod_digit, d_pod_tol, int(node_base), d_keys,
                                          stream or None)
        if rc:
            self._check(rc)

    def decode_keys_device(self, p: int, d_pod_digit: int, d_pod_tol: int, d_keys: int, d_idx: int,
                           d_score: int, d_status: int, stream: int = 0) -> None:
        rc = self._fast.decode_keys_device(self._hv(), p, d_pod_digit, d_pod_tol, d_keys, d_idx, d_score, d_status,
                                           stream or None)
        if rc:
            self._check(rc)

    def keys_slot1_is_any(self) -> bool:
        v = C.c_int32(0)
        self._check(self._lib.msh_keys_slot1_is_any(self.handle, C.byref(v)))
        return bool(v.value)

    # -- node-sharded scheduling with the merge in the library (ABI v8: RCCL communicator) --
    @staticmethod
    def comm_unique_id() -> bytes:
        """msh_comm_unique_id: the MSH_COMM_ID_BYTES id rank 0 makes and ships to every rank."""
        buf = (C.c_uint8 * N.COMM_ID_BYTES)()
        N.check(N.lib().msh_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, comm_id: bytes, world: int, rank: int) -> None:
        """msh_comm_init (collective over the `world` ranks)."""
        if len(comm_id) != N.COMM_ID_BYTES:
            raise ValueError(f"a comm id is {N.COMM_ID_BYTES} bytes")
        buf = (C.c_uint8 * N.COMM_ID_BYTES).from_buffer_copy(comm_id)
        self._check(self._lib.msh_comm_init(self.handle, buf, int(world), int(rank)))

    def comm_info(self) -> tuple[int, int]:
        w, r = C.c_int32(), C.c_int32()
        self._check(self._lib.msh_comm_info(self.handle, C.byref(w), C.byref(r)))
        return w.value, r.value

    def schedule_nodeshard_device(self, p: int, d_pod_digit: int, d_pod_tol: int, node_base: int, d_idx: int,
                                  d_score: int, d_status: int, stream: int = 0) -> None:
        """msh_schedule_nodeshard_device: shard kernel, all-reduce(s) over the communicator, decode, on
        `stream`; every rank ends with the global decisions."""
        rc = self._fast.schedule_nodeshard_device(self._hv(), p, d_pod_digit, d_pod_tol, int(node_base), d_idx,
                                                  d_score, d_status, stream or None)
        if rc:
            self._check(rc)

    def schedule_nodeshard(self, pod_digit: np.ndarray, pod_tol: np.ndarray, node_base: int, out=None):
        """msh_schedule_nodeshard: the host-buffer form (synchronous)."""
        pod_digit = np.ascontiguousarray(pod_digit, np.int8)
        pod_tol = np.ascontiguousarray(pod_tol, np.uint8)
        p = _same_len("schedule_nodeshard", pod_digit, pod_tol)
        idx, score, status = self._outputs(p, out)
        self._check(self._lib.msh_schedule_nodeshard(self.handle, p, N.ptr(pod_digit), N.ptr(pod_tol), int(node_base),
                                                     N.ptr(idx), N.ptr(score), N.ptr(status)))
        return idx, score, status

    # -- node-sharded generic pipeline (msh_generic_*: any plugin list, score columns included) --
    def generic_ext_len(self, p: int) -> int:
        """int64 entries of the per-pod extents msh_generic_extents_device writes (0: no plugin
        normalizes, nothing to merge before the bests)."""
        v = C.c_int64(0)
        self._check(self._lib.msh_generic_ext_len(self.handle, int(p), C.byref(v)))
        return int(v.value)

    def generic_extents_device(self, p: int, d_pod_digit: int, d_pod_tol: int, d_ext: int, stream: int = 0) -> None:
        self._check(self._lib.msh_generic_extents_device(self.handle, int(p), d_pod_digit, d_pod_tol, d_ext,
                                                         stream or None))

    def generic_best_device(self, p: int, d_pod_digit: int, d_pod_tol: int, d_ext: int, node_base: int,
                            d_best_total: int, d_best_idx: int, stream: int = 0) -> None:
        self._check(self._lib.msh_generic_best_device(self.handle, int(p), d_pod_digit, d_pod_tol, d_ext or None,
                                                      int(node_base), d_best_total, d_best_idx, stream or None))

    def generic_candidates_device(self, p: int, d_local_total: int, d_merged_total: int, d_best_idx: int,
                                  stream: int = 0) -> None:
        self._check(self._lib.msh_generic_candidates_device(self.handle, int(p), d_local_total, d_merged_total,
                                                            d_best_idx, stream or None))

    def generic_decode_device(self, p: int, d_pod_digit: int, d_merged_total: int, d_merged_idx: int, d_idx: int,
                              d_score: int, d_status: int, stream: int = 0) -> None:
        self._check(self._lib.msh_generic_decode_device(self.handle, int(p), d_pod_digit, d_merged_total,
                                                        d_merged_idx, d_idx, d_score or None, d_status,
                                                        stream or None))


class DeviceGroup:
    """msh_group: shard ctxs in List order (ctxs[k] holds the k-th contiguous slice of the node table), any
    devices; the merge runs on ctxs[0]'s device. The ctxs stay owned by the caller: close the group first."""

    def __init__(self, ctxs: Sequence[DeviceContext]):
        self._lib = N.lib()
        self.ctxs = list(ctxs)
        arr = (C.c_void_p * len(self.ctxs))(*[c.handle for c in self.ctxs])
        h = C.c_void_p()
        rc = self._lib.msh_group_create(arr, len(self.ctxs), C.byref(h))
        if rc != N.MSH_OK:
            raw = self._lib.msh_group_last_error(None)
            raise N.MshError(rc, raw.decode() if raw else "")
        self.handle = h

    def close(self) -> None:
        if self.handle:
            self._lib.msh_group_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def schedule_batch(self, pod_digit: np.ndarray, pod_tol: np.ndarray, scores: bool = True):
        """msh_group_schedule_batch: the decisions over the whole (sharded) table."""
        pod_digit = np.ascontiguousarray(pod_digit, np.int8)
        pod_tol = np.ascontiguousarray(pod_tol, np.uint8)
        p = _same_len("group schedule_batch", pod_digit, pod_tol)
        idx, score, status = np.empty(p, np.int32), (np.empty(p, np.int64) if scores else None), np.empty(p, np.int32)
        rc = self._lib.msh_group_schedule_batch(self.handle, p, N.ptr(pod_digit), N.ptr(pod_tol), N.ptr(idx),
                                                N.ptr(score), N.ptr(status))
        if rc != N.MSH_OK:
            raw = self._lib.msh_group_last_error(self.handle)
            raise N.MshError(rc, raw.decode() if raw else "")
        return idx, score, status


class Scheduler:
    """Batched mirror of minisched.Scheduler (initialize.go:18-29).

    Defaults are the reference's hardcoded plugin lists (initialize.go:80-123):
    filter=[NodeUnschedulable], preScore=[NodeNumber], score=[NodeNumber] (weight 1,
    no NormalizeScore: nodenumber.go:98-100).
    """

    def __init__(self, filter_plugins: Sequence[str] = (NODE_UNSCHEDULABLE,),
                 pre_score_plugins: Sequence[str] = (NODE_NUMBER,),
                 score_plugins: Sequence[ScorePluginConfig | str] = (NODE_NUMBER,),
                 device: int = 0, ctx: DeviceContext | None = None):
        self.filter_plugins = list(filter_plugins)
        self.pre_score_plugins = list(pre_score_plugins)
        self.score_plugins = [c if isinstance(c, ScorePluginConfig) else ScorePluginConfig(c)
                              for c in score_plugins]
        self.ctx = ctx or DeviceContext(device)
        self.ctx.set_plugins(self.filter_plugins, self.pre_score_plugins, self.score_plugins)
        self.nodes: NodeTable | None = None

    def close(self) -> None:
        self.ctx.close()

    # Replaces the per-cycle Nodes().List (minisched.go:40) with one device upload.
    def update_nodes(self, nodes: Iterable[Any]) -> NodeTable:
        self.nodes = pack_nodes(nodes)
        self.ctx.upload_nodes(self.nodes.unsched, self.nodes.digit)
        return self.nodes

    def _results(self, pods: PodTable, idx, score, status) -> list[ScheduleResult]:
        assert self.nodes is not None
        n_nodes = len(self.nodes)
        fit_plugins = frozenset(
            # FitError diagnosis: the filter plugins that rejected at least one node. With the
            # device plugin set that is NodeUnschedulable whenever any node exists.
            [self.filter_plugins[0]] if (self.filter_plugins and n_nodes > 0) else [])
        out = []
        for j, name in enumerate(pods.names):
            st = int(status[j])
            if st == N.MSH_PLACED:
                i = int(idx[j])
                out.append(ScheduleResult(name, Outcome.PLACED, self.nodes.names[i], i, int(score[j])))
            elif st == N.MSH_FIT_ERROR:
                out.append(ScheduleResult(name, Outcome.FIT_ERROR, unschedulable_plugins=fit_plugins))
            else:
                out.append(ScheduleResult(name, Outcome.SCORE_ERROR))
        return out

    def schedule_batch(self, pods: Iterable[Any], nodes: Iterable[Any] | None = None) -> list[ScheduleResult]:
        """scheduleOne's selection part for every pod of the batch against one snapshot."""
        if nodes is not None:
            self.update_nodes(nodes)
        if self.nodes is None:
            raise N.MshError(N.MSH_ERR_STATE, "no node snapshot: call update_nodes() first")
        table = pack_pods(pods)
        idx, score, status = self.ctx.schedule_batch(table.digit, table.tolerates)
        return self._results(table, idx, score, status)

    def schedule_sequential(self, pods: Iterable[Any], nodes: Iterable[Any] | None = None,
                            max_pods_per_node: int = 0) -> list[ScheduleResult]:
        """One pod at a time, committing each placement to node state before the next."""
        if nodes is not None:
            self.update_nodes(nodes)
        if self.nodes is None:
            raise N.MshError(N.MSH_ERR_STATE, "no node snapshot: call update_nodes() first")
        table = pack_pods(pods)
        idx, score, status = self.ctx.schedule_sequential(table.digit, table.tolerates, max_pods_per_node)
        return self._results(table, idx, score, status)
