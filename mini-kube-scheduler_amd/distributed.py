"""Multi-GPU modes of the scheduling core (one process per GPU, torch.distributed over RCCL).

SURVEY.md §8(e). The reference has no distribution at all (one goroutine schedules one pod
at a time, minisched/minisched.go:28-30); the modes below are new:

* Pod sharding (BASELINE C2/C3/C5 at 2/4/8 GPUs). Pods are independent: no plugin reads
  placement-dependent state (NodeInfo is rebuilt per cycle, minisched.go:126; Bind only
  touches the pod, :266-277). Every rank holds the whole node table and schedules its
  contiguous pod range. No data-path collective ("scaling": "weak").

* Node sharding, reference plugins (BASELINE C4: 100k nodes x 1M pods over 8 GPUs). Rank r holds
  the List-order slice [r*N/W, (r+1)*N/W) of the node table and computes int32 keys
  (msh_shard_keys_device), each 0x7FFFFFFF - global_idx, per pod: its first feasible match and its
  first feasible non-match over the slice (ABI v7: both per pod, from the per-pair kernel). Because
  the slices are contiguous and ascending, the element-wise MAX over ranks is the global first
  match / non-match, i.e. exactly the single-GPU inputs of the decode. One RCCL all-reduce(MAX) of
  8 B per pod replaces an all-gather of per-shard bests + merge (same result, ~1/W the bytes per
  link on a ring); msh_decode_keys_device then yields idx / score / status on every rank.

* Node sharding, any plugin list (score-column plugins, any normalizer): GenericNodeShardedScheduler.
  Each rank forms int64 totals per (pod, node) pair of its slice (msh_generic_best_device). A plugin
  that normalizes needs the pod's extent over the feasible nodes of ALL slices first (SURVEY.md §8(e)
  caveat: integer-division normalisation creates ties, so the argmax is not invariant otherwise):
  one all-reduce MAX over the per-pod (max, -min) extents. The bests merge by MAX over the totals,
  then MIN over the global indices of the ranks that hold the maximum (selectHost's first maximum,
  minisched.go:304-325, across ranks).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GKEY_MAX = 0x7FFFFFFF  # int32 key = GKEY_MAX - global node index, 0 = none (include/minisched_hip.h)


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of `total` items for `rank` of `world`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return total * rank // world, total * (rank + 1) // world


def encode_key(global_idx: np.ndarray) -> np.ndarray:
    """Node index (or -1) -> int32 shard key (0 = none)."""
    g = np.asarray(global_idx, np.int64)
    return np.where(g >= 0, GKEY_MAX - g, 0).astype(np.int32)


def decode_key(key: np.ndarray) -> np.ndarray:
    """Shard key -> node index (or -1)."""
    k = np.asarray(key, np.int64)
    return np.where(k > 0, GKEY_MAX - k, -1).astype(np.int64)


def as_torch_stream(stream, device):
    """A torch stream for `stream`: None -> the device's current stream, a torch.cuda.Stream as is,
    an int (a hipStream_t handle, e.g. `Stream.cuda_stream`) wrapped as an ExternalStream."""
    import torch
    if stream is None or (isinstance(stream, int) and stream == 0):
        return torch.cuda.current_stream(device)
    if isinstance(stream, int):
        return torch.cuda.ExternalStream(stream, device=device)
    return stream


def merge_shard_keys_(keys, group=None, stream=None):
    """In-place element-wise MAX of per-shard keys over the process group (RCCL on GPU tensors,
    gloo on CPU or GPU tensors). `keys` is the int32 tensor of msh_shard_keys_len entries.

    For a GPU tensor the collective is issued with `stream` (the stream the keys were produced on and
    the decode will run on; default: the current stream) as torch's current stream, so the process
    group orders it after the keys kernel and the decode after it (ProcessGroupNCCL: its stream waits
    on the current one, and the current one on the collective)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1):
        return keys
    if keys.is_cuda:
        with torch.cuda.stream(as_torch_stream(stream, keys.device)):
            dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=group)
    else:
        dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=group)
    return keys


@dataclass
class NodeShard:
    """This rank's slice of the List-order node table."""
    lo: int
    hi: int

    @property
    def n(self) -> int:
        return self.hi - self.lo


class NodeShardedScheduler:
    """Node-sharded batch scheduling on this rank's GPU (C4 shape).

    `ctx` is a DeviceContext already configured with the plugin set; `unsched` / `digit` are
    the FULL List-order node columns (each rank uploads only its slice)."""

    def __init__(self, ctx, unsched: np.ndarray, digit: np.ndarray, world: int, rank: int, group=None):
        lo, hi = shard_range(len(unsched), world, rank)
        self.shard = NodeShard(lo, hi)
        self.ctx = ctx
        self.group = group
        ctx.upload_nodes(np.ascontiguousarray(unsched[lo:hi]), np.ascontiguousarray(digit[lo:hi]))

    def schedule(self, d_pod_digit, d_pod_tol, d_keys, d_idx, d_score, d_status, stream=None) -> None:
        """All tensors on this rank's GPU (d_keys: int32, >= ctx.shard_keys_len(p) entries);
        every rank ends with the global decisions. `stream`: a torch.cuda.Stream or a hipStream_t
        handle (default: the current stream); the keys kernel, the all-reduce and the decode are
        ordered on it (the cross-shard selectHost, minisched.go:304-325)."""
        p = d_pod_digit.numel()
        klen = self.ctx.shard_keys_len(p)
        s = as_torch_stream(stream, d_keys.device)
        h = s.cuda_stream
        self.ctx.shard_keys_device(p, d_pod_digit.data_ptr(), d_pod_tol.data_ptr(), self.shard.lo,
                                   d_keys.data_ptr(), h)
        merge_shard_keys_(d_keys[:klen], self.group, s)
        self.ctx.decode_keys_device(p, d_pod_digit.data_ptr(), d_pod_tol.data_ptr(), d_keys.data_ptr(),
                                    d_idx.data_ptr(), d_score.data_ptr(), d_status.data_ptr(), h)


class PodShardedScheduler:
    """Pod-sharded batch (or sequential) scheduling: full node table, this rank's pods."""

    def __init__(self, ctx, unsched: np.ndarray, digit: np.ndarray, world: int, rank: int, group=None):
        self.ctx = ctx
        self.world, self.rank, self.group = world, rank, group
        ctx.upload_nodes(unsched, digit)

    def pod_range(self, p_total: int) -> tuple[int, int]:
        return shard_range(p_total, self.world, self.rank)

    def merge_node_counts(self, counts):
        """Sequential mode: the commit state (pods per node) summed over ranks. Exact only when
        no filter reads it (max_pods_per_node == 0), i.e. the reference plugin set."""
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=self.group)
        return counts


def _stream_scope(t, stream):
    """(context manager, hipStream_t handle) for launches on tensor t's device: a CUDA tensor runs on
    `stream` (default: the current stream) made current, so the process group orders its collectives
    there; a CPU tensor (the gloo tests' stand-in context) on no stream."""
    import contextlib
    import torch
    if not t.is_cuda:
        return contextlib.nullcontext(), 0
    s = as_torch_stream(stream, t.device)
    return torch.cuda.stream(s), s.cuda_stream


def _all_reduce(t, op, group):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=op, group=group)
    return t


class GenericNodeShardedScheduler:
    """Node-sharded batch scheduling for ANY plugin list on this rank's GPU (msh_generic_*).

    `ctx` is a DeviceContext already configured with the plugin set; `unsched` / `digit` and the
    score columns (`columns`: {"ScoreColumnK": int64 array}) are the FULL List-order node columns:
    each rank uploads only its slice. One batch is five launches and three collectives (two when no
    plugin normalizes): extents -> all-reduce MAX -> per-shard bests -> all-reduce MAX of the totals
    -> candidates -> all-reduce MIN of the indices -> decode. Every rank ends with the decisions of
    msh_schedule_batch over the whole table."""

    def __init__(self, ctx, unsched: np.ndarray, digit: np.ndarray, world: int, rank: int,
                 columns: dict | None = None, group=None):
        lo, hi = shard_range(len(unsched), world, rank)
        self.shard = NodeShard(lo, hi)
        self.ctx = ctx
        self.group = group
        ctx.upload_nodes(np.ascontiguousarray(unsched[lo:hi]), np.ascontiguousarray(digit[lo:hi]))
        for name, col in (columns or {}).items():
            ctx.upload_score_column(name, np.ascontiguousarray(np.asarray(col, np.int64)[lo:hi]))

    def schedule(self, d_pod_digit, d_pod_tol, d_idx, d_score, d_status, stream=None) -> None:
        """All tensors on this rank's device (int8 digit, uint8 tolerates; int32 idx, int64 score or
        None, int32 status outputs)."""
        import torch
        import torch.distributed as dist
        p = d_pod_digit.numel()
        scope, h = _stream_scope(d_pod_digit, stream)
        dev = d_pod_digit.device
        with scope:
            n_ext = self.ctx.generic_ext_len(p)
            ext = None
            if n_ext:
                ext = torch.empty(n_ext, dtype=torch.int64, device=dev)
                self.ctx.generic_extents_device(p, d_pod_digit.data_ptr(), d_pod_tol.data_ptr(), ext.data_ptr(), h)
                _all_reduce(ext, dist.ReduceOp.MAX, self.group)  # (max, -min) per pod and plugin
            total = torch.empty(p, dtype=torch.int64, device=dev)
            idx = torch.empty(p, dtype=torch.int32, device=dev)
            self.ctx.generic_best_device(p, d_pod_digit.data_ptr(), d_pod_tol.data_ptr(),
                                         ext.data_ptr() if ext is not None else 0, self.shard.lo,
                                         total.data_ptr(), idx.data_ptr(), h)
            merged = total.clone()
            _all_reduce(merged, dist.ReduceOp.MAX, self.group)
            self.ctx.generic_candidates_device(p, total.data_ptr(), merged.data_ptr(), idx.data_ptr(), h)
            _all_reduce(idx, dist.ReduceOp.MIN, self.group)
            self.ctx.generic_decode_device(p, d_pod_digit.data_ptr(), merged.data_ptr(), idx.data_ptr(),
                                           d_idx.data_ptr(), d_score.data_ptr() if d_score is not None else 0,
                                           d_status.data_ptr(), h)
