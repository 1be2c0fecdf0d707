"""ctypes binding of libminisched_hip.so (the C-ABI declared in include/minisched_hip.h).

The product path has no CPU fallback: if the library cannot be loaded, `lib()` raises.
Only plain pointers and sizes cross the boundary (numpy arrays for host buffers, integer
device addresses — e.g. `torch.Tensor.data_ptr()` — for the `_device` entry points).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("MSH_LIBRARY", PKG_DIR / "libminisched_hip.so"))

# ---- mirrors of the header's enums ----
MSH_OK = 0
MSH_ERR_INVALID = -1
MSH_ERR_NO_DEVICE = -2
MSH_ERR_HIP = -3
MSH_ERR_STATE = -4
MSH_ERR_UNSUPPORTED = -5
MSH_ERR_NOMEM = -6
ERR_NAMES = {
    MSH_ERR_INVALID: "MSH_ERR_INVALID",
    MSH_ERR_NO_DEVICE: "MSH_ERR_NO_DEVICE",
    MSH_ERR_HIP: "MSH_ERR_HIP",
    MSH_ERR_STATE: "MSH_ERR_STATE",
    MSH_ERR_UNSUPPORTED: "MSH_ERR_UNSUPPORTED",
    MSH_ERR_NOMEM: "MSH_ERR_NOMEM",
}

MSH_PLACED = 0
MSH_FIT_ERROR = 1
MSH_SCORE_ERROR = 2

MSH_PLUGIN_NODE_UNSCHEDULABLE = 1
MSH_PLUGIN_NODE_NUMBER = 2
MSH_PLUGIN_SCORE_COLUMN0 = 16  # .. 19: score-column plugins (generic pipeline)

MSH_EXPORT_NONE = -(1 << 63)  # msh_export_results: no score recorded

MSH_NORMALIZE_NONE = 0
MSH_NORMALIZE_DEFAULT = 1
MSH_NORMALIZE_DEFAULT_REVERSE = 2
MSH_NORMALIZE_MINMAX = 3

# Every symbol include/minisched_hip.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "msh_abi_version", "msh_device_count", "msh_host_alloc", "msh_host_free", "msh_create", "msh_create_ex",
    "msh_destroy", "msh_last_error",
    "msh_set_plugins", "msh_set_plugins_ex", "msh_upload_nodes", "msh_upload_score_column", "msh_num_nodes",
    "msh_patch_nodes", "msh_export_results",
    "msh_schedule_batch", "msh_schedule_batch_async", "msh_wait", "msh_schedule_batch_device",
    "msh_schedule_batches_device", "msh_schedule_sequential",
    "msh_schedule_sequential_device", "msh_node_pod_counts", "msh_reset_node_pod_counts",
    "msh_shard_keys_len", "msh_shard_keys_device", "msh_decode_keys_device", "msh_keys_slot1_is_any",
    "msh_generic_ext_len", "msh_generic_extents_device", "msh_generic_best_device",
    "msh_generic_candidates_device", "msh_generic_decode_device",
    "msh_comm_unique_id", "msh_comm_init", "msh_comm_info", "msh_schedule_nodeshard_device", "msh_schedule_nodeshard",
    "msh_group_create", "msh_group_destroy", "msh_group_last_error", "msh_group_schedule_batch",
    "msh_timing_begin", "msh_timing_end",
    "msh_pack_nodes", "msh_pack_pods", "msh_toleration_tolerates_unschedulable",
)


class MshError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERR_NAMES.get(code, code)}: {msg}")
        self.code = code


class Toleration(C.Structure):
    """msh_toleration (k8s.io/api core/v1 Toleration subset)."""
    _fields_ = [("key", C.c_char_p), ("op", C.c_char_p), ("value", C.c_char_p), ("effect", C.c_char_p)]


class Batch(C.Structure):
    """msh_batch: one batch of msh_schedule_batches_device (device pointers)."""
    _fields_ = [("p", C.c_int32), ("reserved", C.c_int32), ("pod_digit", C.c_void_p), ("pod_tol", C.c_void_p),
                ("out_idx", C.c_void_p), ("out_score", C.c_void_p), ("out_status", C.c_void_p)]


class Options(C.Structure):
    """msh_options (ABI v8): kernel-selection overrides for msh_create_ex, 0 = automatic."""
    _fields_ = [("struct_size", C.c_int32), ("batch_kernel", C.c_int32), ("pair_planes", C.c_int32),
                ("pair_noax", C.c_int32), ("pair_slices", C.c_int32), ("seq_waves", C.c_int32),
                ("seq_split", C.c_int32), ("seq_pod_waves", C.c_int32), ("gen_keys", C.c_int32),
                ("gen_nnkey", C.c_int32)]


# Named values of the msh_options fields (an int passes through unchanged, for the library to check).
OPTION_NAMES = {
    "batch_kernel": {"auto": 0, "pair": 0, "generic": 1},
    "pair_planes": {"auto": 0, "sgpr": 1, "lds": 2},
    "pair_noax": {"auto": 0, "noax": 1, "axlast": 2},
    "pair_slices": {"auto": 0},
    "seq_waves": {"auto": 0},
    "seq_split": {"auto": 0, "serial": 1, "blocks": 2},
    "seq_pod_waves": {"auto": 0},
    "gen_keys": {"auto": 0, "f53": 0, "u64": 1},
    "gen_nnkey": {"auto": 0, "select": 1},
}


def make_options(opts: dict | None) -> "Options | None":
    """msh_options from {field: value}: a name of OPTION_NAMES[field], or an int (digit strings too)."""
    if not opts:
        return None
    o = Options()
    o.struct_size = C.sizeof(Options)
    for k, v in opts.items():
        if k not in OPTION_NAMES:
            raise ValueError(f"unknown msh_options field {k!r}")
        if isinstance(v, str):
            v = OPTION_NAMES[k][v] if v in OPTION_NAMES[k] else int(v)
        setattr(o, k, int(v))
    return o


COMM_ID_BYTES = 128  # MSH_COMM_ID_BYTES
GROUP_MAX_SHARDS = 16  # MSH_GROUP_MAX_SHARDS
BATCHES_PER_LAUNCH = 32  # MSH_BATCHES_PER_LAUNCH
ASYNC_DEPTH = 4  # MSH_ASYNC_DEPTH

COMMIT_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32, C.c_int64)

_P = C.c_void_p
_I32 = C.c_int32
_I64 = C.c_int64

_SIGS = {
    "msh_abi_version": (C.c_int, []),
    "msh_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "msh_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(_P)]),
    "msh_host_free": (None, [_P]),
    "msh_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "msh_create_ex": (C.c_int, [C.c_int, C.POINTER(Options), C.POINTER(_P)]),
    "msh_destroy": (None, [_P]),
    "msh_last_error": (C.c_char_p, [_P]),
    "msh_set_plugins": (C.c_int, [_P, _P, _I32, _P, _P, _I32]),
    "msh_set_plugins_ex": (C.c_int, [_P, _P, _I32, _P, _I32, _P, _P, _P, _I32]),
    "msh_upload_nodes": (C.c_int, [_P, _I32, _P, _P]),
    "msh_num_nodes": (C.c_int, [_P, C.POINTER(_I32)]),
    "msh_upload_score_column": (C.c_int, [_P, _I32, _I32, _P]),
    "msh_patch_nodes": (C.c_int, [_P, _I32, _P, _P, _P]),
    "msh_export_results": (C.c_int, [_P, _I32, _P, _P, _P, _P, _P]),
    "msh_schedule_batch": (C.c_int, [_P, _I32, _P, _P, _P, _P, _P]),
    "msh_schedule_batch_device": (C.c_int, [_P, _I32, _P, _P, _P, _P, _P, _P]),
    "msh_schedule_batches_device": (C.c_int, [_P, _I32, _P, _P]),
    "msh_schedule_batch_async": (C.c_int, [_P, _I32, _P, _P, _P, _P, _P, C.POINTER(C.c_uint64)]),
    "msh_wait": (C.c_int, [_P, C.c_uint64]),
    "msh_timing_begin": (C.c_int, [_P, _I32]),
    "msh_timing_end": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "msh_schedule_sequential": (C.c_int, [_P, _I32, _P, _P, _I32, _P, _P, _P, COMMIT_CB, _P]),
    "msh_schedule_sequential_device": (C.c_int, [_P, _I32, _P, _P, _I32, _P, _P, _P, _P]),
    "msh_node_pod_counts": (C.c_int, [_P, _P]),
    "msh_reset_node_pod_counts": (C.c_int, [_P]),
    "msh_shard_keys_len": (C.c_int, [_P, _I32, C.POINTER(_I32)]),
    "msh_shard_keys_device": (C.c_int, [_P, _I32, _P, _P, _I64, _P, _P]),
    "msh_decode_keys_device": (C.c_int, [_P, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "msh_keys_slot1_is_any": (C.c_int, [_P, C.POINTER(_I32)]),
    "msh_generic_ext_len": (C.c_int, [_P, _I32, C.POINTER(_I64)]),
    "msh_generic_extents_device": (C.c_int, [_P, _I32, _P, _P, _P, _P]),
    "msh_generic_best_device": (C.c_int, [_P, _I32, _P, _P, _P, _I64, _P, _P, _P]),
    "msh_generic_candidates_device": (C.c_int, [_P, _I32, _P, _P, _P, _P]),
    "msh_generic_decode_device": (C.c_int, [_P, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "msh_comm_unique_id": (C.c_int, [_P]),
    "msh_comm_init": (C.c_int, [_P, _P, _I32, _I32]),
    "msh_comm_info": (C.c_int, [_P, C.POINTER(_I32), C.POINTER(_I32)]),
    "msh_schedule_nodeshard_device": (C.c_int, [_P, _I32, _P, _P, _I64, _P, _P, _P, _P]),
    "msh_schedule_nodeshard": (C.c_int, [_P, _I32, _P, _P, _I64, _P, _P, _P]),
    "msh_group_create": (C.c_int, [C.POINTER(_P), _I32, C.POINTER(_P)]),
    "msh_group_destroy": (None, [_P]),
    "msh_group_last_error": (C.c_char_p, [_P]),
    "msh_group_schedule_batch": (C.c_int, [_P, _I32, _P, _P, _P, _P, _P]),
    "msh_pack_nodes": (C.c_int, [_I32, C.c_char_p, _P, _P, _P, _P, _P]),
    "msh_pack_pods": (C.c_int, [_I32, C.c_char_p, _P, C.POINTER(Toleration), _P, _P, _P]),
    "msh_toleration_tolerates_unschedulable": (C.c_int, [C.POINTER(Toleration)]),
}

_LIB: C.CDLL | None = None
_HIP_RUNTIME: C.CDLL | None = None


def _share_hip_runtime_with_torch() -> None:
    """Make this library and PyTorch share ONE HIP runtime in the process.

    PyTorch-ROCm wheels bundle their own libamdhip64 (SONAME libamdhip64.so.7, the same as
    /opt/rocm's). If libminisched_hip.so were loaded first it would pull in /opt/rocm's copy
    and torch would later load its bundled copy: two runtimes in one process, and torch then
    reports "No HIP GPUs are available". Loading torch's runtime RTLD_GLOBAL first makes our
    NEEDED libamdhip64.so.7 resolve to it (and torch's later load reuse it), so device pointers
    and streams are interchangeable. Without torch installed, /opt/rocm's runtime is used.
    Set MSH_HIP_RUNTIME=system to skip.
    """
    global _HIP_RUNTIME
    if _HIP_RUNTIME is not None or os.environ.get("MSH_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    cand = Path(list(spec.submodule_search_locations)[0]) / "lib" / "libamdhip64.so"
    if cand.exists():
        _HIP_RUNTIME = C.CDLL(str(cand), mode=C.RTLD_GLOBAL)


def lib() -> C.CDLL:
    """Load libminisched_hip.so (in-tree). Raises if it is missing: no fallback path."""
    global _LIB
    if _LIB is None:
        _share_hip_runtime_with_torch()
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        h = C.CDLL(str(LIB_PATH))
        for name, (res, args) in _SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = h
    return _LIB


_FAST = None


def fast():
    """The CPython fast-call module (csrc/msh_pyfast.c) for the per-batch device entry points;
    it links this package's libminisched_hip.so. Raises if it is missing: no fallback path."""
    global _FAST
    if _FAST is None:
        lib()  # the HIP runtime shared with torch, and the library, loaded first
        import importlib.util
        path = next(LIB_PATH.parent.glob("_msh_fast*.so"), None)
        if path is None:
            raise RuntimeError(f"_msh_fast*.so is missing next to {LIB_PATH}: build it with __graft_entry__.build()")
        spec = importlib.util.spec_from_file_location("_msh_fast", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _FAST = mod
    return _FAST


def ptr(a: np.ndarray | None):
    """Host numpy array -> void* (None for an absent optional array)."""
    if a is None:
        return None
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data_as(C.c_void_p)


def check(rc: int, ctx=None) -> None:
    if rc != MSH_OK:
        msg = ""
        if ctx is not None:
            raw = lib().msh_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise MshError(rc, msg)


def device_count() -> int:
    n = C.c_int(0)
    check(lib().msh_device_count(C.byref(n)))
    return n.value
