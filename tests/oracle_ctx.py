"""Test infrastructure: a DeviceContext stand-in computed by the CPU oracle.

Used only to exercise the HOST logic around the device path (queue, node cache, Permit/Bind,
the loop) on machines without a GPU, and as the checker the GPU pipeline tests compare
against. It is never importable from the product package.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O


class OracleCtx:
    def __init__(self):
        self.plugins = O.PluginSet()
        self.unsched = np.zeros(0, np.uint8)
        self.digit = np.zeros(0, np.int8)
        self.calls: list[tuple] = []
        self.n_nodes = 0

    def close(self) -> None:
        pass

    def set_plugins(self, filters, prescore, score) -> None:
        self.plugins = O.PluginSet(list(filters), list(prescore), [c.name for c in score],
                                   [int(c.weight) for c in score], [int(c.normalize) for c in score])
        self.calls.append(("set_plugins",))

    def upload_nodes(self, unsched, digit) -> None:
        self.unsched = np.array(unsched, np.uint8)
        self.digit = np.array(digit, np.int8)
        self.n_nodes = len(self.unsched)
        self.calls.append(("upload", len(self.unsched)))

    def patch_nodes(self, idx, unsched, digit) -> None:
        idx = np.asarray(idx, np.int64)
        assert len(np.unique(idx)) == len(idx) and (idx >= 0).all() and (idx < self.n_nodes).all()
        self.unsched[idx] = unsched
        self.digit[idx] = digit
        self.calls.append(("patch", sorted(int(i) for i in idx)))

    def schedule_batch(self, pod_digit, pod_tol):
        idx, score, status, _ = O.c_schedule_batch(self.unsched, self.digit, pod_digit, pod_tol, self.plugins)
        self.calls.append(("batch", len(pod_digit)))
        return idx, score, status
