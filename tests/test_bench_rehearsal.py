"""The driver's multi-GPU bench command, rehearsed on one GPU (verdict r4, next #4).

At round end the driver runs `python -m torch.distributed.run --nnodes=1 --nproc-per-node N
--master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W` on an 8-GPU node.
These tests launch exactly that command as a fresh child process at N = 2 with MSH_BENCH_REHEARSE=1
(every rank on cuda:0, the process group on gloo: RCCL refuses two ranks on one device), in each mode
bench.py has: pod-sharded batches (the default), the node-sharded C4 shape (keys merged by an
all-reduce MAX across the ranks) and pod-sharded sequential commit. Each must print one JSON line
whose outputs were checked bit-exact against the closed form on rank 0, with n_gpus = 2.
Not a measurement: the ranks share one device.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("extra", [[], ["--mode", "nodeshard", "--nodes", "20000", "--pods", "100000"],
                                   ["--mode", "sequential"]], ids=["batch", "nodeshard", "sequential"])
def test_driver_command_two_ranks(msh, extra):
    env = dict(os.environ, MSH_BENCH_REHEARSE="1", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "1", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["check"] == "bit-exact vs closed form", line["check"]
    assert line["config"].get("rehearsal"), line["config"]
    assert line["value"] > 0 and line["steps"] == 4 and line["warmup"] == 1
