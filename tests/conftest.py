"""Shared fixtures. `gpu`-marked tests need an MI355X; everything else runs on CPU."""
from __future__ import annotations

import importlib
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


def _build():
    importlib.import_module("mini-kube-scheduler_amd.build").build()
    importlib.import_module("oracle.build").build_oracle()


@pytest.fixture(scope="session")
def msh():
    """The product package (builds libminisched_hip.so in-tree when missing or stale)."""
    _build()
    return importlib.import_module("mini-kube-scheduler_amd")


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (test infrastructure only)."""
    _build()
    return importlib.import_module("oracle.oracle")


@pytest.fixture(scope="session")
def synth():
    return importlib.import_module("mini-kube-scheduler_amd.synthetic")


@pytest.fixture(scope="session")
def gpu_ctx(msh):
    if msh.device_count() < 1:
        pytest.skip("no GPU")
    ctx = msh.DeviceContext(0)
    yield ctx
    ctx.close()
