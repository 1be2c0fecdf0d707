"""The GPU evidence runs a library built from this tree's sources on the machine that runs it (verdict r5,
next #3): on a GPU box the session fixture rebuilds libminisched_hip.so with that box's hipcc (conftest._build,
force) before any GPU test, and build.py records what it built from."""
from __future__ import annotations

import hashlib
import importlib
import socket

import pytest

import conftest


@pytest.mark.gpu
def test_library_built_here_from_these_sources(msh):
    if not conftest.on_gpu_box():
        pytest.skip("not a GPU box")
    b = importlib.import_module("mini-kube-scheduler_amd.build")
    prov = b.load_provenance()
    assert prov is not None, "no build provenance: the library was not compiled in this session"
    assert prov["forced"] and prov["host"] == socket.gethostname(), prov
    assert prov["sources_sha256"] == b.sources_digest(), "library built from other sources"
    assert prov["lib_sha256"] == hashlib.sha256(b.LIB.read_bytes()).hexdigest(), "library replaced after the build"
    assert b.LIB.stat().st_mtime >= conftest._SESSION_T0, "library older than this test session"
    assert "HIP version" in prov["hipcc"], prov
    # the process runs that very file
    lib = msh._native.lib()
    maps = open("/proc/self/maps").read()
    assert str(b.LIB) in maps and lib.msh_abi_version() == 8
    print(f"[build provenance] {prov}")


def test_provenance_record_shape(msh):
    """build.py's digest covers every source and header of the library (CPU)."""
    b = importlib.import_module("mini-kube-scheduler_amd.build")
    d = b.sources_digest()
    assert len(d) == 64 and d == b.sources_digest()
    assert "HIP version" in b.hipcc_version()
