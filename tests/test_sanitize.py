"""ASan+UBSan and TSan over the C-ABI's host-only code: the snapshot packer (msh_pack.cpp) and the
process-wide host thread pool (msh_pool.h), driven by tests/sanitize/pack_stress.cpp (large packs
on the pool, concurrent packers, malformed offsets, a fork after the pool exists, node sorting,
lease contention). The recipe is tests/sanitize/Makefile; no GPU needed."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent / "sanitize"


def test_packer_and_pool_under_asan_and_tsan():
    if not shutil.which("make") or not shutil.which("g++"):
        pytest.skip("make / g++ missing")
    r = subprocess.run(["make", "-C", str(HERE)], capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    if r.returncode != 0 and ("cannot find -lasan" in out or "cannot find -ltsan" in out):
        pytest.skip("sanitizer runtimes missing")
    assert r.returncode == 0, out[-4000:]
    assert out.count("pack_stress: ok") == 2, out[-4000:]
