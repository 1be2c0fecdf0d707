"""Build recipe for libminisched_hip.so (gfx950) — in-tree, no JIT cache.

`python -m` is not needed: `build()` is called by `__graft_entry__.build()` and by the tests'
session fixture when the library is missing or stale. The oracle (test infrastructure) is built
by oracle/build.py, not from here. Objects go to `build/` next to this
file; the shared library lands in the package directory so it travels with the repo
snapshot to the GPU box.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import socket
import subprocess
import sysconfig
import time
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
OBJ = PKG_DIR / "build"
LIB = PKG_DIR / "libminisched_hip.so"
INCLUDE = REPO / "include"
ARCH = os.environ.get("MSH_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    # (source, compiler, extra flags): one translation unit per kernel family, compiled in parallel
    ("msh_pair.hip", "hipcc", ["-x", "hip"]),
    ("msh_generic.hip", "hipcc", ["-x", "hip"]),
    ("msh_seq.hip", "hipcc", ["-x", "hip"]),
    ("msh_seq_cap.hip", "hipcc", ["-x", "hip"]),
    ("msh_prep.hip", "hipcc", ["-x", "hip"]),
    ("msh_capi.cpp", "hipcc", []),
    ("msh_shard.cpp", "hipcc", []),
    ("msh_pack.cpp", "g++", []),
]
HEADERS = [CSRC / "msh_internal.h", CSRC / "msh_device.h", CSRC / "msh_pool.h", CSRC / "msh_ctx.h", CSRC / "msh_seq_kernel.h",
           INCLUDE / "minisched_hip.h"]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the gfx950 build needs ROCm (/opt/rocm/bin/hipcc)")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile the kernels + C-ABI for gfx950, link libminisched_hip.so, and the CPython
    fast-call module on top of it. A build that compiled the library records its provenance
    (PROVENANCE: this machine's hipcc, the sources' digest, the seconds it took)."""
    t0 = time.time()
    compiled = _build_lib(force, verbose)
    build_fast(force, verbose)
    if compiled:
        _write_provenance(time.time() - t0, force)
    return LIB


# Where the last build that compiled the library wrote what it built from (build/ never travels to the
# GPU box: it is in .gpurunignore, so a provenance file there was written by a build on that machine).
PROVENANCE = OBJ / "provenance.json"


def sources_digest() -> str:
    """sha256 over the library's sources and headers (name + bytes, sorted by name)."""
    h = hashlib.sha256()
    for f in sorted({CSRC / s for s, _, _ in SOURCES} | set(HEADERS) | {FAST_SRC}, key=lambda x: x.name):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()


def hipcc_version() -> str:
    out = subprocess.run([_hipcc(), "--version"], capture_output=True, text=True).stdout
    keep = [ln.strip() for ln in out.splitlines() if ln.startswith(("HIP version", "AMD clang version"))]
    return "; ".join(keep) or out.strip().splitlines()[0]


def _write_provenance(seconds: float, forced: bool) -> None:
    rec = {"library": str(LIB), "built_at": time.strftime("%Y-%m-%dT%H:%M:%S%z"), "host": socket.gethostname(),
           "hipcc": hipcc_version(), "offload_arch": ARCH, "seconds": round(seconds, 1), "forced": forced,
           "sources_sha256": sources_digest(), "lib_sha256": hashlib.sha256(LIB.read_bytes()).hexdigest()}
    OBJ.mkdir(exist_ok=True)
    PROVENANCE.write_text(json.dumps(rec, indent=1) + "\n")


def load_provenance() -> dict | None:
    try:
        return json.loads(PROVENANCE.read_text())
    except (OSError, ValueError):
        return None


def _build_lib(force: bool, verbose: bool) -> bool:
    if not force and not _stale(LIB, [CSRC / src for src, _, _ in SOURCES] + HEADERS):
        return False  # up to date (objects need not be present, e.g. on the GPU box)
    OBJ.mkdir(exist_ok=True)
    objs, jobs = [], []
    for src, cc, extra in SOURCES:
        s = CSRC / src
        o = OBJ / (s.stem + ".o")
        objs.append(o)
        if not force and not _stale(o, [s, *HEADERS]):
            continue
        if cc == "hipcc":
            cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                   "-Wall", "-Wno-unused-result", "-Wno-unused-value", *extra,
                   "-c", str(s), "-o", str(o)]
        else:
            cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wextra", "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        jobs.append((src, subprocess.Popen(cmd)))
    failed = [src for src, pr in jobs if pr.wait() != 0]
    if failed:
        raise RuntimeError(f"compile failed: {', '.join(failed)}")
    if force or _stale(LIB, objs):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-ldl", "-o", str(LIB)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return True


FAST_SRC = CSRC / "msh_pyfast.c"
FAST = PKG_DIR / ("_msh_fast" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def build_fast(force: bool = False, verbose: bool = False) -> Path:
    """The CPython fast-call module for the per-batch device entry points (msh_pyfast.c)."""
    if not force and not _stale(FAST, [FAST_SRC, LIB, INCLUDE / "minisched_hip.h"]):
        return FAST
    cmd = ["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-Wall", "-Wextra",
           f"-I{sysconfig.get_paths()['include']}", f"-I{INCLUDE}", str(FAST_SRC),
           f"-L{PKG_DIR}", "-lminisched_hip", "-Wl,-rpath,$ORIGIN", "-o", str(FAST)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return FAST


DEMO = PKG_DIR / "abi_demo"
DEMO_SRC = REPO / "examples" / "abi_demo.c"


def build_demo(verbose: bool = False) -> Path:
    """examples/abi_demo.c: a plain-C consumer of the ABI (what a cgo binding calls), linked
    against the in-tree library; binary next to it so it travels with the snapshot."""
    lib = build(verbose=verbose)
    if _stale(DEMO, [DEMO_SRC, INCLUDE / "minisched_hip.h", lib]):
        cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", f"-I{INCLUDE}", str(DEMO_SRC), f"-L{PKG_DIR}",
               "-lminisched_hip", "-Wl,-rpath,$ORIGIN", "-o", str(DEMO)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return DEMO


if __name__ == "__main__":
    print(build(verbose=True))
    print(build_demo(verbose=True))
