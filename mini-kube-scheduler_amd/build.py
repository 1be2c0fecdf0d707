"""Build recipe for libminisched_hip.so (gfx950) — in-tree, no JIT cache.

`python -m` is not needed: `build()` is called by `__graft_entry__.build()` and by the tests'
session fixture when the library is missing or stale. Objects go to `build/` next to this
file; the shared library lands in the package directory so it travels with the repo
snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
OBJ = PKG_DIR / "build"
LIB = PKG_DIR / "libminisched_hip.so"
INCLUDE = REPO / "include"
ARCH = os.environ.get("MSH_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    # (source, compiler, extra flags)
    ("msh_kernels.hip", "hipcc", ["-x", "hip"]),
    ("msh_capi.cpp", "hipcc", []),
    ("msh_pack.cpp", "g++", []),
]
HEADERS = [CSRC / "msh_internal.h", INCLUDE / "minisched_hip.h"]


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
    """Compile the kernels + C-ABI for gfx950 and link libminisched_hip.so."""
    if not force and not _stale(LIB, [CSRC / src for src, _, _ in SOURCES] + HEADERS):
        return LIB  # up to date (objects need not be present, e.g. on the GPU box)
    OBJ.mkdir(exist_ok=True)
    objs = []
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
            cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    if force or _stale(LIB, objs):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(LIB)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


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


def build_diagnostic(verbose: bool = False) -> Path:
    """Diagnostic variant with per-wave phase stamps (-DMSH_STAMPS): libminisched_hip_stamps.so.
    Used only by scripts/stamps.py; never loaded by the product path."""
    return build_variant(["-DMSH_STAMPS"], "stamps", verbose)


def build_variant(defines: list[str], tag: str, verbose: bool = False) -> Path:
    """A/B build of the library with extra -D flags: libminisched_hip_<tag>.so (tuning only)."""
    out = PKG_DIR / f"libminisched_hip_{tag}.so"
    if not _stale(out, [CSRC / src for src, _, _ in SOURCES] + HEADERS):
        return out
    OBJ.mkdir(exist_ok=True)
    objs = []
    for src, cc, extra in SOURCES:
        s = CSRC / src
        o = OBJ / (s.stem + f".{tag}.o")
        objs.append(o)
        if not _stale(o, [s, *HEADERS]):
            continue
        if cc == "hipcc":
            cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *defines,
                   "-Wno-unused-result", "-Wno-unused-value", *extra, "-c", str(s), "-o", str(o)]
        else:
            cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    if _stale(out, objs):
        subprocess.run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(out)],
                       check=True)
    return out


def build_oracle(verbose: bool = False) -> Path:
    """Compile the C oracle (test infrastructure) into oracle/build/libmsh_oracle.so."""
    odir = REPO / "oracle"
    out = odir / "build" / "libmsh_oracle.so"
    srcs = [odir / "msh_oracle.c", odir / "msh_oracle_omp.c", odir / "msh_oracle.h"]
    if _stale(out, srcs):
        cmd = ["make", "-C", str(odir)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, stdout=None if verbose else subprocess.DEVNULL)
    return out


if __name__ == "__main__":
    print(build(verbose=True))
    print(build_demo(verbose=True))
    print(build_oracle(verbose=True))
