"""Build recipe of the C oracle (test infrastructure; building the checker is not using it):
oracle/msh_oracle.c + msh_oracle_omp.c -> oracle/build/libmsh_oracle.so via oracle/Makefile.
Called by tests/conftest.py, __graft_entry__.build() and bench.py's cpu_baseline leg."""
from __future__ import annotations

import subprocess
from pathlib import Path

ODIR = Path(__file__).resolve().parent
LIB = ODIR / "build" / "libmsh_oracle.so"
SRCS = [ODIR / "msh_oracle.c", ODIR / "msh_oracle_omp.c", ODIR / "msh_oracle.h", ODIR / "Makefile"]


def build_oracle(verbose: bool = False) -> Path:
    if not LIB.exists() or any(s.stat().st_mtime > LIB.stat().st_mtime for s in SRCS):
        cmd = ["make", "-C", str(ODIR)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, stdout=None if verbose else subprocess.DEVNULL)
    return LIB


if __name__ == "__main__":
    print(build_oracle(verbose=True))
