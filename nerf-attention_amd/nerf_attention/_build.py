"""Build the HIP engine (libnerfhip.so) in-tree for gfx950.

`hipcc --offload-arch=gfx950` cross-compiles without a GPU, so this runs in
the build container; the resulting .so travels to the GPU box with the repo
snapshot (it is git-ignored, not gpurun-ignored).
"""

from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent                      # nerf-attention_amd/
CSRC = ROOT / "csrc"
INCLUDE = ROOT.parent / "include"
LIB_DIR = PKG / "_lib"
LIB = LIB_DIR / "libnerfhip.so"
SOURCES = [CSRC / "nerfhip.hip"]
HEADERS = [INCLUDE / "nerfhip.h"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("NERFHIP_ARCH", "gfx950")


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = True) -> Path:
    if not force and not _stale():
        return LIB
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-Wall", "-I", str(INCLUDE), "-o", str(tmp), *map(str, SOURCES)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr, flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(LIB)
