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
SOURCES = [CSRC / "nerfhip.hip", CSRC / "nerfhip_svd.hip", CSRC / "nerfhip_analysis.hip",
           CSRC / "nerfhip_rng.cpp"]
HEADERS = [INCLUDE / "nerfhip.h", CSRC / "nerfhip_layout.h"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("NERFHIP_ARCH", "gfx950")


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in SOURCES + HEADERS)


N_PARTS = 9   # NERFHIP_PART 0 = host ABI + small kernels, 1..8 = (W, precision) kernels

# Every (W, precision) part is compiled twice: its row kernels (NERFHIP_KIND=1)
# and its parameter kernels (NERFHIP_KIND=2), so each gets its own flags.  The
# parameter kernels' staging split (split3 + bf16 packing of 16 floats per
# thread and block) is SLP-vectorised by default into v_pk_add_f32 plus the
# register moves that pair its operands; packed fp32 VALU beside MFMAs costs
# more than the scalar ops (MI355X_MICROARCH.md), and without it the W = 64..512
# parameter kernels measured 3-10 % faster (profiles/r02/ab_noslp.log), while
# the W = 256 row kernel measured ~2 % slower — so only the parameter side
# drops SLP.
KIND_FLAGS = {1: [], 2: ["-fno-slp-vectorize"]}
# NERFHIP_KIND 3: the 32-row kernel (k_step_rows32), part 6 (W = 256, bf16x3)
# only.  Its MFMAs take the B operand from accumulator registers and keep the
# accumulators in VGPRs; -amdgpu-mfma-vgpr-form makes the compiler select the
# VGPR form of the MFMA destination (without it the accumulators go to AGPRs
# too, and 192 AGPRs of B plus 32 of accumulators do not fit beside them).
# Also without SLP vectorisation, like the parameter kernels: 2-3 % faster
# (profiles/r05/ab_r32_variants.log, v_r32noslp).
# The unit exists only in NERFHIP_VARIANTS builds (tools/build_variant.py with
# -DNERFHIP_VARIANTS): the kernel measured slower than the 16-row one
#  and is not part of the product library.
R32_UNITS = [(6, 3, ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"])]


def units(defines=()) -> list:
    """(part, kind, flags) of every translation unit of nerfhip.hip; the
    32-row unit only when `defines` carries -DNERFHIP_VARIANTS."""
    out = [(0, 0, [])] + [(part, kind, KIND_FLAGS[kind]) for part in range(1, N_PARTS)
                          for kind in KIND_FLAGS]
    return out + (R32_UNITS if "-DNERFHIP_VARIANTS" in defines else [])


def build(force: bool = False, verbose: bool = True) -> Path:
    """Compile the NERFHIP_PART translation units in parallel (the host part,
    then one per hidden width × precision × kernel kind), then link them into
    libnerfhip.so."""
    if not force and not _stale():
        return LIB
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    obj_dir = LIB_DIR / "obj"
    obj_dir.mkdir(exist_ok=True)
    base = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-unused-function", "-I", str(INCLUDE)]
    objs, procs = [], []
    for part, kind, flags in units():
        obj = obj_dir / (f"nerfhip_p{part}.o" if kind == 0 else f"nerfhip_p{part}k{kind}.o")
        cmd = base + flags + [f"-DNERFHIP_PART={part}",
                                                 f"-DNERFHIP_KIND={kind}", "-c", str(SOURCES[0]),
                                                 "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr, flush=True)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    for extra in SOURCES[1:]:                       # further translation units
        obj = obj_dir / f"{extra.stem}.o"
        cmd = base + ["-c", str(extra), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr, flush=True)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    failed = [p.args for p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr, flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(LIB)
