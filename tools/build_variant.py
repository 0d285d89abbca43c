"""Build an experiment variant of libnerfhip.so: the given NERFHIP_PART
translation units recompiled with extra -D flags, every other object reused
from the main build (nerf_attention/_lib/obj), linked to
build/variants/v_<name>.so.  Diagnostic only (kbench / ab.sh via NERFHIP_LIB).

usage: python tools/build_variant.py <name> [-DFLAG ...] [--parts 6,8]

The opt-in kernels that are not in the product library (the 32-row row
kernel, the fused split-K reduction) need -DNERFHIP_VARIANTS over every part
that launches them: the host part and the parameter parts, e.g.
  python tools/build_variant.py variants -DNERFHIP_VARIANTS --parts 0,1,2,3,4,5,6,7,8
"""

import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
from nerf_attention import _build  # noqa: E402


def main():
    name, rest = sys.argv[1], sys.argv[2:]
    parts = [6, 8]
    if "--parts" in rest:
        i = rest.index("--parts")
        parts = [int(p) for p in rest[i + 1].split(",")]
        rest = rest[:i] + rest[i + 2:]
    _build.build(verbose=False)
    out = ROOT / "build" / "variants"
    odir = out / f"obj_{name}"
    odir.mkdir(parents=True, exist_ok=True)
    base = [_build.HIPCC, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC",
            "-Wno-unused-function", "-I", str(_build.INCLUDE), *rest]
    objs, procs = [], []
    units = _build.units(rest)
    for part, kind, flags in units:
        fname = f"nerfhip_p{part}.o" if kind == 0 else f"nerfhip_p{part}k{kind}.o"
        if part in parts or kind == 3:                  # (the 32-row unit: variant builds only)
            obj = odir / fname
            procs.append(subprocess.Popen(base + flags + [
                f"-DNERFHIP_PART={part}", f"-DNERFHIP_KIND={kind}", "-c",
                str(_build.SOURCES[0]), "-o", str(obj)]))
        else:
            obj = _build.LIB_DIR / "obj" / fname
        objs.append(obj)
    objs += [_build.LIB_DIR / "obj" / f"{s.stem}.o" for s in _build.SOURCES[1:]]
    if any(p.wait() != 0 for p in procs):
        sys.exit("variant compile failed")
    lib = out / f"v_{name}.so"
    subprocess.run([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o",
                    str(lib), *map(str, objs)], check=True)
    print(lib)


if __name__ == "__main__":
    main()
