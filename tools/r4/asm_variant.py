"""Build a libnerfhip.so variant whose part-P kind-K device code comes from a
hand-patched assembly file (ISA-level bisection; diagnostic only).

  python tools/r4/asm_variant.py emit  <part> <kind> <out.s> [-DFLAG ...]
      compile that translation unit's device code to assembly
  python tools/r4/asm_variant.py build <name> <part> <kind> <patched.s> [-DFLAG ...]
      assemble <patched.s> (llvm-mc via clang), link it to a code object,
      bundle it, compile the host side of the same unit against that bundle
      (the host command is taken from `hipcc -###`), and link
      build/variants/v_<name>.so with every other object from the main build.

The host side and the device side must come from the same source and flags.
"""

from __future__ import annotations

import shlex
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
from nerf_attention import _build  # noqa: E402

LLVM = Path("/opt/rocm/lib/llvm/bin")


def base_cmd(part, kind, extra):
    return [_build.HIPCC, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-fPIC",
            "-Wno-unused-function", "-I", str(_build.INCLUDE), *extra,
            *_build.KIND_FLAGS.get(kind, []), f"-DNERFHIP_PART={part}", f"-DNERFHIP_KIND={kind}"]


def emit(part, kind, out, extra):
    subprocess.run(base_cmd(part, kind, extra) + ["--cuda-device-only", "-S", "-o", out,
                                                  str(_build.SOURCES[0])], check=True)


def build(name, part, kind, patched, extra):
    odir = ROOT / "build" / "variants" / f"obj_{name}"
    odir.mkdir(parents=True, exist_ok=True)
    dev_o, dev_out, hipfb = odir / "dev.o", odir / "dev.out", odir / "dev.hipfb"
    subprocess.run([str(LLVM / "clang"), "-target", "amdgcn-amd-amdhsa", f"-mcpu={_build.ARCH}",
                    "-c", str(patched), "-o", str(dev_o)], check=True)
    subprocess.run([str(LLVM / "lld"), "-flavor", "gnu", "-m", "elf64_amdgpu", "--no-undefined",
                    "-shared", "-o", str(dev_out), str(dev_o)], check=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "-type=o", "-bundle-align=4096",
                    f"-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--{_build.ARCH}",
                    "-input=/dev/null", f"-input={dev_out}", f"-output={hipfb}"], check=True)
    fname = f"nerfhip_p{part}.o" if kind == 0 else f"nerfhip_p{part}k{kind}.o"
    host_o = odir / fname
    cmds = subprocess.run(base_cmd(part, kind, extra) + ["-c", str(_build.SOURCES[0]), "-o",
                                                         str(host_o), "-###"],
                          capture_output=True, text=True).stderr.splitlines()
    host = [shlex.split(c) for c in cmds if c.strip().startswith('"') and "-triple\" \"x86_64" in
            c.replace(" ", "\" \"") or (c.strip().startswith('"') and "x86_64-unknown-linux-gnu" in
                                        c.split("-aux-triple")[0] and "-cc1" in c)]
    host = [h for h in host if "-cc1" in h and h[h.index("-triple") + 1].startswith("x86_64")]
    assert len(host) == 1, cmds
    h = host[0]
    i = h.index("-fcuda-include-gpubinary")
    h[i + 1] = str(hipfb)
    subprocess.run(h, check=True)
    objs = []
    units = [(0, 0)] + [(p, k) for p in range(1, _build.N_PARTS) for k in _build.KIND_FLAGS]
    for p, k in units:
        f = f"nerfhip_p{p}.o" if k == 0 else f"nerfhip_p{p}k{k}.o"
        objs.append(host_o if (p, k) == (part, kind) else _build.LIB_DIR / "obj" / f)
    objs += [_build.LIB_DIR / "obj" / f"{s.stem}.o" for s in _build.SOURCES[1:]]
    lib = ROOT / "build" / "variants" / f"v_{name}.so"
    subprocess.run([_build.HIPCC, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o",
                    str(lib), *map(str, objs)], check=True)
    print(lib)


if __name__ == "__main__":
    what = sys.argv[1]
    if what == "emit":
        emit(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5:])
    else:
        build(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], sys.argv[6:])
