"""Per-kernel resources of the built libnerfhip.so, read from its gfx950 code
objects (no GPU): scratch (private segment) bytes, VGPR/AGPR/SGPR counts and
spills.  The .hip_fatbin section holds one offload bundle per translation unit;
each gfx950 entry is an ELF code object whose metadata note lists its kernels.

    python tools/kernel_resources.py [lib.so]     # one line per kernel
"""

from __future__ import annotations

import re
import struct
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "nerf-attention_amd" / "nerf_attention" / "_lib" / "libnerfhip.so"
LLVM = Path("/opt/rocm/lib/llvm/bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FIELDS = ("private_segment_fixed_size", "vgpr_count", "agpr_count", "sgpr_count",
          "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size")


def code_objects(lib: Path, tmp: Path) -> list[Path]:
    # objcopy rewrites its input file when given no output: dump from a copy,
    # so the shipped library (and the hash the PMC summaries are stamped with)
    # never changes under a resource check
    fb, cp = tmp / "fatbin", tmp / "lib_copy.so"
    shutil.copyfile(lib, cp)
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", str(cp), str(tmp / "lib_out.so")],
                   check=True, capture_output=True)
    data = fb.read_bytes()
    out = []
    for s in (m.start() for m in re.finditer(re.escape(MAGIC), data)):
        (nb,) = struct.unpack_from("<Q", data, s + 24)
        p = s + 32
        for _ in range(nb):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if triple.endswith("gfx950"):
                co = tmp / f"co{len(out)}.o"
                co.write_bytes(data[s + off:s + off + size])
                out.append(co)
    return out


def kernels(lib: Path = LIB) -> dict[str, dict[str, int]]:
    """{demangled kernel name: {field: value}} over every code object."""
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(lib, Path(d)):
            notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True,
                                   capture_output=True, text=True).stdout
            # one YAML list item per kernel: "  - .agpr_count: …" up to the next item
            for block in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
                block = ".agpr_count:" + block
                name = re.search(r"\.name:\s+(\S+)", block).group(1)
                vals = {f: int(m.group(1)) for f in FIELDS
                        if (m := re.search(rf"\.{f}:\s+(\d+)", block))}
                res[name] = vals
    names = list(res)
    dem = subprocess.run(["c++filt"], input="\n".join(names), check=True,
                         capture_output=True, text=True).stdout.split("\n")
    return {dem[i].replace("(anonymous namespace)::", ""): res[n] for i, n in enumerate(names)}


if __name__ == "__main__":
    ks = kernels(Path(sys.argv[1]) if len(sys.argv) > 1 else LIB)
    for n, v in sorted(ks.items()):
        print(f"{n:70s} " + " ".join(f"{k}={x}" for k, x in v.items()))
