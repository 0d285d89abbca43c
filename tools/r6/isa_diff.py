"""Compare the gfx950 device code of two builds (objects or libraries with a
.hip_fatbin section), kernel by kernel: instruction streams with addresses
and encodings stripped.  Used to show that a source refactor leaves the
machine code unchanged.

usage: python tools/r6/isa_diff.py OLD NEW
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import kernel_resources  # noqa: E402


def kernels_isa(path: Path) -> dict:
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for co in kernel_resources.code_objects(path, Path(d)):
            dis = subprocess.run([str(kernel_resources.LLVM / "llvm-objdump"), "-d",
                                  "--no-show-raw-insn", "--mcpu=gfx950", str(co)],
                                 capture_output=True, text=True, check=True).stdout
            name, body = None, []
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
                if m:
                    if name:
                        out[name] = body
                    name, body = m.group(1), []
                    continue
                s = re.sub(r"^\s*[0-9a-f]+:\s*", "", line).split("//")[0].strip()
                s = re.sub(r"<[^>]*>", "<>", s)           # branch targets by label
                if name and s:
                    body.append(s)
            if name:
                out[name] = body
    return out


if __name__ == "__main__":
    a, b = kernels_isa(Path(sys.argv[1])), kernels_isa(Path(sys.argv[2]))
    only_a, only_b = sorted(set(a) - set(b)), sorted(set(b) - set(a))
    diff = [k for k in sorted(set(a) & set(b)) if a[k] != b[k]]
    print(f"kernels: {len(a)} old, {len(b)} new, {len(set(a) & set(b))} common, "
          f"{len(diff)} differ, {len(only_a)} only old, {len(only_b)} only new")
    for k in diff[:20]:
        print("  differs:", k[:120])
    for k in only_a[:20]:
        print("  only old:", k[:120])
    for k in only_b[:20]:
        print("  only new:", k[:120])
    sys.exit(1 if diff or only_a or only_b else 0)
