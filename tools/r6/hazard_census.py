"""Census of tools/r4/exec_war_scan.py's pattern (an EXEC write, or a write of
an SGPR a vector-memory instruction reads, within WS wait states of that
instruction) over EVERY kernel of the shipped library.

Writes a JSON summary: per kernel the EXEC and SGPR site counts, and the
totals.  Round 4 named the pattern as the cause of the K-split co-residency
fault; this census is the evidence that it is not a fault mechanism on its
own: the kernels that carry the most sites are the ones
every sweep launches thousands of times, concurrently, without a fault.

usage: python tools/r6/hazard_census.py [LIB] [--ws 8] [--json OUT]
"""
import argparse
import json
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tools"))
sys.path.insert(0, str(ROOT / "tools" / "r4"))
import exec_war_scan  # noqa: E402
import kernel_resources  # noqa: E402


def census(lib: Path, ws: int = 8) -> dict:
    per = {}
    with tempfile.TemporaryDirectory() as t:
        for co in kernel_resources.code_objects(lib, Path(t)):
            dis = subprocess.run([str(kernel_resources.LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950",
                                  str(co)], capture_output=True, text=True, check=True).stdout
            names = subprocess.run(["c++filt"],
                                   input="\n".join(l[l.index("<") + 1:l.index(">")] for l in dis.splitlines()
                                                   if l.endswith(">:") and "<" in l),
                                   capture_output=True, text=True).stdout.splitlines()
            mangled = [l[l.index("<") + 1:l.index(">")] for l in dis.splitlines()
                       if l.endswith(">:") and "<" in l]
            demangle = dict(zip(mangled, names))
            res = exec_war_scan.scan(dis.splitlines(), ws)
            for m in mangled:
                if m.startswith("_Z") and ("k_" in m):
                    ex, sg = res.get(m, [0, 0])
                    per[demangle.get(m, m)] = {"exec_sites": ex, "sgpr_sites": sg}
    flagged = {k: v for k, v in per.items() if v["exec_sites"] or v["sgpr_sites"]}
    return {"wait_states": ws, "kernels": len(per), "kernels_with_sites": len(flagged),
            "exec_sites": sum(v["exec_sites"] for v in per.values()),
            "sgpr_sites": sum(v["sgpr_sites"] for v in per.values()), "per_kernel": per}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=str(kernel_resources.LIB))
    ap.add_argument("--ws", type=int, default=8)
    ap.add_argument("--json")
    a = ap.parse_args()
    c = census(Path(a.lib), a.ws)
    print(f"{c['kernels']} kernels, {c['kernels_with_sites']} with sites; "
          f"{c['exec_sites']} EXEC, {c['sgpr_sites']} SGPR sites (WS={c['wait_states']})")
    top = sorted(c["per_kernel"].items(), key=lambda kv: -(kv[1]["exec_sites"] + kv[1]["sgpr_sites"]))
    for k, v in top[:12]:
        print(f"  exec {v['exec_sites']:4d} sgpr {v['sgpr_sites']:4d}  {k[:110]}")
    if a.json:
        Path(a.json).write_text(json.dumps(c, indent=1, sort_keys=True))
