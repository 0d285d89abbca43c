"""Summarise tools/r4/iso_prof.sh output: rocprof kernel-trace average vs the
in-process hipEvent average of the isolated leg, and the per-launch PMC
figures of the same launches (FETCH_SIZE x2 per MI355X_MICROARCH.md §HBM,
WRITE_SIZE, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8)).  Only the training instantiation counts
(`<W, 128, X3, true>`; the forward-only final-eval launch is excluded).

usage: python tools/r4/iso_summary.py <iso_prof out dir>
"""

from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

N_SIMD, N_XCD = 1024, 8
ROOT = Path(__file__).resolve().parents[2]


def lib_sha16() -> str:
    """The measured library's hash (bench.py reports these counters only for
    the same build)."""
    import hashlib
    import os
    lib = os.environ.get("NERFHIP_LIB") or ROOT / "nerf-attention_amd/nerf_attention/_lib/libnerfhip.so"
    return hashlib.sha256(Path(lib).read_bytes()).hexdigest()[:16]


def summarise(d: Path, ev: dict, kind: str, hip_ms: float) -> tuple:
    """Per-launch PMC figures and the rocprof average of one kernel kind
    (`k_step_rows` / `k_step_params`) of the isolated leg."""
    W = int(ev["kernel"].split("<")[1].split(",")[0])
    x3 = "true" if ev["precision"] == "bf16x3" else "false"
    pat = re.compile(rf"{kind}<{W}, 128, {x3}, (true|false)(, false)*>" if kind == "k_step_rows"
                     else rf"{kind}<{W}, 128, {x3}, false(, false)?(, \d+)?(, false)?>")
    # the 32-row training kernel (k_step_rows32<W, 128, TRAIN>, variant builds)
    # stands in for k_step_rows when the library selects it
    pat32 = re.compile(rf"k_step_rows32<{W}, 128, true>")

    def match(name):
        if kind == "k_step_rows" and pat32.search(name):
            return True
        m = pat.search(name)
        return bool(m) and (kind != "k_step_rows" or m.group(1) == "true")

    stats = None
    for r in csv.DictReader(open(d / "kernel_stats.csv")):
        if match(r["Name"]):
            stats = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                     "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    acc = defaultdict(list)
    for i in (1, 2, 3):
        f = d / f"pmc{i}.csv"
        if not f.exists():
            continue
        for r in csv.DictReader(open(f)):
            if match(r["Kernel_Name"]):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = {k: sum(v) / len(v) for k, v in acc.items()}
    rd = 2 * 1024 * per.get("FETCH_SIZE", 0.0)
    wr = 1024 * per.get("WRITE_SIZE", 0.0)
    key = f"{kind}<{W},128>[{ev['precision']}]"
    return key, {
        "bytes": rd + wr, "read_bytes": rd, "write_bytes": wr,
        "mfma_busy": (per["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * per["GRBM_GUI_ACTIVE"] / N_XCD)
                      if per.get("GRBM_GUI_ACTIVE") else None),
        "pmc_launches": {k: len(v) for k, v in acc.items()},
        "rocprof_avg_ms": stats and round(stats["avg_ms"], 5),
        "rocprof_calls": stats and stats["calls"],
        "rocprof_min_ms": stats and round(stats["min_ms"], 5),
        "hipevent_avg_ms": hip_ms,
        "rocprof_vs_hipevent": stats and round(stats["avg_ms"] / hip_ms - 1, 4),
        "fits": ev["fits"], "epochs": ev["epochs"],
        "lib_sha16": lib_sha16(),
        "source": "tools/r4/iso_prof.sh (rocprofv3 of tools/r4/isokernel.py)"}


def main():
    """Both kernels of the isolated chunk-epoch (the leg launches the row and
    the parameter kernel once per epoch; bench.py reports their bytes together
    against SURVEY.md §8d's algorithmic bytes of the chunk-epoch)."""
    d = Path(sys.argv[1])
    ev = None
    for line in (d / "trace.log").read_text().splitlines():
        if line.startswith("{"):
            ev = json.loads(line)
    primary = ev["kernel"].split("<")[0]
    partner = "k_step_params" if primary == "k_step_rows" else "k_step_rows"
    out = {}
    for kind, ms in ((primary, ev["avg_launch_ms"]), (partner, ev["partner_kernel_avg_ms"])):
        key, rec = summarise(d, ev, kind, ms)
        if kind == primary:
            rec["flops_per_launch"] = ev["flops_per_launch"]
        out[key] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
