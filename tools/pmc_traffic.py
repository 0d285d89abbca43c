"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from the L2's
memory-side request counters, in KB; on gfx950 FETCH_SIZE reports exactly half
the bytes of wide (16 B/lane) coalesced reads, so it is doubled here.
WRITE_SIZE is exact for 16 B/lane stores; the engine also issues 4 B/lane
stores (activation scratch), for which the guide gives no calibration — the
write figure is reported as measured.

A third, optional pass (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE) gives the
matrix-core busy fraction of each kernel: SQ_VALU_MFMA_BUSY_CYCLES is the sum
over SIMDs of MFMA pipe cycles (calibrated: it equals 16 x the number of
v_mfma_f32_16x16x32_bf16 the row kernel issues, tools/pmc_groups.sh), and
GRBM_GUI_ACTIVE the GPU-active cycles summed over the 8 XCDs, so
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
PMC passes serialise the dispatches, so these are per-kernel figures.

usage: python tools/pmc_traffic.py <fetch.csv> <write.csv> [out.json] [mfma.csv]
"""

from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    """k_step_rows<512, 128, true, true> -> k_step_rows<512,128>[bf16x3]"""
    m = re.search(r"(k_\w+)<(\d+), (\d+)(?:, (true|false))?", name)
    if not m:
        return name.split("(")[0][-40:]
    prec = "[bf16x3]" if m.group(4) == "true" else "[fp32]"
    return f"{m.group(1)}<{m.group(2)},{m.group(3)}>{prec}"


def per_launch(path: str, counter: str) -> dict:
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


N_SIMD = 256 * 4          # MI355X: 256 CUs x 4 SIMDs
N_XCD = 8


def main():
    fetch = per_launch(sys.argv[1], "FETCH_SIZE")
    write = per_launch(sys.argv[2], "WRITE_SIZE")
    mfma = per_launch(sys.argv[4], "SQ_VALU_MFMA_BUSY_CYCLES") if len(sys.argv) > 4 else {}
    active = per_launch(sys.argv[4], "GRBM_GUI_ACTIVE") if len(sys.argv) > 4 else {}
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_step"):
            continue
        rd = 2 * 1024 * fetch.get(k, 0.0)        # KB → B, ×2 gfx950 correction
        wr = 1024 * write.get(k, 0.0)
        out[k] = {"bytes": rd + wr, "read_bytes": rd, "write_bytes": wr}
        if active.get(k):
            out[k]["mfma_busy"] = mfma.get(k, 0.0) / (N_SIMD * active[k] / N_XCD)
            out[k]["mfma_busy_cycles"] = mfma.get(k, 0.0)
            out[k]["gpu_active_cycles_per_xcd"] = active[k] / N_XCD
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
