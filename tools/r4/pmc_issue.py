"""Per-launch issue / stall counters of the bench's isolated row-kernel leg,
from a rocprofv3 --pmc counter_collection CSV (tools/sessions/r4/s4pmc.sh):
sums per dispatch of k_step_rows<256, 128, true, true>, averaged over the
dispatches.  Ratios: SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES (share of wave time
waiting to issue an LDS instruction), SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES,
instructions per wave-cycle by type.
usage: python tools/r4/pmc_issue.py [--kernel=<name prefix>] <counter_collection.csv> [...]"""
import csv
import json
import re
import sys
from collections import defaultdict

args = sys.argv[1:]
kern = r"k_step_rows<256, 128, true, true"
if args and args[0].startswith("--kernel="):
    kern = re.escape(args.pop(0).split("=", 1)[1])
pat = re.compile(kern)
per = defaultdict(lambda: defaultdict(float))
for path in args:
    for r in csv.DictReader(open(path)):
        if not pat.search(r.get("Kernel_Name", "")):
            continue
        per[(path, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
tot = defaultdict(float)
n = defaultdict(int)
for d in per.values():
    for k, v in d.items():
        tot[k] += v
        n[k] += 1
avg = {k: tot[k] / n[k] for k in tot}
out = {"dispatches": max(n.values()) if n else 0, "per_launch": avg}
wc = avg.get("SQ_WAVE_CYCLES")
if wc:
    out["ratios_of_wave_cycles"] = {k: avg[k] / wc for k in avg if k.startswith("SQ_") and k != "SQ_WAVE_CYCLES"}
print(json.dumps(out, indent=1))
