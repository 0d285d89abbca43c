"""Launch gaps of a lone fit's epoch (VERDICT r03 item 5's premise): from a
rocprofv3 --kernel-trace CSV, the idle time between the end of one step
kernel and the start of the next on the same queue, and each kernel's
duration, medians over the run.  usage: python tools/r4/gaps.py <kernel_trace.csv>"""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if re.search(r"k_step|k_adam", r["Kernel_Name"])]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(list)
gaps = defaultdict(list)
prev = None
for r in rows:
    name = re.search(r"(k_\w+)", r["Kernel_Name"]).group(1)
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[name].append(e - s)
    if prev is not None:
        gaps[f"{prev[0]} -> {name}"].append(s - prev[1])
    prev = (name, e)
out = {"kernels": {k: {"n": len(v), "median_us": round(statistics.median(v) / 1e3, 2)}
                   for k, v in dur.items()},
       "gaps": {k: {"n": len(v), "median_us": round(statistics.median(v) / 1e3, 2),
                    "p90_us": round(sorted(v)[int(0.9 * len(v))] / 1e3, 2)}
                for k, v in gaps.items() if len(v) > 10}}
epoch = sum(statistics.median(v) for v in dur.values()) / 1e3
gap = sum(statistics.median(v) for v in gaps.values() if len(v) > 10) / 1e3
out["epoch_kernel_us"] = round(epoch, 2)
out["epoch_gap_us"] = round(gap, 2)
print(json.dumps(out, indent=1))
