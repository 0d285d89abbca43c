"""Per-stream (group / chunk) elapsed time of one sweep: which stream sets the
makespan.  usage: python tools/group_times.py [--epochs 200]"""
import argparse
import json
import os
import sys
from pathlib import Path

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8 and "SWEEP_KEEP_QUEUES" not in os.environ:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import torch  # noqa: E402
from nerf_attention import engine  # noqa: E402
from nerf_attention.workloads import sweep_280  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--epochs", type=int, default=200)
args = ap.parse_args()
_, specs = sweep_280(2048, seed=0)
job = engine.FitJob(specs, args.epochs, devices=[0])
for rep in range(2):
    job.launch()
    job.wait()
    secs = job.group_seconds()
    print(json.dumps([{"W": g.W, "fits": g.n, "L": sorted({specs[i].config.hidden_layers for i in g.members}),
                       "s": round(t, 3)} for g, t in zip(job.groups, secs)]), flush=True)
