"""Schedule experiments on the 280-fit sweep (development tool): one process
per setting (env vars must be set before HIP initialises).  Prints the sweep
wall clock of `--steps` timed sweeps after one warm-up, and per-group seconds.
usage: GPU_MAX_HW_QUEUES=8 NERFHIP_GROUP_MAX=40 python tools/r4/sweep_sched.py --epochs 400
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8 and "SWEEP_KEEP_QUEUES" not in os.environ:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import torch  # noqa: E402
from nerf_attention import engine  # noqa: E402
from nerf_attention.workloads import sweep_280  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--epochs", type=int, default=400)
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--tag", default="")
args = ap.parse_args()
_, specs = sweep_280(2048, seed=0)
job = engine.FitJob(specs, args.epochs, devices=[0])
job.launch()
job.wait()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.steps):
    job.launch()
    job.wait()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / args.steps
secs = job.group_seconds()
print(json.dumps({"tag": args.tag, "queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                  "group_max": os.environ.get("NERFHIP_GROUP_MAX", "40"),
                  "chunks": os.environ.get("NERFHIP_CHUNKS", "depth"), "epochs": args.epochs,
                  "s_per_sweep": round(dt, 4), "fits_per_s_2000ep_equiv":
                  round(280 / (dt * 2000 / args.epochs), 3),
                  "groups": [[g.W, g.n, g.L_max, round(t, 3)] for g, t in zip(job.groups, secs)]}),
      flush=True)
