"""Predict multi-GPU strong scaling of the 280-fit sweep on ONE GPU: for each
world size N, run every rank's LPT share (farm.rank_share) alone on this GPU
for a few hundred epochs and report the slowest rank's time — what
`bench.py --gpus N` would see, minus the collectives.  Diagnostic only.

usage: python tools/rank_probe.py [--epochs 200] [--worlds 1,2,4,8] [--all-ranks]
"""

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))

import torch  # noqa: E402

from nerf_attention import engine, farm  # noqa: E402
from nerf_attention.workloads import sweep_280  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--all-ranks", action="store_true")
    ap.add_argument("--partition", default="lpt")
    ap.add_argument("--reverse", action="store_true", help="time the ranks last to first")
    args = ap.parse_args()
    plan, specs = sweep_280(2048, seed=0)
    costs = [engine.fit_flops(2048, 128, s.config, args.epochs) for s in specs]
    widths = [s.config.hidden_features for s in specs]
    engine.FitJob(specs[:8], 5, devices=[0]).launch()        # warm-up (module load)
    torch.cuda.synchronize()
    for n in [int(x) for x in args.worlds.split(",")]:
        times = []
        ranks = list(range(n)) if args.all_ranks else [0]
        for r in (ranks[::-1] if args.reverse else ranks):
            mine = farm.rank_share(costs, n, r, widths, args.partition)
            job = engine.FitJob([specs[i] for i in mine], args.epochs, devices=[0])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            job.launch()
            job.wait()
            times.append(time.perf_counter() - t0)
            del job
        t = max(times)
        if args.reverse:
            times = times[::-1]          # report in rank order
        print(json.dumps({"world": n, "partition": args.partition, "epochs": args.epochs, "rank_s": [round(x, 3) for x in times],
                          "pred_fits_per_s": round(280 / (t * 2000 / args.epochs), 2)}), flush=True)


if __name__ == "__main__":
    main()
