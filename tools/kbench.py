"""Isolated per-group kernel timing (development tool, not the bench contract).

Runs ONE group of identical-width fits (no concurrent groups) for a few
epochs through nerfhip_siren_fit_timed and prints per-kernel average launch
time and algorithmic TFLOP/s.  Example:
    python tools/kbench.py --config large --fits 40 --epochs 50
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
sys.path.insert(0, str(ROOT))

import torch

from nerf_attention import CONFIGS_FULL, CONFIG_WIDE, SIREN, engine
from nerf_attention.synthetic import kv_slice
from bench import params_flops, rows_flops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="medium")
    ap.add_argument("--fits", type=int, default=40)
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16x3"])
    args = ap.parse_args()
    cfgs = {c.name: c for c in CONFIGS_FULL + [CONFIG_WIDE]}
    names = args.config.split(",")
    keys, vals = kv_slice(16, 2, seq_len=args.seq_len)
    specs = []
    torch.manual_seed(0)
    for i in range(args.fits):
        cfg = cfgs[names[i % len(names)]]
        specs.append(engine.FitSpec(keys if i % 2 == 0 else vals, cfg,
                                    SIREN(cfg, 128).flat_parameters()))
    job = engine.FitJob(specs, args.epochs, devices=[0], precision=args.precision)
    assert len(job.groups) == 1, "kbench times one group: use configs of one width"
    g = job.groups[0]
    cf = [specs[i].config for i in g.members]
    out = []
    for rep in range(args.repeat):
        job.launch(timed=True)
        job.wait()
        t = job.timing[0]
        if t.launches == 0:   # the timed variant times every 4th epoch from epoch 3
            sys.exit(f"kbench needs --epochs >= 4 (got {args.epochs}): no timed launch")
        rows_ms, par_ms = t.rows_ms / t.launches, t.params_ms / t.launches
        fr, fp = rows_flops(args.seq_len, 128, cf), params_flops(args.seq_len, 128, cf)
        out.append({"rep": rep, "config": args.config, "precision": args.precision, "fits": g.n, "W": g.W,
                    "rows_ms": round(rows_ms, 4), "params_ms": round(par_ms, 4),
                    "rows_tflops": round(fr / rows_ms / 1e9, 2),
                    "params_tflops": round(fp / par_ms / 1e9, 2),
                    "epoch_ms": round(job.group_seconds()[0] * 1e3 / args.epochs, 4)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
