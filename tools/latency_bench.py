"""SIREN inference latency on one MI355X (the reference's
evaluate.py:173-242 loop).  Random-init models of every architecture (the
forward cost is data-independent), positions linspace(0, 1, N).

Per (arch, N) one JSON line:
  wall_ms     reference loop: perf_counter over 100 model(positions) calls
  device_ms   the same calls between HIP events (kernel + per-call copies)
  plan_ms     engine.ForwardPlan replay, HIP events, 100 launches
  layer16_ms  one launch regenerating 16 models (8 KV heads x K/V of a layer)
  hbm_fp16_ms the raw fp16 KV read at 8 TB/s, for the reference's comparison

usage: python tools/latency_bench.py [--seq-lens 2048] [--scan]
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))

import torch

from nerf_attention import CONFIG_WIDE, CONFIGS_FULL, SIREN, engine
from nerf_attention.latency import HBM_MI355X, time_forward


def plan_ms(cfg, n, models, runs=100):
    torch.manual_seed(0)
    params = torch.stack([SIREN(cfg, 128).flat_parameters() for _ in range(models)]).cuda()
    pos = torch.linspace(0, 1, n).cuda()
    plan = engine.ForwardPlan(cfg, 128, pos, models).load(params)
    for _ in range(10):
        plan()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(runs):
        plan()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / runs


def one(cfg, n):
    torch.manual_seed(0)
    model = SIREN(cfg, 128).cuda().eval()
    wall, dev = time_forward(model, n)
    p1, p16 = plan_ms(cfg, n, 1), plan_ms(cfg, n, 16)
    flops = 2 * n * (cfg.hidden_layers * cfg.hidden_features ** 2 + cfg.hidden_features * 128)
    print(json.dumps({"arch": cfg.name, "seq_len": n, "wall_ms": round(wall, 4),
                      "device_ms": round(dev, 4), "plan_ms": round(p1, 4),
                      "layer16_ms": round(p16, 4), "layer16_per_model_ms": round(p16 / 16, 4),
                      "plan_tflops": round(flops / p1 / 1e9, 2),
                      "layer16_tflops": round(16 * flops / p16 / 1e9, 2),
                      "hbm_fp16_ms": n * 128 * 2 / HBM_MI355X * 1e3}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq-lens", default="2048")
    ap.add_argument("--scan", action="store_true", help="medium at N = 512 .. 8192 as well")
    args = ap.parse_args()
    for n in [int(x) for x in args.seq_lens.split(",")]:
        for cfg in CONFIGS_FULL + [CONFIG_WIDE]:
            one(cfg, n)
    if args.scan:
        medium = {c.name: c for c in CONFIGS_FULL}["medium"]
        for n in (512, 1024, 4096, 8192):
            one(medium, n)


if __name__ == "__main__":
    main()
