"""Fused split-K Adam probe: one small group, E epochs, NERFHIP_SPLIT_FUSED=0
vs 1 (set per run via the env the library reads at launch): parameter
differences per region and the arrival counters after the run."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import torch

from nerf_attention import SIREN, SIRENConfig, engine
from nerf_attention.synthetic import kv_slice


def run(fused, cfg, N, n, E, precision):
    os.environ["NERFHIP_SPLIT_FUSED"] = fused
    keys, vals = kv_slice(3, 1, seq_len=N, num_layers=32, num_kv_heads=8)
    specs = []
    for i in range(n):
        torch.manual_seed(i)
        specs.append(engine.FitSpec(target=keys if i % 2 == 0 else vals, config=cfg,
                                    init=SIREN(cfg, 128).flat_parameters()))
    job = engine.FitJob(specs, E, devices=[0], split=True, precision=precision)
    job.launch()
    job.wait()
    g = job.groups[0]
    gp = g.grad_partial
    outs = job.outputs()
    return outs, g.plan(), gp


for cfg, N, n, prec in [(SIRENConfig(256, 2, 30.0, "medium"), 2048, 2, "bf16x3"),
                        (SIRENConfig(256, 2, 30.0, "medium"), 2048, 2, "fp32"),
                        (SIRENConfig(256, 2, 30.0, "medium"), 2048, 1, "bf16x3")]:
    for E in (1, 3):
        o0, p0, _ = run("0", cfg, N, n, E, prec)
        o1, p1, gp = run("1", cfg, N, n, E, prec)
        W, D, L = 256, 128, 2
        P = 2 * W + L * (W * W + W) + W * D + D
        regions = {"w0": (0, W), "b0": (W, 2 * W)}
        for i in range(L):
            o = 2 * W + i * (W * W + W)
            regions[f"w{i+1}"] = (o, o + W * W)
            regions[f"b{i+1}"] = (o + W * W, o + W * W + W)
        o = 2 * W + L * (W * W + W)
        regions["wf"] = (o, o + W * D)
        regions["bf"] = (o + W * D, o + W * D + D)
        a, b = o0[0].params.cpu(), o1[0].params.cpu()
        diff = {k: float((a[s:e] - b[s:e]).abs().max()) for k, (s, e) in regions.items()}
        from nerf_attention import _native
        sp = _native.group_sizes(W, D, N, L, E).grad_split
        cnt = gp[0, sp * P:].contiguous().view(torch.int32).cpu()[:64].tolist()
        print(json.dumps({"prec": prec, "n": n, "E": E, "plan0": p0, "plan1": p1, "diff": diff,
                          "cos": [float(o0[0].row_cos.mean()), float(o1[0].row_cos.mean())],
                          "counters": cnt}), flush=True)
