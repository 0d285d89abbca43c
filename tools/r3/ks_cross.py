"""K-split vs regular row kernel crossover after the xoff_ks layout: group
seconds per epoch of small bf16x3 groups with NERFHIP_ROWS_KS forced 0 / 1
(200 epochs, split-K as the engine plans it).  usage: python tools/r3/ks_cross.py"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import torch

from nerf_attention import SIREN, SIRENConfig, engine
from nerf_attention.synthetic import kv_slice

MED, WIDE = SIRENConfig(256, 2, 30.0, "medium"), SIRENConfig(512, 3, 30.0, "wide")
CASES = [(MED, 4096, 1), (MED, 8192, 1), (WIDE, 8192, 1), (WIDE, 4096, 1), (MED, 4096, 2),
         (MED, 2048, 4), (MED, 2048, 8), (MED, 1024, 8), (MED, 512, 16)]


def run(cfg, N, n, ks, epochs=200):
    os.environ["NERFHIP_ROWS_KS"] = ks
    specs = []
    for k in range(n):
        keys, vals = kv_slice(k // 8, k % 8, seq_len=N, num_layers=32, num_kv_heads=8)
        torch.manual_seed(k)
        specs.append(engine.FitSpec(target=keys, config=cfg, init=SIREN(cfg, 128).flat_parameters()))
    outs = engine.run_fits(specs, epochs, devices=[0], precision="bf16x3")
    return outs[0].group_seconds / epochs * 1e3, outs[0].plan


for cfg, N, n in CASES:
    run(cfg, N, n, "0", epochs=5)
    for rep in range(2):
        r0, p0 = run(cfg, N, n, "0")
        r1, p1 = run(cfg, N, n, "1")
        print(json.dumps({"arch": cfg.name, "seq": N, "fits": n, "regular_ms": round(r0, 4),
                          "ksplit_ms": round(r1, 4), "plan_reg": p0["rows_variant"],
                          "plan_ks": p1["rows_variant"], "grad_split": p1["grad_split"]}), flush=True)
