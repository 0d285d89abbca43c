"""Train a fixed set of groups (all widths, split-K and fused reductions,
d_head 64 and 128) for a few epochs and save every fit's parameters and
losses; run it under two NERFHIP_LIB builds and compare the files bitwise.
usage: python tools/bitwise_ab.py out.npz [bf16x3|fp32]   |   python tools/bitwise_ab.py --cmp a.npz b.npz"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))

import numpy as np


def main():
    if sys.argv[1] == "--cmp":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
        print(f"{len(a.files) - len(bad)}/{len(a.files)} arrays bitwise equal", bad[:5])
        sys.exit(1 if bad else 0)
    import torch
    from nerf_attention import SIREN, SIRENConfig, engine
    from nerf_attention.synthetic import kv_slice
    precision = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
    out = {}
    cases = [("medium40", SIRENConfig(256, 2, 30.0, "medium"), 40, 512, 128),
             ("deep9", SIRENConfig(256, 3, 30.0, "deep"), 9, 512, 128),
             ("large5", SIRENConfig(512, 2, 30.0, "large"), 5, 512, 128),
             ("large8", SIRENConfig(512, 2, 30.0, "large"), 8, 256, 128),
             ("tiny12", SIRENConfig(64, 1, 30.0, "tiny"), 12, 192, 128),
             ("small3", SIRENConfig(128, 1, 30.0, "small"), 3, 320, 64),
             ("w256d64", SIRENConfig(256, 2, 60.0, "x"), 10, 256, 64),
             # split-K slices of exactly 8 blocks (the prefetch-all parameter path)
             ("medium1_2048", SIRENConfig(256, 2, 30.0, "medium"), 1, 2048, 128),
             ("medium2_1024", SIRENConfig(256, 2, 30.0, "medium"), 2, 1024, 128),
             ("small5_2048", SIRENConfig(128, 1, 30.0, "small"), 5, 2048, 128),
             ("tiny5_2048", SIRENConfig(64, 1, 30.0, "tiny"), 5, 2048, 128)]
    for name, cfg, n, N, D in cases:
        specs = []
        for i in range(n):
            k, v = kv_slice(i % 32, i % 8, seq_len=N, num_layers=32, num_kv_heads=8)
            torch.manual_seed(i)
            specs.append(engine.FitSpec(target=(k if i % 2 else v)[:, :D].contiguous(), config=cfg,
                                        init=SIREN(cfg, D).flat_parameters()))
        outs = engine.run_fits(specs, 12, devices=[0], precision=precision)
        for i, o in enumerate(outs):
            out[f"{name}_{i}_params"] = o.params.cpu().numpy()
            out[f"{name}_{i}_losses"] = np.asarray(o.losses, np.float32)
    np.savez(sys.argv[1], **out)
    print("saved", len(out))


if __name__ == "__main__":
    main()
