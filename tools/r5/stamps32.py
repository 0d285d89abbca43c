"""Per-phase cycle breakdown (train launches only) of k_step_rows32 from the NERFHIP_STAMPS variant
(development tool).  usage:
    NERFHIP_LIB=build/variants/v_r32stamps.so python tools/r5/stamps32.py --config medium
Stamps (s_memtime) per wave: 0 start, 1 after layer 0, 2 after the hidden
forward, 3 after the final layer, 4 after W_fᵀ, 5 end; slots 8-11 the
per-sub-chunk DMA issue / k-steps / wait + barrier / count sums."""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from nerf_attention import CONFIGS_FULL, SIREN, engine  # noqa: E402
from nerf_attention.synthetic import kv_slice  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="medium")
ap.add_argument("--fits", type=int, default=40)
ap.add_argument("--epochs", type=int, default=3)
args = ap.parse_args()
cfg = {c.name: c for c in CONFIGS_FULL}[args.config]
keys, _ = kv_slice(16, 2, seq_len=2048)
torch.manual_seed(0)
specs = [engine.FitSpec(keys, cfg, SIREN(cfg, 128).flat_parameters()) for _ in range(args.fits)]
n_waves = 8 * ((args.fits + 7) // 8) * (2048 // 128) * 4
buf = torch.zeros(262144 + n_waves * 32, dtype=torch.int64, device="cuda")
os.environ["NERFHIP_PSTAMPS"] = str(buf.data_ptr())     # read by make_args (KArgs.pstamps)
os.environ.setdefault("NERFHIP_ROWS32", "1")
job = engine.FitJob(specs, args.epochs, devices=[0], precision="bf16x3")
g = job.groups[0]
assert g.plan()["rows_variant"] == "rows32"
job.launch()
job.wait()
st = buf[262144:].view(n_waves, 32).cpu().numpy().astype(np.float64)
st = st[st[:, 0] > 0]
d = np.diff(st[:, :6], axis=1)
W, L, D = cfg.hidden_features, cfg.hidden_layers, 128
k = 6 * 32   # one k-step: six 32x32x16 MFMAs of 32 cycles
mf = {"layer0": 0, "hidden_fwd": L * (W // 32) * (W // 16) * k, "final_fwd": (D // 32) * (W // 16) * k,
      "bwd_final": (W // 32) * (D // 16) * k, "bwd_rest": L * (W // 32) * (W // 16) * k}
out = {}
for i, name in enumerate(mf):
    c = float(d[:, i].mean())
    out[name] = {"cycles": round(c), "mfma_pipe_cycles": mf[name],
                 "ratio": round(c / max(1, mf[name]), 3)}
out["total_cycles"] = round(float((st[:, 5] - st[:, 0]).mean()))
out["total_mfma_pipe"] = sum(mf.values())
for name, b in (("hidden_fwd", 8), ("final_fwd", 12), ("bwd", 16), ("bwd_layer0", 24)):
    n = float(st[:, b + 3].mean())
    out["sub_" + name] = {"n": round(n, 1),
                          "dma_issue_per": round(float(st[:, b].mean()) / max(n, 1)),
                          "ksteps_per": round(float(st[:, b + 1].mean()) / max(n, 1)),
                          "wait_barrier_per": round(float(st[:, b + 2].mean()) / max(n, 1)),
                          "mfma_per": 48 * 32}
out["phase_tails_per_wave"] = round(float(st[:, 28].mean()))
out["phase_head_wait_per_wave"] = round(float(st[:, 29].mean()))
out["phase_head_split_per_wave"] = round(float(st[:, 30].mean()))
out["flush_pre_per_wave"] = round(float(st[:, 31].mean()))
out["next_fragment_per_wave"] = round(float(st[:, 20].mean()))
out["waves"] = int(st.shape[0])
out["spread_total"] = [round(float(np.percentile(st[:, 5] - st[:, 0], q))) for q in (5, 50, 95)]
print(json.dumps(out, indent=1))
