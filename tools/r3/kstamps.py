"""Phase timeline of the K-split row kernel (NERFHIP_STAMPS diagnostic build):
per-wave s_memrealtime stamps (100 MHz) at 0 entry, 1 layer 0 done, 2 hidden
forward done, 3 final forward done, 4 W_f^T backward done, 5 hidden backward
done, 6 end.  One lone medium fit at seq 2048 (config 2), last of 5 epochs.
usage: NERFHIP_LIB=build/variants/v_kstamps.so python tools/r3/kstamps.py"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import numpy as np
import torch
from nerf_attention import SIREN, CONFIGS_FULL, engine
from nerf_attention.synthetic import kv_slice

cfg = {c.name: c for c in CONFIGS_FULL}[sys.argv[1] if len(sys.argv) > 1 else "medium"]
keys, _ = kv_slice(0, 0, seq_len=2048)
buf = torch.zeros(2 * 4096 * 4 * 8, dtype=torch.int64, device="cuda")
os.environ["NERFHIP_PSTAMPS"] = str(buf.data_ptr())
torch.manual_seed(0)
job = engine.FitJob([engine.FitSpec(keys, cfg, SIREN(cfg, 128).flat_parameters())], 5, devices=[0])
print(job.groups[0].plan())
job.launch()
job.wait()
st = buf[131072:].view(-1, 8).cpu().numpy().astype(np.float64)
st = st[st[:, 6] > 0]                    # waves of the last training launch that ran to the end
t0 = st[:, 0].min()
rel = (st[:, :7] - t0) / 100.0            # µs
names = ["layer0", "hidden_fwd", "final_fwd", "bwd_final", "bwd_hidden", "bwd_layer0"]
out = {"waves": int(st.shape[0]), "entry_spread_us": round(float(rel[:, 0].max()), 2),
       "end_max_us": round(float(rel[:, 6].max()), 2)}
for k, n in enumerate(names, start=1):
    d = rel[:, k] - rel[:, k - 1]
    out[n] = {"mean_us": round(float(d.mean()), 2), "max_us": round(float(d.max()), 2)}
print(json.dumps(out, indent=1))
