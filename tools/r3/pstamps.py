"""Timeline of the split-K parameter kernel (NERFHIP_STAMPS diagnostic build):
per-wave s_memrealtime stamps (100 MHz) at 0 entry, 1 loads issued, 2 first
block staged, 3 MFMA loop done, 4 epilogue issued.  (The round-3 measurement ran a variant that issued all 8 blocks of a slice up front.)  One lone medium fit at
seq 2048 (config 2), a few epochs; the last epoch's stamps are kept.
usage: NERFHIP_LIB=build/variants/v_pstamps.so python tools/r3/pstamps.py"""
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

cfg = {c.name: c for c in CONFIGS_FULL}["medium"]
keys, _ = kv_slice(0, 0, seq_len=2048)
buf = torch.zeros(4096 * 4 * 8, dtype=torch.int64, device="cuda")
os.environ["NERFHIP_PSTAMPS"] = str(buf.data_ptr())
torch.manual_seed(0)
job = engine.FitJob([engine.FitSpec(keys, cfg, SIREN(cfg, 128).flat_parameters())], 5, devices=[0])
print(job.groups[0].plan())
job.launch()
job.wait()
st = buf.view(-1, 8).cpu().numpy().astype(np.float64)
st = st[st[:, 0] > 0]
t0 = st[:, 0].min()
rel = (st[:, :5] - t0) / 100.0        # µs
ok = st[:, 1] > 0                       # waves of MFMA tiles
out = {"waves": int(st.shape[0]), "mfma_waves": int(ok.sum()),
       "entry_spread_us": float(rel[:, 0].max()),
       "end_max_us": float(rel[ok, 4].max())}
for k, name in enumerate(["issue_loads", "first_block", "mfma_loop", "epilogue"], start=1):
    d = rel[ok, k] - rel[ok, k - 1]
    out[name] = {"mean_us": round(float(d.mean()), 2), "max_us": round(float(d.max()), 2)}
out["entry_hist_us"] = np.histogram(rel[:, 0], bins=8)[0].tolist()
print(json.dumps(out, indent=1))
