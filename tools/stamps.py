"""Per-phase cycle breakdown of k_step_rows from the NERFHIP_STAMPS diagnostic
build (development tool).  usage:
    NERFHIP_LIB=build/variants/v_stamps.so python tools/stamps.py --config medium --fits 160
Stamps (s_memtime, shader clock) per wave: 0 start, 1 after layer 0, 2 after the
hidden forward, 3 after the final layer, 4 after the backward of the final
layer, 5 end; 12 / 13 s_memrealtime at start / end (the clock the chip held).
Build with -DNERFHIP_STAMPS_NOADD too for undistorted totals (no per-sub-chunk
read-modify-write counters).  Prints mean cycles per phase next to the wave's MFMA cycles."""

import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))

import numpy as np
import torch

from nerf_attention import CONFIGS_FULL, CONFIG_WIDE, SIREN, engine, _native
from nerf_attention.synthetic import kv_slice

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="medium")
ap.add_argument("--fits", type=int, default=40)
ap.add_argument("--epochs", type=int, default=3)
ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16x3"])
args = ap.parse_args()
cfgs = {c.name: c for c in CONFIGS_FULL + [CONFIG_WIDE]}
cfg = cfgs[args.config]
keys, _ = kv_slice(16, 2, seq_len=2048)
torch.manual_seed(0)
specs = [engine.FitSpec(keys, cfg, SIREN(cfg, 128).flat_parameters()) for _ in range(args.fits)]
job = engine.FitJob(specs, args.epochs, devices=[0], precision=args.precision)
g = job.groups[0]
n_waves = 8 * ((g.n + 7) // 8) * (g.n_pad // 16)    # every wave of the grid, any rows/WG
# the row kernel's stamps sit at kRowStampsOff of the NERFHIP_PSTAMPS buffer
# (the kernel arguments' pstamps pointer, read when the job's arguments are made)
ROW_OFF = 1 << 20
buf = torch.zeros(ROW_OFF + n_waves * 16, dtype=torch.int64, device="cuda")
if not _native.load().nerfhip_build_flags() & 2:
    sys.exit("not a NERFHIP_STAMPS library (set NERFHIP_LIB)")
os.environ["NERFHIP_PSTAMPS"] = str(buf.data_ptr())
job.launch()
job.wait()
st = buf[ROW_OFF:].view(n_waves, 16).cpu().numpy().astype(np.float64)
st = st[st[:, 0] > 0]                         # waves that ran (mapped blocks)
d = np.diff(st[:, :6], axis=1)
W, L, D = cfg.hidden_features, cfg.hidden_layers, 128
mf = {"layer0": 0, "hidden_fwd": L * (W // 16) * (W // 16) * 4, "final_fwd": (D // 16) * (W // 16) * 4,
      "bwd_final": (W // 16) * (D // 16) * 4, "bwd_hidden": L * (W // 16) * (W // 16) * 4}
# MFMA pipe cycles per wave: f32 16x16x4 = 32 cycles each; bf16x3 = 6 x 16x16x32
# (16 cycles) per 8 f32 16x16x4 = 12 cycles per f32-MFMA equivalent
cyc = 32 if args.precision == "fp32" else 12
out = {"precision": args.precision}
for i, name in enumerate(mf):
    out[name] = {"cycles": round(float(d[:, i].mean())), "mfma_f32_equiv": mf[name],
                 "mfma_pipe_cycles": mf[name] * cyc,
                 "ratio": round(float(d[:, i].mean()) / max(1, mf[name] * cyc), 3)}
out["total_cycles"] = round(float((st[:, 5] - st[:, 0]).mean()))
if st[:, 11].sum() > 0:   # bf16x3 phase counters (per wave, summed over sub-chunks)
    out["x3_phase"] = {"subchunks": round(float(st[:, 11].mean()), 1),
                       "dma_issue": round(float(st[:, 8].mean())),
                       "ksteps": round(float(st[:, 9].mean())),
                       "wait_barrier": round(float(st[:, 10].mean()))}
if st[:, 13].sum() > 0:   # s_memrealtime at entry / exit (100 MHz): the clock held
    rt = st[:, 13] - st[:, 12]
    ok = rt > 0
    clk = (st[ok, 5] - st[ok, 0]) / rt[ok] * 100.0
    mf_total = sum(mf.values()) * cyc
    out["clock_mhz"] = {"p10": round(float(np.percentile(clk, 10)), 1),
                        "p50": round(float(np.median(clk)), 1),
                        "p90": round(float(np.percentile(clk, 90)), 1)}
    # two waves share a SIMD (RowsCfg::WAVES_PER_SIMD at W <= 256): the pipe
    # carries both waves' MFMAs over one wave's lifetime
    out["mfma_pipe_busy_2waves"] = round(2.0 * mf_total / out["total_cycles"], 3)
out["waves"] = int(st.shape[0])
print(json.dumps(out, indent=1))
