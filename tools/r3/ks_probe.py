"""K-split row kernel co-residency probe (round 3).

Runs the lone-fit K-split path (NERFHIP_ROWS_KS=1), pad "0" = two workgroups
may share a CU (NERFHIP_KS_SHARE_CU=1; the round-3 sessions varied the pad
size through NERFHIP_KS_DYN_LDS, since replaced), at seq 8192/16384 for
E = 0 and E = 3 epochs, then compares the final-eval ŷ with the torch forward
of the final parameters, and characterises every wrong element: 16-row block,
output tile J, feature-in-tile (= finalising wave w for fe = 4g + w), size.
usage: NERFHIP_LIB=<lib> python tools/r3/ks_probe.py <tag> [repeats]
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import numpy as np
import torch
from nerf_attention import SIREN, SIRENConfig, engine
from nerf_attention.synthetic import kv_slice

os.environ["NERFHIP_ROWS_KS"] = os.environ.get("ROWS_KS", "1")   # 0: the regular row kernel
tag = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cases = [(256, 2, 8192, 0), (256, 2, 8192, 3), (512, 3, 8192, 0), (256, 2, 16384, 0),
         (128, 1, 8192, 0)]
if os.environ.get("KS_CASES"):      # e.g. "256,2,16384,0;256,2,8192,3"
    cases = [tuple(int(x) for x in c.split(",")) for c in os.environ["KS_CASES"].split(";")]
pads = os.environ.get("KS_PADS", "0,default").split(",")
for pad in pads:
    if pad == "default":
        os.environ.pop("NERFHIP_KS_SHARE_CU", None)
    else:
        os.environ["NERFHIP_KS_SHARE_CU"] = "1"
    for (W, L, N, E) in cases:
        cfg = SIRENConfig(W, L, 30.0, "x")
        keys, _ = kv_slice(0, 0, seq_len=N, num_layers=1, num_kv_heads=1)
        for rep in range(reps):
            torch.manual_seed(rep)
            nf = int(os.environ.get("KS_FITS", "1"))   # 2: two identical fits (ALTFIT builds)
            init = SIREN(cfg, 128).flat_parameters()
            specs = [engine.FitSpec(target=keys, config=cfg, init=init) for _ in range(nf)]
            job = engine.FitJob(specs, E, devices=[0], precision="bf16x3", log_every=0)
            g = job.groups[0]
            g.eval_y.fill_(float("nan"))
            job.launch()
            job.wait()
            out = job.outputs()[0]
            m = SIREN(cfg, 128)
            m.load_flat_parameters(out.params.cpu())
            with torch.no_grad():
                y_ref = m.network(torch.linspace(0, 1, N).unsqueeze(1)).double()
            y = torch.cat([g.eval_y[k, :N] for k in range(nf)]).cpu().double()
            y_ref = torch.cat([y_ref] * nf)
            nan = torch.isnan(y)
            err = (torch.nan_to_num(y, 0.0) - y_ref).abs()
            scale = y_ref.abs().max().item()
            bad = (err > 1e-3 * max(scale, 1.0)) | nan
            rows, cols = np.nonzero(bad.numpy())
            rec = {"tag": tag, "pad": pad, "W": W, "L": L, "N": N, "E": E, "rep": rep,
                   "bad_elems": int(rows.size), "nan_elems": int(nan.sum()),
                   "bad_rows": int(np.unique(rows).size),
                   "bad_blocks": int(np.unique(rows // 16).size), "blocks": N // 16,
                   "max_err": float(err.max()), "scale": scale}
            if rows.size:
                blk = rows // 16
                rec["first_blocks"] = np.unique(blk)[:12].tolist()
                rec["tile_hist"] = np.bincount(cols // 16, minlength=8).tolist()
                rec["fe_hist"] = np.bincount(cols % 16, minlength=16).tolist()
                rec["rows_per_bad_block"] = float(np.mean(
                    [np.unique(rows[blk == b]).size for b in np.unique(blk)]))
                rec["cols_per_bad_row"] = float(bad.numpy()[np.unique(rows)].sum(1).mean())
            print(json.dumps(rec), flush=True)
