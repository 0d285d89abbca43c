"""K-split diagnostic 4: final eval into a NaN-filled eval_y (are the bad rows
never stored, or stored wrong?), with and without LDS padding (one workgroup
per CU)."""
import json, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import numpy as np
import torch
from nerf_attention import SIREN, SIRENConfig, engine
from nerf_attention.synthetic import kv_slice

os.environ["NERFHIP_ROWS_KS"] = "1"
for pad in ("0", "default"):
    if pad == "default":
        os.environ.pop("NERFHIP_KS_DYN_LDS", None)
    else:
        os.environ["NERFHIP_KS_DYN_LDS"] = pad
    for (W, L, N, n, E) in [(256, 2, 8192, 1, 0), (256, 2, 8192, 1, 3), (512, 3, 8192, 1, 0)]:
        cfg = SIRENConfig(W, L, 30.0, "x")
        keys, vals = kv_slice(0, 0, seq_len=N, num_layers=1, num_kv_heads=1)
        torch.manual_seed(0)
        specs = [engine.FitSpec(target=keys, config=cfg, init=SIREN(cfg, 128).flat_parameters())]
        job = engine.FitJob(specs, E, devices=[0], precision="bf16x3", log_every=1 if E else 0)
        g = job.groups[0]
        g.eval_y.fill_(float("nan"))
        if g.probe_y is not None:
            g.probe_y.fill_(float("nan"))
        job.launch()
        job.wait()
        out = job.outputs()[0]
        m = SIREN(cfg, 128)
        m.load_flat_parameters(out.params.cpu())
        with torch.no_grad():
            y_ref = m.network(torch.linspace(0, 1, N).unsqueeze(1))
        y = g.eval_y[0, :N].cpu()
        nanrows = np.nonzero(torch.isnan(y).any(1).numpy())[0]
        dy = (torch.nan_to_num(y, 0.0) - y_ref).abs().max(1).values.numpy()
        bad = np.nonzero(dy > 1e-3)[0]
        pn = None
        if g.probe_y is not None:
            py = g.probe_y.reshape(-1)
            pn = int(torch.isnan(py.reshape(E, -1)[:, :N * 128]).sum().item())
        print(json.dumps({"pad": pad, "W": W, "N": N, "E": E, "nan_rows": int(nanrows.size),
                          "nan_blocks": np.unique(nanrows // 16)[:10].tolist(),
                          "bad_rows": int(bad.size), "probe_nans": pn}), flush=True)
