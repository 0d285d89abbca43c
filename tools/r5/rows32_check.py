"""First GPU check of the 32-row row kernel (k_step_rows32) against the
16-row kernel on the same inputs (development tool): parameters after a few
epochs, 200-epoch cosines, then isolated per-launch timing of both variants.
usage: python tools/r5/rows32_check.py [--quick]"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from nerf_attention import CONFIGS_FULL, SIREN, engine  # noqa: E402
from nerf_attention.synthetic import kv_slice  # noqa: E402
from bench import rows_flops, params_flops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--quick", action="store_true")
args = ap.parse_args()
cfg = {c.name: c for c in CONFIGS_FULL}


def specs_for(names, n, seq):
    keys, vals = kv_slice(16, 2, seq_len=seq)
    torch.manual_seed(0)
    out = []
    for i in range(n):
        c = cfg[names[i % len(names)]]
        out.append(engine.FitSpec(keys if i % 2 == 0 else vals, c, SIREN(c, 128).flat_parameters()))
    return out


def run(specs, epochs, variant, timed=False):
    os.environ["NERFHIP_ROWS32"] = variant
    job = engine.FitJob(specs, epochs, devices=[0], precision="bf16x3")
    plan = job.groups[0].plan()
    job.launch(timed=timed)
    job.wait()
    return job, plan


def compare(names, n, seq, epochs):
    sp = specs_for(names, n, seq)
    ja, pa = run(sp, epochs, "0")
    jb, pb = run(sp, epochs, "1")
    oa, ob = ja.outputs(), jb.outputs()
    dp = max(float((a.params - b.params).abs().max()) for a, b in zip(oa, ob))
    dl = max(abs(x - y) / max(abs(x), 1e-30) for a, b in zip(oa, ob) for x, y in zip(a.losses, b.losses))
    dc = max(abs(float(np.mean(a.row_cos)) - float(np.mean(b.row_cos))) for a, b in zip(oa, ob))
    print(json.dumps({"names": names, "n": n, "seq": seq, "epochs": epochs,
                      "variants": [pa["rows_variant"], pb["rows_variant"]],
                      "max_abs_dparam": dp, "max_rel_dloss": dl, "max_dcos": dc,
                      "cos_b": [round(float(np.mean(o.row_cos)), 6) for o in ob[:4]]}), flush=True)
    return dp, dl, dc


dp, dl, dc = compare(["medium", "deep"], 8, 512, 3)
assert dl < 1e-3 and dp < 1e-4, "rows32 step mismatch"
compare(["medium", "deep", "hifreq"], 8, 512, 200)
if not args.quick:
    compare(["medium", "deep", "hifreq", "lofreq"], 40, 2048, 100)
    for names in (["medium"], ["deep"]):
        sp = specs_for(names, 40, 2048)
        cf = [s.config for s in sp]
        for variant in ("0", "1", "0", "1"):
            job, plan = run(sp, 41, variant, timed=True)
            t = job.timing[0]
            rows_ms, par_ms = t.rows_ms / t.launches, t.params_ms / t.launches
            print(json.dumps({"config": names[0], "fits": 40, "variant": plan["rows_variant"],
                              "rows_ms": round(rows_ms, 4), "params_ms": round(par_ms, 4),
                              "rows_tflops": round(rows_flops(2048, 128, cf) / rows_ms / 1e9, 1),
                              "params_tflops": round(params_flops(2048, 128, cf) / par_ms / 1e9, 1)}),
                  flush=True)
