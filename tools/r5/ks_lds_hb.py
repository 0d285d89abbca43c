"""Inter-wave LDS happens-before check of the K-split row kernel
(k_step_rows_ks), from a per-lane trace of every LDS
access (NERFHIP_EXP_KS_TRACE variant build, nerfhip.hip ks_tr).

Every traced access carries (barrier count, read/write, LDS byte address).
All four waves of a workgroup pass the same barriers in the same order, so
two accesses of one address by different waves are ordered iff their barrier
counts differ; a pair with at least one write and equal counts is a race.
Checked per address for both launches of a 1-epoch fit — the training launch
(mode 0) and the final-eval forward-only launch (mode 1, which returns early
after the final phase) — for two workgroups each.

usage (GPU box):
  NERFHIP_LIB=build/variants/v_kstrace.so python tools/r5/ks_lds_hb.py
"""
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nerf_attention import SIREN, SIRENConfig, engine  # noqa: E402
from nerf_attention.synthetic import kv_slice  # noqa: E402

MAXEV = 4096          # kKsTrMax
TRACES = 4            # (mode, workgroup) = (0,0) (0,1) (1,0) (1,1)


def check(tr, bc_override=None):
    """tr: [4 waves][MAXEV][64] uint32 (0xffffffff = no event)."""
    acc = defaultdict(lambda: defaultdict(lambda: [set(), set()]))   # addr -> bc -> [readers, writers]
    n_ev, last_bc, truncated = [], [], False
    for w in range(4):
        ev = tr[w]
        n = int((ev[:, 0] != 0xFFFFFFFF).sum())
        n_ev.append(n)
        truncated |= n >= MAXEV
        e = ev[:n].astype(np.int64)
        bc = (e >> 18) if bc_override is None else np.zeros_like(e)
        rw = (e >> 17) & 1
        ad = e & 0x1FFFF
        last_bc.append(int(bc.max()) if n else 0)
        for b, r, a in zip(bc.ravel(), rw.ravel(), ad.ravel()):
            acc[int(a)][int(b)][int(r)].add(w)
    races = []
    for a, by_bc in acc.items():
        for b, (rd, wr) in by_bc.items():
            for wa in wr:
                others = (rd | wr) - {wa}
                if others:
                    races.append((a, b, wa, sorted(others)))
                    break
    return {"events_per_wave": n_ev, "barriers_per_wave": last_bc, "truncated": truncated,
            "addresses": len(acc), "races": len(races), "race_examples": races[:5]}


def run(cfg, N, precision="bf16x3"):
    buf = torch.full((TRACES * 4 * MAXEV * 64,), -1, dtype=torch.int32, device="cuda")
    os.environ["NERFHIP_PSTAMPS"] = str(buf.data_ptr())      # KArgs.pstamps (make_args)
    keys, _ = kv_slice(0, 0, seq_len=N, num_layers=1, num_kv_heads=1)
    torch.manual_seed(0)
    job = engine.FitJob([engine.FitSpec(keys, cfg, SIREN(cfg, 128).flat_parameters())], 1,
                        devices=[0], precision=precision)
    plan = job.groups[0].plan()
    job.launch()
    job.wait()
    tr = buf.view(TRACES, 4, MAXEV, 64).cpu().numpy().view(np.uint32)
    out = {"W": cfg.hidden_features, "L": cfg.hidden_layers, "N": N,
           "rows_variant": plan["rows_variant"]}
    for k in range(TRACES):
        r = check(tr[k])
        r["races_if_barriers_ignored"] = check(tr[k], bc_override=True)["races"]   # checker sensitivity
        out[f"mode{k // 2}_wg{k % 2}"] = r
    return out


def main():
    ok = True
    for cfg, N in ((SIRENConfig(256, 2, 30.0, "medium"), 2048),
                   (SIRENConfig(512, 3, 30.0, "wide"), 1024),
                   (SIRENConfig(128, 1, 30.0, "small"), 1024)):
        r = run(cfg, N)
        print(json.dumps(r), flush=True)
        for k, v in r.items():
            if isinstance(v, dict):
                # (barriers_per_wave is the count at each wave's LAST LDS access:
                # waves with no access after the final barriers show fewer)
                ok &= (v["races"] == 0 and not v["truncated"] and v["events_per_wave"][0] > 0
                       and v["races_if_barriers_ignored"] > 0)
    print(json.dumps({"all_clear": bool(ok)}))


if __name__ == "__main__":
    main()
