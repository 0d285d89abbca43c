"""BASELINE.json configs 2, 4 and 5 on one GPU (bench.py covers config 3, the
280-fit sweep; config 1 is the reference's CPU plumbing run).

  single   config 2: one medium fit, synthetic L0 H0 key, seq 2048, 2000 epochs
  wide     config 5: one (512, 3) fit at seq 8192, 2000 epochs
  scan     config 4: medium on every layer × KV head × K/V (512 fits) at each
           seq_len in {512, 1024, 2048, 4096}, 2000 epochs (the BASELINE runs
           this on 8 GPUs; one GPU here)

Prints one JSON line per measurement.  usage:
    python tools/configs_bench.py single wide scan [--scan-lens 512,1024]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nerf-attention_amd"))

import torch

from nerf_attention import CONFIG_WIDE, CONFIGS_FULL, SIREN, engine, fit_siren
from nerf_attention.synthetic import kv_slice
from nerf_attention.workloads import sweep_280


def single(cfg, seq_len, epochs, label):
    keys, _ = kv_slice(0, 0, seq_len=seq_len)
    fit_siren(keys[:256], cfg, epochs=5, device="cuda", verbose=False)    # warm-up
    torch.manual_seed(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fit_siren(keys, cfg, epochs=epochs, device="cuda", verbose=False)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    fl = engine.fit_flops(seq_len, 128, cfg, epochs)
    print(json.dumps({"config": label, "arch": cfg.name, "seq_len": seq_len, "epochs": epochs,
                      "wall_s": round(wall, 3), "device_s": round(r.train_time_seconds, 3),
                      "ms_per_epoch": round(r.train_time_seconds / epochs * 1e3, 4),
                      "tflops": round(fl / r.train_time_seconds / 1e12, 1),
                      "final_cosine_mean": r.final_cosine_mean}), flush=True)


def svd_baseline(seq_len):
    """Config 5's SVD rank-k baseline: the svd.py selection (layers 0/16/31 x
    4 heads x K/V = 24 slices) at seq_len, all four target ratios, on the
    engine; next to the reference's CPU op sequence (oracle) on one slice."""
    import sys
    sys.path.insert(0, str(ROOT / "oracle"))
    import svd_oracle
    from nerf_attention.svd import rank_metrics, svd_rank
    from nerf_attention.synthetic import kv_layer
    sl = []
    for layer in (0, 16, 31):
        t = kv_layer(layer, seq_len, 32, 8, 128, heads=range(4))
        for h in range(4):
            sl += [t["keys"][h], t["values"][h]]
    x = torch.stack(sl).cuda()
    ranks = sorted({svd_rank(seq_len, 128, tc) for tc in (2.0, 4.0, 8.0, 16.0)})
    rank_metrics(x[:2], ranks)                                   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = rank_metrics(x, ranks)
    torch.cuda.synchronize()
    gpu_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    for r in ranks:
        svd_oracle.slice_metrics(sl[0], r)
    cpu_s = (time.perf_counter() - t0) * len(sl)
    print(json.dumps({"config": "5 svd baseline", "seq_len": seq_len, "slices": len(sl),
                      "ranks": ranks, "gpu_s": round(gpu_s, 4),
                      "cpu_oracle_s_extrapolated": round(cpu_s, 2),
                      "cpu_threads": torch.get_num_threads(),
                      "mean_cos_per_rank": [round(float(v), 4)
                                            for v in out["stats"][:, :, 0].mean(0)]}), flush=True)


def analysis(seq_len):
    """Pre-fit KV structure analysis (analyze.py selection: layers 0/8/16/24/31
    x 4 heads x K/V = 40 slices) at seq_len on the engine, next to the
    reference's CPU op sequence (oracle) on two slices, extrapolated."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import analysis_oracle
    from nerf_attention.analyze import analyze_slices, select_layers
    from nerf_attention.synthetic import kv_layer
    sl, names = [], []
    for layer in select_layers(32):
        t = kv_layer(layer, seq_len, 32, 8, 128, heads=range(4))
        for h in range(4):
            sl += [t["keys"][h], t["values"][h]]
            names += [f"L{layer}_H{h}_K", f"L{layer}_H{h}_V"]
    x = torch.stack(sl).cuda()
    analyze_slices(x[:2], names[:2])                             # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = analyze_slices(x, names)
    torch.cuda.synchronize()
    gpu_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    for i in range(2):
        analysis_oracle.analyze_tensor(sl[i], names[i])
    cpu_s = (time.perf_counter() - t0) / 2 * len(sl)
    print(json.dumps({"config": "pre-fit KV analysis", "seq_len": seq_len, "slices": len(sl),
                      "gpu_s": round(gpu_s, 4), "cpu_oracle_s_extrapolated": round(cpu_s, 2),
                      "cpu_threads": torch.get_num_threads(),
                      "mean_lag1": round(sum(o["lag1_autocorrelation"] for o in out) / len(out), 4)}),
          flush=True)


def scan(lens, epochs):
    for n in lens:
        t0 = time.perf_counter()
        plan, specs = sweep_280(n, seed=0, select="all", configs=["medium"])
        gen = time.perf_counter() - t0
        job = engine.FitJob(specs, epochs, devices=[0])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        job.launch()
        job.wait()
        wall = time.perf_counter() - t0
        fl = sum(engine.fit_flops(n, 128, s.config, epochs) for s in specs)
        cos = [float(torch.from_numpy(o.row_cos).mean()) for o in job.outputs()]
        k = [c for c, p in zip(cos, plan) if p[3] == "key"]
        v = [c for c, p in zip(cos, plan) if p[3] == "value"]
        print(json.dumps({"config": "4 scan", "seq_len": n, "fits": len(specs),
                          "epochs": epochs, "wall_s": round(wall, 2),
                          "fits_per_s": round(len(specs) / wall, 2),
                          "tflops": round(fl / wall / 1e12, 1), "datagen_s": round(gen, 1),
                          "mean_cos_keys": round(sum(k) / len(k), 4),
                          "mean_cos_values": round(sum(v) / len(v), 4)}), flush=True)
        del job


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="+", choices=["single", "wide", "scan", "svd", "analysis"])
    ap.add_argument("--epochs", type=int, default=2000)
    ap.add_argument("--scan-lens", default="512,1024,2048,4096")
    args = ap.parse_args()
    medium = {c.name: c for c in CONFIGS_FULL}["medium"]
    if "single" in args.which:
        single(medium, 2048, args.epochs, "2 single fit")
    if "wide" in args.which:
        single(CONFIG_WIDE, 8192, args.epochs, "5 wide SIREN")
    if "svd" in args.which:
        svd_baseline(8192)
    if "analysis" in args.which:
        analysis(8192)
    if "scan" in args.which:
        scan([int(x) for x in args.scan_lens.split(",")], args.epochs)


if __name__ == "__main__":
    main()
