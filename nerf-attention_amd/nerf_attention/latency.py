"""Inference-latency harness: SIREN forward vs reading the raw KV from memory.

SURVEY §8f row 1.  The reference measures this in two places:
  * `evaluate.profile_latency` (nerf_attention/evaluate.py:173-242): up to 8
    `*_model.pt` checkpoints, 10 warm-up + 100 timed `model(positions)` calls,
    `latency_results.json` with the per-model record below;
  * `experiments.scaling._profile_siren_latency`
    (nerf_attention/experiments/scaling.py:225-262): the mean forward time of
    up to 4 checkpoints at a given seq_len.
Both are restated here with the same loop, the same JSON keys and the same
stdout line.  The forward runs on the HIP engine (SIREN.forward on a CUDA
device → engine.ForwardPlan → nerfhip_siren_forward).  Added to the record: the
HBM read time of the raw fp16 KV on MI355X (8 TB/s) and the device time of
one forward measured with HIP events (no host overhead).  The figures
(`latency_comparison.png`) are out of scope.
"""

from __future__ import annotations

import json
import time
from pathlib import Path

import numpy as np
import torch

from .siren import SIREN
from .types import SIRENConfig

HBM_4060 = 272e9       # B/s, evaluate.py:210
HBM_H100 = 3350e9      # B/s, evaluate.py:211
HBM_MI355X = 8e12      # B/s, MI355X HBM3E peak


def load_model_from_checkpoint(checkpoint: dict, device: str) -> SIREN:
    """evaluate.py:34-45."""
    cfg = checkpoint['config']
    config = SIRENConfig(hidden_features=cfg['hidden_features'],
                         hidden_layers=cfg['hidden_layers'], omega_0=cfg['omega_0'],
                         name=cfg.get('name', 'medium'))
    model = SIREN(config, out_features=cfg['out_features']).to(device)
    model.load_state_dict(checkpoint['model_state'])
    model.eval()
    return model


def time_forward(model: SIREN, seq_len: int, device: str = 'cuda', warmup: int = 10,
                 runs: int = 100) -> tuple[float, float]:
    """(wall ms, device ms) per forward.  Wall: the reference's loop, perf_counter
    around `runs` no-grad calls + synchronize (evaluate.py:187-200).  Device: the
    same calls bracketed by HIP events on the current stream."""
    positions = torch.linspace(0, 1, seq_len).unsqueeze(1).to(device)
    on_gpu = positions.is_cuda
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    with torch.no_grad():
        for _ in range(warmup):
            model(positions)
        sync()
        start = time.perf_counter()
        for _ in range(runs):
            model(positions)
        sync()
        wall = (time.perf_counter() - start) / runs
        if not on_gpu:        # a CPU model (the reference's device='cpu' case)
            return wall * 1e3, wall * 1e3
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(runs):
            model(positions)
        e1.record()
        e1.synchronize()
    return wall * 1e3, e0.elapsed_time(e1) / runs


def latency_record(name: str, config_name: str, model: SIREN, raw_bytes: int,
                   wall_ms: float, device_ms: float) -> dict:
    """The evaluate.py:206-216 record (same keys, same order), plus MI355X fields."""
    elapsed = wall_ms / 1e3
    return {
        'name': name,
        'config': config_name,
        'siren_time_ms': wall_ms,
        'hbm_time_4060_ms': raw_bytes / HBM_4060 * 1000,
        'hbm_time_h100_ms': raw_bytes / HBM_H100 * 1000,
        'speedup_vs_4060': (raw_bytes / HBM_4060) / max(elapsed, 1e-10),
        'speedup_vs_h100': (raw_bytes / HBM_H100) / max(elapsed, 1e-10),
        'num_params': sum(p.numel() for p in model.parameters()),
        'siren_device_time_ms': device_ms,
        'hbm_time_mi355x_ms': raw_bytes / HBM_MI355X * 1000,
    }


def profile_latency(siren_dir: Path, output_dir: Path, device: str = 'cuda') -> list[dict]:
    """evaluate.py:173-242 without the figure: writes latency_results.json."""
    siren_dir, output_dir = Path(siren_dir), Path(output_dir)
    model_files = sorted(siren_dir.glob('*_model.pt'))
    if not model_files:
        print("  No models found for latency profiling")
        return []
    results = []
    for model_file in model_files[:8]:
        checkpoint = torch.load(model_file, map_location=device, weights_only=True)
        metrics = checkpoint['metrics']
        model = load_model_from_checkpoint(checkpoint, device)
        wall_ms, dev_ms = time_forward(model, metrics['seq_len'], device)
        r = latency_record(metrics['name'], metrics['config_name'], model,
                           metrics['raw_size_bytes'], wall_ms, dev_ms)
        results.append(r)
        print(f"  {r['name']}: SIREN={wall_ms:.3f}ms | "
              f"HBM(4060)={r['hbm_time_4060_ms']:.3f}ms | "
              f"HBM(H100)={r['hbm_time_h100_ms']:.3f}ms")
    output_dir.mkdir(parents=True, exist_ok=True)
    with open(output_dir / 'latency_results.json', 'w') as f:
        json.dump(results, f, indent=2)
    return results


def profile_siren_latency(fits_dir: Path, seq_len: int, device: str) -> float:
    """scaling.py:225-262: mean forward ms over up to 4 checkpoints."""
    model_files = sorted(Path(fits_dir).glob('*_model.pt'))
    if not model_files:
        return 0.0
    times = []
    for mf in model_files[:4]:
        checkpoint = torch.load(mf, map_location=device, weights_only=True)
        model = load_model_from_checkpoint(checkpoint, device)
        times.append(time_forward(model, seq_len, device)[0])
    return float(np.mean(times)) if times else 0.0
