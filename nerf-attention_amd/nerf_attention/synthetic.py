"""Deterministic synthetic KV cache — the input format of the fit path.

Restates `extract_kv_cache_synthetic` (reference extract.py:182-259): each
(layer, head) is drawn from its own `np.random.RandomState(layer*H + head)`
(extract.py:207) and each head dimension is a low-frequency base + a
mid-frequency term + layer-sharpened Gaussian spikes + noise for keys, a
sine + noise for values (extract.py:211-234).  The RNG draw order and the
numpy expression forms (and hence dtypes under NEP-50 promotion) are the
reference's, so the tensors are bit-identical — pinned by the SHA-256
fixtures in tests/golden/synthetic.json.

Because every (layer, head) has its own RNG stream, `kv_slice` produces any
single slice without generating the rest (the sweep needs 20 of 256).
"""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import torch

from .types import KVMetadata


def _sharpness(layer: int, num_layers: int) -> float:
    return 1.0 + 2.0 * (layer / max(num_layers - 1, 1))        # extract.py:204


def _spike_train(rng, seq_len: int, sharp: float) -> np.ndarray:
    """Sparse Gaussian bumps, narrower and more numerous in deeper layers
    (extract.py:219-228)."""
    out = np.zeros(seq_len)
    for _ in range(int(3 * sharp)):
        centre = rng.randint(0, seq_len)
        width = rng.randint(1, max(2, int(5 / sharp)))
        amp = rng.uniform(0.5, 2.0)
        for off in range(-width, width + 1):
            at = centre + off
            if 0 <= at < seq_len:
                out[at] += amp * np.exp(-0.5 * (off / max(1, width / 2)) ** 2)
    return out


def kv_slice(layer: int, head: int, seq_len: int = 2048, num_layers: int = 32,
             num_kv_heads: int = 8, head_dim: int = 128):
    """(keys[seq_len, head_dim], values[seq_len, head_dim]) of one (layer, head)."""
    rng = np.random.RandomState(layer * num_kv_heads + head)
    tt = torch.linspace(0, 1, seq_len).numpy()
    sharp = _sharpness(layer, num_layers)
    keys = np.empty((seq_len, head_dim), dtype=np.float32)
    vals = np.empty((seq_len, head_dim), dtype=np.float32)
    for j in range(head_dim):
        f_lo, f_hi = rng.uniform(1, 5), rng.uniform(3, 10)
        smooth = (0.5 * np.sin(2 * np.pi * f_lo * tt) +
                  0.3 * np.cos(2 * np.pi * f_hi * tt))
        f_mid = rng.uniform(10, 30)
        ripple = 0.2 * np.sin(2 * np.pi * f_mid * tt + rng.uniform(0, 2 * np.pi))
        bumps = _spike_train(rng, seq_len, sharp)
        noise = rng.randn(seq_len) * 0.1
        keys[:, j] = smooth + ripple + bumps + noise
        v_wave = 0.6 * np.sin(2 * np.pi * rng.uniform(1, 8) * tt)
        vals[:, j] = v_wave + rng.randn(seq_len) * 0.15
    return torch.from_numpy(keys), torch.from_numpy(vals)


def kv_layer(layer: int, seq_len: int = 2048, num_layers: int = 32, num_kv_heads: int = 8,
             head_dim: int = 128, heads=None):
    """{'keys': [H', N, d], 'values': [H', N, d]} for heads (default: all)."""
    heads = range(num_kv_heads) if heads is None else heads
    ks, vs = zip(*(kv_slice(layer, h, seq_len, num_layers, num_kv_heads, head_dim)
                   for h in heads))
    return {'keys': torch.stack(ks), 'values': torch.stack(vs)}


def extract_kv_cache_synthetic(
    seq_len: int = 2048,
    num_layers: int = 32,
    num_kv_heads: int = 8,
    head_dim: int = 128,
    output_dir: Path = Path('results/kv_cache_synthetic'),
) -> KVMetadata:
    """Write layer_XX.pt + metadata.json exactly as extract.py:182-259 does."""
    print("Generating synthetic KV cache...")
    print(f"  {num_layers} layers, {num_kv_heads} heads, seq_len={seq_len}, head_dim={head_dim}")
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    for layer in range(num_layers):
        torch.save(kv_layer(layer, seq_len, num_layers, num_kv_heads, head_dim),
                   output_dir / f'layer_{layer:02d}.pt')
    meta = KVMetadata(model_name='synthetic', num_layers=num_layers, num_kv_heads=num_kv_heads,
                      seq_len=seq_len, head_dim=head_dim, actual_tokens=seq_len)
    with open(output_dir / 'metadata.json', 'w') as f:
        json.dump(meta.to_dict(), f, indent=2)
    total_mb = num_layers * num_kv_heads * seq_len * head_dim * 2 * 4 / 1024 / 1024
    print(f"Saved to {output_dir}/ ({total_mb:.1f} MB)")
    return meta
