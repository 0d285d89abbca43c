"""Configuration and result types of the SIREN KV-fit path.

Mirrors the reference's API surface (nerf_attention/types.py:10-100) so that
callers of `fit_siren` / `fit_kv_cache` see the same objects:

* `SIRENConfig`  — frozen (hidden_features, hidden_layers, omega_0, name),
  reference types.py:10-15.
* `FitResult`    — the 18-field result of one fit, reference types.py:18-37.
* `KVMetadata`   — `metadata.json` of an extracted KV cache, types.py:40-63.
* `CONFIGS_QUICK` / `CONFIGS_FULL` — the sweep architectures, types.py:87-100.
"""

from __future__ import annotations

from dataclasses import dataclass, fields

import numpy as np
import torch
import torch.nn as nn


@dataclass(frozen=True)
class SIRENConfig:
    hidden_features: int = 256
    hidden_layers: int = 2
    omega_0: float = 30.0
    name: str = 'medium'

    def num_parameters(self, out_features: int) -> int:
        """P = 2W + L(W² + W) + W·d + d (first SineLayer, L hidden, final Linear)."""
        w, l, d = self.hidden_features, self.hidden_layers, out_features
        return 2 * w + l * (w * w + w) + w * d + d


@dataclass
class FitResult:
    model: nn.Module
    config: SIRENConfig
    target_mean: torch.Tensor
    target_std: torch.Tensor
    losses: list[float]
    final_mse: float
    final_cosine_mean: float
    final_cosine_min: float
    final_cosine_std: float
    per_pos_mse: np.ndarray
    cosine_sims: np.ndarray
    compression_ratio: float
    raw_size_bytes: int
    siren_size_bytes: int
    train_time_seconds: float
    seq_len: int
    d_head: int
    num_parameters: int


@dataclass
class KVMetadata:
    model_name: str
    num_layers: int
    num_kv_heads: int
    seq_len: int
    head_dim: int
    actual_tokens: int
    dtype: str = 'float32'

    def to_dict(self) -> dict:
        return {f.name: getattr(self, f.name) for f in fields(self)}

    @classmethod
    def from_dict(cls, d: dict) -> 'KVMetadata':
        known = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in known})


@dataclass
class LayerSummary:
    """Per-layer averages of the KV structure analysis (reference types.py:66-74)."""
    layer: int
    avg_autocorr_k: float
    avg_autocorr_v: float
    avg_energy_10pct_k: float
    avg_energy_10pct_v: float
    avg_rank_ratio_k: float
    avg_rank_ratio_v: float


@dataclass
class AnalysisResult:
    """Result of `analyze_kv_cache` (reference types.py:77-84)."""
    metadata: KVMetadata
    layer_summaries: list
    avg_autocorr_keys: float
    avg_autocorr_values: float
    avg_spectral_keys: float
    avg_spectral_values: float


CONFIGS_QUICK: list[SIRENConfig] = [
    SIRENConfig(128, 1, 30.0, 'small'),
    SIRENConfig(256, 2, 30.0, 'medium'),
]

CONFIGS_FULL: list[SIRENConfig] = [
    SIRENConfig(64, 1, 30.0, 'tiny'),
    SIRENConfig(128, 1, 30.0, 'small'),
    SIRENConfig(256, 2, 30.0, 'medium'),
    SIRENConfig(512, 2, 30.0, 'large'),
    SIRENConfig(256, 3, 30.0, 'deep'),
    SIRENConfig(256, 2, 60.0, 'hifreq'),
    SIRENConfig(256, 2, 15.0, 'lofreq'),
]

# BASELINE.json config 5: the wide SIREN at seq_len 8192.
CONFIG_WIDE = SIRENConfig(512, 3, 30.0, 'wide')
