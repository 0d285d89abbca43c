"""ORACLE — CPU restatement of the reference KV structure analysis (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this.  Restates, per KV slice, the reference
`_analyze_tensor` (ruskaruma/nerf-attention, nerf_attention/analyze.py:61-80)
with its helpers `_autocorrelation` (:20-30), `_spectral_energy` (:33-44) and
`_effective_rank` (:47-58), in the same numpy / torch CPU operations.
tests/test_analysis.py pins it against the reference's own per-slice results
(tests/golden/make_golden_analysis.py): parity PINNED.
"""

from __future__ import annotations

import numpy as np
import torch


def autocorrelation(signal: np.ndarray, max_lag: int = 50) -> np.ndarray:
    n = len(signal)
    signal = signal - signal.mean()
    var = (signal ** 2).sum()
    if var < 1e-10:
        return np.zeros(max_lag + 1)
    out = np.zeros(max_lag + 1)
    for lag in range(min(max_lag + 1, n)):
        out[lag] = (signal[:n - lag] * signal[lag:]).sum() / var
    return out


def spectral_energy(signal: np.ndarray) -> dict:
    windowed = (signal - signal.mean()) * np.hanning(len(signal))
    spectrum = np.abs(np.fft.rfft(windowed))
    total = (spectrum ** 2).sum()
    if total < 1e-10:
        return {'top_5pct': 1.0, 'top_10pct': 1.0, 'top_25pct': 1.0, 'top_50pct': 1.0}
    n_freqs = len(spectrum)
    return {f'top_{int(pct * 100)}pct': float((spectrum[:max(1, int(n_freqs * pct))] ** 2).sum()
                                             / total)
            for pct in (0.05, 0.10, 0.25, 0.50)}


def effective_rank(matrix: torch.Tensor, threshold: float = 0.99) -> dict:
    _, S, _ = torch.linalg.svd(matrix)
    total = S.sum()
    cumulative = torch.cumsum(S, dim=0)
    rank = (cumulative < threshold * total).sum().item() + 1
    return {'effective_rank_99': rank, 'full_rank': len(S), 'rank_ratio': rank / len(S),
            'top_sv_fraction': (S[0] / total).item(),
            'top_10_sv_fraction': (S[:10].sum() / total).item() if len(S) >= 10 else 1.0}


def analyze_tensor(tensor: torch.Tensor, name: str, max_lag: int = 50) -> dict:
    seq_len, d_head = tensor.shape
    dims = range(0, d_head, max(1, d_head // min(d_head, 16)))
    ac = np.array([autocorrelation(tensor[:, d].numpy(), max_lag) for d in dims])
    mean_ac = ac.mean(axis=0)
    ratios = [spectral_energy(tensor[:, d].numpy()) for d in dims]
    return {'name': name, 'shape': list(tensor.shape),
            'lag1_autocorrelation': float(mean_ac[1]) if len(mean_ac) > 1 else 0.0,
            'mean_autocorrelation': mean_ac.tolist(),
            'spectral_energy': {k: float(np.mean([r[k] for r in ratios])) for k in ratios[0]},
            'rank': effective_rank(tensor)}
