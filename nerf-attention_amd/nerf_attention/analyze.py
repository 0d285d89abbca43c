"""KV structure analysis on the MI355X engine.

Drop-in for the reference's `nerf_attention/analyze.py` (`analyze_kv_cache`,
analyze.py:95-213): same layer/head selection, same per-slice measures
(lag-1 autocorrelation of 16 sampled dimensions, Hann-windowed spectral
energy concentration, SVD effective rank), same layer summaries, stdout lines,
feasibility assessment and `analysis_results.json`.  The per-dimension numpy
loops become one `nerfhip_kv_analysis` launch for every slice and dimension,
and the per-slice `torch.linalg.svd` one `nerfhip_svd_rank_metrics` launch.
The figure (`_plot_analysis`) is out of scope.
"""

from __future__ import annotations

import ctypes
import json
from pathlib import Path

import numpy as np
import torch

from . import _native, engine
from .svd import rank_metrics
from .types import AnalysisResult, KVMetadata, LayerSummary

MAX_LAG = 50


def select_layers(num_layers: int) -> list[int]:
    """analyze.py:83-84."""
    return sorted({0, num_layers // 4, num_layers // 2, 3 * num_layers // 4, num_layers - 1})


def sampled_dims(d_head: int) -> list[int]:
    """analyze.py:63-64: up to 16 evenly strided head dimensions."""
    return list(range(0, d_head, max(1, d_head // min(d_head, 16))))


def feasibility_label(val: float, good: float = 0.5, bad: float = 0.2) -> str:
    """analyze.py:87-92."""
    if val > good:
        return 'GOOD'
    if val > bad:
        return 'CONCERNING'
    return 'BAD'


def effective_rank(S: torch.Tensor, threshold: float = 0.99) -> dict:
    """analyze.py:47-58 on given singular values (fp32, descending)."""
    total = S.sum()
    cumulative = torch.cumsum(S, dim=0)
    rank = (cumulative < threshold * total).sum().item() + 1
    return {
        'effective_rank_99': rank,
        'full_rank': len(S),
        'rank_ratio': rank / len(S),
        'top_sv_fraction': (S[0] / total).item(),
        'top_10_sv_fraction': (S[:10].sum() / total).item() if len(S) >= 10 else 1.0,
    }


ENGINE_MAX_SEQ = 8192   # nerfhip_kv_analysis keeps a column + twiddles in LDS


def _host_measures(slices: torch.Tensor, dims, max_lag: int) -> dict:
    """The same measures on the CPU with numpy, per column as analyze.py:20-44
    defines them (explicit device='cpu' only, e.g. quickstart --cpu)."""
    x = slices.detach().to('cpu', torch.float32).numpy()
    T, N, _ = x.shape
    ac = np.zeros((T, len(dims), max_lag + 1))
    en = np.ones((T, len(dims), 4))
    hann = np.hanning(N)
    for t in range(T):
        for i, d in enumerate(dims):
            col = x[t, :, d]
            c = col - col.mean()
            var = (c ** 2).sum()
            if var >= 1e-10:
                for lag in range(min(max_lag + 1, N)):
                    ac[t, i, lag] = (c[:N - lag] * c[lag:]).sum() / var
            p = np.abs(np.fft.rfft((col - col.mean()) * hann)) ** 2
            tot = p.sum()
            if tot >= 1e-10:
                en[t, i] = [p[:max(1, int(len(p) * f))].sum() / tot for f in (0.05, 0.10, 0.25, 0.50)]
    return {"autocorr": ac, "energy": en}


def kv_measures(slices: torch.Tensor, dims, max_lag: int = MAX_LAG) -> dict:
    """Autocorrelation [T, n_dims, max_lag+1] and spectral-energy fractions
    [T, n_dims, 4] (top 5/10/25/50 %) of the given columns of every slice:
    on the engine for a HIP tensor, with numpy for a CPU tensor."""
    if slices.device.type == 'cpu':
        return _host_measures(slices, [int(d) for d in dims], max_lag)
    dev = engine.resolve_device(slices.device)
    x = slices.detach().to(dev, torch.float32).contiguous()
    T, N, D = x.shape
    if N > ENGINE_MAX_SEQ:
        raise _native.NerfhipError(
            f"KV analysis on the engine takes seq_len <= {ENGINE_MAX_SEQ} (got {N}); analyse "
            "longer caches with device='cpu'")
    dims = [int(d) for d in dims]
    f64 = dict(dtype=torch.float64, device=dev)
    ac = torch.empty(T, len(dims), max_lag + 1, **f64)
    en = torch.empty(T, len(dims), 4, **f64)
    b = _native.NerfhipKvAnalysisBatch(n_tensors=T, N=N, D=D, n_dims=len(dims), max_lag=max_lag,
                                       x=x.data_ptr(), autocorr=ac.data_ptr(),
                                       energy=en.data_ptr())
    for i, d in enumerate(dims):
        b.dims[i] = d
    stream = torch.cuda.current_stream(dev)
    _native.check(_native.load().nerfhip_kv_analysis(ctypes.byref(b), stream.cuda_stream))
    return {"autocorr": ac.cpu().numpy(), "energy": en.cpu().numpy()}


def analyze_slices(slices: torch.Tensor, names: list) -> list[dict]:
    """`_analyze_tensor` (analyze.py:61-80) for every slice of [T, N, D]."""
    T, N, D = slices.shape
    dims = sampled_dims(D)
    m = kv_measures(slices, dims)
    if slices.device.type == 'cpu':     # torch.linalg.svd's singular values (analyze.py:48)
        sigma = torch.linalg.svdvals(slices.to(torch.float32)).double().numpy()
    else:
        # fp64, descending; the D x D Gram gives D values, the SVD of an N x D
        # slice has min(N, D) (the rest are zero up to rounding)
        sigma = rank_metrics(slices, [1])["sigma"][:, :min(N, D)]
    keys = ('top_5pct', 'top_10pct', 'top_25pct', 'top_50pct')
    out = []
    for t in range(T):
        mean_ac = m["autocorr"][t].mean(axis=0)
        S = torch.from_numpy(sigma[t]).to(torch.float32)
        out.append({
            'name': names[t],
            'shape': [N, D],
            'lag1_autocorrelation': float(mean_ac[1]) if len(mean_ac) > 1 else 0.0,
            'mean_autocorrelation': mean_ac.tolist(),
            'spectral_energy': {k: float(np.mean(m["energy"][t, :, i])) for i, k in enumerate(keys)},
            'rank': effective_rank(S),
        })
    return out


def analyze_kv_cache(kv_dir: Path, output_dir: Path, device: str | None = None) -> AnalysisResult:
    """analyze.py:95-213 on the engine (without the figure).  The reference's
    signature has no device (it analyses on the CPU); here device=None means
    the HIP device when there is one, else the CPU (the reference's own
    computation, as quickstart --cpu needs); 'cuda' / 'cpu' force either."""
    if device is None:
        device = 'cuda' if torch.cuda.is_available() else 'cpu' 
    kv_dir, output_dir = Path(kv_dir), Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    with open(kv_dir / 'metadata.json') as f:
        metadata = KVMetadata.from_dict(json.load(f))
    dev = torch.device('cpu') if torch.device(device).type == 'cpu' else \
        engine.resolve_device(device)
    print(f"Analyzing KV cache: {metadata.num_layers} layers x {metadata.num_kv_heads} heads")
    print(f"Sequence length: {metadata.seq_len}, Head dim: {metadata.head_dim}")

    present, slices, names = [], [], []
    for layer_idx in select_layers(metadata.num_layers):
        filepath = kv_dir / f'layer_{layer_idx:02d}.pt'
        if not filepath.exists():
            present.append((layer_idx, False))
            continue
        present.append((layer_idx, True))
        data = torch.load(filepath, map_location='cpu', weights_only=True)
        for head_idx in range(min(metadata.num_kv_heads, 4)):
            for tag, t in (('K', data['keys'][head_idx]), ('V', data['values'][head_idx])):
                slices.append(t)
                names.append(f'L{layer_idx}_H{head_idx}_{tag}')
    results = analyze_slices(torch.stack(slices).to(dev), names) if slices else []
    by_name = {r['name']: r for r in results}

    layer_summaries: list[LayerSummary] = []
    for layer_idx, ok in present:
        if not ok:
            print(f"  Skipping layer {layer_idx} (not found)")
            continue
        heads = range(min(metadata.num_kv_heads, 4))
        ks = [by_name[f'L{layer_idx}_H{h}_K'] for h in heads]
        vs = [by_name[f'L{layer_idx}_H{h}_V'] for h in heads]
        summary = LayerSummary(
            layer=layer_idx,
            avg_autocorr_k=float(np.mean([r['lag1_autocorrelation'] for r in ks])),
            avg_autocorr_v=float(np.mean([r['lag1_autocorrelation'] for r in vs])),
            avg_energy_10pct_k=float(np.mean([r['spectral_energy']['top_10pct'] for r in ks])),
            avg_energy_10pct_v=float(np.mean([r['spectral_energy']['top_10pct'] for r in vs])),
            avg_rank_ratio_k=float(np.mean([r['rank']['rank_ratio'] for r in ks])),
            avg_rank_ratio_v=float(np.mean([r['rank']['rank_ratio'] for r in vs])),
        )
        layer_summaries.append(summary)
        print(f"\n  Layer {layer_idx}:")
        print(f"    Keys   - Autocorr: {summary.avg_autocorr_k:.3f} | "
              f"Spectral: {summary.avg_energy_10pct_k:.3f} | "
              f"Rank: {summary.avg_rank_ratio_k:.3f}")
        print(f"    Values - Autocorr: {summary.avg_autocorr_v:.3f} | "
              f"Spectral: {summary.avg_energy_10pct_v:.3f} | "
              f"Rank: {summary.avg_rank_ratio_v:.3f}")

    avg_ac_k = float(np.mean([s.avg_autocorr_k for s in layer_summaries]))
    avg_ac_v = float(np.mean([s.avg_autocorr_v for s in layer_summaries]))
    avg_en_k = float(np.mean([s.avg_energy_10pct_k for s in layer_summaries]))
    avg_en_v = float(np.mean([s.avg_energy_10pct_v for s in layer_summaries]))

    print(f"\n{'=' * 60}")
    print("SIREN FEASIBILITY ASSESSMENT")
    print(f"{'=' * 60}")
    print("\nAutocorrelation (lag-1):")
    print(f"  Keys:   {avg_ac_k:.3f}  {feasibility_label(avg_ac_k)} (>0.5)")
    print(f"  Values: {avg_ac_v:.3f}  {feasibility_label(avg_ac_v)} (>0.5)")
    print("\nSpectral concentration (energy in lowest 10% frequencies):")
    print(f"  Keys:   {avg_en_k:.3f}  {feasibility_label(avg_en_k)} (>0.5)")
    print(f"  Values: {avg_en_v:.3f}  {feasibility_label(avg_en_v)} (>0.5)")
    print("\nOverall prediction:")
    if avg_ac_k > 0.5 and avg_en_k > 0.5:
        print("  PROMISING: KV cache has significant structure. SIREN should compress well.")
    elif avg_ac_k > 0.2 or avg_en_k > 0.3:
        print("  MIXED: Some structure. SIREN may work partially.")
    else:
        print("  CHALLENGING: Noisy/unstructured. Document why it fails.")

    result = AnalysisResult(metadata=metadata, layer_summaries=layer_summaries,
                            avg_autocorr_keys=avg_ac_k, avg_autocorr_values=avg_ac_v,
                            avg_spectral_keys=avg_en_k, avg_spectral_values=avg_en_v)
    results_data = {
        'metadata': metadata.to_dict(),
        'layer_summaries': [
            {'layer': s.layer, 'avg_autocorr_k': s.avg_autocorr_k,
             'avg_autocorr_v': s.avg_autocorr_v, 'avg_energy_10pct_k': s.avg_energy_10pct_k,
             'avg_energy_10pct_v': s.avg_energy_10pct_v, 'avg_rank_ratio_k': s.avg_rank_ratio_k,
             'avg_rank_ratio_v': s.avg_rank_ratio_v}
            for s in layer_summaries
        ],
        'assessment': {'avg_autocorr_keys': avg_ac_k, 'avg_autocorr_values': avg_ac_v,
                       'avg_spectral_keys': avg_en_k, 'avg_spectral_values': avg_en_v},
    }
    with open(output_dir / 'analysis_results.json', 'w') as f:
        json.dump(results_data, f, indent=2)
    print(f"\nResults saved to {output_dir}/")
    return result


def main() -> None:
    """`python -m nerf_attention.analyze` (analyze.py:216-269 CLI, no figure)."""
    import argparse
    ap = argparse.ArgumentParser(description='Analyze KV cache structure (MI355X engine)')
    ap.add_argument('--kv_dir', type=str, default='results/kv_cache')
    ap.add_argument('--output_dir', type=str, default='results/analysis')
    ap.add_argument('--device', type=str, default=None)
    args = ap.parse_args()
    analyze_kv_cache(Path(args.kv_dir), Path(args.output_dir), args.device)


if __name__ == '__main__':
    main()
