"""Truncated-SVD baseline on the MI355X engine.

Drop-in for the reference's `nerf_attention/experiments/svd.py`
(`run_svd_experiment`, svd.py:19-85): same slice selection (layers
{0, L/2, L-1}, up to 4 KV heads, K then V), same rank rule (svd.py:48-51),
same 15-key records, `svd_results.json` (indent=2) and stdout lines.  The
per-slice `torch.linalg.svd` + reconstruction + `F.cosine_similarity` loop
becomes ONE engine call for every slice and rank (`nerfhip_svd_rank_metrics`:
fp64 Gram, Jacobi eigen-solver, projection cosines, fp64 statistics).  The
figure (`plot_siren_vs_svd`) is out of scope.
"""

from __future__ import annotations

import ctypes
import json
from pathlib import Path

import numpy as np
import torch

from . import _native, engine
from .types import KVMetadata


def svd_rank(seq_len: int, d_head: int, target_cr: float) -> int:
    """svd.py:48-51: rank whose fp32 factors match the fp16 KV at ratio target_cr."""
    raw_bytes = seq_len * d_head * 2
    rank = max(1, int(raw_bytes / (target_cr * 4 * (seq_len + 1 + d_head))))
    return min(rank, min(seq_len, d_head))


def rank_metrics(slices: torch.Tensor, ranks, max_sweeps: int = 0) -> dict:
    """Row cosines of the rank-r reconstructions of every slice.

    slices: [T, N, D] fp32 on a HIP device (D in {64, 128}); ranks: up to 8
    ranks in [1, min(N, D)].  Returns {'row_cos': [T, R, N] fp32 tensor,
    'stats': [T, R, 3] float64 numpy (mean, min, unbiased std),
    'sigma': [T, D] float64 numpy (singular values, descending),
    'vectors': [T, D, D] float64 tensor (rows = right singular vectors)}."""
    dev = engine.resolve_device(slices.device)
    x = slices.detach().to(dev, torch.float32).contiguous()
    T, N, D = x.shape
    ranks = [int(r) for r in ranks]
    if not 1 <= len(ranks) <= _native.SVD_MAX_RANKS:
        raise ValueError(f"1..{_native.SVD_MAX_RANKS} ranks, got {len(ranks)}")
    f64 = dict(dtype=torch.float64, device=dev)
    gram = torch.empty(T, D, D, **f64)
    evec = torch.empty(T, D, D, **f64)
    eval_ = torch.empty(T, D, **f64)
    order = torch.empty(T, D, dtype=torch.int32, device=dev)
    row_cos = torch.empty(T, len(ranks), N, dtype=torch.float32, device=dev)
    stats = torch.empty(T, len(ranks), 3, **f64)
    b = _native.NerfhipSvdBatch(n_tensors=T, N=N, D=D, n_ranks=len(ranks),
                                max_sweeps=max_sweeps, x=x.data_ptr(), gram=gram.data_ptr(),
                                evec=evec.data_ptr(), eval=eval_.data_ptr(),
                                order=order.data_ptr(), row_cos=row_cos.data_ptr(),
                                stats=stats.data_ptr())
    for k, r in enumerate(ranks):
        b.ranks[k] = r
    stream = torch.cuda.current_stream(dev)
    _native.check(_native.load().nerfhip_svd_rank_metrics(ctypes.byref(b), stream.cuda_stream))
    sigma = eval_.clamp_min(0).sqrt()
    return {"row_cos": row_cos, "stats": stats.cpu().numpy(), "sigma": sigma.cpu().numpy(),
            "vectors": evec}


def run_svd_experiment(kv_dir: Path, base_dir: Path, target_compressions: list | None = None,
                       device: str = 'cuda') -> list[dict]:
    """svd.py:19-85 on the engine; returns the records it writes."""
    kv_dir, base_dir = Path(kv_dir), Path(base_dir)
    base_dir.mkdir(parents=True, exist_ok=True)
    if target_compressions is None:
        target_compressions = [2.0, 4.0, 8.0, 16.0]
    with open(kv_dir / 'metadata.json') as f:
        metadata = KVMetadata.from_dict(json.load(f))
    dev = engine.resolve_device(device)
    layers_to_fit = sorted({0, metadata.num_layers // 2, metadata.num_layers - 1})

    slices, keys = [], []                     # selection and order of svd.py:37-44
    for layer_idx in layers_to_fit:
        filepath = kv_dir / f'layer_{layer_idx:02d}.pt'
        if not filepath.exists():
            continue
        data = torch.load(filepath, map_location='cpu', weights_only=True)
        for head_idx in range(min(metadata.num_kv_heads, 4)):
            for kv_type, tensor in (('key', data['keys'][head_idx]),
                                    ('value', data['values'][head_idx])):
                slices.append(tensor)
                keys.append((layer_idx, head_idx, kv_type))
    all_results: list[dict] = []
    if slices:
        seq_len, d_head = slices[0].shape
        ranks = [svd_rank(seq_len, d_head, tc) for tc in target_compressions]
        uniq = sorted(set(ranks))
        out = rank_metrics(torch.stack(slices).to(dev), uniq)
        stats = out["stats"]
        raw_bytes = seq_len * d_head * 2
        for t, (layer_idx, head_idx, kv_type) in enumerate(keys):
            for target_cr, rank in zip(target_compressions, ranks):
                mean, mn, std = stats[t, uniq.index(rank)]
                svd_bytes = (seq_len * rank + rank + rank * d_head) * 4
                all_results.append({
                    'name': f'L{layer_idx}_H{head_idx}_{kv_type}_svd_r{rank}',
                    'method': 'svd', 'layer': layer_idx, 'head': head_idx, 'kv_type': kv_type,
                    'rank': rank, 'target_compression': target_cr,
                    'actual_compression': float(raw_bytes / svd_bytes),
                    'final_cosine_mean': float(np.float32(mean)),
                    'final_cosine_min': float(np.float32(mn)),
                    'final_cosine_std': float(np.float32(std)),
                    'raw_size_bytes': raw_bytes, 'svd_size_bytes': svd_bytes,
                    'seq_len': seq_len, 'd_head': d_head,
                })
            prefix = f'L{layer_idx}_H{head_idx}_{kv_type}'
            print(f"  {prefix}: " + " | ".join(
                f"r{r['rank']}={r['final_cosine_mean']:.4f}@{r['actual_compression']:.1f}x"
                for r in all_results if r['name'].startswith(prefix)))
    with open(base_dir / 'svd_results.json', 'w') as f:
        json.dump(all_results, f, indent=2)
    _print_summary(all_results, target_compressions)
    return all_results


def _print_summary(all_results: list[dict], target_compressions: list) -> None:
    """svd.py:88-97."""
    key_r = [r for r in all_results if r['kv_type'] == 'key']
    val_r = [r for r in all_results if r['kv_type'] == 'value']
    print("\nSVD Summary:")
    for tc in target_compressions:
        kr = [r for r in key_r if r['target_compression'] == tc]
        vr = [r for r in val_r if r['target_compression'] == tc]
        if kr and vr:
            print(f"  {tc:.0f}x: keys CosSim={np.mean([r['final_cosine_mean'] for r in kr]):.4f}, "
                  f"values CosSim={np.mean([r['final_cosine_mean'] for r in vr]):.4f}")


def main() -> None:
    """`python -m nerf_attention.svd` — the 'svd' experiment of the reference CLI
    (experiments/__main__.py:69-78) without its figure."""
    import argparse
    ap = argparse.ArgumentParser(description='SVD baseline comparison (MI355X engine)')
    ap.add_argument('--kv_dir', type=str, default='results/kv_cache')
    ap.add_argument('--output_dir', type=str, default='results/svd')
    ap.add_argument('--device', type=str, default='cuda')
    args = ap.parse_args()
    print("\n" + "=" * 60)
    print("EXPERIMENT 3: SVD Baseline Comparison")
    print("=" * 60)
    run_svd_experiment(Path(args.kv_dir), Path(args.output_dir), device=args.device)


if __name__ == '__main__':
    main()
