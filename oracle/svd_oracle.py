"""ORACLE — CPU restatement of the reference SVD baseline (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this.  It restates, per KV slice, the reference
`run_svd_experiment` body (ruskaruma/nerf-attention,
nerf_attention/experiments/svd.py:45-75): the rank rule (:48-51), the
factorisation `torch.linalg.svd(tensor, full_matrices=False)` (:53), the
rank-r reconstruction (:54), `F.cosine_similarity(dim=1)` (:57) and the
record's statistics (:67-69).  The arithmetic lives in torch (LAPACK gesdd on
CPU); tests/test_svd.py pins this restatement against the reference's own
svd_results.json (tests/golden/make_golden_svd.py): parity PINNED.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F


def rank_for(seq_len: int, d_head: int, target_cr: float) -> int:
    raw_bytes = seq_len * d_head * 2
    rank = max(1, int(raw_bytes / (target_cr * 4 * (seq_len + 1 + d_head))))
    return min(rank, min(seq_len, d_head))


def slice_metrics(tensor: torch.Tensor, rank: int) -> dict:
    """svd.py:53-69 for one slice and one rank."""
    U, S, Vt = torch.linalg.svd(tensor, full_matrices=False)
    reconstructed = U[:, :rank] @ torch.diag(S[:rank]) @ Vt[:rank, :]
    cos = F.cosine_similarity(reconstructed, tensor, dim=1)
    return {"cosine_sims": cos, "final_cosine_mean": float(cos.mean().item()),
            "final_cosine_min": float(cos.min().item()),
            "final_cosine_std": float(cos.std().item()), "singular_values": S}
