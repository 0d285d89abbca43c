"""The explicit host path: `fit_siren(..., device='cpu')`.

BASELINE.json config 1 is `quickstart --cpu`: one SIREN fit on a 512×128
synthetic tensor on a machine without a GPU, run as plumbing.  The MI355X
engine is the only path for a HIP device and never falls back here — a
'cuda' request on a host without a GPU raises (engine.resolve_device).  This
module runs only when the caller names the CPU.

On the CPU the fit is the training loop itself, in eager PyTorch: module
forward, `F.mse_loss`, autograd, `torch.optim.Adam` (single-tensor on CPU)
and `CosineAnnealingLR(T_max=epochs, eta_min=lr/100)`, one epoch after the
other, exactly the arithmetic of the reference loop (siren.py:80-149), so a
seeded CPU fit reproduces the reference's numbers at the same thread count.
"""

from __future__ import annotations

import time

import torch
import torch.nn.functional as F

from .types import FitResult, SIRENConfig


def _real(pred_norm, mean, std):
    return pred_norm * std + mean


def fit_on_host(kv_tensor: torch.Tensor, config: SIRENConfig, model, epochs: int, lr: float,
                log_every: int, on_probe=None) -> FitResult:
    """Train `model` (already initialised, on the CPU) to `kv_tensor` [N, d].
    Every `log_every` epochs on_probe(epoch, norm_mse, real_mse, cos) receives
    the verbose probe of siren.py:107-115 (None: no probes)."""
    n, d = kv_tensor.shape
    x = torch.linspace(0, 1, n).unsqueeze(1)
    y = kv_tensor.to('cpu')
    mean = y.mean(dim=0, keepdim=True)
    std = y.std(dim=0, keepdim=True).clamp(min=1e-3)
    y_norm = (y - mean) / std

    opt = torch.optim.Adam(model.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=epochs, eta_min=lr * 0.01)
    losses: list[float] = []
    t0 = time.time()
    for e in range(1, epochs + 1):
        opt.zero_grad()
        pred = model(x)
        loss = F.mse_loss(pred, y_norm)
        loss.backward()
        opt.step()
        sched.step()
        losses.append(loss.item())
        if on_probe is not None and e % log_every == 0:
            with torch.no_grad():
                real = _real(pred, mean, std)
                on_probe(e, loss.item(), F.mse_loss(real, y).item(),
                         F.cosine_similarity(real, y, dim=1).mean().item())
    train_time = time.time() - t0

    model.eval()
    with torch.no_grad():
        real = _real(model(x), mean, std)
        final_mse = F.mse_loss(real, y).item()
        cos = F.cosine_similarity(real, y, dim=1)
        row_mse = ((real - y) ** 2).mean(dim=1)
    raw, size = n * d * 2, model.size_bytes()
    return FitResult(model=model, config=config, target_mean=mean, target_std=std,
                     losses=losses, final_mse=final_mse,
                     final_cosine_mean=cos.mean().item(), final_cosine_min=cos.min().item(),
                     final_cosine_std=cos.std().item(), per_pos_mse=row_mse.numpy(),
                     cosine_sims=cos.numpy(), compression_ratio=raw / size,
                     raw_size_bytes=raw, siren_size_bytes=size, train_time_seconds=train_time,
                     seq_len=n, d_head=d, num_parameters=model.count_parameters())
