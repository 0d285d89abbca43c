"""PyTorch custom ops over the HIP engine (torch.library).

`torch.ops.nerfhip.siren_fit` trains a batch of same-width fits and returns
plain tensors, so the engine composes with torch code (streams, devices,
torch.compile graphs via the registered fake) without touching ctypes:

    params, losses, row_cos, row_mse = torch.ops.nerfhip.siren_fit(
        targets,            # [n, N, D] fp32, CUDA
        init,               # [n, P_max] fp32, state_dict-order flat params (zero padded)
        hidden_features,    # int
        hidden_layers,      # list[int], one per fit
        omega_0,            # list[float], one per fit
        epochs, lr)

`torch.ops.nerfhip.siren_forward(params, positions, W, L, omega, D)` is the
inference forward (reference SIREN.forward, siren.py:60-61).
"""

from __future__ import annotations

import torch

from . import engine
from .types import SIRENConfig


def _p(W, L, D):
    return SIRENConfig(W, L, 30.0, "x").num_parameters(D)


@torch.library.custom_op("nerfhip::siren_fit", mutates_args=())
def siren_fit(targets: torch.Tensor, init: torch.Tensor, hidden_features: int,
              hidden_layers: list[int], omega_0: list[float], epochs: int,
              lr: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    dev = engine.resolve_device(targets.device)
    n, N, D = targets.shape
    specs = []
    for i in range(n):
        cfg = SIRENConfig(hidden_features, hidden_layers[i], omega_0[i], f"fit{i}")
        specs.append(engine.FitSpec(targets[i], cfg, init[i, :_p(hidden_features,
                                                                   hidden_layers[i], D)]))
    outs = engine.run_fits(specs, epochs, lr=lr, devices=[dev.index])
    params = torch.zeros_like(init)
    for i, o in enumerate(outs):
        params[i, :o.params.numel()] = o.params.to(init.device)
    losses = torch.tensor([o.losses for o in outs], dtype=torch.float32).reshape(n, epochs)
    row_cos = torch.stack([torch.from_numpy(o.row_cos) for o in outs])
    row_mse = torch.stack([torch.from_numpy(o.row_mse) for o in outs])
    return params, losses.to(dev), row_cos.to(dev), row_mse.to(dev)


@siren_fit.register_fake
def _(targets, init, hidden_features, hidden_layers, omega_0, epochs, lr):
    n, N, _ = targets.shape
    return (torch.empty_like(init), targets.new_empty(n, epochs), targets.new_empty(n, N),
            targets.new_empty(n, N))


@torch.library.custom_op("nerfhip::siren_forward", mutates_args=())
def siren_forward(params: torch.Tensor, positions: torch.Tensor, hidden_features: int,
                  hidden_layers: int, omega_0: float, out_features: int) -> torch.Tensor:
    engine.resolve_device(params.device)
    cfg = SIRENConfig(hidden_features, hidden_layers, omega_0, "x")
    return engine.forward(params, cfg, out_features, positions).clone()


@siren_forward.register_fake
def _(params, positions, hidden_features, hidden_layers, omega_0, out_features):
    return params.new_empty(positions.numel(), out_features)
