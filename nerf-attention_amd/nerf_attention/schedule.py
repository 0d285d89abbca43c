"""Per-epoch optimiser scalars, computed on the host in float64.

The reference builds `torch.optim.Adam(lr)` and
`CosineAnnealingLR(T_max=epochs, eta_min=lr*0.01)` (siren.py:90-93) and steps
the scheduler after every Adam step (siren.py:103-104).  Adam step t = e+1
uses the learning rate lr_e that the scheduler holds at epoch e, with bias
corrections 1-β1^t and 1-β2^t evaluated as Python floats
(TORCH/optim/adam.py:531-547).

The scheduler itself is torch's own class, stepped exactly as the reference
steps it (its *recursive* closed form, TORCH/optim/lr_scheduler.py), so the
lr sequence is the reference's to the last bit.  Only the two fp32 scalars
per epoch that the device update needs leave the host:
    step_size = lr_e / (1 - β1^t),   bc2_sqrt = (1 - β2^t) ** 0.5
"""

from __future__ import annotations

import functools
import warnings

import numpy as np
import torch

BETA1, BETA2, EPS = 0.9, 0.999, 1e-8


@functools.lru_cache(maxsize=32)
def lr_sequence(epochs: int, lr: float = 1e-4) -> tuple[float, ...]:
    """lr_e for e = 0..epochs-1, as the reference's scheduler produces them."""
    holder = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([holder], lr=lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=max(epochs, 1),
                                                       eta_min=lr * 0.01)
    out = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for _ in range(epochs):
            out.append(float(opt.param_groups[0]["lr"]))
            opt.step()  # no grads: a no-op that keeps the scheduler's order check quiet
            sched.step()
    return tuple(out)


def adam_table(epochs: int, lr: float = 1e-4) -> np.ndarray:
    """[epochs, 2] float32: (lr_e / bias_correction1, sqrt(bias_correction2))."""
    tab = np.zeros((epochs, 2), dtype=np.float32)
    for e, lr_e in enumerate(lr_sequence(epochs, lr)):
        step = float(e + 1)
        bc1 = 1 - BETA1 ** step
        bc2 = 1 - BETA2 ** step
        tab[e, 0] = lr_e / bc1
        tab[e, 1] = bc2 ** 0.5
    return tab
