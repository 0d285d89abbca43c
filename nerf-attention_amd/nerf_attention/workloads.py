"""The benchmark workloads of BASELINE.json, on the synthetic KV stand-in.

Real Llama-3.1-8B KV cannot be produced offline, so the
sweep runs on the reference's own synthetic generator at the Llama shape
(32 layers × 8 KV heads × seq_len × 128), which `synthetic.kv_slice`
reproduces bit-for-bit.
"""

from __future__ import annotations

import torch

from .engine import FitSpec
from .fit import select_fits, sweep_plan
from .siren import init_flat
from .synthetic import kv_cache
from .types import KVMetadata

LLAMA_SHAPE = dict(num_layers=32, num_kv_heads=8, head_dim=128)


def sweep_280(seq_len: int = 2048, seed: int | None = 0, quick: bool = False,
              select: str = 'sweep', configs=None):
    """(plan, specs) of the full 280-fit sweep (fit.py:43-47 selection, reference
    record order).  With `seed` set, torch.manual_seed(seed) precedes the inits,
    which are drawn in the reference's loop order.
    select='all', configs=['medium'] gives BASELINE config 4's per-seq-len scan
    (32 layers × 8 heads × K/V = 512 fits)."""
    meta = KVMetadata(model_name='synthetic', seq_len=seq_len, actual_tokens=seq_len,
                      **LLAMA_SHAPE)
    layers, heads, configs = select_fits(meta, quick, select, configs)
    # every slice the selection reads, in one request (a process pool when large)
    cache = kv_cache(layers, seq_len, LLAMA_SHAPE['num_layers'], LLAMA_SHAPE['num_kv_heads'],
                     LLAMA_SHAPE['head_dim'], heads=range(heads))

    def load(layer):
        return cache[layer]

    plan, _ = sweep_plan(layers, heads, configs, load)
    if seed is not None:
        torch.manual_seed(seed)
    specs = [FitSpec(target=tensor, config=cfg, init=init_flat(cfg, int(tensor.shape[1])))
             for _name, _l, _h, _kv, cfg, tensor in plan]
    return plan, specs
