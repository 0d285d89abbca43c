"""numpy-only core of the synthetic KV generator (no torch import, so pool
workers start fast).  See synthetic.py for what it restates."""

from __future__ import annotations

import numpy as np


def _sharpness(layer: int, num_layers: int) -> float:
    return 1.0 + 2.0 * (layer / max(num_layers - 1, 1))        # extract.py:204


_BUMP = {}


def _bump(width: int) -> np.ndarray:
    """exp(-½(off/max(1, width/2))²) for off = -width..width, each value
    evaluated as the reference evaluates it (one Python-scalar np.exp per
    offset, extract.py:226-228), cached per width (the widths are 1..4)."""
    w = _BUMP.get(width)
    if w is None:
        w = np.array([np.exp(-0.5 * (off / max(1, width / 2)) ** 2)
                      for off in range(-width, width + 1)])
        _BUMP[width] = w
    return w


def _spike_train(rng, seq_len: int, sharp: float) -> np.ndarray:
    """Sparse Gaussian bumps, narrower and more numerous in deeper layers
    (extract.py:219-228).  One slice add per bump: every element receives its
    bumps' contributions in the same order and with the same products
    (amp·weight) as the reference's per-offset loop, so the sum is bitwise
    the same."""
    out = np.zeros(seq_len)
    for _ in range(int(3 * sharp)):
        centre = rng.randint(0, seq_len)
        width = rng.randint(1, max(2, int(5 / sharp)))
        amp = rng.uniform(0.5, 2.0)
        lo, hi = max(centre - width, 0), min(centre + width + 1, seq_len)
        out[lo:hi] += amp * _bump(width)[lo - (centre - width):hi - (centre - width)]
    return out


def slice_np(tt: np.ndarray, layer: int, head: int, num_layers: int, num_kv_heads: int,
             head_dim: int, out_k: np.ndarray, out_v: np.ndarray) -> None:
    """keys / values [seq_len, head_dim] float32 of one (layer, head) into
    out_k / out_v; tt = torch.linspace(0, 1, seq_len) as float32 numpy.

    The RandomState draws run column by column in the reference's order
    (they are inherently sequential); everything else is evaluated once for
    the whole slice as [head_dim, seq_len] arrays with the reference's
    per-element operations and dtypes: the sin/cos arguments are the
    reference's Python-float coefficient rounded to float32 (NEP-50 weak
    scalar) times the float32 positions, the float32 terms are summed first,
    then the float64 spikes and noise, then one cast to float32."""
    rng = np.random.RandomState(layer * num_kv_heads + head)
    sharp = _sharpness(layer, num_layers)
    D, N = head_dim, tt.shape[0]
    c_lo, c_hi, c_mid, phase, c_v = (np.empty((D, 1), np.float32) for _ in range(5))
    spikes, k_noise, v_noise = _scratch((3, D, N), np.float64)
    a32, b32 = _scratch((2, D, N), np.float32, 1)
    for j in range(D):
        f_lo, f_hi = rng.uniform(1, 5), rng.uniform(3, 10)
        c_lo[j], c_hi[j] = 2 * np.pi * f_lo, 2 * np.pi * f_hi
        c_mid[j] = 2 * np.pi * rng.uniform(10, 30)
        phase[j] = rng.uniform(0, 2 * np.pi)
        spikes[j] = _spike_train(rng, N, sharp)
        k_noise[j] = rng.randn(N)
        c_v[j] = 2 * np.pi * rng.uniform(1, 8)
        v_noise[j] = rng.randn(N)
    # keys: ((0.5 sin + 0.3 cos) + 0.2 sin) in float32, + spikes, + 0.1 noise in float64
    np.sin(np.multiply(c_lo, tt, out=a32), out=a32)
    np.multiply(a32, 0.5, out=a32)
    np.cos(np.multiply(c_hi, tt, out=b32), out=b32)
    np.add(a32, np.multiply(b32, 0.3, out=b32), out=a32)
    np.sin(np.add(np.multiply(c_mid, tt, out=b32), phase, out=b32), out=b32)
    np.add(a32, np.multiply(b32, 0.2, out=b32), out=a32)
    np.add(a32, spikes, out=spikes)
    np.add(spikes, np.multiply(k_noise, 0.1, out=k_noise), out=spikes)
    out_k[...] = spikes.T                                    # one rounding to float32
    # values: 0.6 sin in float32, + 0.15 noise in float64
    np.sin(np.multiply(c_v, tt, out=a32), out=a32)
    np.multiply(a32, 0.6, out=a32)
    np.add(a32, np.multiply(v_noise, 0.15, out=v_noise), out=v_noise)
    out_v[...] = v_noise.T


_SCRATCH = {}


def _scratch(shape: tuple, dtype, slot: int = 0) -> np.ndarray:
    """Per-process reusable work arrays (a fresh [128, N] float64 temporary per
    operation costs more in page faults than the arithmetic)."""
    key = (shape, np.dtype(dtype).str, slot)
    a = _SCRATCH.get(key)
    if a is None:
        a = _SCRATCH[key] = np.empty(shape, dtype)
    return a


_SHARED = None      # fork pool: the parent's anonymous shared mapping, inherited


def pool_job_fork(shape: tuple, tt: np.ndarray, jobs: list, num_layers: int,
                  num_kv_heads: int) -> int:
    """Forked worker: like pool_job, into the inherited shared mapping."""
    buf = np.frombuffer(_SHARED, dtype=np.float32).reshape(shape)
    for k, layer, head in jobs:
        slice_np(tt, layer, head, num_layers, num_kv_heads, shape[3], buf[k, 0], buf[k, 1])
    return len(jobs)


def pool_job(path: str, shape: tuple, tt: np.ndarray, jobs: list, num_layers: int,
             num_kv_heads: int) -> int:
    """Worker: fill slots [k] of the shared [n, 2, seq_len, head_dim] float32
    file mapping at `path` (the parent removes it) with slice (layer, head)
    for every (k, layer, head) in jobs."""
    buf = np.memmap(path, dtype=np.float32, mode="r+", shape=shape)
    for k, layer, head in jobs:
        slice_np(tt, layer, head, num_layers, num_kv_heads, shape[3], buf[k, 0], buf[k, 1])
    buf.flush()
    del buf
    return len(jobs)


if __name__ == "__main__":   # a worker process of synthetic.kv_slices (spawn path)
    import json
    import sys
    with open(sys.argv[1]) as f:
        job = json.load(f)
    pool_job(job["path"], tuple(job["shape"]), np.asarray(job["tt"], dtype=np.float32),
             [tuple(j) for j in job["jobs"]], job["num_layers"], job["num_kv_heads"])
