"""Deterministic synthetic KV cache — the input format of the fit path.

Restates `extract_kv_cache_synthetic` (reference extract.py:182-259): each
(layer, head) is drawn from its own `np.random.RandomState(layer*H + head)`
(extract.py:207) and each head dimension is a low-frequency base + a
mid-frequency term + layer-sharpened Gaussian spikes + noise for keys, a
sine + noise for values (extract.py:211-234).  The RNG draw order and the
numpy expression forms (and hence dtypes under NEP-50 promotion) are the
reference's, so the tensors are bit-identical — pinned by the SHA-256
fixtures in tests/golden/synthetic.json.

Because every (layer, head) has its own RNG stream, `kv_slice` produces any
single slice without generating the rest (the sweep needs 20 of 256).
"""

from __future__ import annotations

import json
import os
from pathlib import Path

import numpy as np
import torch

from ._synth_core import slice_np
from .types import KVMetadata


def kv_slice(layer: int, head: int, seq_len: int = 2048, num_layers: int = 32,
             num_kv_heads: int = 8, head_dim: int = 128):
    """(keys[seq_len, head_dim], values[seq_len, head_dim]) of one (layer, head)."""
    tt = torch.linspace(0, 1, seq_len).numpy()
    keys = np.empty((seq_len, head_dim), np.float32)
    vals = np.empty((seq_len, head_dim), np.float32)
    slice_np(tt, layer, head, num_layers, num_kv_heads, head_dim, keys, vals)
    return torch.from_numpy(keys), torch.from_numpy(vals)


def _threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", n))))


POOL_MIN_ROWS = 32 * 4096     # slices x seq_len below which one process is faster



def _hip_untouched() -> bool:
    """True while nothing in this process can have created HIP runtime state:
    torch has not initialised its HIP context and the engine library
    (libnerfhip, whose calls initialise HIP on their own) is not loaded.
    Only then may the generator fork its workers; otherwise it spawns fresh
    interpreters.  (torch.cuda.device_count() on ROCm counts through amdsmi
    and does not initialise HIP.)"""
    from . import _native
    return _native._lib is None and not torch.cuda.is_initialized()

def kv_slices(pairs, seq_len: int = 2048, num_layers: int = 32, num_kv_heads: int = 8,
              head_dim: int = 128) -> list:
    """kv_slice for every (layer, head) in `pairs`.  Large requests run on a
    pool of fresh worker processes (the RandomState draws are a sequential
    Python loop per slice, so threads serialise on the GIL): every slice has
    its own RandomState, so the bits do not depend on the split; the workers
    write into one shared-memory buffer."""
    pairs = list(pairs)
    workers = min(_threads(), len(pairs))
    if workers <= 1 or len(pairs) * seq_len < POOL_MIN_ROWS:
        return [kv_slice(l, h, seq_len, num_layers, num_kv_heads, head_dim) for l, h in pairs]
    import mmap
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    from . import _synth_core
    tt = torch.linspace(0, 1, seq_len).numpy()
    shape = (len(pairs), 2, seq_len, head_dim)
    nbytes = int(np.prod(shape)) * 4
    jobs = [(k, l, h) for k, (l, h) in enumerate(pairs)]
    parts = [jobs[w::workers] for w in range(workers)]
    if _hip_untouched():
        # fork: the workers inherit an anonymous shared mapping and write the
        # slices straight into it; the result is a view of it (no copy)
        mm = mmap.mmap(-1, nbytes, flags=mmap.MAP_SHARED)
        _synth_core._SHARED = mm
        try:
            with ProcessPoolExecutor(max_workers=workers,
                                     mp_context=mp.get_context("fork")) as ex:
                for f in [ex.submit(_synth_core.pool_job_fork, shape, tt, part, num_layers,
                                    num_kv_heads) for part in parts]:
                    f.result()
        finally:
            _synth_core._SHARED = None
        out = torch.from_numpy(np.frombuffer(mm, dtype=np.float32).reshape(shape))
    else:
        # this process has HIP state: fresh interpreters — plain child
        # processes running _synth_core.py as a script (numpy only), not a
        # multiprocessing spawn pool, whose start method launches a resource
        # tracker process that outlives the caller (the process BENCH_r04
        # found left at the end) — writing into a memory-mapped file under
        # /dev/shm
        import subprocess
        import sys
        import tempfile
        shm_dir = "/dev/shm" if os.path.isdir("/dev/shm") else None
        fd, path = tempfile.mkstemp(prefix="nerf_synth_", dir=shm_dir)
        specs = []
        try:
            os.ftruncate(fd, nbytes)
            procs = []
            for w, part in enumerate(parts):
                spec = f"{path}.job{w}.json"
                specs.append(spec)
                with open(spec, "w") as f:
                    json.dump({"path": path, "shape": list(shape), "tt": tt.tolist(),
                               "jobs": part, "num_layers": num_layers,
                               "num_kv_heads": num_kv_heads}, f)
                procs.append(subprocess.Popen([sys.executable, _synth_core.__file__, spec]))
            bad = [p.args for p in procs if p.wait() != 0]
            if bad:
                raise RuntimeError(f"synthetic KV worker failed: {bad[0]}")
            buf = np.memmap(path, dtype=np.float32, mode="r", shape=shape)
            out = torch.from_numpy(np.array(buf))
            del buf
        finally:
            os.close(fd)
            os.unlink(path)
            for spec in specs:
                if os.path.exists(spec):
                    os.unlink(spec)
    return [(out[k, 0], out[k, 1]) for k in range(len(pairs))]


def kv_layer(layer: int, seq_len: int = 2048, num_layers: int = 32, num_kv_heads: int = 8,
             head_dim: int = 128, heads=None):
    """{'keys': [H', N, d], 'values': [H', N, d]} for heads (default: all)."""
    heads = range(num_kv_heads) if heads is None else heads
    ks, vs = zip(*kv_slices([(layer, h) for h in heads], seq_len, num_layers, num_kv_heads,
                            head_dim))
    return {'keys': torch.stack(ks), 'values': torch.stack(vs)}


def kv_cache(layers, seq_len: int = 2048, num_layers: int = 32, num_kv_heads: int = 8,
             head_dim: int = 128, heads=None) -> dict:
    """{layer: kv_layer(layer)} for several layers, all slices generated on
    one thread pool (BASELINE config 4 needs 32 x 8 of them per seq_len)."""
    layers = list(layers)
    heads = list(range(num_kv_heads) if heads is None else heads)
    flat = kv_slices([(l, h) for l in layers for h in heads], seq_len, num_layers,
                     num_kv_heads, head_dim)
    out, k = {}, 0
    for l in layers:
        ks, vs = zip(*flat[k:k + len(heads)])
        out[l] = {'keys': torch.stack(ks), 'values': torch.stack(vs)}
        k += len(heads)
    return out


def write_kv_cache(output_dir: Path, seq_len: int = 2048, num_layers: int = 32,
                   num_kv_heads: int = 8, head_dim: int = 128, layers=None) -> KVMetadata:
    """The on-disk cache format (layer_XX.pt + metadata.json, extract.py:
    238-259) for `layers` only (default all), without the progress lines."""
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    layers = range(num_layers) if layers is None else layers
    for layer, data in kv_cache(layers, seq_len, num_layers, num_kv_heads, head_dim).items():
        torch.save(data, output_dir / f'layer_{layer:02d}.pt')
    meta = KVMetadata(model_name='synthetic', num_layers=num_layers, num_kv_heads=num_kv_heads,
                      seq_len=seq_len, head_dim=head_dim, actual_tokens=seq_len)
    with open(output_dir / 'metadata.json', 'w') as f:
        json.dump(meta.to_dict(), f, indent=2)
    return meta


def extract_kv_cache_synthetic(
    seq_len: int = 2048,
    num_layers: int = 32,
    num_kv_heads: int = 8,
    head_dim: int = 128,
    output_dir: Path = Path('results/kv_cache_synthetic'),
) -> KVMetadata:
    """Write layer_XX.pt + metadata.json exactly as extract.py:182-259 does."""
    print("Generating synthetic KV cache...")
    print(f"  {num_layers} layers, {num_kv_heads} heads, seq_len={seq_len}, head_dim={head_dim}")
    meta = write_kv_cache(output_dir, seq_len, num_layers, num_kv_heads, head_dim)
    total_mb = num_layers * num_kv_heads * seq_len * head_dim * 2 * 4 / 1024 / 1024
    print(f"Saved to {output_dir}/ ({total_mb:.1f} MB)")
    return meta
