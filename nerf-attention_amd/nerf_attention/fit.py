"""Sweep driver: fit SIRENs to an extracted KV cache — `python -m nerf_attention.fit`.

Drop-in for the reference driver (nerf_attention/fit.py:20-196): same
signature, CLI flags, selection rules, record order, stdout lines,
`fit_results.json` schema (19 keys, indent=2) and `{name}_model.pt`
checkpoints for the medium architecture.

What changes is HOW the fits run.  The reference trains them one after
another (fit.py:54-76).  Here every model is first initialised on the host in
the reference's loop order — init is the only consumer of the torch RNG, so
each fit gets exactly the parameters the sequential reference would give it —
and then ALL fits are trained together on the HIP engine (grouped by width,
one stream per group, optionally over several GPUs).  Each fit's stdout block
(the `[k/N] name` line, its probe lines and the `-> CosSim` line,
fit.py:66-86) is printed as soon as its group has finished and every fit
before it in the reference's record order has been printed, so stdout keeps
the reference's order; a line per finished group goes to stderr.

`train_time_seconds` (siren.py:96,117: the wall clock of the fit's epoch
loop) is measured: the device-clock interval of the group that trained the
fit, from before its first launch to after its last (engine.FitOutput).  A
lone fit gets its own loop time; fits of concurrent groups overlap, so a
sweep's records sum to more than its wall clock (printed at the end by the
CLI).

With `gpus=N` (or `--gpus N`) the fits are farmed over N GPUs, one worker
process per GPU (farm.run_farm), the same one-process-per-GPU design as
bench.py.
"""

from __future__ import annotations

import argparse
import os
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

from . import engine
from .siren import SIREN, _finish, init_flat, probe_line, uninitialised
from .types import CONFIG_WIDE, CONFIGS_FULL, CONFIGS_QUICK, FitResult, KVMetadata, SIRENConfig


def select_fits(metadata: KVMetadata, quick: bool, select: str = 'sweep', configs=None):
    """(layers, heads_per_layer, configs) — reference fit.py:39-48.

    Extensions (default off = reference behaviour): select='all' takes every
    layer and every KV head (BASELINE config 4's "all layers×heads" scan,
    SURVEY §3.3); `configs` (names) restricts the architecture list, e.g.
    ['medium'] or ['wide'] for CONFIG_WIDE."""
    nl = metadata.num_layers
    if quick:
        layers = [0, nl // 2, nl - 1]
        heads, cfgs = 1, CONFIGS_QUICK
    else:
        layers = [0, nl // 4, nl // 2, 3 * nl // 4, nl - 1]
        heads, cfgs = min(metadata.num_kv_heads, 4), CONFIGS_FULL
    if select == 'all':
        layers, heads = list(range(nl)), metadata.num_kv_heads
    elif select != 'sweep':
        raise ValueError(f"select must be 'sweep' or 'all', got {select!r}")
    if configs:
        known = {c.name: c for c in CONFIGS_FULL + [CONFIG_WIDE]}
        cfgs = [known[n] for n in configs]
    layers = sorted(set(l for l in layers if l < nl))
    return layers, heads, cfgs


def sweep_plan(layers, heads, configs, load_layer):
    """Fits in the reference record order layer → head → (key, value) → config
    (fit.py:54-65).  load_layer(l) returns {'keys','values'} or None (skip)."""
    plan, skipped = [], []
    for layer in layers:
        data = load_layer(layer)
        if data is None:
            skipped.append(layer)
            continue
        for head in range(heads):
            for kv_type, tensor in (('key', data['keys'][head]), ('value', data['values'][head])):
                for cfg in configs:
                    plan.append((f"L{layer}_H{head}_{kv_type}_{cfg.name}", layer, head, kv_type,
                                 cfg, tensor))
    return plan, skipped


def _host_plan(plan, epochs: int, log_every: int, on_ready=None):
    """device='cpu' (BASELINE config 1): the fits one after the other in eager
    PyTorch, each model initialised right before its fit as the reference
    does (fit.py:70-76); on_ready(k, result, probes) after each."""
    from .host_fit import fit_on_host
    out = []
    for k, (_name, _l, _h, _kv, cfg, tensor) in enumerate(plan):
        m = SIREN(cfg, out_features=int(tensor.shape[1]))
        probes = []
        res = fit_on_host(tensor, cfg, m, epochs, 1e-4, log_every,
                          lambda *probe: probes.append(probe))
        out.append((res, probes))
        if on_ready:
            on_ready(k, res, probes)
    return out


def _devices(device, gpus) -> list:
    """Device indices to train on.  One GPU: the requested device.  Several:
    one farm worker process per GPU (farm.run_farm); counted without
    initialising HIP in this process (the workers are started first)."""
    if not gpus or gpus <= 1:
        return [engine.resolve_device(device).index]
    if torch.device(device).type != 'cuda':
        return [engine.resolve_device(device).index]     # raises: no CPU path
    have = torch.cuda.device_count()
    if have < gpus:
        raise engine._native.NerfhipError(f"--gpus {gpus} but only {have} HIP device(s) visible")
    return list(range(gpus))


def _stream_ok(plan, epochs, devices, log_every, precision) -> bool:
    """The streaming path needs one device, one memory wave and at least one
    fit (an empty selection — every layer file missing — takes train_plan,
    which returns no results, as the reference's loop does)."""
    if not plan:
        return False
    if devices is None or len(devices) != 1 or os.environ.get("NERFHIP_STREAM", "1") == "0":
        return False
    need = 0
    for _n, _l, _h, _kv, cfg, tensor in plan:
        proto = engine.FitSpec(target=tensor, config=cfg, init=None)
        need += engine.fit_device_bytes(proto, epochs, log_every, precision)
    return need <= engine.memory_budget(devices[0])


def train_plan_streaming(plan, epochs: int, device: int, log_every: int, precision=None,
                         on_ready=None):
    """train_plan with the host work overlapped (engine.StreamingJob): the
    inits are drawn in plan order (the reference's RNG order; siren.init_flat,
    bit-identical to building each SIREN) and each group of same-width fits
    starts training the moment its last init exists; every finished group is
    copied back and turned into FitResults while the others still train, and
    on_ready(k, result, probes) is called for each of its fits (fit_kv_cache
    prints and saves from there).  train_time_seconds: the group's measured
    device time (engine.FitOutput)."""
    protos = [engine.FitSpec(target=tensor, config=cfg, init=None)
              for _n, _l, _h, _kv, cfg, tensor in plan]
    job = engine.StreamingJob(protos, epochs, log_every=log_every, device=device,
                              precision=precision)
    for k, (_name, _l, _h, _kv, cfg, tensor) in enumerate(plan):
        job.add(k, engine.FitSpec(target=tensor, config=cfg,
                                  init=init_flat(cfg, int(tensor.shape[1]))))
    results = [None] * len(plan)
    dev = torch.device('cuda', device)
    for n, gi in enumerate(job.finished(), 1):
        done = job.outputs(gi)
        for k, o in done:
            n_rows, d = int(plan[k][5].shape[0]), int(plan[k][5].shape[1])
            m = uninitialised(plan[k][4], d, dev)
            m.load_flat_parameters(o.params)
            m.eval()
            results[k] = (_finish(m, plan[k][4], o, n_rows, d), o.probes)
        if done:
            o = done[0][1]
            print(f"[nerf-attention-amd] group {n}/{len(job.plan)} done: {len(done)} x "
                  f"{plan[done[0][0]][4].name if len({plan[k][4].name for k, _ in done}) == 1 else 'mixed'}"
                  f" (W={plan[done[0][0]][4].hidden_features}) in {o.group_seconds:.2f}s device time",
                  file=sys.stderr, flush=True)
        if on_ready:
            for k, _o in done:
                on_ready(k, *results[k])
    return results


def train_plan(plan, epochs: int, devices, log_every: int, precision=None, on_ready=None):
    """Draw every model's init in plan order (the reference's RNG order;
    siren.init_flat), then train them all on the engine; the returned models
    are built storage-only (siren.uninitialised) around the trained parameters.  Returns [(FitResult, probes)]."""
    specs = [engine.FitSpec(target=tensor, config=cfg, init=init_flat(cfg, int(tensor.shape[1])))
             for _name, _l, _h, _kv, cfg, tensor in plan]
    outs = engine.run_fits(specs, epochs, log_every=log_every, devices=devices,
                           precision=precision)
    results = []
    for (name, _l, _h, _kv, cfg, tensor), o in zip(plan, outs):
        m = uninitialised(cfg, int(tensor.shape[1]), torch.device('cuda', o.device))
        m.load_flat_parameters(o.params)
        m.eval()
        results.append((_finish(m, cfg, o, int(tensor.shape[0]), int(tensor.shape[1])),
                        o.probes))
    if on_ready:
        for k, (res, probes) in enumerate(results):
            on_ready(k, res, probes)
    return results


class _Report:
    """The per-fit output of fit_kv_cache (fit.py:54-86) in the reference's
    order — layer by layer, a missing layer's 'Skipping' line in its place,
    then the layer's fits in plan order — each block (`[k/N] name`, the probe
    lines, `-> CosSim`), record and medium checkpoint emitted the moment its
    fit has finished and everything before it has been emitted."""

    def __init__(self, plan, layers, skipped, total, epochs, output_dir):
        self.plan, self.total, self.epochs, self.output_dir = plan, total, epochs, output_dir
        self.order = []
        for layer in layers:
            if layer in skipped:
                self.order.append(('skip', layer))
            else:
                self.order += [('fit', k) for k, p in enumerate(plan) if p[1] == layer]
        self.ready, self.at, self.count, self.records = {}, 0, 0, []
        self._flush()

    def fit_done(self, k, res, probes):
        self.ready[k] = (res, probes)
        self._flush()

    def _flush(self):
        while self.at < len(self.order):
            kind, v = self.order[self.at]
            if kind == 'skip':
                print(f"  Skipping layer {v} (not found)")
            else:
                if v not in self.ready:
                    return
                res, probes = self.ready.pop(v)
                name, layer, head, kv_type, cfg, _t = self.plan[v]
                self.count += 1
                print(f"\n[{self.count}/{self.total}] {name}")
                for ep, nm, rm, cs in probes:
                    print(probe_line(ep, self.epochs, nm, rm, cs))
                record = _result_to_record(name, layer, head, kv_type, res)
                self.records.append(record)
                if cfg.name == 'medium':
                    _save_model(self.output_dir, name, res, record)
                print(f"  -> CosSim: {res.final_cosine_mean:.4f} | "
                      f"Compress: {res.compression_ratio:.1f}x | "
                      f"Time: {res.train_time_seconds:.1f}s", flush=True)
            self.at += 1

    def finish(self) -> list:
        self._flush()
        if self.at != len(self.order):
            raise RuntimeError(f"fit {self.order[self.at][1]} never reported")
        return self.records


def fit_kv_cache(
    kv_dir: Path,
    output_dir: Path,
    epochs: int = 5000,
    device: str = 'cuda',
    quick: bool = False,
    *,
    gpus: int | None = None,
    select: str = 'sweep',
    configs=None,
    precision: str | None = None,
) -> list[dict]:
    """Fit SIRENs to an extracted KV cache and record metrics (fit.py:20-92).
    Extensions: `gpus` farms the fits over this many local GPUs; `select` and
    `configs` widen / narrow the selection (see select_fits); `precision` picks
    the GEMM arithmetic (engine.PRECISIONS)."""
    kv_dir, output_dir = Path(kv_dir), Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    with open(kv_dir / 'metadata.json') as f:
        metadata = KVMetadata.from_dict(json.load(f))

    print(f"KV Cache: {metadata.num_layers} layers x {metadata.num_kv_heads} heads")
    print(f"Per tensor: ({metadata.seq_len}, {metadata.head_dim}) = "
          f"{metadata.seq_len * metadata.head_dim * 2 / 1024:.1f} KB (float16 baseline)")
    print(f"Device: {device}, Epochs: {epochs}")

    host = torch.device(device).type == 'cpu'
    devices = None if host else _devices(device, gpus)
    layers, heads, configs = select_fits(metadata, quick, select, configs)
    total = len(layers) * heads * 2 * len(configs)

    def load_layer(layer):
        p = kv_dir / f'layer_{layer:02d}.pt'
        if not p.exists():
            return None
        return torch.load(p, map_location='cpu', weights_only=True)

    plan, skipped = sweep_plan(layers, heads, configs, load_layer)
    log_every = max(epochs // 5, 100)
    report = _Report(plan, layers, skipped, total, epochs, output_dir)
    if host:
        _host_plan(plan, epochs, log_every, on_ready=report.fit_done)
    elif _stream_ok(plan, epochs, devices, log_every, precision):
        train_plan_streaming(plan, epochs, devices[0], log_every, precision,
                             on_ready=report.fit_done)
    else:
        train_plan(plan, epochs, devices, log_every=log_every, precision=precision,
                   on_ready=report.fit_done)
    all_results = report.finish()

    with open(output_dir / 'fit_results.json', 'w') as f:
        json.dump(all_results, f, indent=2)
    _print_summary(all_results, layers)
    return all_results


RECORD_KEYS = ('name', 'layer', 'head', 'kv_type', 'config_name', 'hidden_features',
               'hidden_layers', 'omega_0', 'final_mse', 'final_cosine_mean',
               'final_cosine_min', 'final_cosine_std', 'compression_ratio', 'raw_size_bytes',
               'siren_size_bytes', 'train_time_seconds', 'num_parameters', 'seq_len', 'd_head')


def _result_to_record(name: str, layer: int, head: int, kv_type: str,
                      result: FitResult) -> dict:
    """The 19-key JSON record of fit.py:95-118, in that key order."""
    c = result.config
    values = (name, layer, head, kv_type, c.name, c.hidden_features, c.hidden_layers, c.omega_0,
              result.final_mse, result.final_cosine_mean, result.final_cosine_min,
              result.final_cosine_std, result.compression_ratio, result.raw_size_bytes,
              result.siren_size_bytes, result.train_time_seconds, result.num_parameters,
              result.seq_len, result.d_head)
    return dict(zip(RECORD_KEYS, values))


def _save_model(output_dir: Path, name: str, result: FitResult, record: dict) -> None:
    """{name}_model.pt as fit.py:121-137 writes it (read by evaluate.py:34-45)."""
    c = result.config
    ckpt = {
        'model_state': result.model.state_dict(),
        'config': {'hidden_features': c.hidden_features, 'hidden_layers': c.hidden_layers,
                   'omega_0': c.omega_0, 'name': c.name, 'out_features': result.d_head},
        'target_mean': result.target_mean,
        'target_std': result.target_std,
        'metrics': record,
    }
    torch.save(ckpt, output_dir / f'{name}_model.pt')


def _print_summary(all_results: list[dict], layers_to_fit: list[int]) -> None:
    """Results table and per-architecture / K-V / layer means (fit.py:140-180)."""
    bar = '=' * 80
    print(f"\n{bar}\nRESULTS SUMMARY\n{bar}")
    print(f"{'Name':<35} {'CosSim':>8} {'MSE':>10} {'Compress':>10} {'Time':>8}")
    print(f"{'-' * 35} {'-' * 8} {'-' * 10} {'-' * 10} {'-' * 8}")
    for r in sorted(all_results, key=lambda x: x['final_cosine_mean'], reverse=True):
        print(f"{r['name']:<35} {r['final_cosine_mean']:>8.4f} "
              f"{r['final_mse']:>10.6f} {r['compression_ratio']:>9.1f}x "
              f"{r['train_time_seconds']:>7.1f}s")
    print(f"\n{bar}\nKEY FINDINGS\n{bar}")
    for cn in sorted({r['config_name'] for r in all_results}):
        cr = [r for r in all_results if r['config_name'] == cn]
        print(f"  {cn:<10}: avg CosSim={np.mean([r['final_cosine_mean'] for r in cr]):.4f}, "
              f"avg Compression={np.mean([r['compression_ratio'] for r in cr]):.1f}x")
    keys = [r['final_cosine_mean'] for r in all_results if r['kv_type'] == 'key']
    vals = [r['final_cosine_mean'] for r in all_results if r['kv_type'] == 'value']
    if keys and vals:
        k_avg, v_avg = np.mean(keys), np.mean(vals)
        print(f"\n  Keys avg CosSim:   {k_avg:.4f}")
        print(f"  Values avg CosSim: {v_avg:.4f}")
        diff = v_avg - k_avg
        if diff > 0.01:
            print("  -> Values compress better (smoother signal)")
        elif diff < -0.01:
            print("  -> Keys compress better (stronger positional structure)")
        else:
            print("  -> Similar compressibility")
    for layer in layers_to_fit:
        lr = [r['final_cosine_mean'] for r in all_results
              if r['layer'] == layer and r['config_name'] == 'medium']
        if lr:
            print(f"  Layer {layer:2d} (medium): avg CosSim={np.mean(lr):.4f}")


def main() -> None:
    # one HIP hardware queue per group stream (before the runtime initialises;
    # unset or HIP's default of 4 is raised to 8, any other value wins; see bench.py)
    if (os.environ.get("NERFHIP_KEEP_HW_QUEUES") != "1"
            and os.environ.get("GPU_MAX_HW_QUEUES", "").strip() in ("", "4")):
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    parser = argparse.ArgumentParser(description='Fit SIRENs to KV cache')
    parser.add_argument('--kv_dir', type=str, default='results/kv_cache')
    parser.add_argument('--output_dir', type=str, default='results/fits')
    parser.add_argument('--epochs', type=int, default=5000)
    parser.add_argument('--device', type=str, default='cuda')
    parser.add_argument('--quick', action='store_true')
    parser.add_argument('--gpus', type=int, default=1,
                        help='farm the fits over this many local GPUs (extension)')
    parser.add_argument('--seed', type=int, default=None,
                        help='torch.manual_seed before the sweep (extension; the reference '
                             'is unseeded)')
    parser.add_argument('--select', choices=['sweep', 'all'], default='sweep',
                        help="'all' = every layer x every KV head (extension)")
    parser.add_argument('--configs', type=str, default=None,
                        help='comma-separated architecture names, e.g. medium or wide (extension)')
    parser.add_argument('--precision', choices=['bf16x3', 'fp32'], default=None,
                        help='GEMM arithmetic (extension; default bf16x3 = exact 3-way bf16 '
                             'split, fp32-class; fp32 = f32 MFMA)')
    args = parser.parse_args()
    # The reference's CLI falls back to the CPU when no GPU is present
    # (fit.py:192-194).  The CPU run is this package's explicit host path
    # (host_fit.py: eager PyTorch, the reference arithmetic); a HIP request made
    # through the Python API (fit_siren / fit_kv_cache with device='cuda') still
    # raises on such a host.  device_count() counts without initialising HIP,
    # so a later --gpus farm can still start its workers cleanly.
    if args.device == 'cuda' and torch.cuda.device_count() == 0:
        print("CUDA not available, falling back to CPU")
        args.device = 'cpu'
    if args.seed is not None:
        torch.manual_seed(args.seed)
    t0 = time.time()
    fit_kv_cache(Path(args.kv_dir), Path(args.output_dir), args.epochs, args.device,
                 args.quick, gpus=args.gpus, select=args.select,
                 configs=args.configs.split(',') if args.configs else None,
                 precision=args.precision)
    print(f"\n[nerf-attention-amd] sweep wall clock {time.time() - t0:.2f}s")


if __name__ == '__main__':
    main()
