"""The fit farm: packs independent SIREN fits into device groups and runs them
through the HIP engine (include/nerfhip.h) in one asynchronous call.

Reference behaviour being replaced: `fit_kv_cache` calls `fit_siren` once per
(layer, head, K|V, architecture) in a strictly sequential Python loop
(nerf_attention/fit.py:303-319 of the reference = fit.py:54-76), each fit
running its own 2000-iteration eager loop with a host sync per epoch
(siren.py:98-105).  Here:

* fits sharing (device, W, d_head, seq_len) form ONE group = one pair of
  kernel launches per epoch for all of them (hidden_layers and omega_0 may
  differ inside a group: medium/deep/hifreq/lofreq share W = 256);
* every group gets its own HIP stream and the C side interleaves the groups'
  launches epoch by epoch, so the groups run concurrently;
* a FitJob lives on ONE device; several devices mean several processes
  (`run_fits(devices=[0, 1, ...])` hands the fits to `farm.run_farm`, one
  worker process per GPU with its longest-processing-time share on the FLOP
  model of SURVEY §8d; `bench.py` runs one rank per GPU the same way).

There is deliberately no CPU path: a non-CUDA device raises.
"""

from __future__ import annotations

import ctypes
import math
import os
import threading
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native
from .schedule import adam_table
from .types import SIRENConfig


@dataclass
class FitSpec:
    """One fit: the raw KV slice [seq_len, d_head], its architecture and the
    flat initial parameters in state_dict order (siren.py:89)."""
    target: torch.Tensor
    config: SIRENConfig
    init: torch.Tensor


@dataclass
class FitOutput:
    params: torch.Tensor          # flat fp32 [P] on the fit's device (state_dict order)
    target_mean: torch.Tensor     # CPU [1, d]
    target_std: torch.Tensor      # CPU [1, d]
    losses: list                  # per-epoch normalised MSE (siren.py:105)
    row_cos: np.ndarray           # [seq_len] final per-row cosine (siren.py:124)
    row_mse: np.ndarray           # [seq_len] final per-row MSE (siren.py:125)
    final_mse: float              # siren.py:123
    probes: list = field(default_factory=list)  # (epoch, norm_mse, real_mse, cos)
    # the reference's quantity (siren.py:96,117) is the wall clock of the epoch
    # loop that trained this fit.  Here a fit trains inside its group's launches
    # (all fits of a group step together, one kernel pair per epoch), so the
    # measured interval of ITS training is the group's: hipEvents on the
    # group's stream before its first and after its last launch (device clock).
    # A lone fit (fit_siren) gets exactly its own loop time; fits of concurrent
    # groups overlap, so a sweep's records sum to more than its wall clock.
    train_time_seconds: float = 0.0
    flop_share_seconds: float = 0.0   # group time x this fit's share of its group's FLOPs
    group_seconds: float = 0.0
    device: int = 0
    plan: dict = field(default_factory=dict)   # how its group ran (_Group.plan)


def fit_flops(seq_len: int, d_head: int, cfg: SIRENConfig, epochs: int) -> float:
    """Algorithmic FLOPs of one fit: GEMM multiply-adds × 2 of
    forward + backward over `epochs`, plus the final evaluation forward."""
    n, d, w, l = seq_len, d_head, cfg.hidden_features, cfg.hidden_layers
    per_epoch = 6 * n * (l * w * w + w * d) + 4 * n * w
    return float(epochs * per_epoch + 2 * n * (w + l * w * w + w * d))


def fit_bytes(seq_len: int, d_head: int, cfg: SIRENConfig, epochs: int) -> float:
    """Algorithmic HBM bytes of one fit: per epoch the target
    once plus params/m/v read+written (24·P), activations assumed on-chip."""
    p = cfg.num_parameters(d_head)
    return float(epochs * (4 * seq_len * d_head + 24 * p) + 4 * seq_len * d_head)


def lpt_partition(costs: list, n_bins: int) -> list:
    """Longest-processing-time-first assignment of items to bins; returns the
    bin index per item.  Deterministic (ties broken by item index)."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0.0] * n_bins
    out = [0] * len(costs)
    for i in order:
        b = min(range(n_bins), key=lambda k: (load[k], k))
        out[i] = b
        load[b] += costs[i]
    return out


def resolve_device(device) -> torch.device:
    dev = torch.device(device)
    if dev.type != "cuda":
        raise _native.NerfhipError(
            f"the MI355X engine needs a HIP device (device={device!r}); there is no CPU "
            "fallback on the engine path (only fit_siren/fit_kv_cache take an explicit "
            "device='cpu', host_fit.py)")
    if not torch.cuda.is_available():
        raise _native.NerfhipError("no HIP device visible (torch.cuda.is_available() is False)")
    return torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())


SPLIT_MAX_FITS = 8   # groups below this size split the gradient reduction (grad_partial)
# ... but only while the fused one-pass grid (one workgroup per weight tile and
# fit) stays under SPLIT_MIN_TILES workgroups: 5 large fits (220 tiles) train
# faster fused (parameter kernel 0.17 -> 0.14 ms, 8-rank share prediction
# 168 -> 185 fits/s), 5 small fits (20 tiles) 3.5x slower fused
# (profiles/r02/split_probe.log)
SPLIT_MIN_TILES = 128
# FitJob.launch: one launcher thread per group (each group's enqueue blocks on
# its own stream's queue depth only) instead of one thread interleaving the
# groups epoch by epoch
LAUNCH_THREADS = os.environ.get("NERFHIP_LAUNCH_THREADS", "0") == "1"


def wants_split(n_fits: int, W: int, D: int, L_max: int, grad_split: int) -> bool:
    """Whether a group of this shape gets the split-K workspace (grad_partial):
    under SPLIT_MAX_FITS fits, with a fused parameter grid under
    SPLIT_MIN_TILES workgroups, and row slices available (grad_split > 1).
    A function of the group's own shape only — not of how many other groups
    train beside it on the device (round 5's engine.split_allowed, removed in
    round 6: DESIGN.md §13) — so a fit's numerics are the same in every job
    that forms the same group (farm worker or single process).
    NERFHIP_SPLIT_MAX_FITS caps the group size (0 = never; any setting also
    lifts the SPLIT_MIN_TILES condition, diagnostics)."""
    env = os.environ.get("NERFHIP_SPLIT_MAX_FITS")
    split_max = int(env) if env is not None else SPLIT_MAX_FITS
    small = n_fits * param_tiles(W, D, L_max) < SPLIT_MIN_TILES
    return (n_fits < min(split_max, SPLIT_MAX_FITS) and grad_split > 1
            and (small or env is not None))


def param_tiles(W: int, D: int, L: int) -> int:
    """Workgroups of one fit's parameter step (nerfhip.hip ParamsCfg::tiles)."""
    T = min(W, 128)
    nt = W // T
    return L * nt * nt + (D // min(D, T)) * nt + W // 64

# GEMM arithmetic of the engine (include/nerfhip.h nerfhip_precision):
#   "fp32"   exact fp32 MFMA (v_mfma_f32_*_f32), the reference's arithmetic;
#   "bf16x3" fp32 operands split exactly into three bf16 parts, six bf16 MFMA
#            products per pair, fp32 accumulation: fp32-class accuracy at 2.7x
#            the matrix-core rate.
PRECISIONS = tuple(_native.PRECISIONS)
DEFAULT_PRECISION = os.environ.get("NERFHIP_PRECISION", "bf16x3")


def check_precision(precision):
    p = DEFAULT_PRECISION if precision is None else precision
    if p not in _native.PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {precision!r}")
    return p


class _Group:
    """Device buffers + descriptor of one (device, W, d, seq_len) group."""

    def __init__(self, members, specs, epochs, lr, log_every, device, split=True,
                 precision="fp32", priority=0):
        self.members = members
        self.precision = precision
        cfgs = [specs[i].config for i in members]
        t0 = specs[members[0]].target
        self.N, self.D = int(t0.shape[0]), int(t0.shape[1])
        self.W = cfgs[0].hidden_features
        self.L = [c.hidden_layers for c in cfgs]
        self.L_max = max(self.L)
        self.epochs = epochs
        self.log_every = log_every if (log_every > 0 and epochs // log_every > 0) else 0
        self.n_probe = epochs // self.log_every if self.log_every else 0
        self.device = device
        s = _native.group_sizes(self.W, self.D, self.N, self.L_max, epochs)
        self.sizes = s
        n, n_pad = len(members), int(s.n_pad)
        self.n, self.n_pad = n, n_pad
        dev = torch.device("cuda", device)
        f32 = dict(dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            # (high priority for the light W=64/128 groups: +3 % on one box, ±0 on
            # another — box-to-box spread is ±2 %; not adopted)
            self.stream = torch.cuda.Stream(device=dev, priority=priority)
            self.stream.wait_stream(torch.cuda.current_stream(dev))  # callers' prior work
            self.ev_start = torch.cuda.Event(enable_timing=True)
            self.ev_end = torch.cuda.Event(enable_timing=True)
        # uploads and allocations on the group's own stream: a copy on the
        # default stream would queue behind whatever other groups keep the
        # device busy with (StreamingJob builds groups while others train)
        with torch.cuda.stream(self.stream):
            self._build(members, specs, lr, dev, f32, cfgs, s, split, precision)

    def _build(self, members, specs, lr, dev, f32, cfgs, s, split, precision):
        n, n_pad, epochs = self.n, self.n_pad, self.epochs
        # packing (the reference's H2D copies, siren.py:82-89): on the host and
        # one copy per buffer when the inputs are host tensors, directly on the
        # device when the caller already holds them there (torch.ops.nerfhip)
        on_dev = all(specs[i].target.device == dev and specs[i].init.device == dev
                     for i in members)
        pack = dict(dtype=torch.float32, device=dev if on_dev else "cpu")
        pos = torch.zeros(n_pad, **pack)
        pos[:self.N] = torch.linspace(0, 1, self.N)
        tgt = torch.zeros(n, n_pad, self.D, **pack)
        prm = torch.zeros(n, int(s.params), **pack)
        for k, i in enumerate(members):
            sp = specs[i]
            if tuple(sp.target.shape) != (self.N, self.D):
                raise ValueError("all fits of a group must share (seq_len, d_head)")
            tgt[k, :self.N] = sp.target.detach().to(tgt.device, torch.float32)
            p = sp.init.detach().to(prm.device, torch.float32).reshape(-1)
            if p.numel() != sp.config.num_parameters(self.D):
                raise ValueError(f"init has {p.numel()} params, expected "
                                 f"{sp.config.num_parameters(self.D)}")
            prm[k, :p.numel()] = p
        self.layers = torch.tensor(self.L, dtype=torch.int32, device=dev)
        self.omega = torch.tensor([c.omega_0 for c in cfgs], **f32)
        self.pos = pos.to(dev)
        self.target = tgt.to(dev)
        self.params_init = prm.to(dev)
        self.params = self.params_init.clone()
        self.sched = torch.from_numpy(adam_table(epochs, lr)).to(dev) if epochs > 0 \
            else torch.zeros(1, 2, **f32)
        self.target_norm = torch.empty(n, n_pad, self.D, **f32)
        self.mean = torch.empty(n, self.D, **f32)
        self.std = torch.empty(n, self.D, **f32)
        self.params_t = torch.empty(n, int(s.params_t), **f32)
        self.adam_m = torch.empty(n, int(s.params), **f32)
        self.adam_v = torch.empty(n, int(s.params), **f32)
        self.scratch = torch.empty(n, int(s.scratch), **f32)
        self.loss_partial = torch.empty(n, max(int(s.loss_partial), 1), **f32)
        self.eval_y = torch.empty(n, n_pad, self.D, **f32)
        self.row_cos = torch.empty(n, n_pad, **f32)
        self.row_sq = torch.empty(n, n_pad, **f32)
        # groups of < SPLIT_MAX_FITS fits reduce the weight gradient in row
        # slices (nerfhip.h grad_partial); the sweep's groups never need it
        self.grad_partial = torch.empty(n, int(s.grad_partial), **f32) \
            if split and wants_split(n, self.W, self.D, self.L_max, int(s.grad_split)) else None
        self.wsplit = torch.empty(n, int(s.wsplit), dtype=torch.int16, device=dev) \
            if precision == "bf16x3" else None
        if self.n_probe:
            self.probe_y = torch.empty(n, self.n_probe, n_pad, self.D, **f32)
            self.probe_row_cos = torch.empty(n, self.n_probe, n_pad, **f32)
            self.probe_row_sq = torch.empty(n, self.n_probe, n_pad, **f32)
        else:
            self.probe_y = self.probe_row_cos = self.probe_row_sq = None

        ptr = lambda t: None if t is None else t.data_ptr()
        self.desc = _native.NerfhipGroup(
            W=self.W, D=self.D, N=self.N, n_fits=n, L_max=self.L_max, epochs=epochs,
            log_every=self.log_every, device=self.device, precision=_native.PRECISIONS[precision],
            fit_layers=ptr(self.layers), fit_omega=ptr(self.omega), positions=ptr(self.pos),
            target=ptr(self.target), target_norm=ptr(self.target_norm), mean=ptr(self.mean),
            std=ptr(self.std), params=ptr(self.params), params_t=ptr(self.params_t),
            adam_m=ptr(self.adam_m), adam_v=ptr(self.adam_v), scratch=ptr(self.scratch),
            sched=ptr(self.sched), loss_partial=ptr(self.loss_partial),
            probe_y=ptr(self.probe_y), eval_y=ptr(self.eval_y), row_cos=ptr(self.row_cos),
            row_sq=ptr(self.row_sq), probe_row_cos=ptr(self.probe_row_cos),
            probe_row_sq=ptr(self.probe_row_sq), grad_partial=ptr(self.grad_partial),
            wsplit=ptr(self.wsplit))

    def plan(self) -> dict:
        """How the engine runs this group's epoch (nerfhip_group_plan): the row
        variant ('regular' / 'ksplit'), the gradient row slices, the grids and
        the launches per epoch."""
        p = _native.NerfhipPlan()
        _native.check(_native.load().nerfhip_group_plan(ctypes.byref(self.desc), ctypes.byref(p)))
        return {"rows_variant": _native.ROWS_VARIANTS[p.rows_variant], "grad_split": p.grad_split,
                "rows_workgroups": p.rows_workgroups, "params_workgroups": p.params_workgroups,
                "launches_per_epoch": p.launches_per_epoch}

    def outputs(self, specs, group_seconds):
        N, D, n = self.N, self.D, self.n
        numel = float(N * D)
        E = self.epochs
        if E > 0:
            lp = self.loss_partial[:, :E * (self.n_pad // 16)].view(n, E, self.n_pad // 16)
            losses = (lp.double().sum(-1) / numel).float().cpu().numpy()
        else:
            losses = np.zeros((n, 0), np.float32)
        row_cos = self.row_cos[:, :N].cpu().numpy()
        row_sq = self.row_sq[:, :N].cpu()
        final_mse = (row_sq.double().sum(-1) / numel).float().numpy()
        row_mse = (row_sq / D).numpy()
        mean = self.mean.cpu()
        std = self.std.cpu()
        if self.n_probe:
            p_cos = torch.from_numpy(self.probe_row_cos[:, :, :N].cpu().numpy())
            p_sq = self.probe_row_sq[:, :, :N].cpu().double().sum(-1) / numel
            p_cos_mean = p_cos.mean(-1)
        flops = [fit_flops(N, D, specs[i].config, E) for i in self.members]
        tot = sum(flops) or 1.0
        plan = self.plan()
        outs = []
        for k, i in enumerate(self.members):
            P = specs[i].config.num_parameters(D)
            probes = []
            for q in range(self.n_probe):
                ep = (q + 1) * self.log_every
                probes.append((ep, float(losses[k, ep - 1]), float(np.float32(p_sq[k, q])),
                               float(p_cos_mean[k, q])))
            outs.append(FitOutput(
                params=self.params[k, :P], target_mean=mean[k].view(1, D).clone(),
                target_std=std[k].view(1, D).clone(),
                losses=[float(x) for x in losses[k]], row_cos=row_cos[k].copy(),
                row_mse=row_mse[k].copy(), final_mse=float(final_mse[k]), probes=probes,
                train_time_seconds=group_seconds,
                flop_share_seconds=group_seconds * flops[k] / tot,
                group_seconds=group_seconds, device=self.device, plan=dict(plan)))
        return outs


GROUP_MAX = 40


def _chunks(members: list, cap: int) -> list:
    """Split `members` into ceil(len/cap) chunks whose sizes are multiples of
    8 (the last one takes the remainder); cap <= 0 keeps one chunk."""
    n = len(members)
    k = -(-n // cap) if cap > 0 else 1
    octets, rem = divmod(n, 8)
    if k <= 1 or octets < k:
        return [members]
    sizes = [8 * (octets // k + (1 if j < octets % k else 0)) for j in range(k)]
    sizes[-1] += rem
    out, at = [], 0
    for z in sizes:
        out.append(members[at:at + z])
        at += z
    return out


XCDS = 8          # map_block (nerfhip.hip): fit k of a group of >= 8 runs on XCD k mod 8


def xcd_order(members: list, costs: list) -> list:
    """Permute one group's members so that every XCD carries the same work.

    The kernels map fit k of a group (of at least 8 fits) to XCD k mod 8
    (nerfhip.hip map_block: all tiles of a fit share an XCD's L2).  So the
    position of a fit in its group decides its XCD, and a group laid out in
    reference order puts every fit of a periodic pattern on the same XCDs —
    in the sweep's W = 256 group (medium, deep, hifreq, lofreq repeating) all
    deep fits had k = 1 mod 4, i.e. XCDs 1 and 5, which then held 1.4x the
    work of the others.  Here: longest-first assignment of the
    fits to the 8 XCD classes, each class holding exactly as many fits as
    the positions k = x, x+8, ... that exist in a group of this size; then
    fit j of class x goes to position x + 8j.  A fit's arithmetic does not
    depend on its position (bitwise, test_xcd_order_bitwise), only the
    placement changes."""
    n = len(members)
    if n < XCDS:
        return list(members)
    slots = [len(range(x, n, XCDS)) for x in range(XCDS)]
    bins = [[] for _ in range(XCDS)]
    load = [0.0] * XCDS
    for i in sorted(members, key=lambda i: (-costs[i], i)):
        x = min((x for x in range(XCDS) if len(bins[x]) < slots[x]), key=lambda x: (load[x], x))
        bins[x].append(i)
        load[x] += costs[i]
    out = [None] * n
    for x, b in enumerate(bins):
        for j, i in enumerate(sorted(b)):
            out[x + XCDS * j] = i
    return out


CHUNK_POLICIES = ("depth", "mixed", "spec")


def plan_groups(specs: list, device: int) -> list:
    """[(device, [spec indices])] — fits grouped by (W, d, seq_len), large
    groups chunked, every chunk laid out XCD-balanced (xcd_order).

    A group's kernels depend on its size: bf16x3 groups of at most 128
    regular row workgroups run the K-split row kernel, and groups under 8
    fits reduce the weight gradient in split-K slices.  Both
    regroup the same sums, so a fit's result can differ at the rounding level
    (|Δcos| well under 1e-4) with the chunking or the farm partition that put
    it in a smaller or larger group; `test_group_chunks_row_variant_rounding`
    pins that, `test_group_chunks_equal_one_group` the bitwise case.  Both
    choices depend on the group's shape alone (wants_split, rows_ks_for), not
    on the other groups of the job: the same group trains bitwise the same in
    a farm worker and in a single process (test_farm_lone_split_fits_bitwise).
    Records are written in the reference's order whatever the grouping:
    outputs are indexed by spec."""
    costs = [fit_flops(int(s.target.shape[0]), int(s.target.shape[1]), s.config, 1)
             for s in specs]
    keys = {}
    for i, s in enumerate(specs):
        k = (device, s.config.hidden_features, int(s.target.shape[1]),
             int(s.target.shape[0]))
        keys.setdefault(k, []).append(i)
    # Large groups are split into chunks of <= GROUP_MAX fits, each with its
    # own stream: one chunk's row kernel (MFMA/LDS-bound) then overlaps another
    # chunk's parameter kernel (HBM-bound) instead of the two alternating on
    # one stream.  Chunk sizes stay multiples of 8 so the XCD-aware block map
    # keeps every XCD busy.  Measured on the 280-fit sweep: +5 % (160-fit group
    # -> 4 x 40), with GPU_MAX_HW_QUEUES = 8 so the streams get their own queues.
    cap = int(os.environ.get("NERFHIP_GROUP_MAX", str(GROUP_MAX)))
    # per-width override, e.g. NERFHIP_GROUP_MAX_512=8 (schedule experiments)
    caps = {w: int(v) for w, v in ((int(k.rsplit("_", 1)[1]), v) for k, v in os.environ.items()
                                   if k.startswith("NERFHIP_GROUP_MAX_"))}
    # Which fits share a chunk (NERFHIP_CHUNKS):
    #   depth  (default) chunks cut from the width's fits sorted by depth,
    #          deepest first: the sweep's W = 256 group becomes one chunk of
    #          40 deep (L = 3) fits and three of 40 L = 2 fits, so no chunk's
    #          parameter grid carries dead layer-3 tiles for its L = 2 fits
    #          (the grid is n_fits x tiles(L_max));
    #   mixed  every chunk gets an equal share of each depth (dealt round
    #          robin from the depth-sorted list);
    #   spec   reference order (the round-4 plan; diagnostics).
    policy = os.environ.get("NERFHIP_CHUNKS", "depth")
    if policy not in CHUNK_POLICIES:
        raise ValueError(f"NERFHIP_CHUNKS must be one of {CHUNK_POLICIES}, got {policy!r}")
    parts = []
    for k, m in keys.items():
        if policy != "spec":
            m = sorted(m, key=lambda i: (-specs[i].config.hidden_layers, -costs[i], i))
        chunks = _chunks(m, caps.get(k[1], cap))
        if policy == "mixed" and len(chunks) > 1:
            sizes = [len(c) for c in chunks]
            dealt = [[] for _ in chunks]
            at = 0
            for i in m:
                while len(dealt[at % len(chunks)]) >= sizes[at % len(chunks)]:
                    at += 1
                dealt[at % len(chunks)].append(i)
                at += 1
            chunks = dealt
        for c in chunks:
            parts.append((k[0], c if policy == "spec" else xcd_order(c, costs)))
    # heaviest groups first: they are enqueued (and start) first
    return sorted(parts, key=lambda dm: -sum(costs[i] for i in dm[1]))


class FitJob:
    """A set of fits with every input already resident on its device.

    launch() enqueues the whole training (all groups, all epochs) and returns;
    wait() blocks; outputs() reads the results.  reset() restores the initial
    parameters so the same job can be launched again (bench.py's steps)."""

    def __init__(self, specs: list, epochs: int, lr: float = 1e-4, log_every: int = 0,
                 devices=None, split: bool = True, precision: str | None = None):
        _native.load()
        self.precision = check_precision(precision)
        if devices is None:
            devices = [resolve_device("cuda").index]
        if len(devices) != 1:
            raise ValueError("a FitJob runs on one device; farm several with run_fits("
                             "devices=[...]) / farm.run_farm (one process per GPU)")
        self.device = resolve_device(torch.device("cuda", devices[0])).index
        self.devices = [self.device]
        self.specs = specs
        self.epochs = epochs
        self.plan = plan_groups(specs, self.device)
        # (diagnostic: NERFHIP_PRIO_HEAVY=1 gives the heaviest group, the
        # sweep's critical path, a high-priority stream)
        heavy = os.environ.get("NERFHIP_PRIO_HEAVY", "0") == "1"
        self.groups = [_Group(m, specs, epochs, lr, log_every, d, split, self.precision,
                              priority=-1 if (heavy and k == 0) else 0)
                       for k, (d, m) in enumerate(self.plan)]
        G = len(self.groups)
        self._descs = (_native.NerfhipGroup * G)(*[g.desc for g in self.groups])
        self._streams = (ctypes.c_void_p * G)(*[g.stream.cuda_stream for g in self.groups])
        self.fresh = True
        self.timing = None
        self._threads, self._errors = [], {}

    def reset(self) -> None:
        for g in self.groups:
            with torch.cuda.stream(g.stream):
                g.params.copy_(g.params_init, non_blocking=True)
        self.fresh = True

    def launch(self, timed: bool = False) -> None:
        """Enqueue every group.  timed=True brackets every step-kernel launch
        with hipEvents (self.timing[i] per group; synchronises the groups)."""
        for t in self._threads:                      # a previous threaded launch
            t.join()
        if not self.fresh:
            self.reset()
        self.fresh = False
        G = len(self.groups)
        if not timed and G > 1 and LAUNCH_THREADS:
            self.timing = None
            self._threads = [threading.Thread(target=self._launch_one, args=(i,), daemon=True,
                                              name=f"nerfhip-group-{i}") for i in range(G)]
            self._errors = {}
            for t in self._threads:
                t.start()
            return
        for g in self.groups:
            g.ev_start.record(g.stream)
        if not timed:
            _native.check(_native.load().nerfhip_siren_fit(self._descs, G, self._streams))
            self.timing = None
        else:
            t = (_native.NerfhipTiming * G)()
            _native.check(_native.load().nerfhip_siren_fit_timed(self._descs, G, self._streams, t))
            self.timing = list(t)
        for g in self.groups:
            g.ev_end.record(g.stream)

    def _launch_one(self, i: int) -> None:
        g = self.groups[i]
        try:
            g.ev_start.record(g.stream)
            desc = (_native.NerfhipGroup * 1)(g.desc)
            st = (ctypes.c_void_p * 1)(g.stream.cuda_stream)
            _native.check(_native.load().nerfhip_siren_fit(desc, 1, st))
            g.ev_end.record(g.stream)
        except BaseException as e:          # re-raised by wait()
            self._errors[i] = e

    def wait(self) -> None:
        for t in self._threads:
            t.join()
        self._threads = []
        if self._errors:
            raise next(iter(self._errors.values()))
        for g in self.groups:
            g.ev_end.synchronize()

    def group_seconds(self) -> list:
        return [g.ev_start.elapsed_time(g.ev_end) / 1e3 for g in self.groups]

    def outputs(self) -> list:
        outs = [None] * len(self.specs)
        for g, gs in zip(self.groups, self.group_seconds()):
            for i, o in zip(g.members, g.outputs(self.specs, gs)):
                outs[i] = o
        return outs


class StreamingJob:
    """A one-device job whose groups launch as soon as their fits' inputs exist.

    The drop-in driver initialises its models in the reference's RNG order
    (fit.py:54-69), one after the other on the host; a FitJob would wait for
    all of them.  Here the group plan is fixed up front from each fit's
    (config, seq_len, d_head) — `plan_groups` needs nothing else — and
    `add(i, spec)` hands over fit i's target and init: the moment the last
    member of a group (a chunk of same-width fits, plan_groups) arrives, a
    launcher thread of that group packs and uploads its
    buffers and enqueues its whole training on its own stream (that call
    blocks on the stream's queue depth for most of the run), while the
    caller goes on drawing the next inits.
    `finished()` then yields groups in the order they complete, so results,
    checkpoints and progress lines can be produced while the rest still
    trains.  Results are bitwise those of a FitJob over the same groups: the
    grouping is identical and groups never interact."""

    def __init__(self, protos: list, epochs: int, lr: float = 1e-4, log_every: int = 0,
                 device=None, precision: str | None = None):
        _native.load()
        self.precision = check_precision(precision)
        self.device = resolve_device(torch.device("cuda", device) if device is not None
                                     else "cuda").index
        self.epochs, self.lr, self.log_every = epochs, lr, log_every
        self.protos = protos
        self.plan = plan_groups(protos, self.device)
        self.member_of = {i: gi for gi, (_d, m) in enumerate(self.plan) for i in m}
        self.specs = [None] * len(protos)
        self.missing = [len(m) for _d, m in self.plan]
        self.groups = [None] * len(self.plan)
        self.launch_order = []
        self._done = set()
        self._threads, self._errors = {}, {}

    def add(self, i: int, spec: FitSpec) -> None:
        p = self.protos[i]
        if spec.config != p.config or tuple(spec.target.shape) != tuple(p.target.shape):
            raise ValueError(f"fit {i}: spec does not match the planned (config, shape)")
        if self.specs[i] is not None:
            raise ValueError(f"fit {i} added twice")
        self.specs[i] = spec
        gi = self.member_of[i]
        self.missing[gi] -= 1
        if self.missing[gi] == 0:
            self._launch(gi)

    def _launch(self, gi: int) -> None:
        # Enqueueing a group's whole training (≈ 2 launches per epoch) blocks
        # once its stream's hardware queue is full, i.e. for most of the
        # group's run; from the caller's thread that would hold back every
        # later group's launch (and the next inits).  So each group is packed,
        # uploaded (on its own stream) and enqueued by a thread of its own;
        # the C call releases the GIL.
        t = threading.Thread(target=self._run, args=(gi,), name=f"nerfhip-group-{gi}",
                             daemon=True)
        self._threads[gi] = t
        self.launch_order.append(gi)
        t.start()

    def _run(self, gi: int) -> None:
        try:
            d, members = self.plan[gi]
            g = _Group(members, self.specs, self.epochs, self.lr, self.log_every, d, True,
                       self.precision)
            self.groups[gi] = g
            g.ev_start.record(g.stream)
            desc = (_native.NerfhipGroup * 1)(g.desc)
            st = (ctypes.c_void_p * 1)(g.stream.cuda_stream)
            _native.check(_native.load().nerfhip_siren_fit(desc, 1, st))
            g.ev_end.record(g.stream)
        except BaseException as e:          # re-raised by finished()
            self._errors[gi] = e

    def finished(self, poll_s: float = 0.002):
        """Yield group indices as their training completes (every group must
        have been launched, i.e. every fit added).  A group counts once its
        launcher thread is done and its end event has completed."""
        if any(m > 0 for m in self.missing):
            raise ValueError("finished() before every fit was added")
        left = [gi for gi in self.launch_order if gi not in self._done]
        while left:
            ready = []
            for gi in left:
                if self._threads[gi].is_alive():
                    continue
                if gi in self._errors:
                    self._join_all()
                    raise self._errors[gi]
                if self.groups[gi].ev_end.query():
                    ready.append(gi)
            if not ready:
                time.sleep(poll_s)
                continue
            for gi in ready:
                self._done.add(gi)
                left.remove(gi)
                yield gi

    def _join_all(self) -> None:
        for t in self._threads.values():
            t.join()

    def job_seconds(self) -> float:
        """Earliest group start to the last group's end (device clock)."""
        self._join_all()
        if not self.groups:
            return 0.0
        starts = [g.ev_start for g in self.groups]
        first = starts[0]
        for ev in starts[1:]:
            if ev.elapsed_time(first) > 0:        # ev recorded before `first`
                first = ev
        return max(first.elapsed_time(g.ev_end) for g in self.groups) / 1e3

    def outputs(self, gi: int) -> list:
        """[(fit index, FitOutput)] of finished group gi; train_time_seconds
        is the group's measured device time (FitOutput), known the moment the
        group is done."""
        g = self.groups[gi]
        gs = g.ev_start.elapsed_time(g.ev_end) / 1e3
        return list(zip(g.members, g.outputs(self.specs, gs)))


def run_fits(specs: list, epochs: int, lr: float = 1e-4, log_every: int = 0,
             devices=None, precision: str | None = None) -> list:
    """Train every FitSpec for `epochs` Adam steps; returns FitOutput per spec
    (same order).  Blocks until the device work is done.  More than one device:
    one worker process per device (farm.run_farm), outputs' params on the host."""
    if not specs:
        return []
    if devices is not None and len(devices) > 1:
        from . import farm
        return farm.run_farm(specs, epochs, list(devices), lr=lr, log_every=log_every,
                             precision=precision)
    dev = resolve_device(torch.device("cuda", devices[0]) if devices else "cuda").index
    need = [fit_device_bytes(s, epochs, log_every, precision) for s in specs]
    waves = plan_waves(need, memory_budget(dev))
    outs = [None] * len(specs)
    for wave in waves:
        job = FitJob([specs[i] for i in wave], epochs, lr, log_every, [dev], precision=precision)
        job.launch()
        job.wait()
        for i, o in zip(wave, job.outputs()):
            outs[i] = o
        del job
    return outs


def fit_device_bytes(spec: FitSpec, epochs: int, log_every: int = 0, precision=None) -> int:
    """Device bytes one fit occupies in a group (nerfhip_group_sizes buffers,
    as _Group allocates them: params_init, params, adam_m, adam_v; params_t;
    scratch; target, target_norm, eval_y; mean, std; loss partials; row_cos,
    row_sq; the split-K slab (counted even when the group does not take it);
    probes; the bf16x3 split copies; and, once per group but counted per fit,
    the positions, the schedule table and the layer / omega vectors)."""
    N, D = int(spec.target.shape[0]), int(spec.target.shape[1])
    c = spec.config
    s = _native.group_sizes(c.hidden_features, D, N, c.hidden_layers, epochs)
    n_probe = epochs // log_every if log_every > 0 else 0
    floats = (4 * s.params + s.params_t + s.scratch + 3 * s.target + 2 * s.stats
              + max(s.loss_partial, 1) + 2 * s.rows + s.grad_partial
              + n_probe * (s.target + 2 * s.rows)
              + s.rows + 2 * max(epochs, 1) + 2)
    return 4 * int(floats) + (2 * int(s.wsplit) if check_precision(precision) == "bf16x3" else 0)


def memory_budget(device: int) -> int:
    """Bytes a FitJob may allocate at once: NERFHIP_MEM_BUDGET_GB, else 60 % of
    the device's HBM (288 GB on an MI355X)."""
    env = os.environ.get("NERFHIP_MEM_BUDGET_GB")
    if env:
        return int(float(env) * 2 ** 30)
    return int(0.6 * torch.cuda.get_device_properties(device).total_memory)


def plan_waves(need: list, budget: int) -> list:
    """Consecutive runs of fit indices whose summed bytes stay within `budget`
    (a fit larger than the budget runs alone).  One wave when everything fits:
    the 280-fit sweep needs ~6.5 GB.  Waves keep spec order, so results and the
    reference's init order are unaffected (the reference's sequential loop
    runs the same selection in constant memory, fit.py:54-76)."""
    waves, cur, used = [], [], 0
    for i, b in enumerate(need):
        if cur and used + b > budget:
            waves.append(cur)
            cur, used = [], 0
        cur.append(i)
        used += b
    if cur:
        waves.append(cur)
    return waves


class ForwardPlan:
    """A SIREN forward bound to device buffers (inference; siren.py:60-61).

    Everything but the kernel launch happens once here: the padded positions,
    the flat parameter buffer, the per-fit layer/ω tables and the output live
    on the device, so __call__ is one C-ABI call (nerfhip_siren_forward) on
    torch's current stream.  `params` may hold several models of the same
    (config, d_head) as rows [m, P]: one launch evaluates them all, e.g. every
    K/V head of a layer (the decode-time regeneration the reference profiles,
    evaluate.py:173-242)."""

    def __init__(self, config: SIRENConfig, d_head: int, positions: torch.Tensor,
                 n_models: int = 1, device=None):
        dev = resolve_device(device if device is not None else positions.device)
        self.config, self.d_head, self.device = config, d_head, dev
        self.n = int(positions.numel())
        self.n_models = n_models
        s = _native.group_sizes(config.hidden_features, d_head, self.n, config.hidden_layers, 0)
        self.n_pad = int(s.n_pad)
        self.P = config.num_parameters(d_head)
        self.pos = torch.zeros(self.n_pad, dtype=torch.float32, device=dev)
        self.pos[:self.n] = positions.reshape(-1).to(dev, torch.float32)
        self.params = torch.zeros(n_models, int(s.params), dtype=torch.float32, device=dev)
        self.layers = torch.full((n_models,), config.hidden_layers, dtype=torch.int32, device=dev)
        self.omega = torch.full((n_models,), config.omega_0, dtype=torch.float32, device=dev)
        self.y = torch.empty(n_models, self.n_pad, d_head, dtype=torch.float32, device=dev)
        self.desc = _native.NerfhipGroup(
            W=config.hidden_features, D=d_head, N=self.n, n_fits=n_models,
            L_max=config.hidden_layers, epochs=0, log_every=0, device=dev.index,
            fit_layers=self.layers.data_ptr(), fit_omega=self.omega.data_ptr(),
            positions=self.pos.data_ptr(), params=self.params.data_ptr(),
            eval_y=self.y.data_ptr())
        self._lib = _native.load()

    def load(self, params: torch.Tensor) -> "ForwardPlan":
        """Copy flat state_dict-order parameters ([P] or [n_models, P]) in."""
        self.params[:, :self.P].copy_(params.detach().reshape(self.n_models, self.P))
        return self

    def __call__(self, out: torch.Tensor | None = None) -> torch.Tensor:
        """Run the forward.  Without `out` the result is a view of the plan's
        buffer [n_models, n, d_head], overwritten by the next call; `out`
        (fp32, contiguous, [n_models, n_pad, d_head]) receives it instead."""
        y = self.y if out is None else out
        if out is not None and (out.shape != self.y.shape or out.dtype != torch.float32
                                or not out.is_contiguous() or out.device != self.device):
            raise ValueError(f"out must be a contiguous fp32 {tuple(self.y.shape)} tensor "
                             f"on {self.device}")
        self.desc.eval_y = y.data_ptr()
        stream = torch.cuda.current_stream(self.device)
        _native.check(self._lib.nerfhip_siren_forward(ctypes.byref(self.desc),
                                                      stream.cuda_stream))
        return y[:, :self.n]


def forward(params: torch.Tensor, config: SIRENConfig, d_head: int,
            positions: torch.Tensor) -> torch.Tensor:
    """One-shot SIREN forward on the HIP engine (inference; siren.py:60-61).
    params: flat fp32 state_dict-order vector on a CUDA device;
    positions: [n] or [n, 1] on the same device.  Returns [n, d_head].
    For repeated calls build a ForwardPlan once."""
    plan = ForwardPlan(config, d_head, positions, 1, params.device).load(params)
    return plan()[0]
